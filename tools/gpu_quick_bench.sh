# GPU tests + one bench (stage times at one batch in flight + throughput); no CPU baseline.
set -o pipefail
mkdir -p gpurun_out/qb
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/qb/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/qb/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/qb/pytest_gpu.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/qb/bench.log 2>&1 || { tail -20 gpurun_out/qb/bench.log; exit 1; }
tail -1 gpurun_out/qb/bench.log | python3 tools/bench_summary.py
