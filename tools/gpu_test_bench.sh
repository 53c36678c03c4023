# GPU tests, then a short bench (no CPU baseline).
set -o pipefail
mkdir -p gpurun_out/tb
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tb/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/tb/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/tb/pytest_gpu.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/tb/bench.log 2>&1 || { tail -20 gpurun_out/tb/bench.log; exit 1; }
tail -1 gpurun_out/tb/bench.log
