# round-2 check: GPU tests, default bench, 8 batches in flight once, wave phase timing
set -o pipefail
mkdir -p gpurun_out
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python3 tools/bench_summary.py
echo "== bench 8 in flight"; timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --inflight 8 --no-cpu-baseline --no-distinct > gpurun_out/bench8.log 2>&1 || { tail -5 gpurun_out/bench8.log; exit 1; }
tail -1 gpurun_out/bench8.log | python3 tools/bench_summary.py
echo "== wave phase"; timeout -k 10 60 ./tools/ubench/wave_phase
