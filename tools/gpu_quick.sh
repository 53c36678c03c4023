# Quick A/B pass: wave-engine phase timing, GPU tests, the default bench without the slow legs
set -o pipefail
mkdir -p gpurun_out
echo "== wave phase"; timeout -k 5 60 ./tools/ubench/wave_phase && timeout -k 5 60 ./tools/ubench/lin_bench || exit 1
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
echo "== bench"; timeout -k 10 600 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python3 tools/bench_summary.py
