# GPU tests, the invalid-set search profile, then the full default bench (all legs).
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
echo "== invalid search"; timeout -k 10 300 python -u tools/prof_invalid.py 6 3 > gpurun_out/prof_invalid.log 2>&1 || { tail -20 gpurun_out/prof_invalid.log; exit 1; }
tail -5 gpurun_out/prof_invalid.log
bash tools/gpu_bench.sh "$@"
