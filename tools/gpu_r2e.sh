# GPU tests, then the invalid-search profile
set -o pipefail
mkdir -p gpurun_out
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
echo "== invalid search"; timeout -k 10 300 python -u tools/prof_invalid.py 6 3 2>&1 | tee gpurun_out/prof_invalid.log
