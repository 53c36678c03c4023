# grouped Miller microbench, GPU tests, then the default bench without the CPU baseline.
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
echo "== group miller"; timeout -k 5 120 ./tools/ubench/group_miller 6918 || exit 1
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
echo "== bench"; timeout -k 10 900 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python3 tools/bench_summary.py
