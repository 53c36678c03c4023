set -o pipefail
mkdir -p gpurun_out
echo "== ubench"; timeout -k 10 120 ./tools/ubench_int > gpurun_out/ubench.json 2>&1; cat gpurun_out/ubench.json
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -3
echo "== bench"; timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; tail -5 gpurun_out/bench.log; exit $rc
