# GPU suite, the traced invalid-batch search, then the one-invalid-per-slot A/B at the driver's
# step counts.
set -o pipefail
mkdir -p gpurun_out/ab
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python -u tools/prof_invalid.py 6 3 > gpurun_out/prof_invalid.log 2>&1 || { tail -20 gpurun_out/prof_invalid.log; exit 1; }
cat gpurun_out/prof_invalid.log
LB_RUNS="${LB_RUNS:-default}" AB_FLAGS="--steps 20 --warmup 5 --legs invalid" bash tools/gpu_ab_env.sh
