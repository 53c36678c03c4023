# GPU suite on the default library, then A/B: exponentiations with inline products (default) vs
# out-of-line products (build/variants/powcall.so), and roots in input order (LB_ROOT_SHUFFLE=0);
# headline + one-invalid-per-slot + latency legs at the driver's step counts.
set -o pipefail
mkdir -p gpurun_out/ab
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
LB_RUNS="${LB_RUNS:-default lib:powcall env:LB_ROOT_SHUFFLE=0 default lib:powcall env:LB_ROOT_SHUFFLE=0}" AB_FLAGS="--steps 20 --warmup 5 --legs invalid,latency" bash tools/gpu_ab_env.sh
