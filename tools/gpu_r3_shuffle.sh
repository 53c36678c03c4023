# Root numbering A/B (hash-table order vs input order): search-form GPU tests, then the headline
# and one-invalid-per-slot legs at the driver's step counts, alternating.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "forms or search" > gpurun_out/pytest_forms.log 2>&1 || { tail -30 gpurun_out/pytest_forms.log; exit 1; }
echo "== tests: $(tail -1 gpurun_out/pytest_forms.log)"
LB_RUNS="${LB_RUNS:-default env:LB_ROOT_SHUFFLE=0 default env:LB_ROOT_SHUFFLE=0}" AB_FLAGS="--steps 20 --warmup 5 --legs invalid" bash tools/gpu_ab_env.sh
