# Kernel-forms GPU test, then the headline bench at the driver's step counts with the Miller form
# chosen by device load (default), pinned to one lane per root, and pinned to 8 lanes per root.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -k "forms" > gpurun_out/pytest_forms.log 2>&1 || { tail -30 gpurun_out/pytest_forms.log; exit 1; }
tail -2 gpurun_out/pytest_forms.log
LB_RUNS="${LB_RUNS:-default env:LB_MILLER_FORM=lane env:LB_MILLER_FORM=g8}" AB_FLAGS="--steps 20 --warmup 5 --no-extra" bash tools/gpu_ab_env.sh
