# Field-product microbench, then each library variant (build/variants/*.so from
# tools/build_variant.sh) through the golden + kernel-forms GPU tests with the one-lane subgroup
# check forced, then the headline bench A/B at the driver's step counts.
set -o pipefail
mkdir -p gpurun_out/var
VARS=${VARS:-"sub2 ps2 sl sub2ps2"}
if [ -x tools/ubench/fpmul_ps ]; then echo "== fpmul_ps"; timeout -k 5 120 ./tools/ubench/fpmul_ps || exit 1; fi
for v in $VARS; do
  LODESTAR_BLS_LIB=$GRAFT_REPO_ROOT/build/variants/$v.so LB_SUBGROUP_G8_MAX=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "golden or forms" > gpurun_out/var/pytest_$v.log 2>&1 || { echo "tests FAILED for $v"; tail -30 gpurun_out/var/pytest_$v.log; exit 1; }
  echo "== tests $v: $(tail -1 gpurun_out/var/pytest_$v.log)"
done
runs="default"; for v in $VARS; do runs="$runs lib:$v"; done
LB_RUNS="$runs" AB_FLAGS="--steps 20 --warmup 5 --no-extra" bash tools/gpu_ab_env.sh
