# Library variants (build/variants/NAME.so from tools/build_variant.sh NAME -DFLAG=...) and env
# knobs: the golden + kernel-forms + search GPU tests under each, then the headline bench A/B at
# the driver's step counts.  VARS="sub2 ps2" LB_RUNS="default lib:sub2 env:LB_SEARCH_BLOCKS=0"
# LEGS="invalid,latency".  Every GPU step has its own time limit; the first failure ends it.
set -o pipefail
mkdir -p gpurun_out/var
for v in ${VARS:-}; do
  LODESTAR_BLS_LIB=$GRAFT_REPO_ROOT/build/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "golden or forms or search" > gpurun_out/var/pytest_$v.log 2>&1 || { echo "tests FAILED for $v"; tail -30 gpurun_out/var/pytest_$v.log; exit 1; }
  echo "== tests $v: $(tail -1 gpurun_out/var/pytest_$v.log)"
done
runs=${LB_RUNS:-default}
[ -z "${LB_RUNS:-}" ] && for v in ${VARS:-}; do runs="$runs lib:$v"; done
if [ -n "${LEGS:-}" ]; then legs="--legs $LEGS"; else legs="--no-extra"; fi
LB_RUNS="$runs" AB_FLAGS="--steps 20 --warmup 5 $legs" bash tools/gpu_ab_env.sh
