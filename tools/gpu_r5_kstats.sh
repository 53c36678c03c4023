# rocprofv3 kernel statistics at the headline configuration (7 in flight) for the default library
# and each variant in VARIANTS (build/variants/NAME.so): where the time per batch goes.
set -o pipefail
OUT=gpurun_out/kstats
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in default $VARIANTS; do
  unset LODESTAR_BLS_LIB
  [ "$v" != default ] && export LODESTAR_BLS_LIB=$GRAFT_REPO_ROOT/build/variants/$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o $v --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-distinct --no-extra > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
  echo "== $v $(tail -1 $OUT/$v.log | cut -c1-120)"
done
