# Round-6 A/B on the driver's bench flags (headline, 7 in flight, 20 steps): RUNS="default lib:NAME
# env:K=V ..." (lib: build/variants/NAME.so through LODESTAR_BLS_LIB).  Every GPU step has its own
# limit; the first failure ends the script.
set -o pipefail
OUT=gpurun_out/ab_${R:-r6}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for r in $RUNS; do
  i=$((i+1))
  unset LODESTAR_BLS_LIB
  envs=""
  case "$r" in
    env:*) envs="${r#env:}"; envs=${envs//+/ } ;;
    lib:*) export LODESTAR_BLS_LIB=$GRAFT_REPO_ROOT/build/variants/${r#lib:}.so ;;
  esac
  tag=$i_$(echo "$r" | tr ':=/@+' '_____')
  if [ -n "$LEGS" ]; then legs="--legs $LEGS"; else legs="--no-extra"; fi
  env $envs timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline ${BENCH_FLAGS:---no-distinct} $legs > $OUT/$i.$tag.log 2>&1 || { tail -5 $OUT/$i.$tag.log; exit 1; }
  echo "== $r"; tail -1 $OUT/$i.$tag.log | python3 tools/bench_summary.py > $OUT/$i.summary.txt; head -${NLINES:-3} $OUT/$i.summary.txt
done
