# Round-4 A/B: library variants and engine counts on the driver's bench flags (headline + the
# distinct-root leg), RUNS="default lib:millreg default@8 env:LB_MILLER_FORM=g8" (name@N: N in
# flight).  Every GPU step has its own limit; the first failure ends the script.
set -o pipefail
OUT=gpurun_out/ab_${R:-r4}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in $RUNS; do
  unset LODESTAR_BLS_LIB
  envs=""
  base=${r%@*}; inf=7
  [ "$base" != "$r" ] && inf=${r#*@}
  case "$base" in
    env:*) envs="${base#env:}"; envs=${envs//+/ } ;;
    lib:*) export LODESTAR_BLS_LIB=$GRAFT_REPO_ROOT/build/variants/${base#lib:}.so ;;
  esac
  tag=$(echo "$r" | tr ':=/@+' '_____')
  if [ -n "$LEGS" ]; then legs="--legs $LEGS"; else legs="--no-extra"; fi
  env LB_MAX_ENGINES_PER_DEVICE=16 $envs timeout -k 10 300 python3 -u bench.py --inflight $inf --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline $legs > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  echo "== $r"; tail -1 $OUT/$tag.log | python3 tools/bench_summary.py
done
