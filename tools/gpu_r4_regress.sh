# Round-4 headline regression hunt: knobs of the current build against the round-3 tree, one box.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/regress
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in $RUNS; do
  unset LODESTAR_BLS_LIB
  envs=""
  case "$r" in
    r3) (cd build/r3tree && timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $OUT/r3.log 2>&1) || { tail -5 $OUT/r3.log; exit 1; }
        echo "== r3"; tail -1 $OUT/r3.log | python3 tools/bench_summary.py; continue ;;
    env:*) envs="${r#env:}"; envs=${envs//+/ } ;;
    lib:*) export LODESTAR_BLS_LIB=$GRAFT_REPO_ROOT/build/variants/${r#lib:}.so ;;
  esac
  tag=$(echo "$r" | tr ':=/@+' '_____')
  env $envs timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  echo "== $r"; tail -1 $OUT/$tag.log | python3 tools/bench_summary.py
done
