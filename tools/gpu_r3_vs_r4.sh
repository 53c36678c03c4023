# Headline A/B against the round-3 tree (build/r3tree: git archive of the round-3 commit with its own
# library built in place), alternating r3 / r4 runs of each tree's own bench.py on one box.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r3cmp
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for k in 1 2; do
  (cd build/r3tree && timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $OUT/r3_$k.log 2>&1) || { tail -5 $OUT/r3_$k.log; exit 1; }
  echo "== r3 run $k"; tail -1 $OUT/r3_$k.log | python3 tools/bench_summary.py
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $OUT/r4_$k.log 2>&1 || { tail -5 $OUT/r4_$k.log; exit 1; }
  echo "== r4 run $k"; tail -1 $OUT/r4_$k.log | python3 tools/bench_summary.py
done
