# VALU instructions per kernel at the headline configuration (7 in flight) for the round-3 tree
# (build/r3tree) and the current tree: the per-batch instruction budget side by side.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r3pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PM="--steps 2 --warmup 1 --no-cpu-baseline --no-distinct --no-extra"
(cd build/r3tree && timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $OUT/r3 -o r3 --output-format csv -- python3 bench.py $PM > $OUT/r3.log 2>&1) || { tail -5 $OUT/r3.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $OUT/r4 -o r4 --output-format csv -- python3 bench.py $PM > $OUT/r4.log 2>&1 || { tail -5 $OUT/r4.log; exit 1; }
echo done
