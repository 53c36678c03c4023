# 8 batches in flight with the one-lane per-root forms off (LB_MILLER_FORM=g8, no one-lane cofactor
# clearing): every HIP queue's scratch counts against one per-process pool, sized by the largest
# private segment the queue has run.
set -o pipefail
mkdir -p gpurun_out/ab
for k in ${KS:-8}; do
  LB_MILLER_FORM=g8 LB_HASH_G8_MAX=1000000000 LB_MAX_ENGINES_PER_DEVICE=$k timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --inflight $k --no-distinct --no-cpu-baseline --legs invalid > gpurun_out/ab/inflight${k}_g8.log 2>&1; rc=$?
  echo "== $k in flight (g8 forms): rc=$rc OUT_OF_RESOURCES lines: $(grep -c OUT_OF_RESOURCES gpurun_out/ab/inflight${k}_g8.log)"
  [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/ab/inflight${k}_g8.log | python3 tools/bench_summary.py | grep -E "^value"
done
