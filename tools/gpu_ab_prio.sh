# A/B: s1 stream priority (LB_S1_PRIORITY) on the full bench
set -o pipefail
mkdir -p gpurun_out
for P in 0 1; do
  echo "== LB_S1_PRIORITY=$P"
  LB_S1_PRIORITY=$P timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench_prio$P.log 2>&1 || { tail -20 gpurun_out/bench_prio$P.log; exit 1; }
  tail -1 gpurun_out/bench_prio$P.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for k in ['value','value_one_batch_in_flight','value_distinct_roots','value_one_invalid_per_batch','value_slots1','latency_1set_ms','value_dropin','batch_latency_ms']: print(k, d.get(k))
"
done
