# full default bench (all legs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py "$@" > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for k in ['value','value_one_batch_in_flight','value_distinct_roots','value_one_invalid_per_batch','value_slots1','latency_slot1_ms','latency_1set_ms','latency_block_ms','value_dropin','batch_latency_ms']: print(k, d.get(k))
print('invalid stages', d.get('invalid_batch_stage_ms'))
print('per_config', {k: (v['ms_per_batch'], v['sets_per_s']) for k, v in d.get('per_config', {}).items()})
print('cpu', d.get('cpu_baseline', {}).get('value'), 'cpu_c1', (d.get('cpu_c1') or {}).get('value'))
"
