# A/B of the per-config and latency legs (one bench process per setting): RUNS="default env:K=V ..."
set -o pipefail
OUT=gpurun_out/cfgab_${R:-r6}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for r in $RUNS; do
  i=$((i+1))
  envs=""
  case "$r" in env:*) envs="${r#env:}"; envs=${envs//+/ } ;; esac
  env $envs timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-3} --warmup 1 --inflight ${INFL:-7} --no-cpu-baseline --no-distinct --legs ${LEGS:-latency,configs} > $OUT/$i.log 2>&1 || { tail -5 $OUT/$i.log; exit 1; }
  tail -1 $OUT/$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
pc=d.get('per_config') or {}
print('== $r', 'value', round(d['value']/1e6,3), '1set', d.get('latency_1set_ms'), 'block', d.get('latency_block_ms'), 'slot', d.get('latency_slot1_ms'), {c: x['ms_per_batch'] for c,x in pc.items()})"
done
