# A/B of one engine environment setting (AB="NAME=value") against the default on the headline and
# every-root-distinct legs: two runs each, alternating.
set -o pipefail
OUT=gpurun_out/envab_${R:-r6}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for it in 1 2; do
  for f in default ab; do
    if [ $f = default ]; then E=""; else E="$AB"; fi
    timeout -k 10 300 env $E python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --legs none > $OUT/$f.$it.log 2>&1 || { tail -20 $OUT/$f.$it.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', round(d['value']/1e6,3), 'distinct', round((d.get('value_distinct_roots') or 0)/1e6,3))" $OUT/$f.$it.log "$f.$it $E"
  done
done
