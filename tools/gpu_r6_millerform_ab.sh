# A/B of the per-root Miller form under load (LB_MILLER_FORM: default by device load, lane, g8)
# on the headline and every-root-distinct legs: two runs each, alternating.
set -o pipefail
OUT=gpurun_out/mf_${R:-r6}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for it in 1 2; do
  for f in default g8; do
    if [ $f = default ]; then unset LB_MILLER_FORM; else export LB_MILLER_FORM=$f; fi
    timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --legs none > $OUT/$f.$it.log 2>&1 || { tail -20 $OUT/$f.$it.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', round(d['value']/1e6,3), 'distinct', round((d.get('value_distinct_roots') or 0)/1e6,3))" $OUT/$f.$it.log $f.$it
  done
done
