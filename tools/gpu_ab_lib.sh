# A/B: default library vs an alternative build (LODESTAR_BLS_LIB) at 6 batches in flight.
set -o pipefail
mkdir -p gpurun_out
for v in default $LB_VARIANTS; do
  if [ "$v" = default ]; then unset LODESTAR_BLS_LIB; else export LODESTAR_BLS_LIB=$GRAFT_REPO_ROOT/build/variants/$v.so; fi
  for k in 1 6; do
    timeout -k 10 240 python -u bench.py --steps 6 --warmup 1 --inflight $k --no-cpu-baseline > gpurun_out/ab_${v}_k$k.log 2>&1 || { tail -5 gpurun_out/ab_${v}_k$k.log; exit 1; }
    echo "$v k=$k $(tail -1 gpurun_out/ab_${v}_k$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), {k: v["ms"] for k, v in r["stages"].items()})')"
  done
done
