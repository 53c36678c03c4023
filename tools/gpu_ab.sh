# A/B over (library variant, batches in flight, slots per batch): LB_RUNS="default:4:6 msm2:6:3"
set -o pipefail
mkdir -p gpurun_out/ab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in $LB_RUNS; do
  IFS=: read -r v k sl <<< "$r"; sl=${sl:-6}
  if [ "$v" = default ]; then unset LODESTAR_BLS_LIB; else export LODESTAR_BLS_LIB=$GRAFT_REPO_ROOT/build/variants/$v.so; fi
  timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 --inflight $k --slots $sl --no-cpu-baseline --no-distinct > gpurun_out/ab/${v}_${k}_$sl.log 2>&1 || { tail -5 gpurun_out/ab/${v}_${k}_$sl.log; exit 1; }
  echo "== $v inflight=$k slots=$sl"; tail -1 gpurun_out/ab/${v}_${k}_$sl.log | python3 tools/bench_summary.py
done
