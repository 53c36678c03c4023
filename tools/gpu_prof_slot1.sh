# rocprofv3 kernel trace of one-slot batches, one in flight (the latency-bound configuration)
set -o pipefail
mkdir -p gpurun_out/prof_slot1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_slot1 -o run --output-format csv -- python3 bench.py --slots 1 --inflight 1 --steps 10 --warmup 2 --no-extra --no-distinct --no-cpu-baseline > gpurun_out/prof_slot1/bench.log 2>&1 || { tail -20 gpurun_out/prof_slot1/bench.log; exit 1; }
f=$(find gpurun_out/prof_slot1 -name '*kernel_stats.csv' | head -1) && python3 -c "
import csv
r=list(csv.DictReader(open('$f')))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:40]: print(x['Name'][:60].ljust(60), x['Calls'].rjust(6), '%.3f ms avg'%(float(x['AverageNs'])/1e6), '%.2f ms tot'%(float(x['TotalDurationNs'])/1e6))
"
