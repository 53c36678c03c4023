# invalid-set search profile: stage times, search rounds, rocprofv3 kernel stats
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/prof_invalid.py 6 3 2>&1 | tee gpurun_out/prof_invalid.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_inv -o run --output-format csv -- python3 tools/prof_invalid.py 6 1 > gpurun_out/prof_inv_rocprof.log 2>&1 &&
f=$(find gpurun_out/prof_inv -name '*kernel_stats.csv' | head -1) && python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:25]: print(x['Name'][:60].ljust(60), x['Calls'].rjust(6), '%.3f ms avg'%(float(x['AverageNs'])/1e6), '%.2f ms tot'%(float(x['TotalDurationNs'])/1e6))
"
