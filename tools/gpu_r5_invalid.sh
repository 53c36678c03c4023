# The invalid-set leg on the driver's flags, with the search's per-round trace (LB_SEARCH_TRACE)
set -o pipefail
mkdir -p gpurun_out/inv
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LB_SEARCH_TRACE=1 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-distinct --legs invalid > gpurun_out/inv/bench.log 2> gpurun_out/inv/trace.log || { tail -20 gpurun_out/inv/bench.log gpurun_out/inv/trace.log; exit 1; }
tail -1 gpurun_out/inv/bench.log | python3 tools/bench_summary.py | head -8
grep "lb search" gpurun_out/inv/trace.log | tail -12
