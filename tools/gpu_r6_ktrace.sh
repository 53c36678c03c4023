# Kernel trace of the latency legs (1-set, C2 block) at one batch in flight: median duration per
# (kernel, grid) into gpurun_out/kt_$R/kernels.txt.
set -o pipefail
R=${R:-r6}
OUT=gpurun_out/kt_$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o lat -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --slots 1 --no-cpu-baseline --no-distinct --legs ${LEGS:-latency} > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
trace=$(find $OUT/tr -name "*kernel_trace.csv" | head -1)
python3 tools/trace_kernels.py "$trace" > $OUT/kernels.txt
python3 tools/trace_kernels.py "$trace" | awk '$3 < 2000' | head -80
