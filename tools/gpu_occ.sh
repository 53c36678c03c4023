# kernel trace of the default bench (6 batches in flight) for occupancy analysis
set -o pipefail
mkdir -p gpurun_out/occ
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/occ/kt -o occ --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-distinct > gpurun_out/occ/log.txt 2>&1 || { tail -20 gpurun_out/occ/log.txt; exit 1; }
find gpurun_out/occ -name "*.csv" | head
