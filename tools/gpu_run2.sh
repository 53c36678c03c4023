set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "== bench"; timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1; rc=$?; tail -3 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
echo "== rocprof"; timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r1 -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$?; tail -3 gpurun_out/prof.log; find gpurun_out/prof -name "*stats*" | head; exit $rc
