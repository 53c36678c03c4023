set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "== kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o r1 --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof/kt.log 2>&1 || { tail -20 gpurun_out/prof/kt.log; exit 1; }
tail -1 gpurun_out/prof/kt.log | head -c 300; echo
find gpurun_out/prof/kt -name "*stats*"
echo "== pmc: valu"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/prof/pmc1 -o r1 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof/pmc1.log 2>&1 || { tail -5 gpurun_out/prof/pmc1.log; }
echo "== pmc: hbm"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d gpurun_out/prof/pmc2 -o r1 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof/pmc2.log 2>&1 || { tail -5 gpurun_out/prof/pmc2.log; }
find gpurun_out/prof -name "*.csv" | head -20
