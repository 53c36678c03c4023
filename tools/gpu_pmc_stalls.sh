# Two PMC passes over one single-batch bench run: where the per-set kernels spend their cycles.
set -o pipefail
mkdir -p gpurun_out/st
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "== pass A"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_IFETCH SQ_INSTS_VMEM -d gpurun_out/st/a -o r1 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline > gpurun_out/st/a.log 2>&1 || { tail -5 gpurun_out/st/a.log; exit 1; }
echo "== pass B"
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES -d gpurun_out/st/b -o r1 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline > gpurun_out/st/b.log 2>&1 || { tail -5 gpurun_out/st/b.log; exit 1; }
find gpurun_out/st -name "*.csv" | sort
