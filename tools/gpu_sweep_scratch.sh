# in-flight batches with a larger device scratch pool (HSA_SCRATCH_MEM); stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/sw2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_SCRATCH_MEM=${SCR:-34359738368}
for qk in "32 8" "32 10" "32 12" "32 16"; do
  set -- $qk
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 200 python -u bench.py --steps 6 --warmup 1 --inflight $2 --no-cpu-baseline --no-distinct > gpurun_out/sw2/q$1_k$2.log 2>&1 || { echo "q=$1 k=$2 failed rc=$?"; grep -v "^ " gpurun_out/sw2/q$1_k$2.log | grep -i "error\|limit" | head -5; exit 1; }
  echo "q=$1 k=$2 $(tail -1 gpurun_out/sw2/q$1_k$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["value_one_batch_in_flight"]))')"
done
