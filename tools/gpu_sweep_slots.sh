# batches in flight (K) x slots per batch (B), 16 HW queues; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/sw3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for kb in "6 1" "4 2" "6 2" "3 4" "4 4" "6 3"; do
  set -- $kb
  timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --inflight $1 --slots $2 --no-cpu-baseline --no-distinct > gpurun_out/sw3/k$1_b$2.log 2>&1 || { echo "k=$1 b=$2 failed rc=$?"; grep -i "error" gpurun_out/sw3/k$1_b$2.log | head -3; exit 1; }
  echo "k=$1 b=$2 $(tail -1 gpurun_out/sw3/k$1_b$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["value_one_batch_in_flight"]), d["ms_per_step"])')"
done
