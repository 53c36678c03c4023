# batches in flight (K) x slots per batch (B); stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/sw4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for kb in "6 3" "6 4" "4 6" "6 6" "5 4"; do
  set -- $kb
  timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --inflight $1 --slots $2 --no-cpu-baseline --no-distinct > gpurun_out/sw4/k$1_b$2.log 2>&1 || { echo "k=$1 b=$2 failed rc=$?"; grep -i "error" gpurun_out/sw4/k$1_b$2.log | head -3; exit 1; }
  echo "k=$1 b=$2 $(tail -1 gpurun_out/sw4/k$1_b$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d[\"value\"]), d[\"ms_per_step\"], d[\"batch_latency_ms\"])")"
done
