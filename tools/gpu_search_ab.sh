# A/B of the merged search round (LB_SEARCH_MERGE=0/1): search-round latency, then the bench's
# invalid-batch throughput leg
set -o pipefail
mkdir -p gpurun_out/search_ab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in 0 1; do
  echo "== LB_SEARCH_MERGE=$m"
  LB_SEARCH_MERGE=$m timeout -k 10 240 python -u tools/prof_invalid.py 6 3 > gpurun_out/search_ab/prof_$m.log 2>&1 || { tail -20 gpurun_out/search_ab/prof_$m.log; exit 1; }
  grep -E "search|c3_invalid" gpurun_out/search_ab/prof_$m.log
done
LB_RUNS="env:LB_SEARCH_MERGE=0 env:LB_SEARCH_MERGE=1 env:LB_SEARCH_MERGE=0 env:LB_SEARCH_MERGE=1" bash tools/gpu_ab_env.sh
