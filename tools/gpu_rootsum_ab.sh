# root-level search rounds (LB_SEARCH_ROOTSUM=0/1): search GPU tests, the search trace on
# c3_invalid, then the bench's invalid leg
set -o pipefail
mkdir -p gpurun_out/rootsum
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "search or bisection or shared_roots or invalid or fallback" > gpurun_out/rootsum/pytest.log 2>&1 || { tail -30 gpurun_out/rootsum/pytest.log; exit 1; }
tail -2 gpurun_out/rootsum/pytest.log
for m in 0 1; do
  echo "== LB_SEARCH_ROOTSUM=$m"
  LB_SEARCH_ROOTSUM=$m timeout -k 10 240 python -u tools/prof_invalid.py 6 3 > gpurun_out/rootsum/prof_$m.log 2>&1 || { tail -20 gpurun_out/rootsum/prof_$m.log; exit 1; }
  grep -E "search|c3_invalid" gpurun_out/rootsum/prof_$m.log
done
LB_RUNS="env:LB_SEARCH_ROOTSUM=0 env:LB_SEARCH_ROOTSUM=1 env:LB_SEARCH_ROOTSUM=0 env:LB_SEARCH_ROOTSUM=1" bash tools/gpu_ab_env.sh
