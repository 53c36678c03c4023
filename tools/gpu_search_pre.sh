# search with kept per-set terms: search GPU tests, the search trace, the kernel stats, the bench
set -o pipefail
mkdir -p gpurun_out/pre
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LB_SEARCH_PRE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "search or bisection or shared_roots or invalid or fallback" > gpurun_out/pre/pytest.log 2>&1 || { tail -30 gpurun_out/pre/pytest.log; exit 1; }
tail -2 gpurun_out/pre/pytest.log
LB_SEARCH_PRE=1 timeout -k 10 240 python -u tools/prof_invalid.py 6 3 > gpurun_out/pre/prof.log 2>&1 || { tail -20 gpurun_out/pre/prof.log; exit 1; }
grep -E "search|c3_invalid" gpurun_out/pre/prof.log
LB_RUNS="default env:LB_SEARCH_PRE=1" bash tools/gpu_ab_env.sh
