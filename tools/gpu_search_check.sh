# search changes: the search GPU tests, the search trace on c3_invalid, then the default bench
set -o pipefail
mkdir -p gpurun_out/search
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "search or bisection or shared_roots or invalid or fallback" > gpurun_out/search/pytest.log 2>&1 || { tail -30 gpurun_out/search/pytest.log; exit 1; }
tail -3 gpurun_out/search/pytest.log
timeout -k 10 240 python -u tools/prof_invalid.py 6 3 > gpurun_out/search/prof.log 2>&1 || { tail -20 gpurun_out/search/prof.log; exit 1; }
grep -E "search|c3_invalid" gpurun_out/search/prof.log
LB_RUNS="default default" bash tools/gpu_ab_env.sh
