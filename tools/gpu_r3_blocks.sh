# Search first-round forms: GPU search tests, a traced invalid batch per form, then the
# one-invalid-per-slot throughput A/B at 7 in flight (driver step counts).
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "search or invalid or bisection or fallback or forms" > gpurun_out/pytest_search.log 2>&1 || { tail -30 gpurun_out/pytest_search.log; exit 1; }
echo "== tests: $(tail -1 gpurun_out/pytest_search.log)"
for f in 1 0; do
  LB_SEARCH_BLOCKS=$f LB_SEARCH_TRACE=1 timeout -k 10 200 python -u tools/prof_invalid.py 6 2 > gpurun_out/ab/trace_blocks$f.log 2>&1 || { tail -20 gpurun_out/ab/trace_blocks$f.log; exit 1; }
  echo "== trace LB_SEARCH_BLOCKS=$f"; grep -E "lb search|search" gpurun_out/ab/trace_blocks$f.log | tail -12
done
LB_RUNS="${LB_RUNS:-default env:LB_SEARCH_BLOCKS=0 default}" AB_FLAGS="--steps 20 --warmup 5 --legs invalid" bash tools/gpu_ab_env.sh
