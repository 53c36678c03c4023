# GPU test suite, then the invalid-set search forms at the driver's step counts (one wrong
# attestation per slot, 7 batches in flight), then one run at 8 batches in flight with the engine
# cap raised (the round-2 queue abort).
set -o pipefail
mkdir -p gpurun_out/ab
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
LB_RUNS="${LB_RUNS:-default env:LB_SEARCH_ROOTSUM=0 env:LB_SEARCH_MERGE=0 env:LB_SEARCH_ROOTSUM=0+LB_SEARCH_MERGE=0}" AB_FLAGS="--steps 20 --warmup 5 --legs invalid" bash tools/gpu_ab_env.sh || exit 1
echo "== 8 in flight"; LB_MAX_ENGINES_PER_DEVICE=8 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --inflight 8 --no-extra --no-distinct --no-cpu-baseline > gpurun_out/ab/inflight8.log 2>&1; rc=$?
grep -c "OUT_OF_RESOURCES" gpurun_out/ab/inflight8.log; [ $rc -eq 0 ] && tail -1 gpurun_out/ab/inflight8.log | python3 tools/bench_summary.py | head -2
exit $rc
