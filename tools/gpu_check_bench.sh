# GPU parity tests, fp_mul micro-benchmark, then the bench at the default and at 6 batches in flight.
set -o pipefail
mkdir -p gpurun_out
echo "== pytest"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== fpmul"; timeout -k 10 120 tools/ubench/fpmul_asm || exit $?
for cfg in ${LB_CFGS:-4:2 16:6}; do
  set -- ${cfg/:/ }
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 240 python -u bench.py --steps 6 --warmup 1 --inflight $2 --no-cpu-baseline > gpurun_out/bench_q$1_k$2.log 2>&1 || exit $?
  echo "q=$1 k=$2 $(tail -1 gpurun_out/bench_q$1_k$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), round(d["value_one_batch_in_flight"]), {k: v["ms"] for k, v in r["stages"].items()})')"
done
