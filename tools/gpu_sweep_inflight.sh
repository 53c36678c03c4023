# Sweep batches-in-flight x HIP hardware queues (GPU_MAX_HW_QUEUES, HIP's per-process queue count;
# each engine uses two streams).  Also covers the Jacobi is_square change via the GPU parity tests.
set -o pipefail
mkdir -p gpurun_out
echo "== pytest"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for q in 4 8 16; do
  for k in 2 3 4 6; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u bench.py --steps 6 --warmup 1 --inflight $k --no-cpu-baseline > gpurun_out/sweep_q${q}_k${k}.log 2>&1 || exit $?
    echo "q=$q k=$k $(tail -1 gpurun_out/sweep_q${q}_k${k}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["value_one_batch_in_flight"]))')"
  done
done
