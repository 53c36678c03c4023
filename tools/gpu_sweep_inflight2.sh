set -o pipefail
mkdir -p gpurun_out
for q in 16 32; do
  for k in 6 8 12 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u bench.py --steps 6 --warmup 1 --inflight $k --no-cpu-baseline > gpurun_out/sweep2_q${q}_k${k}.log 2>&1 || exit $?
    echo "q=$q k=$k $(tail -1 gpurun_out/sweep2_q${q}_k${k}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["value_one_batch_in_flight"]))')"
  done
done
