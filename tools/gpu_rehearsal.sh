# Multi-rank rehearsal on ONE GPU (no 8-GPU node is ours to launch): 2 ranks sharing device 0 with
# a gloo control plane, weak-scaling mode and --exchange mode (576-byte partial all-gather + one
# final exponentiation per step, batches in flight) at the same in-flight count.
set -o pipefail
mkdir -p gpurun_out/rehearsal
F="--gpus 2 --steps ${STEPS:-5} --warmup 1 --inflight ${INFLIGHT:-3} --no-cpu-baseline --no-distinct --no-extra"
for mode in weak exchange; do
  x=""; [ $mode = exchange ] && x="--exchange"
  LB_BENCH_BACKEND=gloo LB_BENCH_DEVICE=0 timeout -k 10 300 python -u bench.py $F $x > gpurun_out/rehearsal/$mode.log 2>&1 || { tail -20 gpurun_out/rehearsal/$mode.log; exit 1; }
  echo "== $mode"; grep -h '"metric"' gpurun_out/rehearsal/$mode.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['inflight'], d['config']['exchange'], d['config']['world_size_seen'])"
done
