# GPU tests, then the latency / per-config legs for each RUNS entry (tools/gpu_r5_ab.sh with
# LEGS=latency,configs at 5 steps), then (if CAP) the engine cap at 16 with the distinct-roots leg.
set -o pipefail
if [ -z "$SKIP_TESTS" ]; then
  mkdir -p gpurun_out/quick
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/quick/pytest.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/quick/pytest.log | head -20; tail -30 gpurun_out/quick/pytest.log; exit 1; }
  echo "== tests: $(tail -1 gpurun_out/quick/pytest.log)"
fi
LEGS=${LEGS:-latency,configs} STEPS=${STEPS:-5} NLINES=${NLINES:-14} bash tools/gpu_r5_ab.sh || exit 1
if [ -n "$CAP" ]; then
  mkdir -p gpurun_out/cap
  LB_MAX_ENGINES_PER_DEVICE=16 timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 --inflight 16 --no-cpu-baseline --legs roots > gpurun_out/cap/inflight16.log 2>&1 || { tail -20 gpurun_out/cap/inflight16.log; exit 1; }
  echo "== 16 engines"; tail -1 gpurun_out/cap/inflight16.log | python3 tools/bench_summary.py | head -4
fi
