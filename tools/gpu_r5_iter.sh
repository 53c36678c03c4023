# tests (unless SKIP_TESTS), then an A/B of the headline (RUNS, tools/gpu_r5_ab.sh), then the
# latency legs (tools/gpu_quick.sh without tests)
set -o pipefail
if [ -z "$SKIP_TESTS" ]; then
  mkdir -p gpurun_out/quick
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/quick/pytest.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/quick/pytest.log | head -20; tail -30 gpurun_out/quick/pytest.log; exit 1; }
  echo "== tests: $(tail -1 gpurun_out/quick/pytest.log)"
fi
[ -n "$RUNS" ] && { bash tools/gpu_r5_ab.sh || exit 1; }
SKIP_TESTS=1 bash tools/gpu_quick.sh
