# Quick GPU check after a kernel change: the GPU test suite (first failure stops it) and the
# latency / one-batch legs of the bench line.  Each step bounded; the first failure ends the script.
set -o pipefail
OUT=gpurun_out/quick
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
  echo "== tests: $(tail -1 $OUT/pytest.log)"
fi
timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-distinct --legs ${LEGS:-latency,slots1} > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log > $OUT/bench_line.json; python3 tools/bench_summary.py $OUT/bench_line.json
