# Round-6 iteration call: the GPU test suite (-x), then an A/B of the headline (RUNS as in
# tools/gpu_r6_ab.sh), then the driver's bench line.  Each GPU step has its own limit; the first
# failure ends the script.  SKIP_TESTS / SKIP_AB / SKIP_BENCH skip a part.
set -o pipefail
R=${R:-r6}
OUT=gpurun_out/step_$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread ${TESTS:+-k "$TESTS"} > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
  echo "== tests: $(tail -1 $OUT/pytest.log)"
fi
if [ -z "$SKIP_AB" ] && [ -n "$RUNS" ]; then
  R=$R bash tools/gpu_r6_ab.sh || exit 1
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 900 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
  tail -1 $OUT/bench.log > $OUT/bench_line.json; echo "== bench"; python3 tools/bench_summary.py $OUT/bench_line.json
fi
