# Round-4 check: GPU test suite, the driver's default bench line, a headline kernel trace, then
# (last, since it may abort its queue) the 8-engine bench.  Each GPU step has its own limit; the
# first failure ends the script.
set -o pipefail
R=${R:-r4}
OUT=gpurun_out/chk_$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "== KFD scratch properties"
for f in /sys/class/kfd/kfd/topology/nodes/*/properties; do grep -i -E "scratch|max_waves|simd_count|cu_per" $f; done > $OUT/kfd_props.txt 2>&1; cat $OUT/kfd_props.txt | sort | uniq -c | head
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest -m gpu ${TESTS:+-k $TESTS}"
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread ${TESTS:+-k "$TESTS"} > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error|error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
if [ -z "$SKIP_BENCH" ]; then
  echo "== bench ${BENCH_ARGS}"
  timeout -k 10 900 python3 -u bench.py ${BENCH_ARGS} > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
  tail -1 $OUT/bench.log > $OUT/bench_line.json
  python3 tools/bench_summary.py $OUT/bench_line.json 2>/dev/null || tail -1 $OUT/bench.log | cut -c1-1500
fi
if [ -n "$PROF" ]; then
  echo "== kernel trace at the headline's batches in flight"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o $R --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-distinct --no-extra > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
  grep -h '"metric"' $OUT/kt.log | cut -c1-300
fi
if [ -n "$ENGINES" ]; then
  for N in $ENGINES; do
    echo "== $N engines"
    LB_MAX_ENGINES_PER_DEVICE=16 timeout -k 10 300 python3 -u bench.py --inflight $N --steps ${ESTEPS:-10} --warmup 2 --no-cpu-baseline --legs ${ELEGS:-invalid} > $OUT/bench_e$N.log 2>&1; rc=$?
    echo "OUT_OF_RESOURCES lines: $(grep -c OUT_OF_RESOURCES $OUT/bench_e$N.log)  rc=$rc"
    tail -1 $OUT/bench_e$N.log > $OUT/bench_e$N.json
    python3 tools/bench_summary.py $OUT/bench_e$N.json 2>/dev/null | head -4
    [ $rc -eq 0 ] || exit 1
  done
fi
