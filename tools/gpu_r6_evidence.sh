# Round-6 evidence on the final tree: the GPU test suite, the driver's bench line, a rocprofv3
# kernel trace at ONE batch in flight (the configuration the line's stage ms come from) with the
# decode check, the counter passes (VALU utilisation; FETCH_SIZE / WRITE_SIZE traffic), and a
# 2-rank rehearsal on device 0 (gloo control plane) for the N > 1 legs.  Each GPU step has its own
# limit; the first failure ends the script.
set -o pipefail
R=${R:-r6}
OUT=gpurun_out/ev_$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head; tail -20 $OUT/pytest.log; exit 1; }
  echo "== tests: $(tail -1 $OUT/pytest.log)"
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 900 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
  tail -1 $OUT/bench.log > $OUT/bench_line.json; echo "== bench"; python3 tools/bench_summary.py $OUT/bench_line.json > $OUT/bench_summary.txt; head -12 $OUT/bench_summary.txt
fi
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt1 -o ${R}_inflight1 --output-format csv -- python3 bench.py --inflight 1 --steps 5 --warmup 1 --no-cpu-baseline --no-distinct --no-extra > $OUT/kt1.log 2>&1 || { tail -20 $OUT/kt1.log; exit 1; }
  grep -h '"metric"' $OUT/kt1.log | tail -1 > $OUT/kt1_line.json
  trace=$(find $OUT/kt1 -name "*kernel_trace.csv" | head -1)
  NSETS=$(python3 -c "import json; print(json.load(open('$OUT/kt1_line.json'))['config']['sets_per_gpu'])")
  python3 tools/trace_stage_avg.py "$trace" $NSETS $OUT/kt1_line.json > $OUT/decode_check.json && echo "== decode check: $(python3 -c "import json; d=json.load(open('$OUT/decode_check.json')); print(d['stages'], d.get('rocprof_over_hip_event'))")"
fi
if [ -z "$SKIP_VALU" ]; then
  R=$R bash tools/gpu_r6_valu.sh || exit 1
fi
if [ -z "$SKIP_REH" ]; then
  LB_BENCH_BACKEND=gloo LB_BENCH_DEVICE=0 timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 --inflight 3 --no-cpu-baseline --no-distinct --no-extra > $OUT/rehearsal.log 2>&1 || { tail -20 $OUT/rehearsal.log; exit 1; }
  grep -h '"metric"' $OUT/rehearsal.log | tail -1 > $OUT/rehearsal_line.json; echo "== rehearsal $(python3 -c "import json; d=json.load(open('$OUT/rehearsal_line.json')); print(d['value'], d.get('value_exchange'))")"
fi
