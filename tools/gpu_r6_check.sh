# Round-6 check: the GPU test suite, the driver's bench line, a rocprofv3 kernel trace at ONE batch
# in flight (the configuration the line's stage ms come from: DESIGN §7), and a 2-rank rehearsal on
# device 0 (gloo control plane) that prints the N > 1 legs.  Each GPU step has its own limit; the
# first failure ends the script.
set -o pipefail
R=${R:-r6}
OUT=gpurun_out/chk_$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head; tail -20 $OUT/pytest.log; exit 1; }
  echo "== tests: $(tail -1 $OUT/pytest.log)"
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 900 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
  tail -1 $OUT/bench.log > $OUT/bench_line.json; echo "== bench"; python3 tools/bench_summary.py $OUT/bench_line.json
fi
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt1 -o ${R}_inflight1 --output-format csv -- python3 bench.py --inflight 1 --steps 5 --warmup 1 --no-cpu-baseline --no-distinct --no-extra > $OUT/kt1.log 2>&1 || { tail -20 $OUT/kt1.log; exit 1; }
  echo "== kernel trace (1 in flight): $(grep -h '"metric"' $OUT/kt1.log | cut -c1-200)"
fi
if [ -z "$SKIP_REH" ]; then
  LB_BENCH_BACKEND=gloo LB_BENCH_DEVICE=0 timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 --inflight 3 --no-cpu-baseline --no-distinct --no-extra > $OUT/rehearsal.log 2>&1 || { tail -20 $OUT/rehearsal.log; exit 1; }
  echo "== rehearsal"; grep -h '"metric"' $OUT/rehearsal.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('value_exchange'), json.dumps(d.get('range_sync_segments'))[:600])"
fi
