# Round-4 evidence at the HEADLINE configuration (7 batches in flight, the kernel forms the driver's
# bench runs): the GPU test suite, the driver's bench line, a rocprofv3 kernel trace, and PMC passes
# (FETCH_SIZE, WRITE_SIZE, VALU; each its own run; per-dispatch Scratch_Size / VGPR columns come with
# them).  Every GPU step has its own limit; the first failure ends the script.
set -o pipefail
R=${R:-r4}
OUT=gpurun_out/ev_$R
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
HEAD="--steps 5 --warmup 1 --no-cpu-baseline --no-distinct --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o $R --output-format csv -- python3 bench.py $HEAD > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
echo "== kernel trace: $(grep -h '"metric"' $OUT/kt.log | cut -c1-160)"
PM="--steps 1 --warmup 1 --no-cpu-baseline --no-distinct --no-extra"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o $R --output-format csv -- python3 bench.py $PM > $OUT/pmc_fetch.log 2>&1 || { tail -5 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o $R --output-format csv -- python3 bench.py $PM > $OUT/pmc_write.log 2>&1 || { tail -5 $OUT/pmc_write.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU -d $OUT/pmc_valu -o $R --output-format csv -- python3 bench.py $PM > $OUT/pmc_valu.log 2>&1 || { tail -5 $OUT/pmc_valu.log; exit 1; }
NSETS=$(grep -h '"metric"' $OUT/pmc_fetch.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["config"]["sets_per_gpu"])')
python3 tools/pmc_traffic.py $(find $OUT/pmc_fetch -name "*counter_collection.csv") $(find $OUT/pmc_write -name "*counter_collection.csv") $NSETS 7 > $OUT/traffic.json
echo "== pmc done"; find $OUT -name "*.csv" | sort
