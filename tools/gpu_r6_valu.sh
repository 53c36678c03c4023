# Round-6 counter pass: per-kernel VALU utilisation at the headline
# configuration.  bench.py with LB_PROF_MARK=1 brackets the timed region with one
# k_partials_check dispatch each side; tools/valu_util.py keeps the dispatches between them.
# One --pmc pass (8 SQ + 1 GRBM counters: gfx950 has 8 SQ / 2 GRBM slots), then an
# un-profiled line of the same flags for the time base.  Each step has its own limit.
set -o pipefail
R=${R:-r6}
OUT=gpurun_out/valu_$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
FLAGS="--steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-distinct --no-extra"
LB_PROF_MARK=1 timeout -s KILL 420 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE -d $OUT/pmc -o valu --output-format csv -- python3 bench.py $FLAGS > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
echo "== pmc: $(grep -h '"metric"' $OUT/pmc.log | cut -c1-160)"
timeout -k 10 300 python3 bench.py $FLAGS > $OUT/line.log 2>&1 || { tail -20 $OUT/line.log; exit 1; }
tail -1 $OUT/line.log > $OUT/line.json
csv=$(find $OUT/pmc -name "*counter_collection.csv" | head -1)
python3 tools/valu_util.py "$csv" --batches $(( ${STEPS:-3} * 7 )) --line $OUT/line.json --out $OUT/valu_util.json | head -60
if [ -z "$SKIP_TRAFFIC" ]; then
  # HBM traffic at the same configuration: FETCH_SIZE and WRITE_SIZE in their own passes
  PM="--steps 1 --warmup 1 --no-cpu-baseline --no-distinct --no-extra"
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o fetch --output-format csv -- python3 bench.py $PM > $OUT/pmc_fetch.log 2>&1 || { tail -5 $OUT/pmc_fetch.log; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o write --output-format csv -- python3 bench.py $PM > $OUT/pmc_write.log 2>&1 || { tail -5 $OUT/pmc_write.log; exit 1; }
  NSETS=$(grep -h '"metric"' $OUT/pmc_fetch.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["config"]["sets_per_gpu"])')
  python3 tools/pmc_traffic.py $(find $OUT/pmc_fetch -name "*counter_collection.csv") $(find $OUT/pmc_write -name "*counter_collection.csv") $NSETS 7 > $OUT/traffic.json
  echo "== traffic: $(python3 -c "import json; d=json.load(open('$OUT/traffic.json')); print(d['stages'].get('decode_sigs'))")"
fi
