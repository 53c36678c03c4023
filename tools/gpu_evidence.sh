# Evidence pass: PMC traffic passes first (-> profiles/traffic.json on the box, copied back),
# then the default bench (with CPU baseline, reads traffic.json), then a rocprof kernel trace of
# one batch in flight.  Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out/full/ev
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ONE="--steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-distinct --no-extra"
R=${R:-r3}
echo "== pmc: FETCH_SIZE"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/full/ev/pmc_fetch -o $R --output-format csv -- python3 bench.py $ONE > gpurun_out/full/ev/pmc_fetch.log 2>&1 || { tail -3 gpurun_out/full/ev/pmc_fetch.log; exit 1; }
echo "== pmc: WRITE_SIZE"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/full/ev/pmc_write -o $R --output-format csv -- python3 bench.py $ONE > gpurun_out/full/ev/pmc_write.log 2>&1 || { tail -3 gpurun_out/full/ev/pmc_write.log; exit 1; }
echo "== pmc: valu"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU -d gpurun_out/full/ev/pmc_valu -o $R --output-format csv -- python3 bench.py $ONE > gpurun_out/full/ev/pmc_valu.log 2>&1 || { tail -3 gpurun_out/full/ev/pmc_valu.log; exit 1; }
NSETS=$(grep -h '"metric"' gpurun_out/full/ev/pmc_fetch.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["config"]["sets_per_gpu"])')
python3 tools/pmc_traffic.py $(find gpurun_out/full/ev/pmc_fetch -name "*counter_collection.csv") $(find gpurun_out/full/ev/pmc_write -name "*counter_collection.csv") $NSETS > profiles/traffic.json && cp profiles/traffic.json gpurun_out/full/ev/traffic.json
echo "== bench (default flags, with cpu baseline)"
timeout -k 10 600 python3 -u bench.py > gpurun_out/full/ev/bench_default.log 2>&1 || { tail -20 gpurun_out/full/ev/bench_default.log; exit 1; }
tail -1 gpurun_out/full/ev/bench_default.log | cut -c1-400
echo "== rocprof kernel trace (single batch in flight)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/full/ev/kt -o $R --output-format csv -- python3 bench.py --steps 5 --warmup 1 --inflight 1 --no-cpu-baseline --no-distinct --no-extra > gpurun_out/full/ev/kt.log 2>&1 || { tail -20 gpurun_out/full/ev/kt.log; exit 1; }
grep -h '"metric"' gpurun_out/full/ev/kt.log | cut -c1-200
find gpurun_out/full/ev -name "*.csv" | sort
