# Invalid-set search breakdown: tools/prof_invalid.py (c3 then c3_invalid, one batch in flight, the
# search rounds traced) under a rocprofv3 kernel trace; tools/trace_phases.py splits the two phases.
set -o pipefail
OUT=gpurun_out/inv_${R:-r4}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o inv --output-format csv -- python3 tools/prof_invalid.py 6 2 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
grep -v "^\[rocprof" $OUT/prof.log | tail -12
python3 tools/trace_phases.py $(find $OUT/kt -name "*kernel_trace.csv") 30 | tee $OUT/phases.txt
if [ -n "$PMC" ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $OUT/pmc -o inv --output-format csv -- python3 tools/prof_invalid.py 6 1 > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
  python3 tools/trace_phases.py $(find $OUT/pmc -name "*counter_collection.csv") 30 | tee $OUT/phases_valu.txt
fi
