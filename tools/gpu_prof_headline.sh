# Headline-configuration profile: the driver's bench flags (7 batches in
# flight) under rocprofv3 --kernel-trace --stats, so the kernel mix the headline runs is the one
# traced (k_miller_lane / k_hash_finish under load), plus the new signing-root GPU tests.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R=${R:-r4}
OUT=gpurun_out/prof_$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$TESTS" ]; then
  echo "== pytest -m gpu -k '$TESTS'"
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$TESTS" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
HEAD="--steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-distinct --no-extra ${BENCH_ARGS}"
echo "== kernel trace at the headline's batches in flight ($HEAD)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o $R --output-format csv -- python3 bench.py $HEAD > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
grep -h '"metric"' $OUT/kt.log | cut -c1-300
find $OUT/kt -name "*kernel_stats.csv" -exec head -25 {} \;
