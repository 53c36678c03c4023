# A/B: default library vs build/variants/<v>.so (LB_VARIANTS="a b"), bench at the default config.
set -o pipefail
mkdir -p gpurun_out/ab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in default $LB_VARIANTS; do
  if [ "$v" = default ]; then unset LODESTAR_BLS_LIB; else export LODESTAR_BLS_LIB=$GRAFT_REPO_ROOT/build/variants/$v.so; fi
  timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-distinct ${BENCH_ARGS:-} > gpurun_out/ab/$v.log 2>&1 || { tail -5 gpurun_out/ab/$v.log; exit 1; }
  echo "== $v"; tail -1 gpurun_out/ab/$v.log | python3 tools/bench_summary.py
done
