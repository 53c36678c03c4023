# A/B of env knobs / library variants on the default bench (no secondary legs):
# LB_RUNS="default env:LB_SUBGROUP_G8_MAX=1000000 lib:sub1"
set -o pipefail
mkdir -p gpurun_out/ab
for r in $LB_RUNS; do
  unset LODESTAR_BLS_LIB
  envs=""
  case "$r" in
    env:*) envs="${r#env:}"; envs=${envs//+/ } ;;
    lib:*) export LODESTAR_BLS_LIB=$GRAFT_REPO_ROOT/build/variants/${r#lib:}.so ;;
  esac
  tag=$(echo "$r" | tr ':=/' '___')
  env $envs timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-distinct $AB_FLAGS > gpurun_out/ab/$tag.log 2>&1 || { tail -5 gpurun_out/ab/$tag.log; exit 1; }
  echo "== $r"; tail -1 gpurun_out/ab/$tag.log | python3 tools/bench_summary.py
done
