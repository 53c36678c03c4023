# tools/cfg_probe.py under each RUNS setting (env:K=V or default)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cfgprobe
for r in $RUNS; do
  envs=""
  case "$r" in env:*) envs="${r#env:}"; envs=${envs//+/ } ;; esac
  echo "== $r"
  env $envs timeout -k 10 200 python3 -u tools/cfg_probe.py $NAMES > gpurun_out/cfgprobe/$(echo $r | tr ':=+' '___').log 2>&1 || { tail -5 gpurun_out/cfgprobe/*.log; exit 1; }
  cat gpurun_out/cfgprobe/$(echo $r | tr ':=+' '___').log
done
