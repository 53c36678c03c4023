#!/bin/bash
# Offline per-kernel register / scratch usage of the product library (no GPU): every kernel group
# of the split build (lb_kgroup.hip -DLB_KGROUP=g, tools/gen_kdecls.py) with hipcc's
# resource-usage remarks, concatenated:
#   tools/remarks.sh OUT.txt [extra hipcc flags...]  then  python3 tools/resource_usage.py OUT.txt
out=${1:-/tmp/remarks.txt}; shift
cd "$(dirname "$0")/.." || exit 1
n=$(python3 -c 'import sys; sys.path.insert(0, "tools"); import gen_kdecls; print(gen_kdecls.N_GROUPS)')
: > "$out"
pids=()
for g in $(seq 0 $((n - 1))); do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -Wno-unused-result -Wno-unused-value \
    -Iinclude -Ilodestar_amd/csrc -DLB_KGROUP=$g "$@" lodestar_amd/csrc/lb_kgroup.hip -o /tmp/lb_remarks_$g.o \
    -Rpass-analysis=kernel-resource-usage > /tmp/lb_remarks_$g.txt 2>&1 &
  pids+=($!)
  if [ ${#pids[@]} -ge 8 ]; then wait "${pids[0]}"; pids=("${pids[@]:1}"); fi
done
wait
for g in $(seq 0 $((n - 1))); do cat /tmp/lb_remarks_$g.txt >> "$out"; done
