#!/bin/bash
# Offline per-kernel register / scratch usage of the product library (no GPU):
#   tools/remarks.sh OUT.txt [extra hipcc flags...]  then  python3 tools/resource_usage.py OUT.txt
out=${1:-/tmp/remarks.txt}; shift
cd "$(dirname "$0")/.." && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -Wno-unused-result \
  -Wno-unused-value -Iinclude -Ilodestar_amd/csrc "$@" lodestar_amd/csrc/lb_engine.hip -o /tmp/lb_remarks.o \
  -Rpass-analysis=kernel-resource-usage > "$out" 2>&1
