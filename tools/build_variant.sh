# build/variants/$1.so = the product library compiled with extra flags ($2...), for A/B runs
# through LODESTAR_BLS_LIB (tools/gpu_ab.sh).
set -e
name=$1; shift
cd "$(dirname "$0")/.."
mkdir -p build/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -Wno-unused-value \
  -Iinclude -Ilodestar_amd/csrc "$@" lodestar_amd/csrc/lb_engine.hip -o build/variants/$name.so
