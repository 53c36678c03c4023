# build/variants/$1.so = the product library compiled with extra flags ($2...), for A/B runs
# through LODESTAR_BLS_LIB (tools/gpu_ab.sh); the same split build as lodestar_amd/build.py.
set -e
name=$1; shift
cd "$(dirname "$0")/.."
mkdir -p build/variants
python3 -c "import sys; sys.path.insert(0, '.'); from lodestar_amd import build as B; B.build_lib(force=True, extra_flags=tuple(sys.argv[2:]), out='build/variants/' + sys.argv[1] + '.so')" "$name" "$@"
