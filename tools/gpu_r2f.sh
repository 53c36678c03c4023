# GPU tests, the invalid-search profile, then the full bench
set -o pipefail
bash tools/gpu_r2e.sh && bash tools/gpu_bench.sh
