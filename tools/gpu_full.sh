# Full GPU evidence pass: gpu tests, smoke, bench (with CPU baseline), rocprof kernel trace, PMC passes.
set -o pipefail
mkdir -p gpurun_out/full
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "== pytest -m gpu"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/full/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/full/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/full/pytest_gpu.log
echo "== smoke"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1 || { tail -20 gpurun_out/full/smoke.log; exit 1; }
tail -1 gpurun_out/full/smoke.log | cut -c1-300
bash tools/gpu_evidence.sh
