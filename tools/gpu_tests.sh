# The GPU test suite, verbose to gpurun_out/pytest_v.log (progress visible), each test bounded
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_v.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_v.log; grep -E "FAILED|Timeout" gpurun_out/pytest_v.log | head; exit $rc
