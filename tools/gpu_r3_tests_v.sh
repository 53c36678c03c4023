# GPU suite, verbose to a file (progress visible), each test bounded
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_v.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_v.log; grep -E "FAILED|Timeout|timeout" gpurun_out/pytest_v.log | head; exit $rc
