# GPU tests + full default bench (all legs)
set -o pipefail
mkdir -p gpurun_out
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
echo "== bench"; timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d.pop('roofline'); print(json.dumps(d, indent=1))"
