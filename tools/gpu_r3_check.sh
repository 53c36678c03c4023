# GPU suite, the wave-engine phase timing, then the headline at the driver's step counts with the
# invalid and latency legs.  The first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
if [ -x tools/ubench/wave_phase ]; then echo "== wave_phase"; timeout -k 5 60 ./tools/ubench/wave_phase || exit 1; fi
echo "== bench"; timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --legs invalid,latency > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python3 tools/bench_summary.py
