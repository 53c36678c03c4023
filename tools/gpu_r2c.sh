# wave phase timing + full default bench (all legs)
set -o pipefail
mkdir -p gpurun_out
echo "== wave phase"; timeout -k 5 60 ./tools/ubench/wave_phase || exit 1
echo "== bench"; timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d.pop('roofline'); print(json.dumps(d, indent=1))"
