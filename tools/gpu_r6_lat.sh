# Round-6 latency iteration: the GPU test suite (-x; TESTS=-k filter, SKIP_TESTS to skip), then
# a short bench with the latency legs only (1-set, C2 block, slot, per-config), its line summarised.
# Each GPU step has its own limit; the first failure ends the script.
set -o pipefail
R=${R:-r6}
OUT=gpurun_out/lat_$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread ${TESTS:+-k "$TESTS"} > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
  echo "== tests: $(tail -1 $OUT/pytest.log)"
fi
timeout -k 10 400 python3 -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-distinct --legs ${LEGS:-latency,configs,slots1} > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log > $OUT/bench_line.json
python3 - $OUT/bench_line.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value", d["value"])
for k in ("latency_1set_ms", "latency_block_ms", "latency_slot1_ms"):
    print(k, d.get(k))
for k in ("latency_1set_stage_ms", "latency_block_stage_ms"):
    print(k, json.dumps(d.get(k)))
pc = d.get("per_config") or {}
print("per_config", json.dumps({c: {kk: v for kk, v in x.items() if "ms" in kk} for c, x in pc.items()})[:600])
PY
