"""Print the headline numbers and per-stage ms of a bench.py JSON line (stdin)."""
import json
import sys

src = open(sys.argv[1]) if len(sys.argv) > 1 else sys.stdin
d = json.loads(src.read().strip().splitlines()[-1])
r = d["roofline"] or {}
print("value", d["value"], "single", d["value_one_batch_in_flight"], "distinct", d.get("value_distinct_roots"),
      "ms/step", d["ms_per_step"])
print(" ".join(f"{k}={v['ms']}" for k, v in r.get("stages", {}).items()))
for k in ("value_distinct_keys", "distinct_keys", "value_one_invalid_per_batch", "value_e2e", "value_slots1", "latency_slot1_ms", "latency_1set_ms",
          "latency_block_ms", "value_dropin", "batch_latency_ms", "dropin", "signing_roots"):
    if k in d:
        print(k, d[k])
for k in ("slots1_stage_ms", "latency_1set_stage_ms", "latency_block_stage_ms"):
    if k in d:
        print(k, d[k])
if "invalid_batch_stage_ms" in d:
    print("invalid stages", d["invalid_batch_stage_ms"])
if "per_config" in d:
    print("per_config", {k: (v["ms_per_batch"], v["sets_per_s"]) for k, v in d["per_config"].items()})
