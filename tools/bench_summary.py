"""Print the headline numbers and per-stage ms of a bench.py JSON line (stdin)."""
import json
import sys

d = json.loads(sys.stdin.read().strip().splitlines()[-1])
r = d["roofline"] or {}
print("value", d["value"], "single", d["value_one_batch_in_flight"], "distinct", d.get("value_distinct_roots"),
      "ms/step", d["ms_per_step"])
print(" ".join(f"{k}={v['ms']}" for k, v in r.get("stages", {}).items()))
