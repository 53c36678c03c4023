#!/usr/bin/env python3
"""Per-kernel VALU utilisation of the headline configuration from rocprofv3 counters (SURVEY.md
§8(d)).

Input: the counter_collection CSV of
    LB_PROF_MARK=1 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE -- python3 bench.py ...
bench.py brackets the headline's timed region with one k_partials_check dispatch each side
(LB_PROF_MARK=1); only the dispatches between the two markers count, so "per batch" means one
batch of the F-in-flight headline (K x F batches), without the workload generator (k_sign), the
table fill or the one-batch-in-flight profiled steps before the region.

Per kernel:
  valu_G_per_batch   SQ_INSTS_VALU (wave-instructions) / batches
  share              of the region's VALU instructions
  valu_busy          SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: the fraction of its waves' lifetime with a
                     VALU instruction issued (both in quad-cycles on gfx950, MI355X_MICROARCH.md)
  waves              SQ_WAVES per dispatch (mean)
  int64_share        SQ_INSTS_VALU_INT64 / SQ_INSTS_VALU (64-bit integer VALU: the v_mad_u64_u32 of
                     the Fp products, plus 64-bit adds / shifts)
Chip:
  valu_issue_frac    the region's VALU wave-instructions x 2 cycles (wave64 VALU issue on a
                     SIMD-32, MI355X_MICROARCH.md "v_fma_f32 (wave64) 2 cyc") / (1 024 SIMDs x
                     clock x the un-profiled region time), with clock 2.4 GHz (the loaded shader
                     clock read by the wave microbench) unless --clock-ghz; the
                     un-profiled time comes from a bench line (--line, ms_per_step x K x F)
Counter passes serialise dispatches, so no time-based figure here is taken from the profiled run.

  python3 tools/valu_util.py COUNTERS.csv --batches K*F [--line bench_line.json] [--out json]
"""
import argparse
import collections
import csv
import json
import sys

MARK = "k_partials_check"
SIMDS = 1024


def load(path):
    rows = collections.defaultdict(dict)  # dispatch -> {name, counters}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        e = rows[d]
        e["name"] = r["Kernel_Name"].split("(")[0].strip()
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return dict(sorted(rows.items()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--batches", type=int, required=True, help="batches in the timed region (steps x inflight)")
    ap.add_argument("--line", help="an un-profiled bench.py JSON line of the same configuration")
    ap.add_argument("--clock-ghz", type=float, default=2.4)
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = load(a.csv)
    marks = [d for d, e in rows.items() if e["name"].startswith(MARK)]
    if len(marks) < 2:
        sys.exit("need the two LB_PROF_MARK dispatches (k_partials_check) in the trace")
    # the FIRST pair: the headline's region (bench.py's later legs -- the range-sync segments --
    # call lb_fp12_product_is_one too)
    lo, hi = marks[0], marks[1]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    tot = collections.defaultdict(float)
    for d, e in rows.items():
        if not lo < d < hi:
            continue
        k = per[e["name"]]
        k["dispatches"] += 1
        for c, v in e.items():
            if c != "name":
                k[c] += v
                tot[c] += v
    out = {"source": a.csv, "marker_dispatches": [lo, hi], "batches": a.batches,
           "region_dispatches": int(sum(k["dispatches"] for k in per.values())),
           "valu_G_per_batch": round(tot["SQ_INSTS_VALU"] / a.batches / 1e9, 4),
           "salu_G_per_batch": round(tot.get("SQ_INSTS_SALU", 0.0) / a.batches / 1e9, 4),
           "valu_busy_all": round(tot["SQ_ACTIVE_INST_VALU"] / max(tot["SQ_WAVE_CYCLES"], 1.0), 4),
           "int64_share_all": round(tot.get("SQ_INSTS_VALU_INT64", 0.0) / max(tot["SQ_INSTS_VALU"], 1.0), 4),
           "kernels": {}}
    for name, k in sorted(per.items(), key=lambda kv: -kv[1]["SQ_INSTS_VALU"]):
        out["kernels"][name] = {
            "dispatches_per_batch": round(k["dispatches"] / a.batches, 2),
            "valu_G_per_batch": round(k["SQ_INSTS_VALU"] / a.batches / 1e9, 4),
            "share": round(k["SQ_INSTS_VALU"] / max(tot["SQ_INSTS_VALU"], 1.0), 4),
            "valu_busy": round(k["SQ_ACTIVE_INST_VALU"] / max(k["SQ_WAVE_CYCLES"], 1.0), 4),
            "waves_per_dispatch": round(k["SQ_WAVES"] / k["dispatches"], 1),
        }
        if "SQ_INSTS_VALU_INT64" in k:
            out["kernels"][name]["int64_share"] = round(k["SQ_INSTS_VALU_INT64"] / max(k["SQ_INSTS_VALU"], 1.0), 4)
    if a.line:
        line = json.loads(open(a.line).read().strip().splitlines()[-1])
        t = line["ms_per_step"] * 1e-3  # seconds per batch of the headline, un-profiled
        issue = tot["SQ_INSTS_VALU"] / a.batches * 2.0 / (SIMDS * a.clock_ghz * 1e9 * t)
        out["chip"] = {"ms_per_batch": line["ms_per_step"], "clock_ghz_assumed": a.clock_ghz,
                       "valu_issue_frac": round(issue, 4),
                       "note": "VALU wave-instructions per batch x 2 cycles / (1024 SIMDs x clock x ms_per_step)"}
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
