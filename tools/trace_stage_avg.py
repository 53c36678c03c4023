#!/usr/bin/env python3
"""Per-stage kernel time from a rocprofv3 --kernel-trace CSV, restricted to the dispatches of one
batch size (Grid_Size_X = the batch's set count rounded to the 64-lane block), so that the
roofline's HIP-event stage time in bench.py can be checked against rocprof's own durations.

  python tools/trace_stage_avg.py TRACE.csv SETS [stage-ms-json-from-the-line]
"""
import collections
import csv
import json
import sys

STAGE = {"decode_sigs": ["k_decompress_sigs", "k_sig_subgroup", "k_sig_subgroup_g8", "k_job_status"]}


def main():
    path, sets = sys.argv[1], int(sys.argv[2])
    grid = {"k_decompress_sigs": (sets + 63) // 64 * 64, "k_sig_subgroup": (sets + 63) // 64 * 64}
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].split("(")[0].split("<")[0].strip()
        d[(n, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = {"trace": path, "sets_per_batch": sets, "kernels": {}, "stages": {}}
    for st, ks in STAGE.items():
        tot = 0.0
        for k in ks:
            # the batch's dispatch: the grid of its set count, or (k_job_status) the largest grid
            cands = [(g, v) for (n, g), v in d.items() if n == k]
            if not cands:
                continue
            g, v = (next(((g, v) for g, v in cands if g == grid[k]), None) if k in grid
                    else max(cands, key=lambda c: c[0]))
            out["kernels"][k] = {"grid": g, "dispatches": len(v), "avg_ms": round(sum(v) / len(v), 4),
                                 "min_ms": round(min(v), 4)}
            tot += sum(v) / len(v)
        out["stages"][st] = round(tot, 4)
    if len(sys.argv) > 3:
        line = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
        ev = line["roofline"]["stages"]["decode_sigs"]["ms"]
        out["line_hip_event_ms"] = {"decode_sigs": ev}
        out["rocprof_over_hip_event"] = round(out["stages"]["decode_sigs"] / ev, 4)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
