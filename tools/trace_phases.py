"""Per-phase kernel totals from a rocprofv3 kernel trace of tools/prof_invalid.py: the phases are
split at the workload generator's launches (k_sign starts each W.make), so phase 1 is the valid c3
batch and phase 2 the c3_invalid batch, each verified the same number of times.  Prints the
kernels whose device time differs most (the search's own cost) and the phase totals.  Given a
rocprofv3 --pmc counter_collection.csv instead, it sums the counter (e.g. SQ_INSTS_VALU: the
search's issued work, which under load is what it costs) in place of the durations.
    python3 tools/trace_phases.py KERNEL_TRACE.csv|COUNTER_COLLECTION.csv [top]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    rows = list(csv.DictReader(open(path)))
    pmc = "Counter_Value" in rows[0]
    if pmc:  # one row per (dispatch, counter): keep the first counter's rows
        names = {r["Counter_Name"] for r in rows}
        first = "SQ_INSTS_VALU" if "SQ_INSTS_VALU" in names else rows[0]["Counter_Name"]
        rows = [r for r in rows if r["Counter_Name"] == first]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    phases = []
    cur = None
    in_sign = False
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if name == "k_sign":
            if not in_sign:
                cur = defaultdict(lambda: [0, 0.0])
                phases.append(cur)
            in_sign = True
            continue
        in_sign = False
        if cur is None:
            continue
        d = float(r["Counter_Value"]) * 1e-6 if pmc else (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        cur[name][0] += 1
        cur[name][1] += d
    if len(phases) < 2:
        print("fewer than two phases found")
        return
    a, b = phases[0], phases[1]
    names = set(a) | set(b)
    diff = sorted(names, key=lambda k: -(b.get(k, [0, 0.0])[1] - a.get(k, [0, 0.0])[1]))
    unit = "M" if pmc else "ms"
    if pmc:
        print(f"counter {first} (millions)")
    print(f"{'kernel':34s} {'n_valid':>8s} {unit + '_valid':>9s} {'n_inv':>6s} {unit + '_inv':>9s} {'extra':>9s}")
    for k in diff[:top]:
        na, ta = a.get(k, [0, 0.0])
        nb, tb = b.get(k, [0, 0.0])
        print(f"{k[:34]:34s} {na:8d} {ta:9.2f} {nb:6d} {tb:9.2f} {tb - ta:9.2f}")
    ta = sum(v[1] for v in a.values())
    tb = sum(v[1] for v in b.values())
    print(f"total ({unit}): valid phase {ta:.2f}, invalid phase {tb:.2f}, extra {tb - ta:.2f}")


if __name__ == "__main__":
    main()
