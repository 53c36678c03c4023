"""Wave occupancy over time from a rocprofv3 kernel trace: for the busiest window (the last
`--window` seconds of dispatches), the time-average number of resident waves (grid / 64 per
kernel, summed over kernels running at the same instant, capped at the chip's 1024 SIMDs) and
the share of SIMD-time each kernel holds.  A kernel's waves are counted for its whole duration,
so narrow tails over-count; it is an upper bound on SIMD occupancy.

  python tools/occupancy.py gpurun_out/occ/kt/occ_kernel_trace.csv
"""
import collections
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith("k_")]
NU = int(sys.argv[2]) if len(sys.argv) > 2 else 0  # distinct roots per batch (bench JSON)


def active_waves(k, grid):
    """waves that do work: the per-root kernels launch one lane per set and exit past n_u"""
    w = grid // 64
    if not NU:
        return w
    n = grid if k != "k_hash_map" else grid // 2
    mu = 1 << max(n - 1, 1).bit_length()
    if k in ("k_hash_finish", "k_miller_g8", "k_gsum_final"):
        return -(-NU // 64)
    if k == "k_hash_map":
        return -(-2 * NU // 64)
    if k == "k_gsum_chunks":
        return -(-(NU + n // 32) // 64)
    return w


for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["k"] = r["Kernel_Name"].split("(")[0]
    r["w"] = active_waves(r["k"], int(r["Grid_Size_X"]))
    if r["k"] == "k_tree_up_U" and NU:  # one wave per node; nodes past n_u exit
        r["w"] = min(int(r["Grid_Size_X"]) // 64, 64)
t_end = max(r["e"] for r in rows)
# the timed in-flight phase: last 40% of the trace
t0 = t_end - int((t_end - min(r["s"] for r in rows)) * 0.4)
ev = []
share = collections.Counter()
for r in rows:
    s, e = max(r["s"], t0), r["e"]
    if e <= s:
        continue
    ev.append((s, r["w"]))
    ev.append((e, -r["w"]))
    share[r["k"]] += r["w"] * (e - s)
ev.sort()
cur, last, acc, acc_cap = 0, t0, 0.0, 0.0
for t, d in ev:
    acc += cur * (t - last)
    acc_cap += min(cur, 1024) * (t - last)
    cur += d
    last = t
span = t_end - t0
print(f"window {span / 1e6:.1f} ms: mean resident waves {acc / span:.0f}, capped at 1024 SIMDs {acc_cap / span:.0f}"
      f" ({acc_cap / span / 1024:.0%})")
tot = sum(share.values())
for k, v in share.most_common(12):
    print(f"  {k:24s} {v / tot:6.1%}")
