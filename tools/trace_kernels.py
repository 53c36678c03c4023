#!/usr/bin/env python3
"""Median duration per (kernel, grid) from a rocprofv3 --kernel-trace CSV.
  python tools/trace_kernels.py TRACE.csv [name-substring ...]"""
import collections
import csv
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
    d[(n, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
keys = sys.argv[2:]
for (n, g), v in sorted(d.items()):
    if keys and not any(k in n for k in keys):
        continue
    v = sorted(v)
    print("%-28s grid %8d  n %4d  median %.3f ms  max %.3f" % (n, g, len(v), v[len(v) // 2], v[-1]))
