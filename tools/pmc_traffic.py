"""profiles/traffic.json from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py at one
batch in flight: per kernel, average (FETCH_SIZE + WRITE_SIZE) x 1024 bytes per launch.

FETCH_SIZE / WRITE_SIZE are in KB (L2 <-> fabric).  MI355X_MICROARCH.md: FETCH_SIZE under-reports
wide (16 B/lane) streaming reads by 2x; these kernels read 4-byte SoA words and scratch, an
uncalibrated width, so the raw value is reported.

  python tools/pmc_traffic.py FETCH.csv WRITE.csv SETS_PER_LAUNCH > profiles/traffic.json
"""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            d[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}


def main():
    fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
    n = int(sys.argv[3])
    out = {"source": "rocprofv3 --pmc FETCH_SIZE, --pmc WRITE_SIZE (separate passes), bench.py --inflight 1",
           "unit": "bytes per launch", "kernels": {}}
    for k in sorted(set(fetch) & set(write)):
        if not k.startswith("k_"):
            continue
        out["kernels"][k] = {"fetch_bytes": round(fetch[k] * 1024), "write_bytes": round(write[k] * 1024),
                             "bytes_per_launch": round((fetch[k] + write[k]) * 1024), "sets_per_launch": n}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
