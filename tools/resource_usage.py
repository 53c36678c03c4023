#!/usr/bin/env python3
"""Per-kernel register / scratch / LDS usage from hipcc's -Rpass-analysis=kernel-resource-usage
remarks (offline, no GPU): python3 tools/resource_usage.py remarks.txt [name-filter ...]"""
import re
import subprocess
import sys


def parse(text):
    out, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/(?:lane|block)\])?: (\S+) \[", line)
        if m and cur:
            out[cur][m.group(1).strip()] = m.group(2)
    return out


def demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
        return r.stdout.splitlines()
    except OSError:
        return names


if __name__ == "__main__":
    d = parse(open(sys.argv[1]).read())
    flt = sys.argv[2:]
    names = [n for n in d if n.startswith("_Z") and ("k_" in n)]
    for n, dn in zip(names, demangle(names)):
        short = dn.split("(")[0]
        if flt and not any(f in short for f in flt):
            continue
        r = d[n]
        print(f"{short[:34]:34s} vgpr {r.get('VGPRs','?'):>4} agpr {r.get('AGPRs','?'):>4} "
              f"scratch {r.get('ScratchSize','?'):>6} occ {r.get('Occupancy [waves/SIMD]', r.get('Occupancy','?')):>2} "
              f"lds {r.get('LDS Size','?'):>6} spillV {r.get('VGPRs Spill','?')}")
