"""Child process of tests/test_gpu_parity.py::test_engine_cap_reserves_scratch (not a test module):
creates the per-device engine cap's worth of engines (LB_MAX_ENGINES_PER_DEVICE, default 10), each
reserving its three streams' scratch at creation (lb_engine_create_ex), prints the device memory
each creation took, then runs one C1 call on every engine at once and checks the verdicts.
Exits non-zero on a failed creation or a wrong verdict."""
import os
import sys
import threading

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from lodestar_amd.engine import Engine  # noqa: E402
from lodestar_amd import workloads as W  # noqa: E402


def main():
    n = int(os.environ.get("LB_MAX_ENGINES_PER_DEVICE", "10"))
    engines, took = [], []
    for _ in range(n):
        free0 = torch.cuda.mem_get_info(0)[0]
        engines.append(Engine(0))
        took.append((free0 - torch.cuda.mem_get_info(0)[0]) / 2**20)
    print("MiB per engine creation:", " ".join("%.0f" % t for t in took), flush=True)
    wl = W.make(engines[0], "c1")
    packs = [W.indexed_for(e, wl) for e in engines]  # each engine's own resident key table
    bad = []

    def run(k):
        if engines[k].verify_jobs_packed(packs[k]) != [int(x) for x in wl.expected]:
            bad.append(k)
    ths = [threading.Thread(target=run, args=(k,)) for k in range(n)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for e in engines:
        e.close()
    print("engines", n, "bad", len(bad), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
