"""Stage times of the per-config batches (c1, c2, c4, c5, c5_64) at one batch in flight, one engine
(tools/, not product code): python tools/cfg_probe.py [names...]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from lodestar_amd.engine import Engine  # noqa: E402
from lodestar_amd import workloads as W  # noqa: E402

names = sys.argv[1:] or ["c2", "c4", "c5", "c5_64"]
# PROBE_ENGINES > 1: as many engines alive (the bench keeps its 7 in-flight engines), the first used
others = [Engine(0) for _ in range(int(os.environ.get("PROBE_ENGINES", "1")) - 1)]
with Engine(0) as e:
    for name in names:
        wl = W.make(e, name)
        b = e.upload(W.indexed_for(e, wl))
        got = np.asarray(b.verify())
        assert np.array_equal(got, wl.expected), name
        e.set_profiling(True)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            b.verify()
            ts.append((time.perf_counter() - t0) * 1e3)
        prof = e.last_profile()
        e.set_profiling(False)
        b.free()
        print(name, "sets", wl.packed.n_sets, "ms", [round(t, 2) for t in ts],
              json.dumps({k: round(v, 3) for k, v in prof.items() if v > 0}))
