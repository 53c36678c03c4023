"""Profiles the invalid-set search on the bench's c3_invalid batch (one batch in flight):
per-stage times, the search rounds (LB_SEARCH_TRACE) and, under rocprofv3, per-kernel times."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from lodestar_amd import workloads as W  # noqa: E402
from lodestar_amd.engine import Engine  # noqa: E402

slots = int(sys.argv[1]) if len(sys.argv) > 1 else 6
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
eng = Engine(0)
for name in ("c3", "c3_invalid"):
    wl = W.make(eng, name, slots=slots)
    b = eng.upload(W.indexed_for(eng, wl))
    assert np.array_equal(np.asarray(b.verify()), wl.expected)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        b.verify()
        ts.append((time.perf_counter() - t0) * 1e3)
    eng.set_profiling(True)
    os.environ["LB_SEARCH_TRACE"] = "1"
    b.verify()
    os.environ.pop("LB_SEARCH_TRACE")
    prof = eng.last_profile()
    eng.set_profiling(False)
    print(name, wl.packed.n_sets, "sets; ms", [round(t, 2) for t in ts], flush=True)
    print("  stages", {k: round(v, 3) for k, v in prof.items() if v > 0}, flush=True)
    b.free()
