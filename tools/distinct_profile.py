"""Per-stage HIP-event ms of one c3_distinct batch (every signing root distinct) alone on one
engine, and the lane kernels' register use from the build; for the distinct-roots leg's breakdown."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from lodestar_amd import workloads as W  # noqa: E402
from lodestar_amd.engine import Engine  # noqa: E402

eng = Engine(0)
wd = W.make(eng, "c3_distinct", seed=W.SEED)
b = eng.upload(W.indexed_for(eng, wd))
assert np.array_equal(np.asarray(b.verify()), wd.expected)
out = {}
for rep in range(3):
    eng.set_profiling(True)
    b.verify()
    out = {k: round(v, 3) for k, v in eng.last_profile().items() if v > 0}
    eng.set_profiling(False)
print(json.dumps({"sets": int(wd.packed.n_sets), "stage_ms": out}))
b.free()
eng.close()
