"""Child process of tests/test_gpu_parity.py::test_latency_engine_under_load (not a test module):
a latency engine's 1-set calls (upload + verify + readback, as verifyOnMainThread) while two pool engines verify 6-slot C3 batches.  Prints the call
times (ms) on its last line; exits non-zero on any wrong verdict."""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lodestar_amd.engine import Engine  # noqa: E402
from lodestar_amd import workloads as W  # noqa: E402


def main():
    lat = Engine(0, Engine.LATENCY)
    e1, e2 = Engine(0), Engine(0)
    ip = W.indexed_for(lat, W.make(lat, "c1"))
    one = W.PackedJobs(job_off=np.array([0, 1], np.uint32), pk_off=np.array([0, 1], np.uint32), pubkeys=None,
                       msgs=ip.msgs[:32], sigs=ip.sigs[:96], sig_sizes=None, pk_indices=ip.pk_indices[:1])
    wl = W.make(e1, "c3", slots=6)
    b1 = e1.upload(W.indexed_for(e1, wl))
    b2 = e2.upload(W.indexed_for(e2, wl))
    stop = threading.Event()
    bad = []

    def pool(b):
        while not stop.is_set():
            if not np.array_equal(np.asarray(b.verify()), wl.expected):
                bad.append(1)
    assert lat.verify_jobs_packed(one) == [1]
    ths = [threading.Thread(target=pool, args=(b,)) for b in (b1, b2)]
    for t in ths:
        t.start()
    time.sleep(0.3)
    ms = []
    try:
        for _ in range(10):
            t0 = time.perf_counter()
            ok = lat.verify_jobs_packed(one) == [1]
            ms.append((time.perf_counter() - t0) * 1e3)
            if not ok:
                bad.append(2)
    finally:
        stop.set()
        for t in ths:
            t.join()
    for b in (b1, b2):
        b.free()
    for e in (lat, e1, e2):
        e.close()
    print(" ".join("%.3f" % x for x in ms))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
