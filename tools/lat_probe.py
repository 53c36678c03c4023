# Probe (tools/, not a test): a latency engine 1-set call idle and under two pool engines.
import os, sys, threading, time
import numpy as np
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
from lodestar_amd.engine import Engine
from lodestar_amd import workloads as W
flag = int(sys.argv[1]); slots = int(sys.argv[2])
lat = Engine(0, flag)
e1, e2 = Engine(0), Engine(0)
ip = W.indexed_for(lat, W.make(lat, "c1"))
one = W.PackedJobs(job_off=np.array([0, 1], np.uint32), pk_off=np.array([0, 1], np.uint32), pubkeys=None,
                   msgs=ip.msgs[:32], sigs=ip.sigs[:96], sig_sizes=None, pk_indices=ip.pk_indices[:1])
wl = W.make(e1, "c3", slots=slots)
b1 = e1.upload(W.indexed_for(e1, wl)); b2 = e2.upload(W.indexed_for(e2, wl))
def timed(k):
    ms = []
    for _ in range(k):
        t0 = time.perf_counter(); lat.verify_jobs_packed(one); ms.append((time.perf_counter() - t0) * 1e3)
    return sorted(ms)
print("idle", timed(5))
lat.set_profiling(True); lat.verify_jobs_packed(one); print("idle stages", {k: round(v, 2) for k, v in lat.last_profile().items() if v > 0}); lat.set_profiling(False)
stop = threading.Event()
done = [0]
def pool(b):
    while not stop.is_set():
        b.verify(); done[0] += 1
ths = [threading.Thread(target=pool, args=(b,)) for b in (b1, b2)]
for t in ths: t.start()
time.sleep(0.3)
d0, t0 = done[0], time.perf_counter()
print("load", timed(10))
time.sleep(1.0)
print("pool sets/s", round((done[0] - d0) * wl.packed.n_sets / (time.perf_counter() - t0)))
stop.set()
for t in ths: t.join()
