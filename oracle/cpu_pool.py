"""CPU baseline leg of bench.py (test/benchmark infrastructure only): times oracle/cpu_pool.cpp
(the reference worker-pool policy over the engine arithmetic compiled for x86-64, "CPU
stand-in, not blst") on a bounded sample of the same workload."""
import ctypes
import os
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "build", "lb_cpu_pool.so")


def _lib():
    if not os.path.exists(SO):
        from lodestar_amd.build import build_cpu_pool
        build_cpu_pool(verbose=False)
    lib = ctypes.CDLL(SO)
    lib.cpu_verify_jobs.restype = ctypes.c_int
    return lib


def _sub(packed, j0, j1):
    s0, s1 = int(packed.job_off[j0]), int(packed.job_off[j1])
    p0, p1 = int(packed.pk_off[s0]), int(packed.pk_off[s1])
    job_off = (packed.job_off[j0:j1 + 1] - s0).astype(np.uint32)
    pk_off = (packed.pk_off[s0:s1 + 1] - p0).astype(np.uint32)
    return (job_off, pk_off, packed.pubkeys[96 * p0:96 * p1], packed.msgs[32 * s0:32 * s1],
            packed.sigs[96 * s0:96 * s1], s1 - s0)


def run_jobs(packed, j0, j1, threads):
    job_off, pk_off, pks, msgs, sigs, n_sets = _sub(packed, j0, j1)
    out = np.zeros(j1 - j0, dtype=np.int32)
    P = lambda a, t: np.ascontiguousarray(a).ctypes.data_as(ctypes.POINTER(t))  # noqa: E731
    _lib().cpu_verify_jobs(j1 - j0, P(job_off, ctypes.c_uint32), P(pk_off, ctypes.c_uint32), P(pks, ctypes.c_uint8),
                           P(msgs, ctypes.c_uint8), P(sigs, ctypes.c_uint8), threads, P(out, ctypes.c_int32))
    return out, n_sets


def time_cpu_pool(packed, seconds=15.0, threads=16):
    """Sets/s of the CPU pool on a prefix sample of `packed` sized for ~`seconds` of work.
    The sample keeps the workload's job mix by striding over its jobs."""
    n_jobs = packed.n_jobs
    # calibrate on a small strided sample
    stride = max(1, n_jobs // (threads * 4))
    t0 = time.perf_counter()
    sets = 0
    for j in range(0, n_jobs, stride):
        _, ns = run_jobs(packed, j, j + 1, 1)
        sets += ns
        if time.perf_counter() - t0 > 1.0:
            break
    per_set = (time.perf_counter() - t0) / max(sets, 1)
    want_sets = int(seconds * threads / per_set)
    # take evenly spaced contiguous windows to keep the mix
    windows = 8
    per_win = max(1, want_sets // windows)
    spans, total = [], 0
    for w in range(windows):
        j0 = (n_jobs * w) // windows
        j1 = j0
        s = 0
        while j1 < n_jobs and s < per_win:
            s += int(packed.job_off[j1 + 1] - packed.job_off[j1])
            j1 += 1
        spans.append((j0, j1))
    t0 = time.perf_counter()
    for j0, j1 in spans:
        out, ns = run_jobs(packed, j0, j1, threads)
        total += ns
        assert (out == 1).all() or (out <= 1).all()
    el = time.perf_counter() - t0
    return {"value": round(total / el, 1), "unit": "sets/s", "cores": threads, "kind": "port",
            "sample": f"{total} sets ({sum(j1 - j0 for j0, j1 in spans)} jobs, 8 windows of the same workload) "
                      f"in {el:.1f} s; reference worker policy (one batch + one final exp per job) over the "
                      f"engine arithmetic compiled for x86-64 (oracle/cpu_pool.cpp): CPU stand-in, not blst",
            "blst_anchor_sets_s": round(threads / 0.9e-3, 1),
            "blst_anchor": "threads / 0.9 ms per set (packages/beacon-node/src/metrics/metrics/lodestar.ts:505)"}
