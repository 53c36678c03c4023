"""CPU baseline leg of bench.py (test/benchmark infrastructure only): times oracle/cpu_pool.cpp
(the reference worker-pool policy -- 128-set packages, 16-job batch chunks with per-job retry,
plain verify for 1-set jobs -- over the engine arithmetic compiled for x86-64, "CPU stand-in,
not blst") on a bounded sample of the same workload."""
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
    lib.cpu_verify_jobs_policy.restype = ctypes.c_int
    return lib


def _sub(packed, j0, j1):
    s0, s1 = int(packed.job_off[j0]), int(packed.job_off[j1])
    p0, p1 = int(packed.pk_off[s0]), int(packed.pk_off[s1])
    job_off = (packed.job_off[j0:j1 + 1] - s0).astype(np.uint32)
    pk_off = (packed.pk_off[s0:s1 + 1] - p0).astype(np.uint32)
    return (job_off, pk_off, packed.pubkeys[96 * p0:96 * p1], packed.msgs[32 * s0:32 * s1],
            packed.sigs[96 * s0:96 * s1], s1 - s0)


def _P(a, t):
    return np.ascontiguousarray(a).ctypes.data_as(ctypes.POINTER(t))


def run_jobs(packed, j0, j1, threads):
    """Each job on its own (verifySignatureSetsMaybeBatch per job): the test checker."""
    job_off, pk_off, pks, msgs, sigs, n_sets = _sub(packed, j0, j1)
    out = np.zeros(j1 - j0, dtype=np.int32)
    _lib().cpu_verify_jobs(j1 - j0, _P(job_off, ctypes.c_uint32), _P(pk_off, ctypes.c_uint32),
                           _P(pks, ctypes.c_uint8), _P(msgs, ctypes.c_uint8), _P(sigs, ctypes.c_uint8), threads,
                           _P(out, ctypes.c_int32))
    return out, n_sets


def run_policy(packed, j0, j1, threads, batchable=True):
    """The reference pool's policy over jobs [j0, j1) (oracle/cpu_pool.cpp cpu_verify_jobs_policy)."""
    job_off, pk_off, pks, msgs, sigs, n_sets = _sub(packed, j0, j1)
    out = np.zeros(j1 - j0, dtype=np.int32)
    _lib().cpu_verify_jobs_policy(j1 - j0, _P(job_off, ctypes.c_uint32), _P(pk_off, ctypes.c_uint32),
                                  _P(pks, ctypes.c_uint8), _P(msgs, ctypes.c_uint8), _P(sigs, ctypes.c_uint8),
                                  1 if batchable else 0, threads, _P(out, ctypes.c_int32))
    return out, n_sets


def time_cpu_pool(packed, seconds=15.0, threads=16, batchable=True):
    """Sets/s of the CPU pool (reference policy) on a sample of `packed` sized for ~`seconds` of
    work: evenly spaced contiguous windows of jobs keep the workload's mix."""
    n_jobs = packed.n_jobs
    # calibrate on one small window
    j1 = 0
    s = 0
    while j1 < n_jobs and s < 128:
        s += int(packed.job_off[j1 + 1] - packed.job_off[j1])
        j1 += 1
    t0 = time.perf_counter()
    _, ns = run_policy(packed, 0, j1, 1, batchable)
    per_set = (time.perf_counter() - t0) / max(ns, 1)
    want_sets = int(seconds * threads / per_set)
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
        out, ns = run_policy(packed, j0, j1, threads, batchable)
        total += ns
        assert (out <= 1).all()
    el = time.perf_counter() - t0
    return {"value": round(total / el, 1), "unit": "sets/s", "cores": threads, "kind": "port",
            "sample": f"{total} sets ({sum(j1 - j0 for j0, j1 in spans)} jobs, 8 windows of the same workload) "
                      f"in {el:.1f} s; reference worker policy (128-set packages, batchable jobs in >= 16-job "
                      f"batch chunks with per-job retry, Signature.verify for 1-set jobs; worker.ts:17-98, "
                      f"maybeBatch.ts:16-39) over the engine arithmetic compiled for x86-64 "
                      f"(oracle/cpu_pool.cpp): CPU stand-in, not blst",
            "blst_anchor_sets_s": round(threads / 0.9e-3, 1),
            "blst_anchor": "threads / 0.9 ms per set (packages/beacon-node/src/metrics/metrics/lodestar.ts:505)"}


def time_c1(packed):
    """configs[0]: one verifySignatureSets call of 128 single-pubkey sets = one job, verified by
    one worker as one batch (non-batchable path, worker.ts:91-98)."""
    t0 = time.perf_counter()
    out, ns = run_policy(packed, 0, packed.n_jobs, 1, batchable=False)
    el = time.perf_counter() - t0
    assert (out == 1).all()
    return {"value": round(ns / el, 1), "unit": "sets/s", "cores": 1, "kind": "port", "ms_per_call": round(el * 1e3, 1),
            "sample": f"c1: one call of {ns} single-pubkey sets (one job, one worker thread)",
            "blst_anchor_ms_per_call": round(ns * 0.9, 1)}
