#!/usr/bin/env python3
"""Benchmark: verified signature sets/s on the mainnet gossip attestation mix (BASELINE.json
metric; workload c3 = configs[2]: per slot 16384 attestation sets + 1024 aggregate-and-proof calls
x 3 sets = 17408 jobs / 19456 sets, signing roots shared per committee as on mainnet).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3] [--slots B] [--inflight F]

One process per GPU.  Under torchrun (WORLD_SIZE set) every rank runs main(); `--gpus N` with
N > 1 and no WORLD_SIZE relaunches itself under torch.distributed.run (127.0.0.1) before any GPU
call.  Each rank verifies its own shard (weak scaling: sets shard across GPUs with no data-path
collective; --exchange adds the 576-byte Fp12 partial all-gather over RCCL and one final
exponentiation per step, SURVEY.md §8(e), with the same batches in flight: one process group per
in-flight slot).  A batch = B slots of gossip drained into one device
batch (default 6); F batches are in flight per GPU (default 7 = the engine cap per device,
independent engines; 5 / 6 / 7 in flight measured 9.7 / 10.4 / 10.9 M sets/s in one A/B call).  A step =
lb_batch_verify over one resident batch: all kernels + CSPRNG scalars + per-job result readback.
Inputs are in HBM before the timed region.  Rank 0 prints one JSON line.

Secondary measurements on the same line (rank 0; N = 1 unless noted):
  value_one_batch_in_flight     one engine, the same batch
  value_distinct_roots          every signing root distinct (the no-sharing bound)
  value_one_invalid_per_batch   one wrong-message attestation per slot (the invalid-set search)
  value_distinct_keys           the headline batches over a mainnet-sized resident table (2^20
                                keys, ~10^6 validators as index2pubkey, pubkeyCache.ts:56-77):
                                every validator id its own key, so the G1 gathers miss the cache
  value_e2e                     the headline batches through lb_verify_jobs_indexed with the same
                                engines in flight: inputs in pinned host memory, so the pinned
                                upload (H2D), the host-side chunk decomposition, every kernel and
                                the per-job readback are inside the timed region (SURVEY §8(d)'s
                                metric definition without the JS ceiling)
  value_slots1                  one slot per batch, one batch in flight (+ its latency)
  latency_1set_ms / latency_block_ms   one 1-set call / one c2 block call through lb_verify_jobs
  per_config                    c1, c2, c4, c5, c5_64 at one batch in flight (resident, lb_batch_verify)
  value_dropin                  c3 through the JS IBlsVerifier (tools/bench_dropin.js): JS
                                marshalling + pinned copy + H2D inside the timed region (median of
                                10 rounds; + verifyOnMainThread 1-set latency under load)
  signing_roots                 getBlockSignatureSets + GPU merkleization from JS (K3 block,
                                128-attestation block, 32-block segment)
  cpu_baseline / cpu_c1         the reference worker policy on host cores (oracle/cpu_pool.cpp)
  value_exchange (N > 1)        the headline batches in flight with the single-verdict exchange:
                                576-byte Fp12 partials all-gathered over RCCL, one final
                                exponentiation of their product per batch (distributed.py)
  range_sync_segments (all N)   configs[4]: a 32- and a 64-block segment sharded over the ranks by
                                cost, partial all-gather + one final exponentiation (strong scaling;
                                per-rank ms and sets)
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Each engine drives three HIP streams; HIP's default of 4 hardware queues per process would make
# the streams of the batches in flight share queues (false dependencies between independent
# batches).  24 queues (HIP reads this at runtime init, before any GPU call below) gives each of
# the 7 engines' 21 streams its own (3 per engine up to 32 for more engines).  Measured on MI355X: profiles/r1_inflight_sweep.txt.  The GPU
# boxes export GPU_MAX_HW_QUEUES=4, so raise it rather than only defaulting it.
def _want_queues():
    """3 streams per in-flight engine, at least 24, at most 32 (the pool's limit)"""
    k = 7
    for i, t in enumerate(sys.argv):
        if t == "--inflight" and i + 1 < len(sys.argv):
            k = int(sys.argv[i + 1])
        elif t.startswith("--inflight="):
            k = int(t.split("=", 1)[1])
    return max(24, min(32, 3 * k))


if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < _want_queues():
    os.environ["GPU_MAX_HW_QUEUES"] = str(_want_queues())

import numpy as np  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--slots", type=int, default=6,
                    help="c3: slots of gossip drained into one device batch (profiles/r1_slots_sweep.txt)")
    ap.add_argument("--exchange", action="store_true", help="RCCL all-gather of Fp12 partials per step")
    ap.add_argument("--inflight", type=int, default=7,
                    help="batches in flight per GPU: independent engines (own streams + workspaces) driven by "
                         "one host thread each, like the reference pool's concurrent workers")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pubkey-bytes", action="store_true", help="ship 96-byte pubkeys instead of table indices")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: the host's cores as the reference pool counts them, "
                         "os.cpus().length in multithread/poolSize.ts:7 -> host_cores())")
    ap.add_argument("--no-distinct", action="store_true",
                    help="skip the secondary measurement with every signing root distinct (c3_distinct)")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the secondary legs (invalid-set, slots1, latencies, per-config, drop-in)")
    ap.add_argument("--legs", default="e2e,keys,invalid,slots1,latency,configs,dropin,roots,exchange,segment",
                    help="secondary legs to run (comma list; A/B runs pick one)")
    ap.add_argument("--dropin-engines", type=int, default=4)
    ap.add_argument("--dropin-rounds", type=int, default=10, help="drop-in leg: timed rounds (median reported)")
    return ap.parse_args()


def host_cores():
    """The CPUs this process may run on, as the reference pool sizes itself (poolSize.ts:7,
    os.cpus().length), bounded by the cgroup CPU quota when one is set (threads beyond the quota
    only time-slice).  Returns (threads, detail)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    n = aff if quota is None else max(1, min(aff, int(quota + 0.999)))
    return n, {"sched_getaffinity": aff, "cgroup_cpu_quota": quota, "os_cpu_count": os.cpu_count()}


def relaunch_distributed(a):
    """`bench.py --gpus N` outside torchrun: start N ranks (one per GPU) under
    torch.distributed.run before this process touches the GPU, and exit with its code."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def load_counts():
    p = os.path.join(ROOT, "profiles", "roofline_counts.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def n_roots(packed):
    """distinct signing roots in the batch (the grouped path hashes and Miller-loops once per root)"""
    return int(np.unique(np.asarray(packed.msgs).reshape(-1, 32), axis=0).shape[0]) if packed.n_sets else 0


def stage_work(counts, packed):
    """Algorithmic Fp multiplications per pipeline stage for this batch (profiles/roofline_counts.json
    from tools/count_ops.py: per-item counts of exactly the arithmetic each kernel runs).  hash_to_G2
    and the Miller loop run once per distinct signing root; group_sum is one mixed G1 addition per
    set plus an affine conversion per root; sig_msm is ~8 mixed G2 additions per set (2 points x 4
    windows of 8 bits, lb_kernels.h k_msm_*; bucket reduction excluded)."""
    c = counts["fp_mul_per_item"]
    n = packed.n_sets
    nu = n_roots(packed)
    n_keys = int(packed.pk_off[-1])
    return {
        "decode_sigs": n * c["decode_sigs"],
        "hash_map": 2 * nu * c["hash_map"],
        "hash_finish": nu * c["hash_finish"],
        "pk_chunks": n_keys * c["pk_key"],
        "pk_blind": n * c["g1_blind"],
        "sig_msm": n * 2 * 4 * c.get("g2_madd", 29),
        "group_sum": n * c["pk_blind_per_extra_key"] + nu * 4,
        "miller": nu * c["miller"],
        "tree_up_P": max(nu - 1, 0) * c["fp12_mul"],
        "ml_S": c["ml_S"],
        "root_check": c["final_exp"] + c["fp12_mul"],
    }


def roofline(counts, packed, stage_ms):
    if not counts or not stage_ms:
        return None
    work = stage_work(counts, packed)
    mac = counts["mac_per_fp_mul"]
    peak = counts["peak_tmac_s"]
    per = {}
    for k, fm in work.items():
        if stage_ms.get(k, 0) > 0:
            t = stage_ms[k] * 1e-3
            per[k] = {"ms": round(stage_ms[k], 3), "fp_mul": int(fm), "tmac_s": round(fm * mac / t / 1e12, 3),
                      "frac": round(fm * mac / t / 1e12 / peak, 4)}
    # dominant kernel = the one carrying the most algorithmic work (the chip's time goes there; the
    # latency-bound per-root kernels run few waves beside it)
    dom = max(per, key=lambda k: per[k]["fp_mul"])
    ach = per[dom]["tmac_s"]
    wall = stage_ms.get("total") or sum(stage_ms.values())
    traffic = traffic_src = None
    tp = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tp):
        with open(tp) as f:
            t = json.load(f)
        k = t.get("stages", {}).get(dom)
        if k and k.get("sets_per_launch") == packed.n_sets and "correction" in t:
            traffic = k["bytes_per_launch"]
            traffic_src = t.get("source")
    return {"bound": "valu-int", "kernel": "stage " + dom, "achieved": ach, "peak": peak,
            "unit": "T int32 MAC/s (v_mad_u64_u32)", "frac": round(ach / peak, 4), "traffic": traffic,
            "traffic_note": "HBM bytes per launch of the stage's kernels (profiles/traffic.json: rocprofv3 --pmc "
                            "FETCH_SIZE and WRITE_SIZE in separate passes at this config, 7 in flight), corrected as "
                            "MI355X_MICROARCH.md prescribes for gfx950: 2 x FETCH_SIZE + WRITE_SIZE; the decode "
                            "stage's algorithmic bytes are ~700 B per set: 96 B read and 2 x 192 B + status written "
                            "by the decompression, 192 B re-read by the subgroup check (DESIGN.md 5.2)",
            "traffic_source": traffic_src,
            "algorithmic_bytes": 700 * packed.n_sets if dom == "decode_sigs" else None,
            "whole_pipeline_frac": round(sum(work.values()) * mac / (wall * 1e-3) / 1e12 / peak, 4),
            "device_ms": round(wall, 3), "stages": per}


def run_inflight(batches, steps, expected, barrier, step_fns=None, mark=None):
    """len(batches) batches in flight: independent engines (own streams + workspaces), one host
    thread each, every engine verifying its own resident copy of the slot `steps` times
    (step_fns[k]() instead of batches[k].verify() when given: the --exchange steps).
    mark(): called right before and right after the timed region (profiling markers)."""
    import threading
    fns = step_fns or [b.verify for b in batches]
    for f in fns[1:]:
        f()
    res = [None] * len(batches)

    def run(k):
        for _ in range(steps):
            res[k] = fns[k]()

    barrier()
    if mark:
        mark()
    t1 = time.perf_counter()
    ths = [threading.Thread(target=run, args=(k,)) for k in range(len(batches))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    barrier()
    el = time.perf_counter() - t1
    if mark:
        mark()
    for r in res:
        assert np.array_equal(np.asarray(r), expected), "verification results differ"
    return el


def median_ms(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    return round(float(np.median(ts)), 3)


def profiled_stages(eng, fn):
    """per-stage HIP-event times (ms) of one profiled call"""
    eng.set_profiling(True)
    fn()
    prof = eng.last_profile()
    eng.set_profiling(False)
    return {k: round(v, 3) for k, v in prof.items() if v > 0}


def pinned_like(lib, arr, keep):
    """a copy of `arr` in pinned host memory (lb_host_alloc); the allocation is appended to keep"""
    import ctypes
    arr = np.ascontiguousarray(arr)
    n = max(arr.nbytes, 1)
    p = lib.lb_host_alloc(n)
    if not p:
        raise MemoryError("lb_host_alloc")
    keep.append(p)
    buf = (ctypes.c_uint8 * n).from_address(p)
    out = np.frombuffer(buf, dtype=arr.dtype, count=arr.size).reshape(arr.shape)
    out[...] = arr
    return out


def e2e_leg(a, engs, barrier, W, wl):
    """value_e2e: every engine uploads + verifies + reads back the headline batch from pinned host
    memory (lb_verify_jobs_indexed through its engine-owned workspace), batches in flight."""
    import threading
    lib = engs[0].lib
    keep = []
    try:
        packs = []
        for e in engs:
            ip = W.indexed_for(e, wl)
            packs.append(W.PackedJobs(job_off=pinned_like(lib, ip.job_off, keep), pk_off=pinned_like(lib, ip.pk_off, keep),
                                      pubkeys=None, msgs=pinned_like(lib, ip.msgs, keep),
                                      sigs=pinned_like(lib, ip.sigs, keep), sig_sizes=None,
                                      pk_indices=pinned_like(lib, ip.pk_indices, keep)))
        for e, pk in zip(engs, packs):  # warm the workspaces
            assert np.array_equal(np.asarray(e.verify_jobs_packed(pk)), wl.expected), "e2e verdicts differ"
        steps = max(2, a.steps // 2)
        res = [None] * len(engs)

        def run(k):
            for _ in range(steps):
                res[k] = engs[k].verify_jobs_packed(packs[k])

        barrier()
        t1 = time.perf_counter()
        ths = [threading.Thread(target=run, args=(k,)) for k in range(len(engs))]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        barrier()
        el = time.perf_counter() - t1
        for r in res:
            assert np.array_equal(np.asarray(r), wl.expected), "e2e verdicts differ"
        return {"value_e2e": round(wl.packed.n_sets * steps * len(engs) / el, 1),
                "e2e": {"engines": len(engs), "steps_per_engine": steps, "seconds": round(el, 3),
                        "input_bytes_per_batch": int(sum(x.nbytes for x in (packs[0].job_off, packs[0].pk_off,
                                                                               packs[0].msgs, packs[0].sigs,
                                                                               packs[0].pk_indices))),
                        "path": "lb_verify_jobs_indexed from pinned host buffers: chunking + H2D + kernels + D2H"}}
    finally:
        for p in keep:
            lib.lb_host_free(p)


def extra_legs(a, engs, barrier, W, wl_main=None):
    """Secondary measurements (rank 0 at N = 1; each bounded to a few seconds)."""
    out = {}
    eng = engs[0]
    legs = set(a.legs.split(","))
    if wl_main is not None and "e2e" in legs:
        out.update(e2e_leg(a, engs, barrier, W, wl_main))
    if "keys" in legs:
        out.update(distinct_keys_leg(a, engs, barrier, W))
    if "invalid" in legs:
        out.update(invalid_leg(a, engs, barrier, W))
    wc1 = W.make(eng, "c1")
    if "slots1" in legs:
        out.update(slots1_leg(a, eng, W))
    if "latency" in legs:
        out.update(latency_leg(eng, W, wc1))
    if "configs" in legs:
        out["per_config"] = configs_leg(a, eng, W)
    return out, wc1


def distinct_keys_leg(a, engs, barrier, W):
    """value_distinct_keys: the c3 batch shape with validator v -> key v of a 2^20-key resident
    table (SURVEY.md §8(d)'s distinct-key variant of the v mod 100 convention), batches in flight"""
    t0 = time.time()
    kp = W.KeyPool(engs[0], W.N_KEYS_MAINNET)
    wk = W.make(engs[0], "c3", keys=kp, slots=a.slots) if a.slots > 1 else W.make(engs[0], "c3", keys=kp)
    batches = [e.upload(W.indexed_for(e, wk)) for e in engs]
    setup_s = time.time() - t0
    assert np.array_equal(np.asarray(batches[0].verify()), wk.expected), "distinct-key verdicts differ"
    steps = max(2, a.steps // 2)
    el = run_inflight(batches, steps, wk.expected, barrier) if len(engs) > 1 else None
    if el is None:
        barrier()
        t1 = time.perf_counter()
        for _ in range(steps):
            batches[0].verify()
        barrier()
        el = time.perf_counter() - t1
    eng = engs[0]
    prof = profiled_stages(eng, batches[0].verify)
    for b in batches:
        b.free()
    idx = wk.packed.pk_indices
    return {"value_distinct_keys": round(wk.packed.n_sets * steps * len(engs) / el, 1),
            "distinct_keys": {"table_keys": len(kp.sks), "table_mb_per_engine": round(len(kp.sks) * 128 / 2 ** 20, 1),
                              "key_gathers_per_batch": int(idx.size),
                              "distinct_keys_per_batch": int(np.unique(idx).size),
                              "pk_chunks_ms_one_batch": prof.get("pk_chunks"), "setup_s": round(setup_s, 1)}}


def invalid_leg(a, engs, barrier, W):
    """one invalid attestation per slot: the failing root's search, batches in flight"""
    out = {}
    eng = engs[0]
    wi = W.make(eng, "c3_invalid", slots=a.slots)
    batches = [e.upload(W.indexed_for(e, wi)) for e in engs]
    codes = batches[0].verify()
    assert np.array_equal(np.asarray(codes), wi.expected), "invalid-set search verdicts differ"
    steps = max(2, a.steps // 2)
    if len(engs) > 1:
        el = run_inflight(batches, steps, wi.expected, barrier)
    else:
        barrier()
        t1 = time.perf_counter()
        for _ in range(steps):
            batches[0].verify()
        barrier()
        el = time.perf_counter() - t1
    out["value_one_invalid_per_batch"] = round(wi.packed.n_sets * steps * len(engs) / el, 1)
    eng.set_profiling(True)
    batches[0].verify()
    prof = eng.last_profile()
    eng.set_profiling(False)
    out["invalid_batch_stage_ms"] = {k: round(v, 3) for k, v in prof.items() if v > 0}
    for b in batches:
        b.free()
    return out


def slots1_leg(a, eng, W):
    """one slot per batch, one batch in flight"""
    out = {}
    w1 = W.make(eng, "c3")
    b1 = eng.upload(W.indexed_for(eng, w1))
    b1.verify()
    lat = median_ms(lambda: b1.verify(), max(3, a.steps))
    out["value_slots1"] = round(w1.packed.n_sets / (lat * 1e-3), 1)
    out["latency_slot1_ms"] = lat
    out["slots1_stage_ms"] = profiled_stages(eng, b1.verify)
    b1.free()
    return out


def latency_leg(eng, W, wc1):
    """small calls through the workspace path (lb_verify_jobs_indexed: upload + verify + readback)"""
    out = {}
    ip = W.indexed_for(eng, wc1)
    one = W.PackedJobs(job_off=np.array([0, 1], np.uint32), pk_off=np.array([0, 1], np.uint32), pubkeys=None,
                       msgs=ip.msgs[:32], sigs=ip.sigs[:96], sig_sizes=None, pk_indices=ip.pk_indices[:1])
    assert eng.verify_jobs_packed(one) == [1]
    out["latency_1set_ms"] = median_ms(lambda: eng.verify_jobs_packed(one), 10)
    out["latency_1set_stage_ms"] = profiled_stages(eng, lambda: eng.verify_jobs_packed(one))
    wc2 = W.make(eng, "c2")
    ip2 = W.indexed_for(eng, wc2)
    assert eng.verify_jobs_packed(ip2) == list(wc2.expected)
    out["latency_block_ms"] = median_ms(lambda: eng.verify_jobs_packed(ip2), 10)
    out["latency_block_stage_ms"] = profiled_stages(eng, lambda: eng.verify_jobs_packed(ip2))
    return out


def configs_leg(a, eng, W):
    """the other BASELINE configs at one batch in flight (resident inputs)"""
    per = {}
    for name in ("c1", "c2", "c4", "c5", "c5_64"):
        wl = W.make(eng, name)
        b = eng.upload(W.indexed_for(eng, wl))
        got = b.verify()
        assert np.array_equal(np.asarray(got), wl.expected), name
        ms = median_ms(lambda: b.verify(), 3)
        per[name] = {"sets": wl.packed.n_sets, "jobs": wl.packed.n_jobs, "ms_per_batch": ms,
                     "sets_per_s": round(wl.packed.n_sets / (ms * 1e-3), 1),
                     "invalid_or_rejected_jobs": int((wl.expected != 1).sum())}
        b.free()
        if not a.no_cpu_baseline:
            # the CPU stand-in pool on the same workload (bounded sample, a few seconds); c4 is
            # gossip (batchable), the block-shaped configs are one non-batchable call per block
            try:
                from oracle.cpu_pool import time_cpu_pool
                c = time_cpu_pool(wl.packed, seconds=2.5, threads=a.cpu_threads, batchable=(name == "c4"))
                per[name]["cpu_sets_per_s"] = c["value"]
                per[name]["cpu_threads"] = c["cores"]
            except Exception as e:  # reported, never fatal
                per[name]["cpu_error"] = repr(e)
    return per


def segment_legs(a, eng, W, rank, world, barrier, coll_dev, backend):
    """configs[4]: a range-sync segment (32 and 64 blocks of ~131 sets, the same segment on every
    rank) sharded over the ranks by cost (distributed.shard_jobs_by_cost), each rank reducing its
    shard to a 576-byte Fp12 partial (lb_batch_partial), the partials all-gathered over RCCL and one
    final exponentiation of their product per rank (distributed.verify_sharded); at N = 1 the
    partial and the product check run locally.  Strong scaling: the segment is fixed as N grows."""
    import torch
    import torch.distributed as dist
    from lodestar_amd.distributed import shard_jobs_by_cost, verify_sharded
    out = {}
    for name, blocks in (("c5", 32), ("c5_64", 64)):
        wl = W.make(eng, name)
        lo, hi = shard_jobs_by_cost(wl.packed.job_off, wl.packed.pk_off, world, rank)
        shard = W.slice_jobs(W.indexed_for(eng, wl), lo, hi)
        b = eng.upload(shard)
        try:
            if world > 1:
                def step():
                    return verify_sharded(b.partial, eng.product_is_one, b.search_after_partial,
                                          device=coll_dev if coll_dev.type == "cuda" else None)
            else:
                def step():
                    f, st = b.partial()
                    ok = eng.product_is_one([f])
                    return ([int(x) for x in st] if ok else [int(x) for x in b.search_after_partial()]), ok
            codes, ok = step()
            assert ok and np.array_equal(np.asarray(codes), wl.expected[lo:hi]), name
            reps = max(3, a.steps)
            barrier()
            t1 = time.perf_counter()
            for _ in range(reps):
                codes, ok = step()
            barrier()
            el = (time.perf_counter() - t1) / reps
            assert ok, name
            mine = torch.tensor([el * 1e3, float(shard.n_sets)], dtype=torch.float64, device=coll_dev)
            if world > 1:
                allv = [torch.zeros_like(mine) for _ in range(world)]
                dist.all_gather(allv, mine)
                allv = [v.cpu().tolist() for v in allv]
            else:
                allv = [mine.cpu().tolist()]
            ms = max(v[0] for v in allv)
            out[name] = {"blocks": blocks, "sets": wl.packed.n_sets, "jobs": wl.packed.n_jobs,
                         "ms_per_segment": round(ms, 3), "sets_per_s": round(wl.packed.n_sets / (ms * 1e-3), 1),
                         "rank_ms": [round(v[0], 3) for v in allv], "rank_sets": [int(v[1]) for v in allv],
                         "sharding": "whole jobs, balanced by cost (distributed.shard_jobs_by_cost)",
                         "exchange": ("all_gather of 576-byte partials (%s) + one final exponentiation" % backend)
                         if world > 1 else "local partial + one final exponentiation",
                         "world_size_seen": world}
        finally:
            b.free()
    return out


def dropin_leg(a, W, eng_factory):
    """c3 through the JS IBlsVerifier in a node child process (tools/bench_dropin.js)."""
    import shutil
    node = shutil.which("node")
    if node is None:
        return {"error": "node not installed"}
    e = eng_factory()
    try:
        wl = W.make(e, "c3", slots=a.slots) if a.slots > 1 else W.make(e, "c3")
    finally:
        e.close()
    p = wl.packed
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        hdr = np.array([0x4C424430, len(wl.pool96), p.n_jobs, p.n_sets, int(p.pk_off[-1]), a.slots], np.uint32)
        for arr in (hdr, np.ascontiguousarray(wl.pool96, np.uint8), p.job_off.astype(np.uint32),
                    p.pk_off.astype(np.uint32), p.pk_indices.astype(np.uint32), p.msgs, p.sigs,
                    wl.expected.astype(np.int32)):
            f.write(np.ascontiguousarray(arr).tobytes())
        path = f.name
    try:
        r = subprocess.run([node, os.path.join(ROOT, "tools", "bench_dropin.js"), path, str(a.dropin_engines),
                            str(a.dropin_rounds)], capture_output=True, text=True, timeout=300)
    finally:
        os.unlink(path)
    if r.returncode != 0:
        return {"error": (r.stdout + r.stderr)[-500:]}
    return json.loads(r.stdout.strip().splitlines()[-1])


def signing_roots_leg():
    """getBlockSignatureSets + GPU merkleization from the TS host's side (lodestar_amd/js/signing_roots.js
    through addon.merkleize): the K3 devnet block, a 128-attestation block and a 32-block segment,
    against the reference's ~45 ms per 100-signature block (verifyBlocksSignatures.ts:41-43)."""
    import shutil
    node = shutil.which("node")
    if node is None:
        return {"error": "node not installed"}
    r = subprocess.run([node, os.path.join(ROOT, "tests", "js", "test_signing_roots.js"), "gpu"],
                       capture_output=True, text=True, timeout=240)
    if r.returncode != 0:
        return {"error": (r.stdout + r.stderr)[-500:]}
    return json.loads(r.stdout.strip().splitlines()[-2])


def main():
    a = parse()
    cores_detail = None
    if a.cpu_threads <= 0:
        a.cpu_threads, cores_detail = host_cores()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_distributed(a))
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (not used by the driver): LB_BENCH_BACKEND=gloo + LB_BENCH_DEVICE=0 run N ranks
    # on one GPU with CPU-side collectives
    backend = os.environ.get("LB_BENCH_BACKEND", "nccl")
    if os.environ.get("LB_BENCH_DEVICE") is not None:
        local = int(os.environ["LB_BENCH_DEVICE"])
    coll_dev = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")
    world_seen = 1
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        world_seen = dist.get_world_size()

    from lodestar_amd.engine import Engine
    from lodestar_amd import workloads as W

    engs = [Engine(local) for _ in range(a.inflight)]
    eng = engs[0]
    t0 = time.time()
    wkw = {"slots": a.slots} if a.workload.startswith("c3") and a.slots > 1 else {}
    wl = W.make(eng, a.workload, seed=W.SEED + rank, **wkw)
    gen_s = time.time() - t0
    # pubkeys as indices into each engine's resident table (the epoch cache's index2pubkey path);
    # --pubkey-bytes ships 96-byte keys instead
    if a.pubkey_bytes:
        batches = [e.upload(W.PackedJobs(job_off=wl.packed.job_off, pk_off=wl.packed.pk_off,
                                         pubkeys=wl.packed.pubkeys, msgs=wl.packed.msgs, sigs=wl.packed.sigs,
                                         sig_sizes=wl.packed.sig_sizes)) for e in engs]
    else:
        batches = [e.upload(W.indexed_for(e, wl)) for e in engs]
    batch = batches[0]
    n_sets, n_jobs = wl.packed.n_sets, wl.packed.n_jobs

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    # --exchange: every batch in flight has its own process group (created in the same order on
    # every rank), so the engines' all-gathers of different batches proceed independently
    # (created whenever world > 1: the N > 1 line also carries the exchange leg)
    groups = [None] * a.inflight
    if world > 1:
        groups = [dist.new_group(list(range(world))) for _ in range(a.inflight)]

    def make_step(k, exchange=a.exchange):
        b, e = batches[k], engs[k]
        if not (exchange and world > 1):
            return b.verify
        from lodestar_amd.distributed import verify_sharded

        def xstep():
            # 576-byte partials over RCCL, one final exponentiation of their product (distributed.py)
            codes, _ = verify_sharded(b.partial, e.product_is_one, b.search_after_partial, group=groups[k],
                                      device=coll_dev if coll_dev.type == "cuda" else None)
            return codes
        return xstep

    step = make_step(0)

    for _ in range(a.warmup):
        codes = step()
    assert np.array_equal(np.asarray(codes), wl.expected), "verification results differ from expected"

    # (1) one batch in flight: K profiled steps (per-stage HIP-event times feed the roofline)
    stage_ms = {}
    eng.set_profiling(True)
    barrier()
    t1 = time.perf_counter()
    for _ in range(a.steps):
        codes = step()
        for k, v in eng.last_profile().items():
            stage_ms[k] = stage_ms.get(k, 0.0) + v
    barrier()
    el_single = time.perf_counter() - t1
    eng.set_profiling(False)
    stage_ms = {k: v / a.steps for k, v in stage_ms.items()}
    el = el_single
    inflight = a.inflight
    # LB_PROF_MARK=1: an empty lb_fp12_product_is_one (one k_partials_check dispatch) right before
    # and after the headline's timed region, so a counter pass (tools/valu_util.py) can keep
    # exactly the timed region's dispatches (not the workload generator's k_sign, nor the one
    # batch in flight above)
    mark = (lambda: engs[0].product_is_one([])) if os.environ.get("LB_PROF_MARK") == "1" else None
    if inflight > 1:
        el = run_inflight(batches, a.steps, wl.expected, barrier, [make_step(k) for k in range(inflight)], mark)
    el_t = torch.tensor([el], dtype=torch.float64, device=coll_dev)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el = float(el_t.item())
    es_t = torch.tensor([el_single], dtype=torch.float64, device=coll_dev)
    if world > 1:
        dist.all_reduce(es_t, op=dist.ReduceOp.MAX)
    value_single = n_sets * world * a.steps / float(es_t.item())
    ms_per_step = el / (a.steps * inflight) * 1e3
    value = n_sets * world * a.steps * inflight / el

    # N > 1: the same batches in flight with the north-star single-verdict exchange (576-byte Fp12
    # partials all-gathered over RCCL, one final exponentiation of their product per step)
    exchange_leg = None
    if world > 1 and not a.exchange and "exchange" in a.legs.split(","):
        elx = run_inflight(batches, a.steps, wl.expected, barrier,
                           [make_step(k, exchange=True) for k in range(inflight)])
        elx_t = torch.tensor([elx], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(elx_t, op=dist.ReduceOp.MAX)
        elx = float(elx_t.item())
        exchange_leg = {"value": round(n_sets * world * a.steps * inflight / elx, 1),
                        "ms_per_step": round(elx / (a.steps * inflight) * 1e3, 3),
                        "collective": "all_gather of 576-byte Fp12 partials per batch (backend %s)" % backend,
                        "world_size_seen": world_seen}
    roof = roofline(load_counts(), wl.packed, stage_ms)
    if roof is not None:
        # the headline's own fraction: all stages' algorithmic MACs per batch over the measured
        # time per batch at this configuration (ms_per_step, batches in flight), against the peak
        cnt = load_counts()
        work = sum(stage_work(cnt, wl.packed).values()) * cnt["mac_per_fp_mul"]
        roof["chip_frac"] = round(work / (ms_per_step * 1e-3) / 1e12 / cnt["peak_tmac_s"], 4)
        roof["chip_frac_note"] = ("sum of every stage's algorithmic Fp-mul x 300 MACs per batch / ms_per_step / "
                                  "peak: the headline's VALU utilisation, reproducible from this line alone")
        roof["stage_ms_source"] = ("HIP events on each stage's own stream, one batch in flight, %d profiled steps; "
                                   "profiles/r6_rocprof_kernel_stats_inflight1.csv holds rocprof's per-kernel "
                                   "averages for the same configuration (the round-6 final tree); "
                                   "tools/trace_stage_avg.py -> profiles/r6_inflight1_decode_check.json compares them" % a.steps)
        roof["valu_util_source"] = ("profiles/r6_valu_util.json: per-kernel VALU instructions per batch and VALU-busy "
                                    "fraction from rocprofv3 counters at this configuration (tools/valu_util.py)")
        roof["resource_table"] = "profiles/r6_resource_usage.txt (VGPR / AGPR / scratch / LDS per kernel, hipcc remarks)"
    segments = None
    if a.workload == "c3" and "segment" in a.legs.split(","):
        segments = segment_legs(a, eng, W, rank, world, barrier, coll_dev, backend)
    # secondary: the same slot shape with every signing root distinct (no sharing to exploit)
    value_distinct = None
    if a.workload == "c3" and not a.no_distinct and not a.exchange:
        wd = W.make(eng, "c3_distinct", seed=W.SEED + rank, **wkw)
        for b in batches:
            b.free()
        batches = [e.upload(W.indexed_for(e, wd)) for e in engs]
        batches[0].verify()
        eld = run_inflight(batches, a.steps, wd.expected, barrier) if a.inflight > 1 else None
        if eld is None:
            barrier()
            t1 = time.perf_counter()
            for _ in range(a.steps):
                batches[0].verify()
            barrier()
            eld = time.perf_counter() - t1
        eld_t = torch.tensor([eld], dtype=torch.float64, device=coll_dev)
        if world > 1:
            dist.all_reduce(eld_t, op=dist.ReduceOp.MAX)
        value_distinct = wd.packed.n_sets * world * a.steps * a.inflight / float(eld_t.item())
    for b in batches:
        b.free()
    solo = rank == 0 and world == 1 and not a.no_extra and a.workload == "c3" and not a.exchange
    extra, dropin, wc1 = {}, None, None
    if solo:
        extra, wc1 = extra_legs(a, engs, barrier, W, wl)
    for e in engs:
        e.close()
    if solo and "dropin" in a.legs.split(","):
        try:
            dropin = dropin_leg(a, W, lambda: Engine(local))
        except Exception as e:  # reported, never fatal
            dropin = {"error": repr(e)}
    if solo and "roots" in a.legs.split(","):
        try:
            extra["signing_roots"] = signing_roots_leg()
        except Exception as e:  # reported, never fatal
            extra["signing_roots"] = {"error": repr(e)}
    cpu = cpu_c1 = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            from oracle.cpu_pool import time_c1, time_cpu_pool
            cpu = time_cpu_pool(wl.packed, seconds=a.cpu_seconds, threads=a.cpu_threads,
                                batchable=a.workload.startswith("c3"))
            cpu["host_cores"] = cores_detail or {"cpu_threads_flag": a.cpu_threads}
            if wc1 is not None:
                cpu_c1 = time_c1(wc1.packed)
        except Exception as e:  # reported, never fatal
            cpu = {"error": repr(e)}

    if rank == 0:
        line = {
            "metric": "verified signature sets/sec (mainnet attestation mix)",
            "value": round(value, 1), "unit": "sets/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32 (381-bit Montgomery; device products on 14x28-bit limbs)",
            "data": "synthetic",
            "config": {"workload": (f"{a.workload}: gossip attestation flood, {a.slots} slot(s) per batch, "
                                    f"{inflight} batches in flight per GPU") if a.workload == "c3" else a.workload,
                       "slots_per_batch": a.slots, "sets_per_gpu": n_sets, "jobs_per_gpu": n_jobs,
                       "pubkeys_per_gpu": int(wl.packed.pk_off[-1]), "parallelism": f"dp{world} (sets sharded)",
                       "exchange": bool(a.exchange), "inflight": inflight, "world_size_seen": world_seen,
                       "pubkeys": "96-byte keys per set" if a.pubkey_bytes else "indices into the GPU-resident table",
                       "signing_roots_per_gpu": n_roots(wl.packed)},
            "value_one_batch_in_flight": round(value_single, 1),
            "batch_latency_ms": round(el / a.steps * 1e3, 1),
            "value_distinct_roots": None if value_distinct is None else round(value_distinct, 1),
        }
        if exchange_leg is not None:
            line["value_exchange"] = exchange_leg["value"]
            line["exchange"] = exchange_leg
        if segments is not None:
            line["range_sync_segments"] = segments
        line.update(extra)
        if dropin is not None:
            line["value_dropin"] = dropin.get("value_dropin")
            line["dropin"] = dropin
        line.update({"roofline": roof, "cpu_baseline": cpu, "cpu_c1": cpu_c1, "gen_s": round(gen_s, 2)})
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
