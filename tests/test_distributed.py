"""World-size-2 gloo runs of the multi-GPU exchange protocol (lodestar_amd/distributed.py): on CPU
with the CPU counterparts of lb_batch_partial / lb_fp12_product_is_one (oracle/cpu_pool.cpp), and
on the GPU box with two ranks sharing device 0, whose partials come from lb_batch_partial."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, load_json


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _jobs(bad_case=None):
    from lodestar_amd.engine import SetInput
    names = ["single_valid_0", "two_valid", "aggregate_valid", "aggregate_duplicate_keys", "k4_like_batch",
             "mixed_valid_with_aggregate"]
    if bad_case:
        names.insert(3, bad_case)
    cases = {c["name"]: c for c in load_json("jobs.json")["cases"]}
    return [[SetInput([bytes.fromhex(p) for p in s["pubkeys"]], bytes.fromhex(s["signing_root"]),
                      bytes.fromhex(s["signature"])) for s in cases[n]["sets"]] for n in names], \
        [cases[n]["expected"] for n in names]


def _worker(rank, world, port, bad_case, out, by_cost=False):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from lodestar_amd.distributed import shard_jobs, shard_jobs_by_cost, verify_sharded
    from lodestar_amd.engine import pack_jobs
    from oracle.cpu_pool import _lib, run_jobs
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    jobs, _ = _jobs(bad_case)
    if by_cost:
        whole = pack_jobs(jobs)
        lo, hi = shard_jobs_by_cost(whole.job_off, whole.pk_off, world, rank)
    else:
        lo, hi = shard_jobs(len(jobs), world, rank)
    packed = pack_jobs(jobs[lo:hi])
    lib = _lib()
    P = lambda a, t: np.ascontiguousarray(a).ctypes.data_as(ctypes.POINTER(t))  # noqa: E731

    def partial():
        buf = (ctypes.c_uint8 * 576)()
        st = np.zeros(packed.n_jobs, dtype=np.int32)
        lib.cpu_partial(packed.n_jobs, P(packed.job_off, ctypes.c_uint32), P(packed.pk_off, ctypes.c_uint32),
                        P(packed.pubkeys, ctypes.c_uint8), P(packed.msgs, ctypes.c_uint8),
                        P(packed.sigs, ctypes.c_uint8), ctypes.c_uint64(0x1234 + rank),
                        ctypes.cast(buf, ctypes.POINTER(ctypes.c_uint8)), P(st, ctypes.c_int32))
        return bytes(buf), list(st)

    def product(parts):
        b = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
        return bool(lib.cpu_product_is_one(P(b, ctypes.c_uint8), len(parts)))

    def local():
        return list(run_jobs(packed, 0, packed.n_jobs, 2)[0])

    codes, ok = verify_sharded(partial, product, local)
    out.put((rank, lo, codes, ok))
    dist.destroy_process_group()


def _run(bad_case, by_cost=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, bad_case, q, by_cost)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    codes = [c for _, _, cs, _ in res for c in cs]
    return codes, [ok for *_, ok in res]


def _expected_codes(exp):
    from lodestar_amd import _native as N
    names = {N.error_name(c): c for c in range(1, 13)}
    return [(1 if e else 0) if isinstance(e, bool) else -names[e] for e in exp]


def test_gloo_two_ranks_all_valid():
    codes, oks = _run(None)
    assert oks == [True, True]
    assert codes == [1] * len(codes)


def test_gloo_two_ranks_invalid_job_localised():
    codes, oks = _run("batch_one_wrong")
    assert oks == [False, False]
    _, exp = _jobs("batch_one_wrong")
    assert codes == _expected_codes(exp)


def test_shard_jobs_by_cost_balances_unequal_jobs():
    """whole jobs per rank, balanced by device work (per-set cost + per-key
    cost), contiguous and covering every job exactly once; a segment of one heavy block job among
    many 1-set jobs splits by work, not by job count."""
    from lodestar_amd.distributed import KEY_COST, SET_COST, job_costs, shard_jobs_by_cost
    rng = np.random.default_rng(5)
    for trial in range(20):
        n_jobs = int(rng.integers(1, 60))
        sets = rng.integers(1, 6, n_jobs)
        job_off = np.concatenate([[0], np.cumsum(sets)])
        keys = np.where(rng.random(job_off[-1]) < 0.2, rng.integers(100, 512, job_off[-1]), 1)
        pk_off = np.concatenate([[0], np.cumsum(keys)])
        cost = job_costs(job_off, pk_off)
        assert cost.sum() == SET_COST * job_off[-1] + KEY_COST * pk_off[-1]
        for world in (1, 2, 3, 4, 8):
            rs = [shard_jobs_by_cost(job_off, pk_off, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n_jobs
            assert all(rs[r][1] == rs[r + 1][0] and rs[r][0] <= rs[r][1] for r in range(world - 1))
            # no rank carries more than its share plus one job
            share = cost.sum() / world
            for lo, hi in rs:
                assert cost[lo:hi].sum() <= share + cost.max() + 1
    # the count-based split would give rank 0 both heavy jobs here; by cost they separate
    job_off = np.arange(0, 11)
    pk_off = np.concatenate([[0], np.cumsum([2048, 2048] + [1] * 8)])
    assert shard_jobs_by_cost(job_off, pk_off, 2, 0) == (0, 1)


def test_gloo_two_ranks_cost_sharded_invalid_job_localised():
    """The exchange protocol over cost-balanced shards (unequal jobs: aggregates of many keys
    beside single sets) localises the invalid job like the count-based split."""
    codes, oks = _run("batch_one_wrong", by_cost=True)
    assert oks == [False, False]
    _, exp = _jobs("batch_one_wrong")
    assert codes == _expected_codes(exp)


def _worker_gpu(rank, world, port, name, out):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from lodestar_amd import workloads as W
    from lodestar_amd.distributed import shard_jobs, verify_sharded
    from lodestar_amd.engine import Engine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    eng = Engine(0)
    try:
        wl = W.make(eng, name)          # deterministic: both ranks build the same workload
        lo, hi = shard_jobs(wl.packed.n_jobs, world, rank)
        shard = W.slice_jobs(wl.packed, lo, hi)
        shard.pk_indices = None         # 96-byte keys
        b = eng.upload(shard)
        try:
            codes, ok = verify_sharded(b.partial, eng.product_is_one, b.search_after_partial)
        finally:
            b.free()
        out.put((rank, codes, ok, [int(x) for x in wl.expected[lo:hi]]))
    finally:
        eng.close()
        dist.destroy_process_group()


def _run_gpu(name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_gpu, args=(r, 2, port, name, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res)


@pytest.mark.gpu
def test_gloo_two_ranks_gpu_partials_valid():
    """c5 (32 block jobs) sharded over two ranks on device 0: lb_batch_partial partials, all-gather,
    one final exponentiation of their product accepts everything."""
    res = _run_gpu("c5")
    assert [ok for _, _, ok, _ in res] == [True, True]
    for _, codes, _, exp in res:
        assert codes == exp == [1] * len(exp)


@pytest.mark.gpu
def test_gloo_two_ranks_gpu_partials_invalid_localised():
    """c4 carries wrong and malformed sets: the product check fails on both ranks and each rank
    localises its invalid jobs from its own partial's state (lb_batch_search_after_partial)."""
    res = _run_gpu("c4")
    assert [ok for _, _, ok, _ in res] == [False, False]
    for _, codes, _, exp in res:
        assert codes == exp


@pytest.mark.gpu
def test_search_after_partial_matches_verify():
    """lb_batch_search_after_partial (the exchange mode's continuation) gives the per-job codes
    of lb_batch_verify on a batch with wrong and malformed sets (c4) and on a valid one (c2); a
    call on the engine in between invalidates the partial's state (LB_ERR_ARGUMENT)."""
    import numpy as np
    from lodestar_amd import workloads as W
    from lodestar_amd.engine import BlsError, Engine
    with Engine(0) as eng:
        for name in ("c4", "c2"):
            wl = W.make(eng, name)
            b = eng.upload(W.indexed_for(eng, wl))
            try:
                _, st = b.partial()
                assert np.array_equal(b.search_after_partial(), wl.expected), name
                b.partial()
                b.verify()
                with pytest.raises(BlsError):
                    b.search_after_partial(fallback=False)
                # the default falls back to a full re-verification of the shard
                assert np.array_equal(b.search_after_partial(), wl.expected), name
            finally:
                b.free()


@pytest.mark.gpu
def test_search_after_partial_rejects_a_successor_batch():
    """partial(b1), free b1, upload b2 (which may reuse b1's address): search_after_partial(b2)
    must not continue from b1's state (round-4 ADVICE: the check compared raw pointers)."""
    from lodestar_amd import workloads as W
    from lodestar_amd.engine import BlsError, Engine
    with Engine(0) as eng:
        w4, w2 = W.make(eng, "c4"), W.make(eng, "c2")
        b1 = eng.upload(W.indexed_for(eng, w4))
        b1.partial()
        b1.free()
        b2 = eng.upload(W.indexed_for(eng, w2))
        try:
            with pytest.raises(BlsError):
                b2.search_after_partial(fallback=False)
            assert np.array_equal(b2.search_after_partial(), w2.expected)
        finally:
            b2.free()


def _cancel_jobs():
    from lodestar_amd.engine import SetInput
    c = load_json("cancel_pair.json")["sets"]
    return [[SetInput([bytes.fromhex(s["pubkey"])], bytes.fromhex(s["signing_root"]),
                      bytes.fromhex(s["signature"]))] for s in c]


def test_cancel_pair_fixture_cancels_only_unblinded():
    """The fixture is a real attack on unblinded 1-set partials: each set alone is invalid, the
    product with r_A = r_B = 1 is one, random blinding rejects it (oracle, pure Python)."""
    import sys
    sys.path.insert(0, ROOT)
    from oracle import bls_oracle as O
    c = load_json("cancel_pair.json")["sets"]
    pk = [O.g1_deserialize(bytes.fromhex(s["pubkey"])) for s in c]
    m = [bytes.fromhex(s["signing_root"]) for s in c]
    sg = [O.g2_decompress(bytes.fromhex(s["signature"])) for s in c]
    assert [O.core_verify(pk[i], m[i], sg[i]) for i in range(2)] == [False, False]
    assert O.verify_multiple_signatures(list(zip(pk, m, sg)), scalars=[1, 1])
    assert not O.verify_multiple_signatures(list(zip(pk, m, sg)), scalars=[3, 5])


@pytest.mark.gpu
def test_single_set_partials_are_blinded():
    """Round-5 ADVICE: lb_batch_partial of a 1-set batch must not be unblinded, or two ranks'
    shards sig_A + D and sig_B - D cancel in lb_fp12_product_is_one.  Each 1-set batch's
    lb_batch_verify stays false (the unblinded single-set path), and the product of the two
    partials is not one."""
    from lodestar_amd.engine import Engine
    jobs = _cancel_jobs()
    with Engine(0) as eng:
        parts = []
        for j in jobs:
            b = eng.upload([j])
            try:
                assert list(b.verify()) == [0]
                f, st = b.partial()
                assert list(st) == [1]
                parts.append(f)
            finally:
                b.free()
        assert not eng.product_is_one(parts)
        assert not eng.product_is_one(parts[::-1])


def _worker_cancel(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from lodestar_amd.distributed import verify_sharded
    from lodestar_amd.engine import Engine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    eng = Engine(0)
    try:
        b = eng.upload([_cancel_jobs()[rank]])   # one single-set shard per rank
        try:
            codes, ok = verify_sharded(b.partial, eng.product_is_one, b.search_after_partial)
        finally:
            b.free()
        out.put((rank, codes, ok))
    finally:
        eng.close()
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gloo_two_ranks_single_set_shards_cannot_cancel():
    """Two ranks, one single-set shard each, with opposite offsets on the two signatures: the
    exchange must reject the segment and each rank must report its job invalid."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_cancel, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [(0, [0], False), (1, [0], False)]


def _worker_nccl(port, out):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from lodestar_amd import workloads as W
    from lodestar_amd.distributed import verify_sharded
    from lodestar_amd.engine import Engine
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    res = {"backend": dist.get_backend()}
    eng = Engine(0)
    try:
        for name in ("c5", "c4"):   # a valid shard, then one with planted wrong / malformed sets
            wl = W.make(eng, name)
            b = eng.upload(W.indexed_for(eng, wl))
            try:
                codes, ok = verify_sharded(b.partial, eng.product_is_one, b.search_after_partial,
                                           device=torch.device("cuda", 0))
            finally:
                b.free()
            res[name] = (codes == [int(x) for x in wl.expected], ok)
        out.put(res)
    finally:
        eng.close()
        dist.destroy_process_group()


@pytest.mark.gpu
def test_nccl_world_one_exchange_on_device():
    """RCCL on hardware: an "nccl" process group of world size 1 on device 0,
    verify_sharded with the 576-B partial as a device tensor (all_gather over RCCL), then
    lb_fp12_product_is_one: a valid shard accepts, a shard with planted invalid jobs rejects and
    the search names them."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_nccl, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert res["backend"] == "nccl"
    assert res["c5"] == (True, True)
    assert res["c4"] == (True, False)
