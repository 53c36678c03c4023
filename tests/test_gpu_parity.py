"""Parity of the HIP path (through the C ABI) with the reference semantics, on MI355X.
Expected values come from the committed golden fixtures (oracle + reference KATs); large
batches use size-independent properties (all-valid accepts; exactly the planted invalid
jobs are rejected; partial products over shards agree)."""
import asyncio
import hashlib
import os

import numpy as np
import pytest

from conftest import load_json
from lodestar_amd.engine import BlsError, SetInput, pack_jobs

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def interop_sk(i):
    d = hashlib.sha256(i.to_bytes(32, "little")).digest()
    return int.from_bytes(d, "little") % R


def case_jobs():
    cases = load_json("jobs.json")["cases"]
    jobs = []
    for c in cases:
        jobs.append([SetInput([bytes.fromhex(p) for p in s["pubkeys"]], bytes.fromhex(s["signing_root"]),
                              bytes.fromhex(s["signature"])) for s in c["sets"]])
    return cases, jobs


def code_to_expected(code, engine):
    if code < 0:
        from lodestar_amd import _native as N
        return N.error_name(-code)
    return bool(code)


def test_golden_jobs_one_batch(engine):
    cases, jobs = case_jobs()
    codes = engine.verify_jobs(jobs)
    for c, code in zip(cases, codes):
        assert code_to_expected(code, engine) == c["expected"], c["name"]


def test_golden_jobs_each_alone_fixed_scalars(engine):
    cases, jobs = case_jobs()
    for c, job in zip(cases, jobs):
        sc = np.arange(1, len(job) + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) | np.uint64(1)
        code = engine.verify_jobs([job], scalars=sc if len(job) else None)[0]
        assert code_to_expected(code, engine) == c["expected"], c["name"]


def test_k2_k4_reference_signatures(engine):
    k = load_json("reference_kats.json")
    k2 = k["K2_deposit_signature"]
    job = [SetInput([bytes.fromhex(k2["pubkey96"])], bytes.fromhex(k2["signing_root"]), bytes.fromhex(k2["signature"]))]
    k4 = [SetInput([bytes.fromhex(s["pubkey96"])], bytes.fromhex(s["signing_root"]), bytes.fromhex(s["signature"]))
          for s in k["K4_multithread_sets"]["sets"]]
    assert engine.verify_jobs([job, k4, k4[:1], k4[1:]]) == [1, 1, 1, 1]


def test_keygen_and_sign_kernels_match_kats(engine):
    k = load_json("reference_kats.json")
    pk48, pk96 = engine.sk_to_pk([interop_sk(i) for i in range(8)])
    for i in range(8):
        assert pk48[i].tobytes().hex() == k["K1_interop_pubkeys"]["pubkeys"][i]
    k2 = k["K2_deposit_signature"]
    sig = engine.sign([interop_sk(0)], np.frombuffer(bytes.fromhex(k2["signing_root"]), np.uint8))
    assert sig[0].tobytes().hex() == k2["signature"]
    for s in k["K4_multithread_sets"]["sets"]:
        sg = engine.sign([int(s["sk"], 16)], np.frombuffer(bytes.fromhex(s["signing_root"]), np.uint8))
        assert sg[0].tobytes().hex() == s["signature"]


def test_aggregate_pubkeys_bytes(engine):
    a = load_json("aggregates.json")
    sets = [[bytes.fromhex(p) for p in g["pubkeys"]] for g in a["aggregate"]]
    out, st = engine.aggregate_pubkeys(sets)
    from lodestar_amd import _native as N
    for g, o_, s in zip(a["aggregate"], out, st):
        assert N.error_name(s) == g["status"]
        if s == 0:
            assert o_.hex() == g["expected96"]


def test_g1_decompress(engine):
    a = load_json("aggregates.json")["g1_decompress"]
    out, st = engine.g1_decompress([bytes.fromhex(x["in48"]) for x in a], validate=True)
    assert st == [0] * len(a)
    assert [o_.hex() for o_ in out] == [x["out96"] for x in a]
    bad = bytes([0xC0]) + bytes(47)
    _, st = engine.g1_decompress([bad], validate=True)
    assert st == [6]  # BLST_PK_IS_INFINITY


def make_batch(engine, n_sets, agg_k=1, seed=1, invalid=()):
    """n_sets single-job sets (k pubkeys each over a 64-key pool) signed on the GPU."""
    rng = np.random.default_rng(seed)
    pool = [interop_sk(i) for i in range(64)]
    _, pk96 = engine.sk_to_pk(pool)
    msgs = rng.integers(0, 256, size=(n_sets, 32), dtype=np.uint8)
    idx = rng.integers(0, 64, size=(n_sets, agg_k))
    sks = [sum(pool[j] for j in row) % R for row in idx]
    sigs = engine.sign(sks, msgs)
    jobs = []
    for i in range(n_sets):
        m = msgs[i].tobytes()
        if i in invalid:
            m = bytes([m[0] ^ 1]) + m[1:]
        jobs.append([SetInput([pk96[j].tobytes() for j in idx[i]], m, sigs[i].tobytes())])
    return jobs


def test_blinding_words_match_oracle_semantics(engine):
    """A blinding word w = hi:lo stands for r = lo + hi * lambda (lambda = -x^2; lb_curve.h
    jac_mul_glv, oracle.blinding_scalar).  On an INVALID batch the root partial depends on r:
    FE(GPU partial) equals FE of the oracle's prod ML(r PK, H(m)) * ML(-G1, sum r sig) with
    r = blinding_scalar(w), and differs when the words are read as plain integers."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import bls_oracle as o
    jobs = make_batch(engine, 3, agg_k=2, seed=33, invalid={1})
    words = np.array([0x0000000500000003, 0xFFFFFFFF00000001, 0x00000001FFFFFFFF], dtype=np.uint64)
    b = engine.upload(jobs)
    try:
        raw, st = b.partial(words)
    finally:
        b.free()
    assert list(st) == [1, 1, 1]
    vals = [int.from_bytes(raw[48 * k:48 * (k + 1)], "big") for k in range(12)]
    f_gpu = tuple(tuple((vals[6 * a + 2 * c], vals[6 * a + 2 * c + 1]) for c in range(3)) for a in range(2))

    def oracle_partial(rs):
        f, ssum = o.F12_ONE, None
        for job, r in zip(jobs, rs):
            (si,) = job
            pk = None
            for k in si.pubkeys:
                pk = o.g1_add(pk, o.g1_deserialize(bytes(k)))
            sig = o.signature_from_bytes(bytes(si.signature), True)
            ssum = o.g2_add(ssum, o.g2_mul(sig, r))
            f = o.f12_mul(f, o.miller_loop(o.g1_mul(pk, r), o.hash_to_g2(bytes(si.signing_root), o.DST_POP)))
        return o.f12_mul(f, o.miller_loop(o.g1_neg(o.G1), ssum))

    e_gpu = o.final_exponentiation(f_gpu)
    assert e_gpu != o.F12_ONE
    assert e_gpu == o.final_exponentiation(oracle_partial([o.blinding_scalar(int(w)) for w in words]))
    assert e_gpu != o.final_exponentiation(oracle_partial([int(w) for w in words]))


def test_bisection_finds_planted_invalid_jobs(engine):
    bad = {3, 77, 200, 201, 511}
    jobs = make_batch(engine, 512, agg_k=1, seed=7, invalid=bad)
    codes = engine.verify_jobs(jobs)
    assert [i for i, c in enumerate(codes) if c != 1] == sorted(bad)
    assert all(codes[i] == 0 for i in bad)


def test_aggregate_sets_and_multi_set_jobs(engine):
    jobs = make_batch(engine, 96, agg_k=33, seed=3)
    merged = [sum(jobs[i:i + 8], []) for i in range(0, 96, 8)]
    assert engine.verify_jobs(merged) == [1] * 12
    bad = make_batch(engine, 96, agg_k=33, seed=3, invalid={50})
    merged = [sum(bad[i:i + 8], []) for i in range(0, 96, 8)]
    assert engine.verify_jobs(merged) == [1] * 6 + [0] + [1] * 5


def test_partials_over_shards(engine):
    jobs = make_batch(engine, 200, seed=11)
    parts = []
    for sh in (jobs[:70], jobs[70:140], jobs[140:]):
        b = engine.upload(sh)
        f, st = b.partial()
        assert list(st) == [1] * len(sh)
        parts.append(f)
        b.free()
    assert engine.product_is_one(parts)
    bad = make_batch(engine, 70, seed=11, invalid={5})
    b = engine.upload(bad)
    fbad, _ = b.partial()
    b.free()
    assert not engine.product_is_one([fbad] + parts[1:])


def test_random_scalars_repeatable_verdicts(engine):
    jobs = make_batch(engine, 64, seed=5, invalid={9})
    b = engine.upload(jobs)
    for _ in range(3):
        codes = list(b.verify())
        assert codes == [1] * 9 + [0] + [1] * 54
    b.free()


def test_pool_multithread_e2e_cases(engine):
    """packages/beacon-node/test/e2e/chain/bls/multithread.test.ts:60-103 on the GPU pool."""
    from lodestar_amd import verifier as V
    k4 = load_json("reference_kats.json")["K4_multithread_sets"]["sets"]
    sets = [V.SingleSignatureSet(V.PublicKey(bytes.fromhex(s["pubkey96"])), bytes.fromhex(s["signing_root"]),
                                 bytes.fromhex(s["signature"])) for s in k4]

    async def many(sleep, opts):
        pool = V.BlsGpuVerifier(engine=engine)
        futs = []
        for _ in range(8):
            futs.append(asyncio.ensure_future(pool.verify_signature_sets(sets, opts)))
            if sleep:
                await asyncio.sleep(0.005)
        res = await asyncio.gather(*futs)
        await pool.close()
        return res

    assert asyncio.run(many(False, None)) == [True] * 8
    assert asyncio.run(many(True, None)) == [True] * 8
    assert asyncio.run(many(True, V.VerifySignatureOpts(batchable=True))) == [True] * 8

    async def first_invalid():
        pool = V.BlsGpuVerifier(engine=engine)
        inv = V.SingleSignatureSet(sets[0].pubkey, sets[0].signing_root, bytes(32))
        bad = asyncio.ensure_future(pool.verify_signature_sets([inv], V.VerifySignatureOpts(batchable=True)))
        goods = [asyncio.ensure_future(pool.verify_signature_sets(sets, V.VerifySignatureOpts(batchable=True)))
                 for _ in range(8)]
        with pytest.raises(BlsError, match="BLST_INVALID_SIZE"):
            await bad
        res = await asyncio.gather(*goods)
        await pool.close()
        return res

    assert asyncio.run(first_invalid()) == [True] * 8

    async def main_thread():
        pool = V.BlsGpuVerifier(engine=engine)
        r = await pool.verify_signature_sets(sets, V.VerifySignatureOpts(verify_on_main_thread=True))
        await pool.close()
        return r

    assert asyncio.run(main_thread()) is True


def test_fp_mul_asm_matches_reference_body():
    """The device Montgomery products -- fp_mul28 (14 x 28-bit limbs, what every kernel's fp_mul
    runs) and the 32-bit inline-asm form (lb_fpmul_gfx950.h) -- agree with the portable
    carry-save form fp_mul_body on 16.4M random and edge-case operands."""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "ubench", "fpmul_asm")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert json.loads(out.stdout.strip().splitlines()[-1])["mismatches"] == 0


def test_pubkey_table_indexed_batches_match_byte_batches(engine):
    """GPU-resident pubkey table: index-based sets give the same per-job
    results as byte-carrying sets; bad indices and bad keys reject their own job only."""
    from lodestar_amd.engine import PackedJobs
    k = load_json("reference_kats.json")
    pk48 = [bytes.fromhex(p) for p in k["K1_interop_pubkeys"]["pubkeys"][:8]]
    first, st = engine.pubkey_table_append(pk48, validate=True)
    assert st == [0] * 8
    # a key that fails decoding (x >= p) and one infinity key
    bad_first, st2 = engine.pubkey_table_append([bytes([0x9f]) + b"\xff" * 47, bytes([0xc0]) + bytes(47)])
    assert st2 == [1, 0]
    jobs = make_batch(engine, 40, agg_k=5, seed=21, invalid={7, 30})
    packed = pack_jobs(jobs)
    ref = engine.verify_jobs(jobs)
    # the same sets expressed as table indices (make_batch draws from a 64-key interop pool)
    _, pk96 = engine.sk_to_pk([interop_sk(i) for i in range(64)])
    base, st3 = engine.pubkey_table_append([pk96[i].tobytes() for i in range(64)])
    assert st3 == [0] * 64
    lookup = {pk96[i].tobytes(): base + i for i in range(64)}
    idx = np.array([lookup[packed.pubkeys[96 * j: 96 * j + 96].tobytes()] for j in range(len(packed.pubkeys) // 96)],
                   dtype=np.uint32)
    ip = PackedJobs(job_off=packed.job_off, pk_off=packed.pk_off, pubkeys=None, msgs=packed.msgs, sigs=packed.sigs,
                    sig_sizes=None, pk_indices=idx)
    b = engine.upload(ip)
    assert list(b.verify()) == ref == [1] * 7 + [0] + [1] * 22 + [0] + [1] * 9
    b.free()
    # bad index / bad key / infinity-only aggregate reject their own jobs
    idx2 = idx.copy()
    idx2[0] = 10 ** 6                      # set 0: index out of range
    idx2[5] = bad_first                    # set 1 (keys 5..9): undecodable key
    idx2[10:15] = bad_first + 1            # set 2: all infinity -> BLST_PK_IS_INFINITY
    ip2 = PackedJobs(job_off=packed.job_off, pk_off=packed.pk_off, pubkeys=None, msgs=packed.msgs, sigs=packed.sigs,
                     sig_sizes=None, pk_indices=idx2)
    b = engine.upload(ip2)
    codes = list(b.verify())
    b.free()
    assert codes[:3] == [-100, -1, -6] and codes[3:] == ref[3:]


def test_pool_with_registered_pubkeys():
    """BlsGpuVerifier with PublicKeys registered in the resident table (index path) gives the same
    answers as with raw keys, including a rejecting job in the same package."""
    from lodestar_amd import verifier as V
    from lodestar_amd.engine import Engine
    k4 = load_json("reference_kats.json")["K4_multithread_sets"]["sets"]

    async def main():
        eng = Engine(0)
        pool = V.BlsGpuVerifier(engine=eng)
        pks = pool.register_pubkeys([bytes.fromhex(s["pubkey96"]) for s in k4])
        assert all(p.index is not None for p in pks)
        sets = [V.SingleSignatureSet(pks[i], bytes.fromhex(s["signing_root"]), bytes.fromhex(s["signature"]))
                for i, s in enumerate(k4)]
        good = [pool.verify_signature_sets(sets, V.VerifySignatureOpts(batchable=True)) for _ in range(6)]
        wrong = V.SingleSignatureSet(pks[0], sets[1].signing_root, sets[0].signature)
        bad = pool.verify_signature_sets([wrong], V.VerifySignatureOpts(batchable=True))
        res = await asyncio.gather(*good, bad)
        await pool.close()
        eng.close()
        return res

    assert asyncio.run(main()) == [True] * 6 + [False]


# ---------------------------------------------------------------- sets sharing a signing root
def make_shared_batch(engine, n_sets, n_msgs, agg_k=1, seed=1, invalid=(), malformed=()):
    """n_sets single-set jobs whose signing roots are drawn from n_msgs distinct roots (a
    committee's attestations sign one AttestationData root).  `invalid`: signed over another
    root (well-formed, wrong); `malformed`: compression flag cleared (BLST_BAD_ENCODING)."""
    rng = np.random.default_rng(seed)
    pool = [interop_sk(i) for i in range(64)]
    _, pk96 = engine.sk_to_pk(pool)
    roots = rng.integers(0, 256, size=(n_msgs, 32), dtype=np.uint8)
    which = rng.integers(0, n_msgs, size=n_sets)
    msgs = roots[which]
    idx = rng.integers(0, 64, size=(n_sets, agg_k))
    sks = [sum(pool[j] for j in row) % R for row in idx]
    sign_msgs = msgs.copy()
    for i in invalid:
        sign_msgs[i, 0] ^= 1
    sigs = engine.sign(sks, sign_msgs)
    jobs = []
    for i in range(n_sets):
        s = bytearray(sigs[i].tobytes())
        if i in malformed:
            s[0] &= 0x7F
        jobs.append([SetInput([pk96[j].tobytes() for j in idx[i]], msgs[i].tobytes(), bytes(s))])
    return jobs


def _verify_profiled(engine, jobs):
    engine.set_profiling(True)
    try:
        codes = engine.verify_jobs(jobs)
        prof = engine.last_profile()
    finally:
        engine.set_profiling(False)
    return codes, prof


def test_shared_roots_grouped_path_accepts(engine):
    # 700 sets over 5 roots: groups of ~140 span several LB_GROUP_CHUNK chunks; aggregates mixed in
    jobs = make_shared_batch(engine, 700, 5, agg_k=3, seed=21)
    codes, prof = _verify_profiled(engine, jobs)
    assert codes == [1] * 700
    assert prof["search_msm"] == 0.0 and prof["search_check"] >= 0.0


def test_shared_roots_invalid_member_found_by_fallback(engine):
    bad = {0, 13, 399}
    jobs = make_shared_batch(engine, 400, 3, seed=22, invalid=bad)
    codes, prof = _verify_profiled(engine, jobs)
    assert [i for i, c in enumerate(codes) if c != 1] == sorted(bad)
    assert all(codes[i] == 0 for i in bad)
    assert prof["search_msm"] > 0.0


def test_shared_roots_malformed_job_excluded_without_fallback(engine):
    from lodestar_amd import _native as N
    mal = {7, 150}
    jobs = make_shared_batch(engine, 300, 2, seed=23, malformed=mal)
    codes, prof = _verify_profiled(engine, jobs)
    for i, c in enumerate(codes):
        if i in mal:
            assert N.error_name(-c) == "BLST_BAD_ENCODING"
        else:
            assert c == 1
    assert prof["search_msm"] == 0.0  # rejected jobs leave the per-root sums; the root still passes


def test_shared_roots_inside_one_job_and_duplicate_sets(engine):
    jobs = make_shared_batch(engine, 64, 2, agg_k=2, seed=24)
    multi = [sum(jobs[i:i + 16], []) for i in range(0, 64, 16)]
    dup = [jobs[0][0], jobs[0][0]]  # the same set twice in one job (same key, root, signature)
    assert engine.verify_jobs(multi + [dup] + [jobs[1]]) == [1] * 6
    bad = make_shared_batch(engine, 64, 2, agg_k=2, seed=24, invalid={37})
    multi = [sum(bad[i:i + 16], []) for i in range(0, 64, 16)]
    assert engine.verify_jobs(multi) == [1, 1, 0, 1]


def test_all_sets_one_root_and_all_distinct(engine):
    one = make_shared_batch(engine, 257, 1, seed=25)
    assert engine.verify_jobs(one) == [1] * 257
    distinct = make_batch(engine, 257, seed=26, invalid={256})
    assert engine.verify_jobs(distinct) == [1] * 256 + [0]


def test_all_valid_distinct_roots_pass_at_the_root(engine):
    """The bucket MSM for sum r_i sig_i and the per-root sums must reproduce the batch equation
    exactly: an all-valid batch is accepted by the root check alone (no fallback)."""
    jobs = make_batch(engine, 300, agg_k=2, seed=27)
    codes, prof = _verify_profiled(engine, jobs)
    assert codes == [1] * 300
    assert prof["search_msm"] == 0.0


@pytest.mark.parametrize("name", ["c1", "c2", "c4", "c5", "c5_64"])
def test_baseline_config_workloads(engine, name):
    """BASELINE.json configs as verification batches (lodestar_amd/workloads.py): per-job verdicts
    equal the planted expectation (c4 carries invalid sets -> fallback + bisection), through both
    the 96-byte-key and the resident-table paths."""
    from lodestar_amd import workloads as W
    wl = W.make(engine, name)
    p = wl.packed
    b = engine.upload(W.PackedJobs(job_off=p.job_off, pk_off=p.pk_off, pubkeys=p.pubkeys, msgs=p.msgs,
                                   sigs=p.sigs, sig_sizes=p.sig_sizes))
    try:
        got = np.asarray(b.verify())[:p.n_jobs]
    finally:
        b.free()
    assert np.array_equal(got, wl.expected), (name, np.nonzero(got != wl.expected))
    bi = engine.upload(W.indexed_for(engine, wl))
    try:
        got = np.asarray(bi.verify())[:p.n_jobs]
    finally:
        bi.free()
    assert np.array_equal(got, wl.expected)
    if name == "c4":
        assert wl.n_invalid_jobs >= 1


@pytest.mark.parametrize("name", ["c3", "c3_mixed"])
def test_c3_one_slot_workload(engine, name):
    """The headline config's one-slot shape (19 456 sets, 17 408 jobs, roots shared per committee)
    through the HIP path; c3_mixed plants the §8(d) invalid mix (wrong-message signatures and
    malformed bytes: 32-byte signatures, cleared compression flags).  Per-job verdicts must equal
    the planted expectation through both the resident-table and the 96-byte-key paths."""
    from lodestar_amd import workloads as W
    wl = W.make(engine, name)
    p = wl.packed
    assert p.n_sets == 19456 and p.n_jobs == 17408
    bi = engine.upload(W.indexed_for(engine, wl))
    try:
        got = np.asarray(bi.verify())[:p.n_jobs]
    finally:
        bi.free()
    assert np.array_equal(got, wl.expected), (name, np.nonzero(got != wl.expected))
    b = engine.upload(W.PackedJobs(job_off=p.job_off, pk_off=p.pk_off, pubkeys=p.pubkeys, msgs=p.msgs,
                                   sigs=p.sigs, sig_sizes=p.sig_sizes))
    try:
        got = np.asarray(b.verify())[:p.n_jobs]
    finally:
        b.free()
    assert np.array_equal(got, wl.expected)
    if name == "c3_mixed":
        assert (wl.expected == 0).sum() >= 4
        assert (wl.expected == -W.LB_INVALID_SIZE).sum() >= 4 and (wl.expected == -W.LB_BAD_ENCODING).sum() >= 4


def test_verify_jobs_workspace_reuse_and_indexed(engine):
    """lb_verify_jobs / lb_verify_jobs_indexed reuse one engine-owned workspace: shrinking and
    growing calls back to back give the same verdicts as resident batches."""
    from lodestar_amd import workloads as W
    wl = W.make(engine, "c1")
    p = W.PackedJobs(job_off=wl.packed.job_off, pk_off=wl.packed.pk_off, pubkeys=wl.packed.pubkeys,
                     msgs=wl.packed.msgs, sigs=wl.packed.sigs, sig_sizes=None)   # 96-byte keys
    ip = W.indexed_for(engine, wl)                                              # table indices
    # uploads up to 1 MiB go up as one staged copy into views of one arena (lb_engine.hip
    # batch_fill), larger ones as owned buffers: alternate the two on the same workspace
    big = W.make(engine, "c3", slots=1)
    bip = W.indexed_for(engine, big)
    for _ in range(2):
        assert engine.verify_jobs_packed(p) == list(wl.expected)
        assert engine.verify_jobs_packed(ip) == list(wl.expected)
        small = make_batch(engine, 3, seed=41, invalid={1})
        assert engine.verify_jobs(small) == [1, 0, 1]
        assert engine.verify_jobs_packed(bip) == list(big.expected)


def test_indexed_null_indices_only_without_keys(engine):
    from lodestar_amd import _native as N
    import ctypes
    lib = N.load()
    job_off = np.array([0, 1], dtype=np.uint32)
    pk_off = np.array([0, 1], dtype=np.uint32)          # one key but no index array
    msgs = np.zeros(32, np.uint8)
    sigs = np.zeros(96, np.uint8)
    out = np.zeros(1, np.int32)
    p32 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))  # noqa: E731
    p8 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))  # noqa: E731
    st = lib.lb_verify_jobs_indexed(engine.h, 1, p32(job_off), p32(pk_off), None, p8(msgs), p8(sigs), None, None,
                                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    assert st == N.LB_ERR_ARGUMENT
    pk0 = np.array([0, 0], dtype=np.uint32)             # no keys: valid call, the set rejects
    st = lib.lb_verify_jobs_indexed(engine.h, 1, p32(job_off), p32(pk0), None, p8(msgs), p8(sigs), None, None,
                                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    assert st == N.LB_OK and out[0] == -N.LB_EMPTY_AGGREGATE_ARRAY


H2 = 0x5D543A95414E7F1091D50792876A202CD91DE4547085ABAA68A205B2E5A7DDFA628F1CB4D9E82EF21537E293A6691AE1616EC6E786F0C70CF1C38E31C7238E5


def small_order_signatures():
    """Signatures on E'(Fp2) of orders 13 and 23 (torsion of the cofactor h2 = 13^2 23^2 ...): the
    psi ladder's prefix at bit 60 is 12 = -1 mod 13, so an order-13 point meets acc == -P at an
    addition (the lane kernel's exceptional branch, then the addition to infinity)."""
    import oracle.bls_oracle as o
    q = o.iso_map(o.map_to_curve_sswu(o.hash_to_field_fp2(bytes(range(32)), 2, o.DST_POP)[0]))
    assert o.g2_mul(q, H2 * o.R) is None
    out = []
    for ell in (13, 23):  # ell^2 divides h2: project onto the ell-primary part, then down to order ell
        Q = o.g2_mul(q, H2 * o.R // (ell * ell))
        if Q is not None and o.g2_mul(Q, ell) is not None:
            Q = o.g2_mul(Q, ell)
        assert Q is not None and o.g2_mul(Q, ell) is None
        out.append(o.g2_compress(Q))
        out.append(o.g2_compress(o.g2_neg(Q)))
    return out


@pytest.mark.parametrize("g8_max,row_fe", [("0", "0"), (str(1 << 31), "0"), (str(1 << 31), "1")])
def test_small_order_signatures_not_in_group(monkeypatch, g8_max, row_fe):
    """Every subgroup-check kernel (one lane per set: k_sig_subgroup; 8 lanes: k_sig_subgroup_g8;
    a row workgroup per set: k_sig_subgroup_row, whose fast ladder meets the exceptional cases of
    small-order points and reruns with the tested additions) rejects points of small order with
    BLST_POINT_NOT_IN_GROUP, in one batch beside valid sets."""
    from lodestar_amd import _native as N
    from lodestar_amd.engine import Engine
    monkeypatch.setenv("LB_SUBGROUP_G8_MAX", g8_max)
    monkeypatch.setenv("LB_ROW_FE", row_fe)
    cases, jobs = case_jobs()
    valid = jobs[[c["name"] for c in cases].index("single_valid_0")]
    pk, root = valid[0].pubkeys, valid[0].signing_root
    bad = [[SetInput(pk, root, sig)] for sig in small_order_signatures()]
    with Engine(0) as e:
        codes = e.verify_jobs(bad + [valid] + bad[:1] + [valid])
    assert codes == [-N.LB_POINT_NOT_IN_GROUP] * 4 + [1, -N.LB_POINT_NOT_IN_GROUP, 1]


def test_search_large_roots_parts_then_sets(engine):
    """Two roots of 750 members: one wrong set in root 0 is named by one weighted test over its
    750 single-set parts (weights up to 750, baby-step / giant-step match); root 1's two wrong sets
    fail that test and are searched in 64 direct parts, then set by set."""
    bad = {5, 777, 1400}
    jobs = make_shared_batch(engine, 1500, 2, seed=31, invalid=bad)
    codes, prof = _verify_profiled(engine, jobs)
    assert [i for i, c in enumerate(codes) if c != 1] == sorted(bad)
    assert prof["search_check"] > 0.0


def test_search_root_above_weighted_part_cap(engine):
    """Two roots of ~1100 members (> LB_WT_MAX = 1024 parts per weighted test): a weighted test runs
    over parts of two sets, then over the named part's sets."""
    bad = {3, 1099, 2150}
    jobs = make_shared_batch(engine, 2200, 2, seed=37, invalid=bad)
    codes, prof = _verify_profiled(engine, jobs)
    assert [i for i, c in enumerate(codes) if c != 1] == sorted(bad)
    assert prof["search_check"] > 0.0


def test_search_c3_invalid_two_slots(engine):
    """c3 with one wrong-message attestation per slot (2 slots, 38 912 sets): the search over
    root subtrees, roots and single sets finds exactly the planted jobs."""
    from lodestar_amd import workloads as W
    wl = W.make(engine, "c3_invalid", slots=2)
    b = engine.upload(W.indexed_for(engine, wl))
    try:
        got = np.asarray(b.verify())
    finally:
        b.free()
    assert np.array_equal(got, wl.expected)
    assert (wl.expected == 0).sum() == 2


@pytest.mark.parametrize("knobs", ["LB_SEARCH_MERGE=0", "LB_ROOT_SHUFFLE=0", "LB_SEARCH_BLOCKS=0",
                                   "LB_SEARCH_BLOCKS=0+LB_SEARCH_MERGE=0",
                                   "LB_SEARCH_BLOCKS=0+LB_SEARCH_ROOTSUM=0", "LB_SEARCH_BLOCKS=0+LB_SEARCH_PRE=1",
                                   "LB_SMSM_FORM=lane", "LB_SMSM_FORM=lane+LB_SEARCH_BLOCKS=0+LB_SEARCH_ROOTSUM=0",
                                   "LB_SEARCH_CHUNK=32", "LB_SEARCH_CHUNK=1"])
def test_search_forms_find_the_same_sets(monkeypatch, knobs):
    """Every selectable form of the invalid-set search (lb_engine.hip: look-ahead tests in a
    separate launch pair; the first round over per-root sums with look-ahead tests instead of
    direct subtree checks from one 4-window MSM; that round over the 6-window bucket MSM; later
    rounds over the kept per-set terms; roots numbered in input order) names exactly the planted jobs of c3 with one wrong
    attestation per slot (2 slots: above LB_SEARCH_SMALL_MAX, so the large-batch rounds run)."""
    from lodestar_amd.engine import Engine
    from lodestar_amd import workloads as W
    for knob in knobs.split("+"):
        k, v = knob.split("=")
        monkeypatch.setenv(k, v)
    with Engine(0) as e:
        wl = W.make(e, "c3_invalid", slots=2)
        b = e.upload(W.indexed_for(e, wl))
        try:
            got = np.asarray(b.verify())
        finally:
            b.free()
    assert np.array_equal(got, wl.expected), (knobs, np.nonzero(got != wl.expected))
    assert (wl.expected == 0).sum() == 2


def test_search_term_forms_trace_the_same_rounds(monkeypatch, capfd):
    """The small rounds' weighted terms one lane per position (k_smsm_terms_lane, the form under
    load) and by 8-lane groups (k_smsm_terms_g8) must be the same points: with the roots in input
    order (LB_ROOT_SHUFFLE=0, one tree shape) the search's rounds, failing nodes and direct checks
    (LB_SEARCH_TRACE) are identical, since a wrong term makes a weighted test match no power and
    sends its node to direct checks one round later.  (The weighted-test counts are not compared:
    the look-ahead tests ride along only while the device runs no other batch.)"""
    from lodestar_amd.engine import Engine
    from lodestar_amd import workloads as W
    monkeypatch.setenv("LB_ROOT_SHUFFLE", "0")
    monkeypatch.setenv("LB_SEARCH_TRACE", "1")
    # both runs with the under-load forms (LB_ALONE=0): an engine created right after another one
    # closed saw the device as loaded, the first one as alone, and the look-ahead tests (alone
    # only) changed the second round
    monkeypatch.setenv("LB_ALONE", "0")
    traces = []
    for form in ("g8", "lane"):
        monkeypatch.setenv("LB_SMSM_FORM", form)
        capfd.readouterr()
        with Engine(0) as e:
            wl = W.make(e, "c3_invalid", slots=2)
            b = e.upload(W.indexed_for(e, wl))
            try:
                got = np.asarray(b.verify())
            finally:
                b.free()
        assert np.array_equal(got, wl.expected), form
        err = capfd.readouterr().err
        # "[lb search] round 1: 1 failing nodes, 109 direct checks, 0 weighted tests: 9.952 ms"
        traces.append([ln.split(", ")[:2] for ln in err.splitlines() if ln.startswith("[lb search]")])
    assert traces[0] and traces[0] == traces[1], traces


def test_aggregate_signatures_golden(engine):
    """bls.Signature.aggregate on the GPU against the oracle's golden
    groups: sums (with duplicates, cancellation to infinity, infinity members), the first bad
    signature's error, EMPTY_AGGREGATE_ARRAY."""
    from lodestar_amd import _native as N
    g = load_json("aggregates.json")["signature_aggregate"]
    out, st = engine.aggregate_signatures([[bytes.fromhex(x) for x in c["signatures"]] for c in g], validate=True)
    for c, o_, s in zip(g, out, st):
        assert N.error_name(s) == c["status"], c
        if c["expected96"] is not None:
            assert o_.hex() == c["expected96"]


def test_direct_verify_callers(engine):
    """state-transition verifySignatureSet and the light client's isValidBlsAggregate (SURVEY.md
    §8(f) row 3) on the golden sets, including the reference's stage-prefixed errors."""
    from lodestar_amd import verifier as V
    cases = {c["name"]: c for c in load_json("jobs.json")["cases"]}
    pool = V.BlsGpuVerifier(engine=engine)
    try:
        def as_set(c, agg):
            s = c["sets"][0]
            pks = [V.PublicKey(bytes.fromhex(p)) for p in s["pubkeys"]]
            root, sig = bytes.fromhex(s["signing_root"]), bytes.fromhex(s["signature"])
            return V.AggregatedSignatureSet(pks, root, sig) if agg else V.SingleSignatureSet(pks[0], root, sig)
        assert pool.verify_signature_set(as_set(cases["single_valid_0"], False)) is True
        assert pool.verify_signature_set(as_set(cases["aggregate_valid"], True)) is True
        assert pool.verify_signature_set(as_set(cases["wrong_message"], False)) is False
        with pytest.raises(BlsError, match="BLST_INVALID_SIZE"):
            pool.verify_signature_set(as_set(cases["invalid_size_32_zero"], False))
        agg = as_set(cases["aggregate_valid"], True)
        assert V.is_valid_bls_aggregate(pool, agg.pubkeys, agg.signing_root, agg.signature) is True
        with pytest.raises(BlsError, match="^Error aggregating pubkeys: EMPTY_AGGREGATE_ARRAY$"):
            V.is_valid_bls_aggregate(pool, [], agg.signing_root, agg.signature)
        bad = as_set(cases["not_in_group"], False)
        with pytest.raises(BlsError, match="^Error deserializing signature: BLST_POINT_NOT_IN_GROUP$"):
            V.is_valid_bls_aggregate(pool, [bad.pubkey], bad.signing_root, bad.signature)
        sigs = [bytes.fromhex(x) for x in load_json("aggregates.json")["signature_aggregate"][2]["signatures"]]
        assert pool.aggregate_signatures(sigs).hex() == load_json("aggregates.json")["signature_aggregate"][2]["expected96"]
    finally:
        asyncio.run(pool.close())


@pytest.mark.parametrize("name", ["c3_mixed", "c2", "c3"])
def test_per_root_kernel_forms_agree(monkeypatch, name):
    """The per-root chain has two forms per step, picked by the batch's distinct-root count: one
    lane per root (k_hash_finish, k_miller_lane) or 8 lanes per root (k_miller_g8, grouped LDS programs) and many
    lanes per root (k_hash_finish_g8: 8-lane G2 doublings / additions; k_miller_wave: the wave
    engine); likewise the signatures'
    subgroup check (k_sig_subgroup / k_sig_subgroup_g8, by set count), S = sum r_i sig_i (bucket
    MSM / per-set terms, one lane or 8 lanes per set, + trees, by set count) and the invalid-set
    search's weighted range sums (bucket MSM / per-position 8-lane terms + segmented sums).
    Engines created with the thresholds at 0 and at 2^31 run the same batch (same blinding
    scalars) through each form; verdicts must match the planted expectation, and the root partials
    (576-byte Fp12 products before the final exponentiation) must be byte-identical."""
    from lodestar_amd.engine import Engine
    from lodestar_amd import workloads as W
    outs = []
    big = str(1 << 31)
    # (all one-lane / MSM forms), (the same with 8-lane Miller loops), (many-lane forms, one-lane
    # S terms), (many-lane forms, 8-lane S terms)
    # + the bucket MSM's lone-lane bucket sums and reduction (LB_MSM_G8=0) against the 8-lane ones,
    # + the one-lane Miller loop with f alone in LDS (LB_MILLER_LDS3_MAX=0: k_miller_lane<2>)
    for lim, s_g8, mform, msm_g8, lds3 in (("0", "0", "lane", "1", big), ("0", "0", "g8", "1", big),
                                           (big, "0", "g8", "1", big), (big, big, "lane", "1", big),
                                           ("0", "0", "lane", "0", big), ("0", "0", "lane", "1", "0")):
        monkeypatch.setenv("LB_MSM_G8", msm_g8)
        monkeypatch.setenv("LB_MILLER_LDS3_MAX", lds3)
        monkeypatch.setenv("LB_MILLER_FORM", mform)
        monkeypatch.setenv("LB_MILLER_WAVE_MAX", lim)
        monkeypatch.setenv("LB_HASH_G8_MAX", lim)
        monkeypatch.setenv("LB_SUBGROUP_G8_MAX", lim)
        monkeypatch.setenv("LB_SMALL_S_MAX", lim)
        monkeypatch.setenv("LB_SMALL_S_G8_MAX", s_g8)
        monkeypatch.setenv("LB_SEARCH_SMALL_MAX", lim)
        with Engine(0) as e:
            wl = W.make(e, name)
            b = e.upload(W.indexed_for(e, wl))
            try:
                sc = np.random.default_rng(5).integers(1, 1 << 63, size=wl.packed.n_sets, dtype=np.uint64)
                got = np.asarray(b.verify(scalars=sc))[:wl.packed.n_jobs]
                part = bytes(b.partial(scalars=sc)[0]) if (wl.expected == 1).all() else None
            finally:
                b.free()
        assert np.array_equal(got, wl.expected), (lim, np.nonzero(got != wl.expected))
        outs.append(part)
    assert outs[0] == outs[1] == outs[2] == outs[3] == outs[4] == outs[5]


@pytest.mark.parametrize("spec", ["1", "0"])
def test_speculative_per_root_chain(monkeypatch, spec):
    """The per-root sums and Miller loops start on speculative liveness (pubkey statuses only,
    LB_SPEC_GSUM=1) and are redone with the full statuses when a signature fails to decode.  c4
    plants malformed signatures in jobs whose roots are shared with valid sets (the sync-committee
    root): verdicts must equal the planted expectation either way; a valid c2 block too."""
    from lodestar_amd.engine import Engine
    from lodestar_amd import workloads as W
    monkeypatch.setenv("LB_SPEC_GSUM", spec)
    with Engine(0) as e:
        for name in ("c4", "c2"):
            wl = W.make(e, name)
            b = e.upload(W.indexed_for(e, wl))
            try:
                assert np.array_equal(np.asarray(b.verify()), wl.expected), name
                _, st = b.partial()
                assert np.array_equal(b.search_after_partial(), wl.expected), name
            finally:
                b.free()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1", "c2", "c3"])
def test_row_engine_forms_agree(monkeypatch, name):
    """The row engine's forms (lb_row.h: a workgroup per root / per product-tree node, every Fp
    product on a 16-lane row) run only while the device is alone: hash_to_G2's cofactor clearing
    (k_hash_finish_row, its fast path and, LB_HASH_ROW_CAREFUL=1, the path with the exceptional-
    case tests), the Miller loops and tree nodes (LB_ROW_MAX), ML(-G1, S), the root checks and
    partials (LB_ROW_FE).  Against the wave / 8-lane forms (all row forms off) on the same batch
    and blinding scalars: same verdicts, byte-identical root partials (576-byte Fp12 products
    before the final exponentiation).  LB_ALONE=1 pins the engine's "device alone" test, so the row
    forms run whatever other engines did just before (round-5 ADVICE: a recent pipeline exit sent
    every configuration to the wave forms and the comparison compared nothing different)."""
    from lodestar_amd.engine import Engine
    from lodestar_amd import workloads as W
    outs = []
    big = str(1 << 20)
    monkeypatch.setenv("LB_ALONE", "1")
    for row_fe, row_max, hash_max, careful in (("1", None, None, "0"), ("0", "0", "0", "0"),
                                               ("1", "64", big, "1")):
        monkeypatch.setenv("LB_ROW_FE", row_fe)
        monkeypatch.setenv("LB_HASH_ROW_CAREFUL", careful)
        for var, val in (("LB_ROW_MAX", row_max), ("LB_HASH_ROW_MAX", hash_max)):
            if val is None:
                monkeypatch.delenv(var, raising=False)
            else:
                monkeypatch.setenv(var, val)
        with Engine(0) as e:
            wl = W.make(e, name)
            b = e.upload(W.indexed_for(e, wl))
            try:
                sc = None
                if wl.packed.n_sets > 1:
                    sc = np.random.default_rng(7).integers(1, 1 << 63, size=wl.packed.n_sets, dtype=np.uint64)
                got = np.asarray(b.verify(scalars=sc))[:wl.packed.n_jobs]
                part = bytes(b.partial(scalars=sc)[0])
            finally:
                b.free()
        assert (wl.expected == 1).all()
        assert np.array_equal(got, wl.expected), (row_fe, row_max, np.nonzero(got != wl.expected))
        outs.append(part)
    assert outs[0] == outs[1] == outs[2]


@pytest.mark.gpu
def test_headline_six_slot_batches_in_flight():
    """The headline's own shape: 6-slot C3 batches (116 736 sets, 104 448 jobs, ~6 900 distinct
    roots) as bench.py runs them, alone and with two engines in flight (so the under-load forms run:
    one lane per root, lone-lane cofactor clearing, bucket MSM), and the same shape with one wrong
    message per slot (the invalid-set search under load).  Per-job verdicts must equal the planted
    expectation (valid: all 1; invalid: the reference's per-job re-verification, worker.ts:76-98)."""
    import threading
    from lodestar_amd.engine import Engine
    from lodestar_amd import workloads as W
    with Engine(0) as e1, Engine(0) as e2:
        wl = W.make(e1, "c3", slots=6)
        wi = W.make(e1, "c3_invalid", slots=6)
        assert wl.packed.n_sets == 116736 and (wl.expected == 1).all()
        assert (wi.expected != 1).sum() >= 6
        b1 = e1.upload(W.indexed_for(e1, wl))
        b2 = e2.upload(W.indexed_for(e2, wi))
        try:
            assert np.array_equal(np.asarray(b1.verify()), wl.expected)
            assert np.array_equal(np.asarray(b2.verify()), wi.expected)
            res = {}

            def run(k, b):
                res[k] = [np.asarray(b.verify()).copy() for _ in range(3)]

            ths = [threading.Thread(target=run, args=(1, b1)), threading.Thread(target=run, args=(2, b2))]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
            for r in res[1]:
                assert np.array_equal(r, wl.expected)
            for r in res[2]:
                assert np.array_equal(r, wi.expected), np.nonzero(r != wi.expected)
        finally:
            b1.free()
            b2.free()


@pytest.mark.gpu
def test_latency_engine_under_load():
    """LB_ENGINE_LATENCY (lb_engine_create_ex): the latency engine, created first, runs on its
    reserved CUs with the latency forms while two engines created after it (the complement of the
    CUs) verify 6-slot C3 batches; every verdict must match, and the 1-set calls must not queue
    behind the pool.  In a child process with GPU_MAX_HW_QUEUES=16, as the drop-in sets it (HIP
    reads it once per process; with the default 4 queues the engines' streams share hardware
    queues and a 1-set call waits behind a pool kernel on its queue)."""
    import subprocess
    import sys
    env = dict(os.environ, GPU_MAX_HW_QUEUES="16")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "gpu_latency_child.py")],
                       env=env, capture_output=True, text=True, timeout=240)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0
    ms = [float(x) for x in r.stdout.strip().splitlines()[-1].split()]
    assert sorted(ms)[len(ms) // 2] < 8.0, ms


@pytest.mark.gpu
def test_latency_partition_released_with_last_latency_engine():
    """Round-5 VERDICT item 7 / ADVICE: the CU partition lives while a latency engine does.  A
    latency engine gets the reserved CUs, a pool engine created beside it the rest; once both are
    gone, a new pool engine reports the device's full CU count (lb_engine_cu_count)."""
    import torch
    from lodestar_amd.engine import Engine
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    with Engine(0) as before:
        assert before.cu_count == ncu
    lat = Engine(0, Engine.LATENCY)
    pool = Engine(0)
    try:
        r = lat.cu_count
        assert 1 <= r <= ncu // 4
        assert pool.cu_count == ncu - r
        with Engine(0, Engine.LATENCY) as lat2:   # a second latency engine shares the partition
            assert lat2.cu_count == r
    finally:
        pool.close()
        lat.close()
    with Engine(0) as after:
        assert after.cu_count == ncu


@pytest.mark.gpu
def test_engine_cap_reserves_scratch():
    """The engine cap's worth of engines (10) each reserve s1, s2 and s3 scratch at creation, then
    verify at once with no queue abort (child process: the engine count is per process)."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "gpu_engines_child.py")],
                       capture_output=True, text=True, timeout=240)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c3_mixed", "c4", "c2"])
def test_per_root_sum_forms_agree(monkeypatch, name):
    """Round 6 per-root sum forms, each pinned with LB_ALONE: under load (LB_ALONE=0) the Straus
    chunk sums with the blinding folded in (k_gsum_straus; the per-set r PK computed only for a
    search) against the per-set ladder + chunk sums (LB_GSUM_STRAUS=0); alone (LB_ALONE=1) the
    segmented shuffle tree (k_gsum_wave) against the k_gsum_tree launches (LB_GSUM_WAVE=0) and the
    serial chunk combine (LB_GSUM_TREE=0).  Same verdicts (c4 carries wrong and malformed sets, so
    its search runs from the Straus form's lazily computed r PK), byte-identical root partials."""
    from lodestar_amd.engine import Engine
    from lodestar_amd import workloads as W
    outs = []
    for alone, straus, wave, tree in (("0", "1", "1", "1"), ("0", "0", "1", "1"), ("1", "1", "1", "1"),
                                      ("1", "1", "0", "1"), ("1", "1", "1", "0")):
        monkeypatch.setenv("LB_ALONE", alone)
        monkeypatch.setenv("LB_GSUM_STRAUS", straus)
        monkeypatch.setenv("LB_GSUM_WAVE", wave)
        monkeypatch.setenv("LB_GSUM_TREE", tree)
        with Engine(0) as e:
            wl = W.make(e, name)
            b = e.upload(W.indexed_for(e, wl))
            try:
                sc = np.random.default_rng(9).integers(1, 1 << 63, size=wl.packed.n_sets, dtype=np.uint64)
                got = np.asarray(b.verify(scalars=sc))[:wl.packed.n_jobs]
                part = bytes(b.partial(scalars=sc)[0])
            finally:
                b.free()
        assert np.array_equal(got, wl.expected), (alone, straus, wave, tree, np.nonzero(got != wl.expected))
        outs.append(part)
    assert all(o == outs[0] for o in outs), [o[:8].hex() for o in outs]
