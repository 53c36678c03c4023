"""The device arithmetic headers (lodestar_amd/csrc/*.h) compiled for x86 (build/lb_harness.so,
test infrastructure) checked stage by stage against the oracle.  CPU only: this is how the
field tower, curve law, hash_to_G2 and pairing are pinned before they ever run on the GPU."""
import ctypes
import random

import pytest

from conftest import load_json
from oracle import bls_oracle as o

P = o.P


@pytest.fixture(scope="module")
def L():
    from lodestar_amd.build import build_harness
    return ctypes.CDLL(build_harness(verbose=False))


def b48(x):
    return (x % P).to_bytes(48, "big")


def fb48(b):
    return int.from_bytes(b, "big")


def b2(a):
    return b48(a[0]) + b48(a[1])


def fb2(b):
    return (fb48(b[:48]), fb48(b[48:96]))


def g2b(pt):
    return b2(pt[0]) + b2(pt[1])


def fg2(b):
    return (fb2(b[:96]), fb2(b[96:]))


def g1b(pt):
    return b48(pt[0]) + b48(pt[1])


def fg1(b):
    return (fb48(b[:48]), fb48(b[48:]))


def buf(n):
    return ctypes.create_string_buffer(n)


def test_fp_fp2(L):
    rnd = random.Random(1)
    edge = [0, 1, 2, P - 1, P - 2, (P - 1) // 2, (P + 1) // 2, 2**383 % P, 2**256]
    vals = edge + [rnd.randrange(P) for _ in range(40)]
    for a in vals:
        b = rnd.choice(vals)
        o_ = buf(48)
        L.h_fp_mul(b48(a), b48(b), o_)
        assert fb48(o_.raw) == a * b % P
        L.h_fp_add(b48(a), b48(b), o_)
        assert fb48(o_.raw) == (a + b) % P
        L.h_fp_sub(b48(a), b48(b), o_)
        assert fb48(o_.raw) == (a - b) % P
        L.h_fp_inv(b48(a), o_)
        assert fb48(o_.raw) == o.fp_inv(a)
        assert L.h_fp_is_square(b48(a)) == o.fp_is_square(a)
        A = (a, rnd.choice(vals))
        B = (rnd.randrange(P), rnd.randrange(P))
        o2 = buf(96)
        L.h_fp2_mul(b2(A), b2(B), o2)
        assert fb2(o2.raw) == o.f2_mul(A, B)
        L.h_fp2_sqr(b2(A), o2)
        assert fb2(o2.raw) == o.f2_sqr(A)
        L.h_fp2_inv(b2(A), o2)
        assert fb2(o2.raw) == o.f2_inv(A)
        ok = L.h_fp2_sqrt(b2(A), o2)
        assert bool(ok) == (o.f2_sqrt(A) is not None)
        if ok:
            assert o.f2_sqr(fb2(o2.raw)) == A
        assert L.h_fp2_sgn0(b2(A)) == o.f2_sgn0(A)


def test_fp_is_square_jacobi(L):
    # binary Jacobi symbol (lb_field.h fp_is_square) vs Euler's criterion in the oracle
    rnd = random.Random(7)
    vals = [rnd.randrange(P) for _ in range(400)] + [x * x % P for x in range(1, 50)] + [P - 1, 2, 3, 5]
    got = [bool(L.h_fp_is_square(b48(a))) for a in vals]
    assert got == [o.fp_is_square(a) for a in vals]
    assert 150 < sum(got[:400]) < 250


def test_fp2_sqrt_special(L):
    rnd = random.Random(2)
    for A in [(rnd.randrange(P), 0), (0, rnd.randrange(P)), (4, 0), (P - 4, 0), (0, 0), (1, 0)]:
        S = o.f2_sqr(A)
        o2 = buf(96)
        assert L.h_fp2_sqrt(b2(S), o2)
        assert o.f2_sqr(fb2(o2.raw)) == S


def test_hash_to_g2_stages(L):
    for msg in [bytes(32), bytes(range(32)), b"\xff" * 32]:
        o256 = buf(256)
        L.h_expand_xmd(msg, o256)
        assert o256.raw == o.expand_message_xmd(msg, o.DST_POP, 256)
        o192 = buf(192)
        L.h_hash_to_field(msg, o192)
        u = o.hash_to_field_fp2(msg, 2, o.DST_POP)
        assert fb2(o192.raw[:96]) == u[0] and fb2(o192.raw[96:]) == u[1]
        for ui in u:
            L.h_map_to_curve(b2(ui), o192)
            assert fg2(o192.raw) == o.iso_map(o.map_to_curve_sswu(ui))
        L.h_hash_to_g2(msg, o192)
        assert fg2(o192.raw) == o.hash_to_g2(msg)


def test_map_to_curve_fold(L):
    # map_to_curve_g2_fold (the Legendre symbol and the inversion folded into the square root's
    # first exponentiation; k_hash_map_row) against the oracle's SSWU + 3-isogeny: random field
    # elements (both branches of the square test), hash_to_field outputs, u = 0 (tv1 = 0)
    rnd = random.Random(11)
    us = [(rnd.randrange(P), rnd.randrange(P)) for _ in range(24)] + [(0, 0), (1, 0), (0, 1), (P - 1, 0)]
    for msg in [bytes(32), bytes(range(32))]:
        us += list(o.hash_to_field_fp2(msg, 2, o.DST_POP))
    branches = set()
    o192 = buf(192)
    for ui in us:
        assert L.h_map_to_curve_fold(b2(ui), o192)
        assert fg2(o192.raw) == o.iso_map(o.map_to_curve_sswu(ui))
        L.h_map_to_curve(b2(ui), o192)
        assert fg2(o192.raw) == o.iso_map(o.map_to_curve_sswu(ui))
        zu2 = o.f2_mul(o.SSWU_Z, o.f2_sqr(ui))
        tv1 = o.f2_add(o.f2_sqr(zu2), zu2)
        if o.f2_is_zero(tv1):
            x1 = o.f2_mul(o.SSWU_B, o.f2_inv(o.f2_mul(o.SSWU_Z, o.SSWU_A)))
        else:
            x1 = o.f2_mul(o.f2_mul(o.f2_neg(o.SSWU_B), o.f2_inv(o.SSWU_A)), o.f2_add(o.F2_ONE, o.f2_inv(tv1)))
        gx1 = o.f2_add(o.f2_add(o.f2_mul(o.f2_sqr(x1), x1), o.f2_mul(o.SSWU_A, x1)), o.SSWU_B)
        branches.add(o.f2_is_square(gx1))
    assert branches == {True, False}


def test_g2_subgroup_cofactor_psi(L):
    msg = bytes(range(32))
    H = o.hash_to_g2(msg)
    assert L.h_g2_in_subgroup(g2b(H)) == 1
    q = o.iso_map(o.map_to_curve_sswu(o.hash_to_field_fp2(msg, 2, o.DST_POP)[0]))
    assert L.h_g2_in_subgroup(g2b(q)) == 0
    o192 = buf(192)
    L.h_g2_clear_cofactor(g2b(q), o192)
    assert fg2(o192.raw) == o.g2_clear_cofactor(q)
    L.h_g2_psi(g2b(q), o192)
    assert fg2(o192.raw) == o.g2_psi(q)


def test_g2_aff_subgroup_matches_jacobian(L):
    # k_decode_sigs runs the affine, mixed-addition form of the psi == [x] test; it must agree
    # with the Jacobian form (and the oracle) on members and non-members of G2
    rnd = random.Random(11)
    for j in range(6):
        msg = bytes(rnd.getrandbits(8) for _ in range(32))
        H = o.hash_to_g2(msg)
        q = o.iso_map(o.map_to_curve_sswu(o.hash_to_field_fp2(msg, 2, o.DST_POP)[j % 2]))
        for P, want in ((H, 1), (q, 0), (o.g2_neg(q), 0), (o.g2_neg(H), 1)):
            assert L.h_g2_aff_in_subgroup(g2b(P)) == want
            assert L.h_g2_in_subgroup(g2b(P)) == want


def test_group_law(L):
    rnd = random.Random(3)
    H = o.hash_to_g2(b"\x01" * 32)
    pk = o.sk_to_pk(12345)
    o192, o96 = buf(192), buf(96)
    for k in [1, 2, 3, rnd.getrandbits(64), 2**64 - 1]:
        L.h_g2_mul(g2b(H), ctypes.c_uint64(k), o192)
        assert fg2(o192.raw) == o.g2_mul(H, k)
        L.h_g1_mul(g1b(pk), ctypes.c_uint64(k), o96)
        assert fg1(o96.raw) == o.g1_mul(pk, k)
    L.h_g1_add(g1b(pk), g1b(pk), o96)
    assert fg1(o96.raw) == o.g1_add(pk, pk)
    L.h_g1_add_aff(g1b(pk), g1b(pk), o96)
    assert fg1(o96.raw) == o.g1_add(pk, pk)
    assert L.h_g1_add(g1b(pk), g1b(o.g1_neg(pk)), o96) == 0   # P + (-P) = infinity
    assert L.h_g1_add_aff(g1b(pk), g1b(o.g1_neg(pk)), o96) == 0
    L.h_g2_add(g2b(H), g2b(H), o192)
    assert fg2(o192.raw) == o.g2_add(H, H)
    L.h_g2_dbl(g2b(H), o192)
    assert fg2(o192.raw) == o.g2_add(H, H)


def test_serialisation_against_fixtures(L):
    k4 = load_json("reference_kats.json")["K4_multithread_sets"]["sets"]
    inf = ctypes.c_int()
    o192, o96, o48 = buf(192), buf(96), buf(48)
    for s in k4:
        sig = bytes.fromhex(s["signature"])
        assert L.h_g2_decompress(sig, o192, ctypes.byref(inf)) == 0
        assert fg2(o192.raw) == o.g2_decompress(sig)
        L.h_g2_compress(o192.raw, o96)
        assert o96.raw == sig
        pk = bytes.fromhex(s["pubkey96"])
        assert L.h_g1_deserialize(pk, o96, ctypes.byref(inf)) == 0
        assert fg1(o96.raw) == o.g1_deserialize(pk)
    for pk48 in load_json("reference_kats.json")["K1_interop_pubkeys"]["pubkeys"][:4]:
        b = bytes.fromhex(pk48)
        assert L.h_g1_decompress(b, o96, ctypes.byref(inf)) == 0
        assert fg1(o96.raw) == o.g1_decompress(b)
        L.h_g1_compress(o96.raw, o48)
        assert o48.raw == b


def test_pairing_and_verify(L):
    msg = bytes(range(32))
    H = o.hash_to_g2(msg)
    pk = o.sk_to_pk(12345)
    sig = o.sign(12345, msg)
    o576 = buf(576)
    L.h_miller_fe(g1b(pk), g2b(H), o576)
    e = o.pairing(pk, H)
    assert o576.raw == o.f12_to_bytes(o.f12_mul(o.f12_mul(e, e), e))   # engine computes e^3
    ng1 = g1b(o.g1_neg(o.G1))
    assert L.h_pairing_check2(g1b(pk), g2b(H), ng1, g2b(sig)) == 1
    assert L.h_pairing_check2(g1b(pk), g2b(H), ng1, g2b(o.g2_add(sig, sig))) == 0
