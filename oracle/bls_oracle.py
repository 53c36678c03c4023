"""CPU ORACLE — test infrastructure only, never part of the product path.

A from-scratch pure-Python (big-int) restatement of the BLS12-381 arithmetic that
the reference's hot path delegates to its un-vendored dependency
``@chainsafe/bls@7.1.1`` -> ``@chainsafe/blst@0.2.7`` (supranational blst),
see SURVEY.md §2 row 8 and §8(c).  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker.

Reference call sites whose observable behaviour this restates:
  * packages/beacon-node/src/chain/bls/maybeBatch.ts:16-39   (verifySignatureSetsMaybeBatch)
  * packages/beacon-node/src/chain/bls/utils.ts:5-16          (getAggregatedPubkey)
  * packages/beacon-node/src/chain/bls/multithread/worker.ts:32-116 (per-job re-verify)
  * packages/state-transition/src/util/interop.ts:19-23       (interop secret keys, fixture K1)

Published algorithms restated (the dependency is absent from /root/reference):
  * IETF draft-irtf-cfrg-bls-signature-04, min-pubkey-size, proof-of-possession
    ciphersuite ``BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_``
  * RFC 9380 hash_to_curve for BLS12381G2_XMD:SHA-256_SSWU_RO_ (expand_message_xmd,
    hash_to_field, simplified SWU on the 3-isogenous curve, 3-isogeny, h_eff cofactor
    clearing via the psi endomorphism).  The 3-isogeny map is *derived* here with
    Velu's formulas from its kernel (x0 = -6+6i) rather than copied as constants;
    the choice among the six normalisations is pinned by fixture K2.
  * ZCash BLS12-381 point serialisation (flags 0x80 compressed / 0x40 infinity / 0x20 sign).
  * Optimal-ate pairing with affine Miller loop on the twist and plain final
    exponentiation f^((p^12-1)/r).
  * blst batch semantics: random non-zero 64-bit blinding scalars, product of Miller
    loops, single final exponentiation.

Pinned by: K1 interop pubkeys, K2 interop deposit signature (tests/test_oracle_kat.py).
"""
from __future__ import annotations

import hashlib
import os
from typing import List, Optional, Sequence, Tuple

# --------------------------------------------------------------------------- params
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
BLS_X = -0xD201000000010000            # curve parameter (negative)
R = BLS_X**4 - BLS_X**2 + 1            # prime subgroup order
assert R == 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
assert P == (BLS_X - 1) ** 2 * R // 3 + BLS_X

DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"

G1_X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1_Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1


# --------------------------------------------------------------------------- Fp
def fp_inv(a: int) -> int:
    a %= P
    if a == 0:
        return 0  # inv0 convention (RFC 9380)
    return pow(a, P - 2, P)


def fp_is_square(a: int) -> bool:
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


def fp_sqrt(a: int) -> Optional[int]:
    a %= P
    s = pow(a, (P + 1) // 4, P)  # p = 3 mod 4
    return s if s * s % P == a else None


# --------------------------------------------------------------------------- Fp2 = Fp[u]/(u^2+1)
Fp2 = Tuple[int, int]
F2_ZERO: Fp2 = (0, 0)
F2_ONE: Fp2 = (1, 0)


def f2(a, b=0) -> Fp2:
    return (a % P, b % P)


def f2_add(a: Fp2, b: Fp2) -> Fp2:
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a: Fp2, b: Fp2) -> Fp2:
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a: Fp2) -> Fp2:
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a: Fp2, b: Fp2) -> Fp2:
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2_sqr(a: Fp2) -> Fp2:
    return f2_mul(a, a)


def f2_muls(a: Fp2, s: int) -> Fp2:
    return (a[0] * s % P, a[1] * s % P)


def f2_conj(a: Fp2) -> Fp2:
    return (a[0], (-a[1]) % P)


def f2_inv(a: Fp2) -> Fp2:
    n = fp_inv(a[0] * a[0] + a[1] * a[1])
    return (a[0] * n % P, (-a[1]) * n % P)


def f2_pow(a: Fp2, e: int) -> Fp2:
    r = F2_ONE
    while e:
        if e & 1:
            r = f2_mul(r, a)
        a = f2_sqr(a)
        e >>= 1
    return r


def f2_is_zero(a: Fp2) -> bool:
    return a[0] == 0 and a[1] == 0


def f2_is_square(a: Fp2) -> bool:
    # a is a square in Fp2 iff its norm is a square in Fp
    return fp_is_square(a[0] * a[0] + a[1] * a[1])


def f2_sqrt(a: Fp2) -> Optional[Fp2]:
    """Complex-method square root in Fp2 (p = 3 mod 4); any root, or None."""
    a0, a1 = a[0] % P, a[1] % P
    if a1 == 0:
        s = fp_sqrt(a0)
        if s is not None:
            return (s, 0)
        s = fp_sqrt(-a0)
        return None if s is None else (0, s)
    alpha = fp_sqrt(a0 * a0 + a1 * a1)
    if alpha is None:
        return None
    inv2 = fp_inv(2)
    delta = (a0 + alpha) * inv2 % P
    x0 = fp_sqrt(delta)
    if x0 is None:
        delta = (a0 - alpha) * inv2 % P
        x0 = fp_sqrt(delta)
        if x0 is None:
            return None
    x1 = a1 * fp_inv(2 * x0) % P
    r = (x0, x1)
    return r if f2_sqr(r) == (a0, a1) else None


def f2_sgn0(a: Fp2) -> int:
    """RFC 9380 §4.1 sgn0 for m = 2."""
    sign_0 = a[0] & 1
    zero_0 = a[0] == 0
    sign_1 = a[1] & 1
    return sign_0 | (zero_0 and sign_1)


XI: Fp2 = (1, 1)  # non-residue 1+u


# --------------------------------------------------------------------------- Fp6 = Fp2[v]/(v^3 - xi)
def f6_add(a, b):
    return (f2_add(a[0], b[0]), f2_add(a[1], b[1]), f2_add(a[2], b[2]))


def f6_sub(a, b):
    return (f2_sub(a[0], b[0]), f2_sub(a[1], b[1]), f2_sub(a[2], b[2]))


def f6_neg(a):
    return (f2_neg(a[0]), f2_neg(a[1]), f2_neg(a[2]))


def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    t0, t1, t2 = f2_mul(a0, b0), f2_mul(a1, b1), f2_mul(a2, b2)
    c0 = f2_add(t0, f2_mul(XI, f2_add(f2_mul(a1, b2), f2_mul(a2, b1))))
    c1 = f2_add(f2_add(f2_mul(a0, b1), f2_mul(a1, b0)), f2_mul(XI, t2))
    c2 = f2_add(f2_add(f2_mul(a0, b2), f2_mul(a2, b0)), t1)
    return (c0, c1, c2)


def f6_mul_by_v(a):
    return (f2_mul(XI, a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    t0 = f2_sub(f2_sqr(a0), f2_mul(XI, f2_mul(a1, a2)))
    t1 = f2_sub(f2_mul(XI, f2_sqr(a2)), f2_mul(a0, a1))
    t2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    d = f2_add(f2_mul(a0, t0), f2_mul(XI, f2_add(f2_mul(a2, t1), f2_mul(a1, t2))))
    di = f2_inv(d)
    return (f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di))


F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)


# --------------------------------------------------------------------------- Fp12 = Fp6[w]/(w^2 - v)
F12_ONE = (F6_ONE, F6_ZERO)


def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = f6_mul(a0, b0)
    t1 = f6_mul(a1, b1)
    c0 = f6_add(t0, f6_mul_by_v(t1))
    c1 = f6_add(f6_mul(a0, b1), f6_mul(a1, b0))
    return (c0, c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    a0, a1 = a
    t = f6_sub(f6_mul(a0, a0), f6_mul_by_v(f6_mul(a1, a1)))
    ti = f6_inv(t)
    return (f6_mul(a0, ti), f6_neg(f6_mul(a1, ti)))


def f12_pow(a, e: int):
    r = F12_ONE
    while e:
        if e & 1:
            r = f12_mul(r, a)
        a = f12_sqr(a)
        e >>= 1
    return r


def f12_from_f2_coeffs(c: Sequence[Fp2]):
    """Element sum_k c[k] * w^k, k = 0..5 (w^2 = v)."""
    # w^0 -> (c0 v^0), w^1 -> c1 part v^0, w^2 -> c0 part v^1, w^3 -> c1 part v^1, w^4 -> c0 v^2, w^5 -> c1 v^2
    return ((c[0], c[2], c[4]), (c[1], c[3], c[5]))


def f12_to_bytes(a) -> bytes:
    """Flat big-endian serialisation (c0.c0.c0, c0.c0.c1, c0.c1.c0, ...), 576 bytes."""
    out = b""
    for six in a:
        for two in six:
            for e in two:
                out += e.to_bytes(48, "big")
    return out


# --------------------------------------------------------------------------- curves (affine, None = infinity)
B1 = 4
B2: Fp2 = (4, 4)  # 4(1+u)


def g1_on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - B1) % P == 0


def g1_add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * fp_inv(2 * y1) % P
    else:
        lam = (y2 - y1) * fp_inv(x2 - x1) % P
    x3 = (lam * lam - x1 - x2) % P
    return (x3, (lam * (x1 - x3) - y1) % P)


def g1_neg(pt):
    return None if pt is None else (pt[0], (-pt[1]) % P)


def g1_mul(pt, k: int):
    if k < 0:
        return g1_mul(g1_neg(pt), -k)
    acc = None
    while k:
        if k & 1:
            acc = g1_add(acc, pt)
        pt = g1_add(pt, pt)
        k >>= 1
    return acc


G1 = (G1_X, G1_Y)


def g2_on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return f2_sub(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), B2)) == F2_ZERO


def g2_add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2:
        if f2_add(y1, y2) == F2_ZERO:
            return None
        lam = f2_mul(f2_muls(f2_sqr(x1), 3), f2_inv(f2_muls(y1, 2)))
    else:
        lam = f2_mul(f2_sub(y2, y1), f2_inv(f2_sub(x2, x1)))
    x3 = f2_sub(f2_sub(f2_sqr(lam), x1), x2)
    return (x3, f2_sub(f2_mul(lam, f2_sub(x1, x3)), y1))


def g2_neg(pt):
    return None if pt is None else (pt[0], f2_neg(pt[1]))


def g2_neg(pt):
    return None if pt is None else (pt[0], f2_neg(pt[1]))


def g2_mul(pt, k: int):
    if k < 0:
        return g2_mul(g2_neg(pt), -k)
    acc = None
    while k:
        if k & 1:
            acc = g2_add(acc, pt)
        pt = g2_add(pt, pt)
        k >>= 1
    return acc


# psi = untwist o Frobenius o twist (RFC 9380 App. G.3)
PSI_CX: Fp2 = f2_inv(f2_pow(XI, (P - 1) // 3))
PSI_CY: Fp2 = f2_inv(f2_pow(XI, (P - 1) // 2))


def g2_psi(pt):
    if pt is None:
        return None
    x, y = pt
    return (f2_mul(f2_conj(x), PSI_CX), f2_mul(f2_conj(y), PSI_CY))


def g2_in_subgroup_slow(pt) -> bool:
    return g2_mul(pt, R) is None


def g2_in_subgroup(pt) -> bool:
    """Scott's test: P in G2 iff psi(P) == [x]P (the check blst performs)."""
    if pt is None:
        return True
    return g2_psi(pt) == g2_mul(pt, BLS_X)


def g2_clear_cofactor(pt):
    """h_eff * P via psi (Budroni-Pintore; RFC 9380 App. G.3)."""
    t1 = g2_mul(pt, BLS_X)
    t2 = g2_psi(pt)
    t3 = g2_psi(g2_psi(g2_add(pt, pt)))
    t3 = g2_add(t3, g2_neg(t2))
    t2 = g2_add(t1, t2)
    t2 = g2_mul(t2, BLS_X)
    t3 = g2_add(t3, t2)
    t3 = g2_add(t3, g2_neg(t1))
    return g2_add(t3, g2_neg(pt))


# --------------------------------------------------------------------------- hash_to_G2 (RFC 9380)
def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    ell = (len_in_bytes + 31) // 32
    assert ell <= 255 and len(dst) <= 255
    dst_prime = dst + bytes([len(dst)])
    msg_prime = bytes(64) + msg + len_in_bytes.to_bytes(2, "big") + b"\x00" + dst_prime
    b0 = hashlib.sha256(msg_prime).digest()
    bi = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = bi
    for i in range(2, ell + 1):
        bi = hashlib.sha256(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out += bi
    return out[:len_in_bytes]


def hash_to_field_fp2(msg: bytes, count: int, dst: bytes) -> List[Fp2]:
    L = 64
    ub = expand_message_xmd(msg, dst, count * 2 * L)
    out = []
    for i in range(count):
        e0 = int.from_bytes(ub[(2 * i) * L:(2 * i + 1) * L], "big") % P
        e1 = int.from_bytes(ub[(2 * i + 1) * L:(2 * i + 2) * L], "big") % P
        out.append((e0, e1))
    return out


# SSWU on E2': y^2 = x^3 + A' x + B'
SSWU_A: Fp2 = (0, 240)
SSWU_B: Fp2 = (1012, 1012)
SSWU_Z: Fp2 = f2(-2, -1)


def map_to_curve_sswu(u: Fp2):
    """RFC 9380 §6.6.2 simplified SWU (plain statement), returns a point on E2'."""
    A, B, Z = SSWU_A, SSWU_B, SSWU_Z
    u2 = f2_sqr(u)
    zu2 = f2_mul(Z, u2)
    tv1 = f2_add(f2_sqr(zu2), zu2)
    tv1 = f2_inv(tv1) if not f2_is_zero(tv1) else F2_ZERO
    if f2_is_zero(tv1):
        x1 = f2_mul(B, f2_inv(f2_mul(Z, A)))
    else:
        x1 = f2_mul(f2_mul(f2_neg(B), f2_inv(A)), f2_add(F2_ONE, tv1))
    gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(A, x1)), B)
    x2 = f2_mul(zu2, x1)
    gx2 = f2_add(f2_add(f2_mul(f2_sqr(x2), x2), f2_mul(A, x2)), B)
    if f2_is_square(gx1):
        x, y = x1, f2_sqrt(gx1)
    else:
        x, y = x2, f2_sqrt(gx2)
    assert y is not None
    if f2_sgn0(u) != f2_sgn0(y):
        y = f2_neg(y)
    return (x, y)


def _derive_iso3():
    """Velu 3-isogeny E2' -> E2 with kernel x0 = -6+6i, normalised by an
    isomorphism (x,y) -> (c^2 x, c^3 y).  Returns the list of 6 candidate maps,
    each as (x0, v, w, c2, c3) so that
       X = c2 * (x + v/(x-x0) + w/(x-x0)^2)
       Y = c3 * y * (1 - v/(x-x0)^2 - 2w/(x-x0)^3)
    """
    x0: Fp2 = f2(-6, 6)
    A = SSWU_A
    # the kernel point must be 3-torsion: psi3(x0) = 3x^4 + 6Ax^2 + 12Bx - A^2 = 0
    x02 = f2_sqr(x0)
    psi3 = f2_sub(f2_add(f2_add(f2_muls(f2_sqr(x02), 3), f2_muls(f2_mul(A, x02), 6)),
                         f2_muls(f2_mul(SSWU_B, x0), 12)), f2_sqr(A))
    assert psi3 == F2_ZERO, "kernel x0 is not a 3-torsion abscissa"
    gx = f2_add(f2_mul(x02, f2_muls(F2_ONE, 3)), A)            # g^x_Q = 3x0^2 + A
    y02 = f2_add(f2_add(f2_mul(x02, x0), f2_mul(A, x0)), SSWU_B)  # y0^2
    v = f2_muls(gx, 2)                                          # v_Q = 2 g^x_Q
    w = f2_muls(y02, 4)                                         # u_Q = (g^y_Q)^2 = 4 y0^2
    a_new = f2_sub(A, f2_muls(v, 5))
    b_new = f2_sub(SSWU_B, f2_muls(f2_add(w, f2_mul(x0, v)), 7))
    assert a_new == F2_ZERO, "Velu codomain is not j=0"
    # need c^6 = B2 / b_new
    target = f2_mul(B2, f2_inv(b_new))
    cands = []
    # sixth roots: solve c^2 = s where s^3 = target
    # cube roots in Fp2: brute force via exponent tricks is awkward; use generic search
    # through a square-root / cube-root over the (small) set of candidates obtained by
    # multiplying one root with 6th roots of unity.
    c = _f2_root6(target)
    assert c is not None
    zeta6 = _f2_primitive_6th_root()
    ck = c
    for _ in range(6):
        c2 = f2_sqr(ck)
        c3 = f2_mul(c2, ck)
        cands.append((x0, v, w, c2, c3))
        ck = f2_mul(ck, zeta6)
    return cands


def _f2_cbrt(a: Fp2) -> Optional[Fp2]:
    """Some cube root of a in Fp2, or None (Tonelli-Shanks style over the 3-Sylow part)."""
    q = P * P - 1
    s, t = 0, q
    while t % 3 == 0:
        t //= 3
        s += 1
    if f2_pow(a, q // 3) != F2_ONE:
        return None
    g = next(z for z in ((c0, c1) for c0 in range(1, 50) for c1 in range(0, 5))
             if f2_pow(z, q // 3) != F2_ONE)
    k = 1 if t % 3 == 2 else 2
    r0 = f2_pow(a, (k * t + 1) // 3)
    h = f2_pow(g, t)
    e = F2_ONE
    for _ in range(3 ** s):
        c = f2_mul(r0, e)
        if f2_mul(f2_sqr(c), c) == a:
            return c
        e = f2_mul(e, h)
    return None


def _f2_root6(a: Fp2) -> Optional[Fp2]:
    s = _f2_cbrt(a)
    if s is None:
        return None
    # try all cube-root variants of s for a square
    om = _f2_primitive_cube_root()
    for k in range(3):
        c = f2_sqrt(s)
        if c is not None:
            return c
        s = f2_mul(s, om)
    return None


def _f2_primitive_cube_root() -> Fp2:
    # omega = (-1 + sqrt(-3))/2 lies in Fp
    s = fp_sqrt(-3)
    return ((-1 + s) * fp_inv(2) % P, 0)


def _f2_primitive_6th_root() -> Fp2:
    om = _f2_primitive_cube_root()
    return f2_neg(om) if f2_pow(f2_neg(om), 3) != F2_ONE else f2_neg(f2_sqr(om))


_ISO_CANDIDATES = None
ISO_INDEX = 2  # which of the 6 normalisations; pinned by KAT K2 (see tests)


def iso_candidates():
    global _ISO_CANDIDATES
    if _ISO_CANDIDATES is None:
        _ISO_CANDIDATES = _derive_iso3()
    return _ISO_CANDIDATES


def iso_map(pt, index: Optional[int] = None):
    if pt is None:
        return None
    x0, v, w, c2, c3 = iso_candidates()[ISO_INDEX if index is None else index]
    x, y = pt
    d = f2_sub(x, x0)
    if f2_is_zero(d):
        return None  # kernel point maps to infinity
    di = f2_inv(d)
    di2 = f2_sqr(di)
    di3 = f2_mul(di2, di)
    X = f2_add(f2_add(x, f2_mul(v, di)), f2_mul(w, di2))
    dX = f2_sub(f2_sub(F2_ONE, f2_mul(v, di2)), f2_muls(f2_mul(w, di3), 2))
    Y = f2_mul(y, dX)
    return (f2_mul(c2, X), f2_mul(c3, Y))


def iso_map_rational_coeffs(index: Optional[int] = None):
    """Expand the isogeny into RFC-style polynomials: x_num (deg 3), x_den (monic deg 2),
    y_num (deg 3), y_den (monic deg 3), coefficients low->high."""
    x0, v, w, c2, c3 = iso_candidates()[ISO_INDEX if index is None else index]
    # d = x - x0 ; X = c2 (x d^2 + v d + w) / d^2 ; Y = c3 y (d^3 - v d - 2w) / d^3
    def pmul(a, b):
        out = [F2_ZERO] * (len(a) + len(b) - 1)
        for i, ai in enumerate(a):
            for j, bj in enumerate(b):
                out[i + j] = f2_add(out[i + j], f2_mul(ai, bj))
        return out

    def padd(a, b):
        n = max(len(a), len(b))
        a = a + [F2_ZERO] * (n - len(a))
        b = b + [F2_ZERO] * (n - len(b))
        return [f2_add(x, y) for x, y in zip(a, b)]

    d = [f2_neg(x0), F2_ONE]
    d2 = pmul(d, d)
    d3 = pmul(d2, d)
    xnum = padd(padd(pmul([F2_ZERO, F2_ONE], d2), [f2_mul(v, c) for c in d]), [w])
    xnum = [f2_mul(c2, c) for c in xnum]
    ynum = padd(padd(d3, [f2_neg(f2_mul(v, c)) for c in d]), [f2_neg(f2_muls(w, 2))])
    ynum = [f2_mul(c3, c) for c in ynum]
    return xnum, d2, ynum, d3


def hash_to_g2(msg: bytes, dst: bytes = DST_POP):
    u0, u1 = hash_to_field_fp2(msg, 2, dst)
    q0 = iso_map(map_to_curve_sswu(u0))
    q1 = iso_map(map_to_curve_sswu(u1))
    return g2_clear_cofactor(g2_add(q0, q1))


# --------------------------------------------------------------------------- serialisation (ZCash)
HALF_P = (P - 1) // 2


class BlsError(Exception):
    """Carries a blst error name as its message, as @chainsafe/blst's ErrorBLST does."""


def g1_compress(pt) -> bytes:
    if pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = pt
    b = bytearray(x.to_bytes(48, "big"))
    b[0] |= 0x80
    if y > HALF_P:
        b[0] |= 0x20
    return bytes(b)


def g1_serialize(pt) -> bytes:
    """96-byte uncompressed (blst PublicKey.toBytes(PointFormat.uncompressed))."""
    if pt is None:
        return bytes([0x40]) + bytes(95)
    return pt[0].to_bytes(48, "big") + pt[1].to_bytes(48, "big")


def g1_decompress(b: bytes):
    if len(b) != 48:
        raise BlsError("BLST_INVALID_SIZE")
    if not (b[0] & 0x80):
        raise BlsError("BLST_BAD_ENCODING")
    if b[0] & 0x40:
        if (b[0] & 0x3F) or any(b[1:]):
            raise BlsError("BLST_BAD_ENCODING")
        return None
    x = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:], "big")
    if x >= P:
        raise BlsError("BLST_BAD_ENCODING")
    y = fp_sqrt(x * x * x + B1)
    if y is None:
        raise BlsError("BLST_POINT_NOT_ON_CURVE")
    if (y > HALF_P) != bool(b[0] & 0x20):
        y = P - y
    return (x, y)


def g1_deserialize(b: bytes):
    """96-byte uncompressed or 48-byte compressed G1, no subgroup check
    (worker.ts:110-116 deserializes pubkeys without validation)."""
    if len(b) == 48:
        return g1_decompress(b)
    if len(b) != 96:
        raise BlsError("BLST_INVALID_SIZE")
    if b[0] & 0x80:
        raise BlsError("BLST_BAD_ENCODING")
    if b[0] & 0x40:
        if (b[0] & 0x3F) or any(b[1:]):
            raise BlsError("BLST_BAD_ENCODING")
        return None
    x = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:48], "big")
    y = int.from_bytes(b[48:], "big")
    if x >= P or y >= P:
        raise BlsError("BLST_BAD_ENCODING")
    pt = (x, y)
    if not g1_on_curve(pt):
        raise BlsError("BLST_POINT_NOT_ON_CURVE")
    return pt


def _f2_lex_larger(y: Fp2) -> bool:
    return y[1] > HALF_P if y[1] != 0 else y[0] > HALF_P


def g2_compress(pt) -> bytes:
    if pt is None:
        return bytes([0xC0]) + bytes(95)
    x, y = pt
    b = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
    b[0] |= 0x80
    if _f2_lex_larger(y):
        b[0] |= 0x20
    return bytes(b)


def g2_decompress(b: bytes):
    """96-byte compressed G2 -> affine point (no subgroup check)."""
    if len(b) != 96:
        raise BlsError("BLST_INVALID_SIZE")
    if not (b[0] & 0x80):
        raise BlsError("BLST_BAD_ENCODING")
    if b[0] & 0x40:
        if (b[0] & 0x3F) or any(b[1:]):
            raise BlsError("BLST_BAD_ENCODING")
        return None
    x1 = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:], "big")
    if x0 >= P or x1 >= P:
        raise BlsError("BLST_BAD_ENCODING")
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise BlsError("BLST_POINT_NOT_ON_CURVE")
    if _f2_lex_larger(y) != bool(b[0] & 0x20):
        y = f2_neg(y)
    return (x, y)


def signature_from_bytes(b: bytes, validate: bool = True):
    """Signature.fromBytes(bytes, CoordType.affine, validate) (maybeBatch.ts:23,36)."""
    pt = g2_decompress(b)
    if validate and not g2_in_subgroup(pt):
        raise BlsError("BLST_POINT_NOT_IN_GROUP")
    return pt


# --------------------------------------------------------------------------- pairing
def _line_eval(lam: Fp2, xt: Fp2, yt: Fp2, pxy):
    """Line through twist point T with twist slope lam, evaluated at P in G1,
    scaled by w^3 (a factor in Fp4, killed by the final exponentiation):
        l = yP w^3 - lam xP w^2 + (lam xT - yT)."""
    px, py = pxy
    c = [F2_ZERO] * 6
    c[0] = f2_sub(f2_mul(lam, xt), yt)
    c[2] = f2_neg(f2_muls(lam, px))
    c[3] = (py % P, 0)
    return f12_from_f2_coeffs(c)


def _vertical_eval(xt: Fp2, pxy):
    # x_P - x_T/w^2, scaled by w^2: xP w^2 - xT
    c = [F2_ZERO] * 6
    c[0] = f2_neg(xt)
    c[2] = (pxy[0] % P, 0)
    return f12_from_f2_coeffs(c)


def miller_loop(p1, q2):
    """f_{|x|,Q}(P), conjugated because x < 0.  Affine arithmetic on the twist."""
    if p1 is None or q2 is None:
        return F12_ONE
    f = F12_ONE
    T = q2
    n = -BLS_X
    for bit in bin(n)[3:]:
        xt, yt = T
        lam = f2_mul(f2_muls(f2_sqr(xt), 3), f2_inv(f2_muls(yt, 2)))
        f = f12_mul(f12_sqr(f), _line_eval(lam, xt, yt, p1))
        T = g2_add(T, T)
        if bit == "1":
            xt, yt = T
            xq, yq = q2
            if xt == xq:
                f = f12_mul(f, _vertical_eval(xt, p1))
            else:
                lam = f2_mul(f2_sub(yq, yt), f2_inv(f2_sub(xq, xt)))
                f = f12_mul(f, _line_eval(lam, xt, yt, p1))
            T = g2_add(T, q2)
    return f12_conj(f)


FE_EXP = (P**12 - 1) // R


def final_exponentiation(f):
    g = f12_mul(f12_conj(f), f12_inv(f))      # f^(p^6-1)
    g = f12_mul(f12_pow(g, P * P), g)          # ^(p^2+1)
    return f12_pow(g, (P**4 - P * P + 1) // R)


def pairing(p1, q2):
    return final_exponentiation(miller_loop(p1, q2))


# --------------------------------------------------------------------------- BLS scheme
def interop_secret_key(index: int) -> int:
    """packages/state-transition/src/util/interop.ts:19-23 with utils/src/bytes.ts
    (intToBytes/bytesToBigInt default little-endian)."""
    d = hashlib.sha256(index.to_bytes(32, "little")).digest()
    return int.from_bytes(d, "little") % R


def sk_to_pk(sk: int):
    return g1_mul(G1, sk)


def sign(sk: int, msg: bytes, dst: bytes = DST_POP):
    return g2_mul(hash_to_g2(msg, dst), sk)


def core_verify(pk, msg: bytes, sig, dst: bytes = DST_POP) -> bool:
    """e(PK, H(m)) * e(-G1, sig) == 1."""
    if pk is None:
        raise BlsError("BLST_PK_IS_INFINITY")
    f = f12_mul(miller_loop(pk, hash_to_g2(msg, dst)), miller_loop(g1_neg(G1), sig))
    return final_exponentiation(f) == F12_ONE


def aggregate_pubkeys(pks):
    """bls.PublicKey.aggregate (utils.ts:11); empty -> EMPTY_AGGREGATE_ARRAY."""
    if len(pks) == 0:
        raise BlsError("EMPTY_AGGREGATE_ARRAY")
    acc = None
    for pk in pks:
        acc = g1_add(acc, pk)
    return acc


GLV_LAMBDA = (-BLS_X * BLS_X) % R  # [lambda]P = (beta x, y) on G1, -psi^2 on G2


def blinding_scalar(word: int) -> int:
    """The blinding value a 64-bit scalar word stands for in the HIP engine (lb_curve.h
    jac_mul_glv): r = lo + hi * lambda mod r_order, lambda = -x^2.  blst draws r as the 64-bit
    integer itself (maybeBatch.ts:18-25 -> verifyMultipleSignatures); both are uniform draws
    from 2^64 - 1 distinct non-zero values, so the verdicts agree except with probability
    2^-64 per invalid batch."""
    return ((word & 0xFFFFFFFF) + (word >> 32) * GLV_LAMBDA) % R


def random_scalar64() -> int:
    while True:
        r = int.from_bytes(os.urandom(8), "little")
        if r:
            return r


def verify_multiple_signatures(sets, scalars=None, dst: bytes = DST_POP) -> bool:
    """blst Pairing + mul_n_aggregate + commit + finalverify (maybeBatch.ts:18-25).
    sets: list of (pk_affine, msg, sig_affine).  Raises BlsError for an infinity pk."""
    f = F12_ONE
    sig_sum = None
    for i, (pk, msg, sig) in enumerate(sets):
        if pk is None:
            raise BlsError("BLST_PK_IS_INFINITY")
        r = scalars[i] if scalars is not None else random_scalar64()
        sig_sum = g2_add(sig_sum, g2_mul(sig, r))
        f = f12_mul(f, miller_loop(g1_mul(pk, r), hash_to_g2(msg, dst)))
    f = f12_mul(f, miller_loop(g1_neg(G1), sig_sum))
    return final_exponentiation(f) == F12_ONE


def verify_sets_maybe_batch(sets, scalars=None) -> bool:
    """verifySignatureSetsMaybeBatch (maybeBatch.ts:16-39).
    sets: list of (pk_affine, msg32, sig_bytes)."""
    if len(sets) >= 2:
        decoded = [(pk, m, signature_from_bytes(s, True)) for pk, m, s in sets]
        return verify_multiple_signatures(decoded, scalars)
    if len(sets) == 0:
        raise BlsError("Empty signature set")
    pk, m, s = sets[0]
    sig = signature_from_bytes(s, True)
    return core_verify(pk, m, sig)


# --------------------------------------------------------------------------- SSZ helpers (fixture K2)
def _sha(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def compute_domain(domain_type: bytes, fork_version: bytes, genesis_validators_root: bytes) -> bytes:
    fork_data_root = _sha(fork_version.ljust(32, b"\x00") + genesis_validators_root)
    return domain_type + fork_data_root[:28]


def deposit_message_root(pubkey48: bytes, withdrawal_credentials: bytes, amount: int) -> bytes:
    pk_root = _sha(pubkey48[:32] + pubkey48[32:].ljust(32, b"\x00"))
    amt = amount.to_bytes(8, "little").ljust(32, b"\x00")
    return _sha(_sha(pk_root + withdrawal_credentials) + _sha(amt + bytes(32)))


def compute_signing_root(object_root: bytes, domain: bytes) -> bytes:
    return _sha(object_root + domain)


# --------------------------------------------------------------------------- job semantics
def verify_job(sets, scalars=None):
    """One BlsWorkReq's result as the reference computes it.
    sets: list of (pubkeys96: list[bytes], signing_root32: bytes, signature: bytes).
    Returns True/False or raises BlsError(name).  Error precedence follows the reference:
      1. main thread getAggregatedPubkey (utils.ts:5-16): empty aggregate -> EMPTY_AGGREGATE_ARRAY
      2. worker deserializeSet (worker.ts:110-116): PublicKey.fromBytes(96 B) decode errors
      3. maybeBatch.ts:18-25 / :36: Signature.fromBytes(sig, affine, validate=true) in set order
      4. mul_n_aggregate / core verify: infinite aggregate pubkey -> BLST_PK_IS_INFINITY
    An infinite signature is skipped in the aggregate (blst), so such a set verifies false
    (parity unpinned: no reference test covers it)."""
    if len(sets) == 0:
        raise BlsError("Empty signature set")
    for pks, _, _ in sets:
        if len(pks) == 0:
            raise BlsError("EMPTY_AGGREGATE_ARRAY")
    agg = []
    for pks, _, _ in sets:
        acc = None
        for pk in pks:
            acc = g1_add(acc, g1_deserialize(pk))
        agg.append(acc)
    sigs = [signature_from_bytes(s, True) for _, _, s in sets]
    for a in agg:
        if a is None:
            raise BlsError("BLST_PK_IS_INFINITY")
    if len(sets) >= 2:
        return verify_multiple_signatures([(a, m, sg) for a, (_, m, _), sg in zip(agg, sets, sigs)], scalars)
    a, (_, m, _), sg = agg[0], sets[0], sigs[0]
    if sg is None:
        return False
    return core_verify(a, m, sg)
