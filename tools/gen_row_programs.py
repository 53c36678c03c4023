#!/usr/bin/env python3
"""Row-engine programs (lodestar_amd/csrc/lb_row.h): the wave programs' formulas re-encoded for
an engine that runs each Fp product on one 16-lane ROW (lane k holds limb k of 14 signed 28-bit
limbs, Montgomery radix R' = 2^392) instead of one lane.

Output: lodestar_amd/csrc/lb_row_progs.h (generated; do not edit).

The programs (MUL12, SQR12, FROB, FROB2, DBL_STEP, ADD_STEP; tools/gen_wave_programs.py traces
them from the tower formulas) keep their slot map and phase schedule; only the encoding changes
(int32 words, signed coefficients, one record per row task):

  program   [n_phases, n_out, out_slot * n_out]
  phase     [kind | flags << 8 | n_tasks << 16, nx | ny << 16], then n_tasks records
  record    kind 0 (product): [dst, x pairs * nx, y pairs * ny]; kind 1 (linear): [dst, pairs * nx]
  pair      (slot & 0xffff) | (coef << 16), coef a signed 16-bit integer; padding: the zero slot,
            coefficient 0
  flags     bit 0: every task's x operand is one slot with coefficient 1 (read as is, no
            reduction); bit 1: the same for y; bit 2: some x operand has a coefficient sum above
            16 (the quotient reduction runs; otherwise only the limb carries); bit 3: the same for y

Arithmetic (mirrored exactly by RowModel below and checked against big integers and the oracle):
a slot value v is an integer in (-2p, 2p) congruent to the element times R' (mod p); an operand
or linear output is the signed limb sum, reduced by a quotient estimate from its top two limbs
(q = floor((l13 2^28 + l12) 2^336 / p) in double precision) to [0, p) up to an error far below p;
a product is the row Montgomery product (lb_row.h rp_mul): |x y| / R' + 1.0001 p.
"""
import math
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import gen_wave_programs as G  # noqa: E402

P = G.P
RP = 1 << 392
M28 = (1 << 28) - 1
PINV = (-pow(P, -1, RP)) % RP
PL = [(P >> (28 * i)) & M28 for i in range(14)]
PPL = [(PINV >> (28 * i)) & M28 for i in range(14)]
INV_P336 = (1 << 336) / P
OUT_PATH = os.path.join(ROOT, "lodestar_amd", "csrc", "lb_row_progs.h")
N_CONST = G.N_CONST


# ------------------------------------------------------------ exact model of lb_row.h
def val(l):
    return sum(v << (28 * k) for k, v in enumerate(l[:14]))


def limbs(v):
    """normalized limbs of a signed integer (limbs 0..12 in [0, 2^28), limb 13 signed)"""
    out = []
    for _ in range(13):
        out.append(v & M28)
        v >>= 28
    return out + [v, 0, 0]


def _shr(v, s):
    return [0] * s + v[:16 - s]


def _shl(v, s):
    return v[s:] + [0] * s


def _i32(x):
    assert -(1 << 31) <= x < (1 << 31), x
    return x


def norm(v, keep_top):
    """lb_row.h rp_norm: two carry rounds (64-bit, then 32-bit); keep_top: limb 13 keeps its
    whole value and takes limb 12's carry whole (the result is a value, not a residue mod 2^392)"""
    for x in v:
        assert -(1 << 63) <= x < (1 << 63)
    q = [x >> 28 for x in v]
    l = [x & M28 for x in v]
    qlo = [x & M28 for x in q]
    qhi = [x >> 28 for x in q]
    if keep_top:
        qlo[12], qhi[12] = q[12], 0
        l[13], qlo[13], qhi[13] = v[13], 0, 0
        for k in (14, 15):
            l[k] = qlo[k] = qhi[k] = 0
    l = [_i32(_i32(a) + b + c) for a, b, c in zip(l, _shr(qlo, 1), _shr(qhi, 2))]
    c = [x >> 28 for x in l]
    l2 = [x & M28 for x in l]
    if keep_top:
        c[13] = 0
        l2[13] = l[13]
    l2 = [_i32(a + b) for a, b in zip(l2, _shr(c, 1))]
    if keep_top:
        l2[14] = l2[15] = 0
    return l2


def rp_mul(x, y):
    y = y[:14] + [0, 0]
    lo, hi = [0] * 16, [0] * 16
    for i in range(14):
        sl = _shr(y, i)
        sh = _shl(y, 16 - i) if i else [0] * 16
        lo = [a + x[i] * b for a, b in zip(lo, sl)]
        hi = [a + x[i] * b for a, b in zip(hi, sh)]
    t = norm(lo, False)
    t = [t[k] if k < 14 else 0 for k in range(16)]
    mc = [0] * 16
    for i in range(14):
        mc = [a + PPL[i] * b for a, b in zip(mc, _shr(t, i))]
    m = norm(mc, False)
    m = [m[k] if k < 14 else 0 for k in range(16)]
    for i in range(14):
        lo = [a + PL[i] * b for a, b in zip(lo, _shr(m, i))]
        hi = [a + PL[i] * b for a, b in zip(hi, _shl(m, 16 - i) if i else [0] * 16)]
    for v in lo + hi:
        assert -(1 << 63) <= v < (1 << 63)
    E = lo[13] + (lo[12] >> 28) + (lo[11] >> 56)
    C = (E + M28) >> 28
    w = [0] * 16
    w[14], w[15] = lo[14] + C, lo[15]
    r = [a + b for a, b in zip(_shl(w, 14), _shr(hi, 2))]
    return norm(r, True)


def lin(terms, reduce=True):
    """signed limb sum of (coef, limbs) terms, then the quotient-estimate reduction"""
    acc = [0] * 16
    for c, l in terms:
        acc = [a + c * x for a, x in zip(acc, l)]
    if not reduce:
        return norm(acc, True)
    w = float(acc[13]) * 268435456.0 + float(acc[12])
    q = int(math.floor(w * INV_P336))
    acc = [a - q * (PL[k] if k < 14 else 0) for k, a in enumerate(acc)]
    return norm(acc, True)


def to_row(x):
    """the R'-form limbs of a field element x (the value x 2^392 mod p, below p)"""
    return limbs(x * RP % P)


def from_row(l):
    return val(l) * pow(RP, -1, P) % P


# ------------------------------------------------------------ programs
class RowProg(G.Prog):
    """(A/B: ROW_PLAIN=1) every product operand one slot with coefficient 1: sums materialised by a
    linear task first.  Measured slower than operand sums inside the product phase (one phase
    more per operation), so the default keeps the wave programs' operand sums."""

    def mul(self, x, y):
        if os.environ.get("ROW_PLAIN") == "1":
            return super().mul(self.mat(x), self.mat(y))
        return super().mul(x, y)

    def mat(self, lin, force=False):
        """Linear tasks of the same stage are inlined into the sum instead of read as slots (one
        level, i.e. one phase and barrier, instead of a chain); tasks left unread are dropped by
        encode.  (A/B: ROW_NO_FLATTEN=1.)"""
        if os.environ.get("ROW_NO_FLATTEN") != "1":
            lin = self._flatten(lin)
        return super().mat(lin, force)

    def _flatten(self, lin):
        st = self._avail(lin)
        defs = {l[2]: l[3] for l in self.lins if l[0] == st}
        if not any(s in defs for s in lin.d):
            return lin
        out = G.Lin()
        for s, c in lin.d.items():
            out = out + (defs[s].scale(c) if s in defs else G.Lin({s: c}))
        if len(out.d) > G.MAXL or sum(abs(c) for c in out.d.values()) > 64:
            return lin
        return out


def f4sqr(t, a0, a1):
    """(a0 + a1 s)^2 in Fp4 = Fp2[s]/(s^2 - xi): (a0^2 + xi a1^2, (a0 + a1)^2 - a0^2 - a1^2)"""
    t0 = t.f2sqr(a0)
    t1 = t.f2sqr(a1)
    r0 = t.f2add(t.f2xi(t1), t0)
    r1 = t.f2sub(t.f2sub(t.f2sqr(t.f2add(a0, a1)), t0), t1)
    return r0, r1


def cyclotomic_sqr(t, a):
    """Granger-Scott squaring of an element of the cyclotomic subgroup (the final exponentiation's
    hard part): three Fp4 squarings, 18 Fp products in one phase instead of SQR12's 36"""
    (a00, a01, a02), (a10, a11, a12) = a
    t0 = f4sqr(t, a00, a11)
    t1 = f4sqr(t, a10, a02)
    t2 = f4sqr(t, a01, a12)

    def lin3m2(x, y, sign):  # 3 x -/+ 2 y
        return (x[0].scale(3) + y[0].scale(2 * sign), x[1].scale(3) + y[1].scale(2 * sign))
    r00 = lin3m2(t0[0], a00, -1)
    r01 = lin3m2(t1[0], a01, -1)
    r02 = lin3m2(t2[0], a02, -1)
    r10 = lin3m2(t.f2xi(t2[1]), a10, 1)
    r11 = lin3m2(t0[1], a11, 1)
    r12 = lin3m2(t1[1], a12, 1)
    return (r00, r01, r02), (r10, r11, r12)


# extra constant slots of the row engine (after the wave programs' 19): psi's coefficients
C_PSI_CX, C_PSI_CY, C_PSI2_CX, C_PSI2_CY = 19, 21, 23, 24
N_CONST_ROW = 25


def g2_in(pg, base):
    return tuple((pg.inp(base + 2 * k), pg.inp(base + 2 * k + 1)) for k in range(3))


def g2_dbl(t, P):
    """2P, dbl-2009-l (as lb_curve.h jac_dbl_i / lb_group.h g8_dbl): 16 products in 3 levels"""
    X, Y, Z = P
    A = t.f2sqr(X)
    B = t.f2sqr(Y)
    YZ = t.f2mul(Y, Z)
    C = t.f2sqr(B)
    D = t.f2dbl(t.f2sub(t.f2sub(t.f2sqr(t.f2add(X, B)), A), C))
    E = t.f2mul3(A)
    F = t.f2sqr(E)
    X3 = t.f2sub(F, t.f2dbl(D))
    C8 = (C[0].scale(8), C[1].scale(8))
    Y3 = t.f2sub(t.f2mul(E, t.f2sub(D, X3)), C8)
    return X3, Y3, t.f2dbl(YZ)


def g2_add(t, P, Q):
    """P + Q, add-2007-bl (as jac_add_i without its exceptional cases; H and r are outputs so the
    caller can detect them): 43 products"""
    X1, Y1, Z1 = P
    X2, Y2, Z2 = Q
    Z1Z1 = t.f2sqr(Z1)
    Z2Z2 = t.f2sqr(Z2)
    U1 = t.f2mul(X1, Z2Z2)
    U2 = t.f2mul(X2, Z1Z1)
    S1 = t.f2mul(t.f2mul(Y1, Z2), Z2Z2)
    S2 = t.f2mul(t.f2mul(Y2, Z1), Z1Z1)
    H = t.f2sub(U2, U1)
    I = t.f2sqr(t.f2dbl(H))
    J = t.f2mul(H, I)
    r = t.f2dbl(t.f2sub(S2, S1))
    V = t.f2mul(U1, I)
    X3 = t.f2sub(t.f2sub(t.f2sqr(r), J), t.f2dbl(V))
    Y3 = t.f2sub(t.f2mul(r, t.f2sub(V, X3)), t.f2dbl(t.f2mul(S1, J)))
    Z3 = t.f2mul(t.f2sub(t.f2sub(t.f2sqr(t.f2add(Z1, Z2)), Z1Z1), Z2Z2), H)
    return (X3, Y3, Z3), H, r


# ---- homogeneous projective G2 (x = X / Z, y = Y / Z), the complete a = 0 formulas of Renes,
# Costello and Batina (2016; Algorithms 7 and 9).  E'(Fp2) has odd order (no 2-torsion), so
# they have no exceptional case: the identity is (0 : Y : 0), P = Q and P = -Q need no tests.
# On the row engine a phase costs ~1 us against a product's 0.45 us, so what counts is product
# LEVELS: the doubling needs 2 (Jacobian dbl-2009-l: 3), the addition 2 (add-2007-bl: 6).
def f2b3(t, a):
    """b3 a with b3 = 3 b = 12 (1 + u) on E': y^2 = x^3 + 4 (1 + u): linear"""
    x = t.f2xi(a)
    return (x[0].scale(12), x[1].scale(12))


def g2_pdbl(t, P):
    """2P, RCB Algorithm 9: products Y^2, YZ, Z^2, XY, then 4 products of level 2"""
    X, Y, Z = P
    t0 = t.f2sqr(Y)
    t1 = t.f2mul(Y, Z)
    t2 = f2b3(t, t.f2sqr(Z))
    z8 = (t0[0].scale(8), t0[1].scale(8))
    x3a = t.f2mul(t2, z8)
    y3s = t.f2add(t0, t2)
    Z3 = t.f2mul(t1, z8)
    t0m = t.f2sub(t0, t.f2mul3(t2))
    Y3 = t.f2add(x3a, t.f2mul(t0m, y3s))
    X3 = t.f2dbl(t.f2mul(t0m, t.f2mul(X, Y)))
    return X3, Y3, Z3


def g2_padd(t, P, Q):
    """P + Q, RCB Algorithm 7 (complete): 6 products, then 6 products"""
    X1, Y1, Z1 = P
    X2, Y2, Z2 = Q
    t0 = t.f2mul(X1, X2)
    t1 = t.f2mul(Y1, Y2)
    t2 = t.f2mul(Z1, Z2)
    t3 = t.f2sub(t.f2mul(t.f2add(X1, Y1), t.f2add(X2, Y2)), t.f2add(t0, t1))
    t4 = t.f2sub(t.f2mul(t.f2add(Y1, Z1), t.f2add(Y2, Z2)), t.f2add(t1, t2))
    sxz = t.f2sub(t.f2mul(t.f2add(X1, Z1), t.f2add(X2, Z2)), t.f2add(t0, t2))
    t0x3 = t.f2mul3(t0)
    t2b = f2b3(t, t2)
    z3a = t.f2add(t1, t2b)
    t1m = t.f2sub(t1, t2b)
    y3b = f2b3(t, sxz)
    X3 = t.f2sub(t.f2mul(t3, t1m), t.f2mul(t4, y3b))
    Y3 = t.f2add(t.f2mul(t1m, z3a), t.f2mul(y3b, t0x3))
    Z3 = t.f2add(t.f2mul(z3a, t4), t.f2mul(t0x3, t3))
    return X3, Y3, Z3


def g2_jtop(t, P):
    """Jacobian (X, Y, Z) -> projective (X Z, Y, Z^3)"""
    X, Y, Z = P
    return t.f2mul(X, Z), Y, t.f2mul(t.f2sqr(Z), Z)


def g2_ptoj(t, P):
    """projective (X, Y, Z) -> Jacobian (X Z, Y Z^2, Z)"""
    X, Y, Z = P
    return t.f2mul(X, Z), t.f2mul(Y, t.f2sqr(Z)), Z


def g2_peqn(t, A, B):
    """(X1 Z2 - X2 Z1, Y1 Z2 + Y2 Z1): both zero iff A = -B for finite A (B = O gives Y2 Z1)"""
    X1, Y1, Z1 = A
    X2, Y2, Z2 = B
    return t.f2sub(t.f2mul(X1, Z2), t.f2mul(X2, Z1)), t.f2add(t.f2mul(Y1, Z2), t.f2mul(Y2, Z1))


def g2_psi(t, pg, P):
    X, Y, Z = P
    cx = (pg.const(C_PSI_CX), pg.const(C_PSI_CX + 1))
    cy = (pg.const(C_PSI_CY), pg.const(C_PSI_CY + 1))
    return t.f2mul(t.f2conj(X), cx), t.f2mul(t.f2conj(Y), cy), t.f2conj(Z)


def g2_psi2(t, pg, P):
    X, Y, Z = P
    return t.f2mulfp(X, pg.const(C_PSI2_CX)), t.f2mulfp(Y, pg.const(C_PSI2_CY)), Z


def g2_flat(P):
    return [c for x in P for c in x]


def build_programs():
    """the wave programs' formulas (tools/gen_wave_programs.py build_programs) traced into
    RowProg, plus CSQR12 and the G2 point programs (G2DBL, G2ADD, PSI, PSI2) of the row engine's
    cofactor clearing (lb_row.h r_g2_*)"""
    saved = G.Prog
    G.Prog = RowProg
    try:
        progs = G.build_programs()
        pg = RowProg("CSQR12")
        t = G.T(pg)
        pg.output(G.fp12_flat(cyclotomic_sqr(t, G.fp12_in(pg, 0))))
        progs["CSQR12"] = pg
        # two chained cyclotomic squarings, the first's outputs never materialised (3 barriers
        # instead of 2 x 2 plus a move out and back in)
        pg = RowProg("CSQR12X2")
        t = G.T(pg)
        pg.output(G.fp12_flat(cyclotomic_sqr(t, cyclotomic_sqr(t, G.fp12_in(pg, 0)))))
        progs["CSQR12X2"] = pg
        pg = RowProg("G2DBL")
        t = G.T(pg)
        pg.output(g2_flat(g2_dbl(t, g2_in(pg, 0))))
        progs["G2DBL"] = pg
        pg = RowProg("G2ADD")
        t = G.T(pg)
        R, H, r = g2_add(t, g2_in(pg, 0), g2_in(pg, 6))
        pg.output(g2_flat(R) + list(H) + list(r))
        progs["G2ADD"] = pg
        pg = RowProg("PSI")
        t = G.T(pg)
        pg.output(g2_flat(g2_psi(t, pg, g2_in(pg, 0))))
        progs["PSI"] = pg
        pg = RowProg("PSI2")
        t = G.T(pg)
        pg.output(g2_flat(g2_psi2(t, pg, g2_in(pg, 0))))
        progs["PSI2"] = pg
        for k in (2, 4):  # k chained doublings, intermediate points never materialised
            pg = RowProg("G2DBL%d" % k)
            t = G.T(pg)
            P = g2_in(pg, 0)
            for _ in range(k):
                P = g2_dbl(t, P)
            pg.output(g2_flat(P))
            progs["G2DBL%d" % k] = pg
        # round 6: projective (complete) point programs
        for k in (1, 2, 4):
            pg = RowProg("PDBL%d" % k)
            t = G.T(pg)
            P = g2_in(pg, 0)
            for _ in range(k):
                P = g2_pdbl(t, P)
            pg.output(g2_flat(P))
            progs["PDBL%d" % k] = pg
        pg = RowProg("PADD")
        t = G.T(pg)
        pg.output(g2_flat(g2_padd(t, g2_in(pg, 0), g2_in(pg, 6))))
        progs["PADD"] = pg
        pg = RowProg("JTOP")
        t = G.T(pg)
        pg.output(g2_flat(g2_jtop(t, g2_in(pg, 0))))
        progs["JTOP"] = pg
        pg = RowProg("PTOJ")
        t = G.T(pg)
        pg.output(g2_flat(g2_ptoj(t, g2_in(pg, 0))))
        progs["PTOJ"] = pg
        pg = RowProg("PEQN")
        t = G.T(pg)
        e1, e2 = g2_peqn(t, g2_in(pg, 0), g2_in(pg, 6))
        pg.output(list(e1) + list(e2))
        progs["PEQN"] = pg
    finally:
        G.Prog = saved
    return progs


# ------------------------------------------------------------ encoding
class RowCode:
    def __init__(self, words, n_prods, n_lins, n_phases, ntemp):
        self.words, self.n_prods, self.n_lins, self.n_phases, self.ntemp = words, n_prods, n_lins, n_phases, ntemp


LBR_NROWS = 64  # lb_row.h: 4 rows per wave, LBR_WAVES 16
ZERO_SLOT = G.CONST_BASE + G.C_ZERO


def _pair(slot, coef):
    assert 0 <= slot < 32768 and -32768 <= coef < 32768
    return (slot & 0xFFFF) | ((coef & 0xFFFF) << 16)


def _live_lins(pg):
    """the linear tasks whose result is read (by a product, a live task or as an output)"""
    live = list(pg.lins)
    while True:
        used = set(pg.outs)
        for p in pg.prods:
            used |= set(p[2].d) | set(p[3].d)
        for l in live:
            used |= set(l[3].d)
        keep = [l for l in live if l[2] in used]
        if len(keep) == len(live):
            return keep
        live = keep


def encode(pg):
    pg.lins = _live_lins(pg)
    nst = max([p[0] for p in pg.prods] + [l[0] for l in pg.lins] + [0])
    # A level-0 linear task of stage s that neither a product of stage s + 1 nor another linear
    # task of stage s reads (typically an output) is deferred into stage s + 1's product phase:
    # it runs on the rows after the products' (header word 1: row offset) with no barrier between
    # (product phase flag 16), one phase and barrier fewer.
    def reads(lin, slot):
        return slot in lin.d
    deferred = {}
    if os.environ.get("ROW_NO_DEFER") != "1":
        for s in range(nst):
            nxt = [p for p in pg.prods if p[0] == s + 1]
            if not nxt:
                continue
            same = [l for l in pg.lins if l[0] == s]
            deferred[s + 1] = [l for l in same if l[1] == 0
                               and not any(reads(p[2], l[2]) or reads(p[3], l[2]) for p in nxt)
                               and not any(reads(o[3], l[2]) for o in same)]
    moved = {id(l) for ls in deferred.values() for l in ls}
    phases = []
    for s in range(nst + 1):
        pr = [p for p in pg.prods if p[0] == s]
        if pr:
            dl = deferred.get(s, [])
            phases.append((0, pr, bool(dl)))
            if dl:
                roff = 4 * ((len(pr) + 3) // 4)
                phases.append((1, dl, roff if roff < LBR_NROWS else 0))
        for v in sorted({l[1] for l in pg.lins if l[0] == s and id(l) not in moved}):
            phases.append((1, [l for l in pg.lins if l[0] == s and l[1] == v and id(l) not in moved], 0))
    out = [len(phases), len(pg.outs)] + list(pg.outs)

    def pad4(n):
        return (n + 3) // 4 * 4

    def pairs(lin, width):
        ps = [_pair(s, c) for s, c in sorted(lin.d.items())]
        assert len(ps) <= width
        return ps + [_pair(ZERO_SLOT, 0)] * (width - len(ps))

    def plain(lins):
        return all(len(l.d) == 1 and list(l.d.values())[0] == 1 for l in lins)

    def reduce(lins):
        # an operand of slot values |v| < 2p with sum |c| <= 16 stays below 32 p < 2^386: its
        # product is below 1.4 p without the quotient reduction (only the limb carries run)
        return any(sum(abs(c) for c in l.d.values()) > 16 for l in lins)

    for kind, tasks, arg in phases:
        if kind == 0:
            xs, ys = [t[2] for t in tasks], [t[3] for t in tasks]
            nx, ny = max(len(x.d) for x in xs), max(len(y.d) for y in ys)
            # operand sums are read in blocks of 4 terms (lb_row.h r_acc4): pad to whole blocks
            # with zero-coefficient pairs, so the interpreter needs no per-term mask
            nx = nx if plain(xs) else pad4(nx)
            ny = ny if plain(ys) else pad4(ny)
            flags = (1 if plain(xs) else 0) | (2 if plain(ys) else 0)
            flags |= (4 if reduce(xs) else 0) | (8 if reduce(ys) else 0)
            flags |= 16 if arg else 0
            out += [kind | (flags << 8) | (len(tasks) << 16), nx | (ny << 16)]
            for t in tasks:
                out += [t[1]] + pairs(t[2], nx) + pairs(t[3], ny)
        else:
            ls = [t[3] for t in tasks]
            nx = pad4(max(len(l.d) for l in ls))
            out += [kind | (len(tasks) << 16), nx | (arg << 16)]
            for t in tasks:
                out += [t[2]] + pairs(t[3], nx)
    code = RowCode(out, len(pg.prods), len(pg.lins), len(phases), pg.ntemp)
    code.n_barriers = sum(1 for k, _, a in phases if not (k == 0 and a))
    return code


def run_row(words, slots):
    """Interpret a row program over slot -> limbs with exactly lb_row.h's arithmetic."""
    n_ph, n_out = words[0], words[1]
    outs = words[2:2 + n_out]
    pos = 2 + n_out
    S = dict(slots)

    def operand(ps, is_plain, red=True):
        terms = []
        for w in ps:
            slot, coef = w & 0xFFFF, (w >> 16) - ((w >> 16) & 0x8000) * 2
            terms.append((coef, S[slot]))
        if is_plain:
            assert len(terms) == 1 and terms[0][0] == 1
            return terms[0][1]
        return lin(terms, reduce=red)

    for _ in range(n_ph):
        h0, h1 = words[pos], words[pos + 1]
        pos += 2
        kind, flags, n = h0 & 0xFF, (h0 >> 8) & 0xFF, h0 >> 16
        nx, ny = h1 & 0xFFFF, h1 >> 16
        rs = 1 + nx + (ny if kind == 0 else 0)  # (a linear phase's ny: its row offset)
        new = {}
        for k in range(n):
            rec = words[pos + k * rs: pos + (k + 1) * rs]
            if kind == 0:
                x = operand(rec[1:1 + nx], flags & 1, flags & 4)
                y = operand(rec[1 + nx:1 + nx + ny], flags & 2, flags & 8)
                new[rec[0]] = rp_mul(x, y)
            else:
                new[rec[0]] = operand(rec[1:1 + nx], False)
        for v in new.values():
            assert abs(val(v)) < 2 * P, "slot bound"
        S.update(new)
        pos += n * rs
    return [S[o] for o in outs]


def consts_values():
    """the CONST slots as field elements (same order as lb_wave.h w_init_consts, then psi's)"""
    sys.path.insert(0, ROOT)
    from oracle import bls_oracle as o
    c = [0] * N_CONST_ROW
    xi = (1, 1)
    cx = o.PSI_CX
    cy = o.PSI_CY
    c[C_PSI_CX], c[C_PSI_CX + 1] = cx
    c[C_PSI_CY], c[C_PSI_CY + 1] = cy
    c[C_PSI2_CX] = o.f2_mul(cx, o.f2_conj(cx))[0]
    c[C_PSI2_CY] = o.f2_mul(cy, o.f2_conj(cy))[0]
    c[G.C_B3], c[G.C_B3 + 1] = 12, 12
    c[G.C_INV2] = pow(2, P - 2, P)
    for k in range(1, 6):
        g = o.f2_pow(xi, k * (P - 1) // 6)
        c[G.C_FROB1 + 2 * (k - 1)], c[G.C_FROB1 + 2 * (k - 1) + 1] = g
        c[G.C_FROB2 + k - 1] = o.f2_pow(xi, k * (P * P - 1) // 6)[0]
    c[G.C_ZERO] = 0
    return c


def _checks(codes):
    sys.path.insert(0, ROOT)
    from oracle import bls_oracle as o
    rnd = random.Random(11)
    cv = consts_values()
    base = {G.CONST_BASE + k: to_row(v) for k, v in enumerate(cv)}

    def f12(v):
        c = [(v[0], v[1]), (v[6], v[7]), (v[2], v[3]), (v[8], v[9]), (v[4], v[5]), (v[10], v[11])]
        return o.f12_from_f2_coeffs(c)

    for _ in range(2):
        a = [rnd.randrange(P) for _ in range(12)]
        b = [rnd.randrange(P) for _ in range(12)]
        S = dict(base)
        S.update({G.IN_BASE + k: to_row(a[k]) for k in range(12)})
        S.update({G.IN_BASE + 12 + k: to_row(b[k]) for k in range(12)})
        got = [from_row(v) for v in run_row(codes["MUL12"].words, S)]
        assert f12(got) == o.f12_mul(f12(a), f12(b)), "MUL12"
        got = [from_row(v) for v in run_row(codes["SQR12"].words, S)]
        assert f12(got) == o.f12_sqr(f12(a)), "SQR12"
        got = [from_row(v) for v in run_row(codes["FROB"].words, S)]
        assert f12(got) == o.f12_pow(f12(a), P), "FROB"
        got = [from_row(v) for v in run_row(codes["FROB2"].words, S)]
        assert f12(got) == o.f12_pow(f12(a), P * P), "FROB2"
    # CSQR12 on an element of the cyclotomic subgroup: f^((p^6 - 1)(p^2 + 1))
    for _ in range(2):
        a = [rnd.randrange(P) for _ in range(12)]
        fa = f12(a)
        g = o.f12_mul(o.f12_conj(fa), o.f12_inv(fa))
        g = o.f12_mul(o.f12_pow(g, P * P), g)
        flat = [e for six in g for two in six for e in two]  # tower order
        assert f12(flat) == g
        S = dict(base)
        S.update({G.IN_BASE + k: to_row(flat[k]) for k in range(12)})
        got = [from_row(v) for v in run_row(codes["CSQR12"].words, S)]
        assert f12(got) == o.f12_sqr(g), "CSQR12"
        got = [from_row(v) for v in run_row(codes["CSQR12X2"].words, S)]
        assert f12(got) == o.f12_sqr(o.f12_sqr(g)), "CSQR12X2"
    # G2 point programs against the oracle's group law (affine results)
    def g2_row_in(Pa):
        (x0, x1), (y0, y1) = Pa
        z = (rnd.randrange(1, P), rnd.randrange(P))  # a random Jacobian representative
        z2 = o.f2_sqr(z)
        X, Y = o.f2_mul(Pa[0], z2), o.f2_mul(Pa[1], o.f2_mul(z2, z))
        return [X[0], X[1], Y[0], Y[1], z[0], z[1]]

    def g2_row_out(v):
        X, Y, Z = (v[0], v[1]), (v[2], v[3]), (v[4], v[5])
        zi = o.f2_inv(Z)
        zi2 = o.f2_sqr(zi)
        return (o.f2_mul(X, zi2), o.f2_mul(Y, o.f2_mul(zi2, zi)))
    for k in range(2):
        Pa = o.hash_to_g2(bytes([k, 1]) * 16)
        Qa = o.hash_to_g2(bytes([k, 2]) * 16)
        S = dict(base)
        S.update({G.IN_BASE + j: to_row(v) for j, v in enumerate(g2_row_in(Pa) + g2_row_in(Qa))})
        got = [from_row(v) for v in run_row(codes["G2DBL"].words, S)]
        assert g2_row_out(got) == o.g2_add(Pa, Pa), "G2DBL"
        got = [from_row(v) for v in run_row(codes["G2ADD"].words, S)]
        assert g2_row_out(got[:6]) == o.g2_add(Pa, Qa), "G2ADD"
        got = [from_row(v) for v in run_row(codes["PSI"].words, S)]
        assert g2_row_out(got) == o.g2_psi(Pa), "PSI"
        got = [from_row(v) for v in run_row(codes["PSI2"].words, S)]
        assert g2_row_out(got) == o.g2_psi(o.g2_psi(Pa)), "PSI2"
        got = [from_row(v) for v in run_row(codes["G2DBL4"].words, S)]
        assert g2_row_out(got) == o.g2_mul(Pa, 16), "G2DBL4"
        got = [from_row(v) for v in run_row(codes["G2DBL2"].words, S)]
        assert g2_row_out(got) == o.g2_mul(Pa, 4), "G2DBL2"
    # projective programs: random representatives (x z, y z, z), results read as (X / Z, Y / Z)
    def p_in(Pa):
        z = (rnd.randrange(1, P), rnd.randrange(P))
        return [c for v in (o.f2_mul(Pa[0], z), o.f2_mul(Pa[1], z), z) for c in v]

    def p_out(v):
        X, Y, Z = (v[0], v[1]), (v[2], v[3]), (v[4], v[5])
        if Z == (0, 0):
            return None
        zi = o.f2_inv(Z)
        return (o.f2_mul(X, zi), o.f2_mul(Y, zi))
    for k in range(2):
        Pa = o.hash_to_g2(bytes([k, 3]) * 16)
        Qa = o.hash_to_g2(bytes([k, 4]) * 16)
        for a, b, want in ((Pa, Qa, o.g2_add(Pa, Qa)), (Pa, Pa, o.g2_add(Pa, Pa)), (Pa, o.g2_neg(Pa), None)):
            S = dict(base)
            S.update({G.IN_BASE + j: to_row(v) for j, v in enumerate(p_in(a) + p_in(b))})
            got = [from_row(v) for v in run_row(codes["PADD"].words, S)]
            assert p_out(got) == want, "PADD"
        S = dict(base)
        S.update({G.IN_BASE + j: to_row(v) for j, v in enumerate(p_in(Pa) + p_in(Qa))})
        got = [from_row(v) for v in run_row(codes["PDBL1"].words, S)]
        assert p_out(got) == o.g2_add(Pa, Pa), "PDBL1"
        got = [from_row(v) for v in run_row(codes["PDBL2"].words, S)]
        assert p_out(got) == o.g2_mul(Pa, 4), "PDBL2"
        got = [from_row(v) for v in run_row(codes["PDBL4"].words, S)]
        assert p_out(got) == o.g2_mul(Pa, 16), "PDBL4"
        got = [from_row(v) for v in run_row(codes["PTOJ"].words, S)]
        assert g2_row_out(got) == Pa, "PTOJ"
        got = [from_row(v) for v in run_row(codes["PSI"].words, S)]
        assert p_out(got) == o.g2_psi(Pa), "PSI (projective)"
        got = [from_row(v) for v in run_row(codes["PSI2"].words, S)]
        assert p_out(got) == o.g2_psi(o.g2_psi(Pa)), "PSI2 (projective)"
        S = dict(base)
        S.update({G.IN_BASE + j: to_row(v) for j, v in enumerate(g2_row_in(Pa))})
        got = [from_row(v) for v in run_row(codes["JTOP"].words, S)]
        assert p_out(got) == Pa, "JTOP"
        for b, zero in ((o.g2_neg(Pa), True), (Pa, False), (Qa, False)):
            S = dict(base)
            S.update({G.IN_BASE + j: to_row(v) for j, v in enumerate(p_in(Pa) + p_in(b))})
            got = [from_row(v) for v in run_row(codes["PEQN"].words, S)]
            assert (got == [0, 0, 0, 0]) == zero, "PEQN"
        # the identity (0 : 1 : 0) on either side of the complete addition and the doubling
        S = dict(base)
        S.update({G.IN_BASE + j: to_row(v) for j, v in enumerate(p_in(Pa) + [0, 0, 1, 0, 0, 0])})
        got = [from_row(v) for v in run_row(codes["PADD"].words, S)]
        assert p_out(got) == Pa, "PADD P + O"
        S = dict(base)
        S.update({G.IN_BASE + j: to_row(v) for j, v in enumerate([0, 0, 1, 0, 0, 0] + p_in(Pa))})
        got = [from_row(v) for v in run_row(codes["PADD"].words, S)]
        assert p_out(got) == Pa, "PADD O + P"
        got = [from_row(v) for v in run_row(codes["PDBL1"].words, S)]
        assert p_out(got) is None, "PDBL1 O"
    # a few Miller steps against the lone-lane programs' interpreter (values, not limbs)
    Pp = o.sk_to_pk(0x1234567)
    Qq = o.hash_to_g2(b"\x07" * 32)
    f = [rnd.randrange(P) for _ in range(12)]
    T = [Qq[0][0], Qq[0][1], Qq[1][0], Qq[1][1], 5, 7]
    for name, vals in (("DBL_STEP", f + T + [Pp[0], Pp[1]]),
                       ("ADD_STEP", f + T + [Qq[0][0], Qq[0][1], Qq[1][0], Qq[1][1], Pp[0], Pp[1]])):
        S = dict(base)
        S.update({G.IN_BASE + k: to_row(v) for k, v in enumerate(vals)})
        got = [from_row(v) for v in run_row(codes[name].words, S)]
        Sw = {G.CONST_BASE + k: v for k, v in enumerate(cv)}
        Sw.update({G.IN_BASE + k: v for k, v in enumerate(vals)})
        want = G.run_encoded(G.build_programs()[name].encode(), Sw)  # the wave programs' own values
        assert got == want, name


ORDER = ["MUL12", "SQR12", "CSQR12", "CSQR12X2", "FROB", "FROB2", "DBL_STEP", "ADD_STEP", "G2DBL", "G2ADD", "PSI", "PSI2", "G2DBL2", "G2DBL4",
         "PDBL1", "PDBL2", "PDBL4", "PADD", "JTOP", "PTOJ", "PEQN"]


def const_limbs(v):
    return limbs(v)[:14]


def render(check=True):
    progs = build_programs()
    codes = {k: encode(v) for k, v in progs.items()}
    if check:
        _checks(codes)
    lines = ["// Generated by tools/gen_row_programs.py -- do not edit.",
             "// Row-engine programs and constants (see the generator's docstring for the encoding).",
             "#pragma once", "#include <stdint.h>", "",
             f"#define LBR_IN {G.IN_BASE}", f"#define LBR_CONST {G.CONST_BASE}", f"#define LBR_TEMP {G.TEMP_BASE}",
             f"#define LBR_C_B3 {G.C_B3}", f"#define LBR_C_INV2 {G.C_INV2}", f"#define LBR_C_FROB1 {G.C_FROB1}",
             f"#define LBR_C_FROB2 {G.C_FROB2}", f"#define LBR_C_ZERO {G.C_ZERO}", f"#define LBR_N_CONST {N_CONST_ROW}",
             f"#define LBR_C_PSI_CX {C_PSI_CX}", f"#define LBR_C_PSI_CY {C_PSI_CY}", f"#define LBR_C_PSI2_CX {C_PSI2_CX}",
             f"#define LBR_C_PSI2_CY {C_PSI2_CY}",
             f"#define LBR_INV_P336 {INV_P336.hex()}  // 2^336 / p, nearest double"]
    image, maxtemp = [], 0
    for name in ORDER:
        c = codes[name]
        maxtemp = max(maxtemp, c.ntemp)
        lines.append(f"// {name}: {c.n_prods} products, {c.n_lins} linear tasks, {c.n_phases} phases, "
                     f"{c.ntemp} temps, offset {len(image)}")
        lines.append(f"#define LBR_{name} {len(image)}")
        image += c.words
        image += [0] * (-len(image) % 4)
        if name == "FROB2":
            lines.append(f"#define LBR_PROGS_FE {len(image)}")
        if name == "ADD_STEP":
            lines.append(f"#define LBR_PROGS_ALL {len(image)}")
    lines.append(f"#define LBR_PROGS_END {len(image)}")
    lines.append(f"#define LBR_MAX_TEMPS {maxtemp}")
    signed = [v - (1 << 32) if v >= (1 << 31) else v for v in image]
    lines.append(f"static __device__ const int32_t __attribute__((aligned(16))) LBR_PROGS[{len(image)}] = "
                 f"{{{', '.join(str(v) for v in signed)}}};")
    # constants: the CONST slots in row form, p, -p^-1 mod 2^392, and the conversion factors
    cv = consts_values()
    rows = [const_limbs(v * RP % P) for v in cv]
    lines.append(f"static __device__ const int32_t __attribute__((aligned(16))) LBR_CONST_LIMBS[{N_CONST_ROW}][16] = {{"
                 + ", ".join("{" + ", ".join(str(x) for x in r + [0, 0]) + "}" for r in rows) + "};")

    def arr(name, v, comment):
        lines.append(f"// {comment}")
        lines.append(f"#define {name} " + ", ".join(str(x) for x in const_limbs(v)))
    arr("LBR_P_LIMBS", P, "p")
    arr("LBR_PINV_LIMBS", PINV, "-p^-1 mod 2^392")
    arr("LBR_K_IMPORT", pow(2, 400, P), "2^400 mod p: rp_mul(x_R, K) = the row form of a 2^384-Montgomery value")
    arr("LBR_K_EXPORT", pow(2, 384, P), "2^384 mod p: rp_mul(x_row, K) = the 2^384-Montgomery value")
    arr("LBR_K_PLAIN", pow(2, 784, P), "2^784 mod p: rp_mul(x, K) = the row form of a plain integer")
    arr("LBR_ONE", RP % P, "1 in row form")
    return progs, codes, "\n".join(lines) + "\n"


def main():
    progs, codes, text = render()
    with open(OUT_PATH, "w") as fh:
        fh.write(text)
    for name in ORDER:
        c = codes[name]
        print(f"{name}: {c.n_prods} products, {c.n_phases} phases, {c.n_barriers} barriers, {len(c.words)} words")
    print("wrote", OUT_PATH)


if __name__ == "__main__":
    main()
