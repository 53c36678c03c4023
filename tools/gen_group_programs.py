#!/usr/bin/env python3
"""Compiles the Miller-loop steps into *grouped* programs: G lanes of a wave run one pairing
instance, so a wave runs 64 / G instances (one per distinct signing root) side by side.

Output: lodestar_amd/csrc/lb_group_progs.h (generated; do not edit).

Why: one lane per root keeps the whole Miller state (f: 144 words, T: 72, P, Q) in registers
and calls an out-of-line Fp product ~6 700 times; every call spills the state (6.7 KB of
scratch per lane, the round-2 engine-cap abort), and a batch of ~7 000 roots runs on ~110
waves for ~12 ms.  The wave engine (lb_wave.h, one root per wave) has the opposite problem:
a Miller step's phases hold 2-47 products, so most of the 64 lanes idle.  Here the step is
traced with the same tower formulas as gen_wave_programs.py (same Karatsuba products, same
linear combinations), but each instance owns a small LDS slot array and the lanes of its group
take the phase's tasks G at a time: ~14 product passes per doubling step at G = 8 instead of
100 serial products, with no register-resident state at all.

Differences from the wave encoding (gen_wave_programs.py):
  * slots are per instance: the persistent state f (12), T (6), P (2), Q (4) lives in slots
    [0, 24); program temps are register-allocated on top (a slot is reused once its last
    reader's phase is done), so an instance needs NSLOT slots instead of 64 + 155;
  * constants live in one shared area per workgroup: a term's slot s < 0 reads constant -1 - s;
  * the outputs (new f and T) are written straight into the state slots when no later or
    same-phase task still reads the old value, else through a final copy phase;
  * records have a per-phase width (header word 6): [dst, 0, A pairs (npa + nna), B pairs
    (npb + nnb)] padded to a multiple of 8 int16 (a pair = one aligned dword: slot, coefficient),
    so the LDS image is ~3x smaller.
Phase header: [kind, n_tasks, npa, nna, npb, nnb, rec_size, 0]; program header [n_phases, 0...]
padded to 8.  A dst with OUT_FLAG is reduced below p (outputs); other temps stay in [0, 3p).
Validated here by interpreting the encoded programs with the device's arithmetic (the quotient
estimate of gen_wave_programs.run_encoded) through a whole Miller loop, checked against the
oracle pairing.
"""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_wave_programs as W  # noqa: E402

ROOT = W.ROOT
P = W.P
OUT_FLAG = W.OUT_FLAG
N_STATE = 24                 # f 0..11, T 12..17, P 18..19, Q 20..23
S_F, S_T, S_P, S_Q = 0, 12, 18, 20
OUT_PATH = os.path.join(ROOT, "lodestar_amd", "csrc", "lb_group_progs.h")


def phases_of(pg):
    """encode()'s phase order: per stage the product phase, then its linear levels."""
    nst = max([p[0] for p in pg.prods] + [l[0] for l in pg.lins] + [0])
    out = []
    for s in range(nst + 1):
        pr = [("P", p[1], p[2], p[3]) for p in pg.prods if p[0] == s]
        if pr:
            out.append(pr)
        for v in sorted({l[1] for l in pg.lins if l[0] == s}):
            out.append([("L", l[2], l[3], None) for l in pg.lins if l[0] == s and l[1] == v])
    return out


def encode_grouped(pg, out_state):
    """pg: a traced Prog whose inputs are the state slots (W.IN_BASE + k); out_state[i] = the
    state slot that program output i replaces.  Returns (code, n_slots)."""
    phases = phases_of(pg)
    is_temp = lambda s: s >= W.TEMP_BASE  # noqa: E731
    # reads per phase
    reads = []
    for ph in phases:
        r = set()
        for t in ph:
            for lin in (t[2], t[3]):
                if lin is not None:
                    r.update(lin.d)
        reads.append(r)
    last_use = {}
    for k, r in enumerate(reads):
        for s in r:
            last_use[s] = k
    def_phase = {}
    for k, ph in enumerate(phases):
        for t in ph:
            def_phase[t[1]] = k
    outs = list(pg.outs)
    assert len(outs) == len(out_state)
    # an output goes straight to its state slot unless a task of its phase or later reads that slot
    direct = {}
    copies = []
    for o, s in zip(outs, out_state):
        d = def_phase[o]
        assert o not in last_use, "output temps have no readers"
        if all(s not in reads[k] for k in range(d, len(phases))):
            direct[o] = s
        else:
            copies.append((o, s))
    # temp register allocation: slots [N_STATE, ...) reused after their last reader's phase
    slot_of = {}
    free = []
    n_slots = N_STATE
    expiring = {}
    for s, k in last_use.items():
        if is_temp(s):
            expiring.setdefault(k, []).append(s)
    for k, ph in enumerate(phases):
        for t in ph:
            dst = t[1]
            if dst in direct:
                continue
            if free:
                slot_of[dst] = free.pop()
            else:
                slot_of[dst] = n_slots
                n_slots += 1
        for s in expiring.get(k, []):
            if s in slot_of:
                free.append(slot_of[s])
        # temps never read (and not outputs) free at once
        for t in ph:
            dst = t[1]
            if dst not in last_use and dst not in direct and dst in slot_of and dst not in dict(copies):
                free.append(slot_of[dst])

    def loc(s):
        if s < W.CONST_BASE:
            assert s < N_STATE
            return s
        if s < W.TEMP_BASE:
            return -1 - (s - W.CONST_BASE)
        return direct.get(s, slot_of.get(s))

    copy_src = {o for o, _ in copies}
    code = [len(phases) + (1 if copies else 0)] + [0] * 7

    def split(lin):
        pos = [(loc(sl), c) for sl, c in lin.d.items() if c > 0]
        neg = [(loc(sl), -c) for sl, c in lin.d.items() if c < 0]
        assert all(c < 1 << 15 for _, c in pos + neg)
        return pos, neg

    def pairs(ops, np_, nn_):
        p, n = ops
        pad = (0, 0)  # coefficient 0 on slot 0
        return [v for k in range(np_) for v in (p[k] if k < len(p) else pad)] + \
               [v for k in range(nn_) for v in (n[k] if k < len(n) else pad)]

    for ph in phases:
        kind = 0 if ph[0][0] == "P" else 1
        if kind == 0:
            xs = [split(t[2]) for t in ph]
            ys = [split(t[3]) for t in ph]
            npa, nna = max(len(p) for p, _ in xs), max(len(n) for _, n in xs)
            npb, nnb = max(len(p) for p, _ in ys), max(len(n) for _, n in ys)
            rs = 2 + 2 * (npa + nna + npb + nnb)
        else:
            xs = [split(t[2]) for t in ph]
            npa, nna = max(len(p) for p, _ in xs), max(len(n) for _, n in xs)
            npb = nnb = 0
            rs = 2 + 2 * (npa + nna)
        rs += -rs % 8
        code += [kind, len(ph), npa, nna, npb, nnb, rs, 0]
        for i, t in enumerate(ph):
            dst = loc(t[1])
            if kind == 1 and (t[1] in direct or t[1] in copy_src):
                dst |= OUT_FLAG
            rec = [dst, 0] + pairs(xs[i], npa, nna) + (pairs(ys[i], npb, nnb) if kind == 0 else [])
            code += rec + [0] * (rs - len(rec))
    if copies:
        rs = 8
        code += [1, len(copies), 1, 0, 0, 0, rs, 0]
        for o, s in copies:
            code += [s | OUT_FLAG, 0, slot_of[o], 1] + [0] * 4
    for v in code:
        assert -32768 <= v < 32768
    return code, n_slots


def run_grouped(code, state, consts):
    """Interpret a grouped program the way lb_group_exec does (state: list of slot values)."""
    S = dict(enumerate(state))
    C = consts
    val = lambda s: S[s] if s >= 0 else C[-1 - s]  # noqa: E731
    nph = code[0]
    pos = 8

    def lin(rec, off, np_, nn_, full):
        pa = [(rec[off + 2 * k + 1], val(rec[off + 2 * k])) for k in range(np_)]
        na = [(rec[off + 2 * (np_ + k) + 1], val(rec[off + 2 * (np_ + k)])) for k in range(nn_)]
        v = sum(c * x for c, x in pa) - sum(c * x for c, x in na)
        r = v - (W.quotient_estimate(pa, na) - 1) * P
        assert 0 <= r < 3 * P, "quotient estimate"
        return r % P if full else r

    for _ in range(nph):
        kind, n, npa, nna, npb, nnb, rs, _z = code[pos:pos + 8]
        pos += 8
        new = {}
        for k in range(n):
            rec = code[pos + k * rs: pos + (k + 1) * rs]
            if kind == 0:
                x = lin(rec, 2, npa, nna, False)
                y = lin(rec, 2 + 2 * (npa + nna), npb, nnb, False)
                new[rec[0]] = x * y % P
            else:
                new[rec[0] & ~OUT_FLAG] = lin(rec, 2, npa, nna, bool(rec[0] & OUT_FLAG))
        S.update(new)
        pos += n * rs
    return [S[k] for k in range(N_STATE)]


def cost(code, g=8):
    """rough per-wave VALU instructions of one program at G lanes per instance (the model used to
    compare schedules: a product pass ~ one 14x28-bit Montgomery product + two reduced operands;
    a term costs 12 multiply-adds, padded to groups of four)"""
    pos, total = 8, 0
    for _ in range(code[0]):
        kind, n, npa, nna, npb, nnb, rs, _z = code[pos:pos + 8]
        pos += 8 + n * rs
        grp = lambda c: 48 * ((c + 3) // 4)  # noqa: E731
        passes = -(-n // g)
        if kind == 0:
            total += passes * (624 + 2 * 110 + grp(npa) + grp(nna) + grp(npb) + grp(nnb))
        else:
            total += passes * (110 + grp(npa) + grp(nna))
    return total


def miller_dbl_relaxed(t, T, xP, yP):
    """miller_dbl of gen_wave_programs (lb_pairing.h: the same T' and line values) traced without
    the intermediate materialisations that kept record coefficients <= 7: the grouped engine's
    linear combinations take 16-bit coefficients, so E = 12 xi(C), F = 3 E and the scalings by 2 and
    4 fold into the operands of the next products (fewer linear phases per step)."""
    X, Y, Z = T
    A = t.f2mul(X, Y)
    B = t.f2sqr(Y)
    C = t.f2sqr(Z)
    YZ2 = t.f2sqr(t.f2add(Y, Z))
    XX = t.f2sqr(X)
    xiC = t.f2xi(C)
    E = (xiC[0].scale(12), xiC[1].scale(12))
    F = (E[0].scale(3), E[1].scale(3))
    H = t.f2sub(YZ2, t.f2add(B, C))
    l0 = t.f2mat(t.f2sub(B, E))
    l2 = t.f2neg(t.f2mulfp((XX[0].scale(3), XX[1].scale(3)), xP))
    l3 = t.f2mulfp(H, yP)
    X3 = t.f2dbl(t.f2mul(A, t.f2sub(B, F)))
    E2 = t.f2sqr(E)
    Y3 = t.f2sub(t.f2sqr(t.f2add(B, F)), (E2[0].scale(12), E2[1].scale(12)))
    BH = t.f2mul(B, H)
    Z3 = (BH[0].scale(4), BH[1].scale(4))
    return (X3, Y3, Z3), (l0, l2, l3)


def miller_add_relaxed(t, T, Q, xP, yP):
    """miller_add (same values) with fewer materialisations, as miller_dbl_relaxed"""
    X, Y, Z = T
    xq, yq = Q
    theta = t.f2mat(t.f2sub(Y, t.f2mul(yq, Z)))
    lam = t.f2mat(t.f2sub(X, t.f2mul(xq, Z)))
    l0 = t.f2sub(t.f2mul(theta, xq), t.f2mul(lam, yq))
    l2 = t.f2neg(t.f2mulfp(theta, xP))
    l3 = t.f2mulfp(lam, yP)
    C = t.f2sqr(theta)
    D = t.f2mat(t.f2sqr(lam))
    E = t.f2mat(t.f2mul(lam, D))
    F = t.f2mul(Z, C)
    G = t.f2mat(t.f2mul(X, D))
    H = t.f2mat(t.f2sub(t.f2add(E, F), t.f2dbl(G)))
    X3 = t.f2mul(lam, H)
    Y3 = t.f2sub(t.f2mul(theta, t.f2sub(G, H)), t.f2mul(E, Y))
    Z3 = t.f2mul(Z, E)
    return (X3, Y3, Z3), (l0, l2, l3)


def build(relaxed=True):
    progs = {}
    # doubling step: f <- f^2 * l_{T,T}(P), T <- 2T
    pg = W.Prog("G_DBL")
    t = W.T(pg)
    f = W.fp12_in(pg, S_F)
    Tt = tuple((pg.inp(S_T + 2 * k), pg.inp(S_T + 2 * k + 1)) for k in range(3))
    xP, yP = pg.inp(S_P), pg.inp(S_P + 1)
    T2, (l0, l2, l3) = (miller_dbl_relaxed if relaxed else W.miller_dbl)(t, Tt, xP, yP)
    if not relaxed:
        l0, l2, l3 = t.f2mat(l0), t.f2mat(l2), t.f2mat(l3)
    f2 = t.f12mat(t.f12sqr(f))
    pg.output(W.fp12_flat(t.f12mulline(f2, l0, l2, l3)) + [c for x in T2 for c in x])
    progs["G_DBL"] = pg
    # addition step: f <- f * l_{T,Q}(P), T <- T + Q
    pg = W.Prog("G_ADD")
    t = W.T(pg)
    f = W.fp12_in(pg, S_F)
    Tt = tuple((pg.inp(S_T + 2 * k), pg.inp(S_T + 2 * k + 1)) for k in range(3))
    xP, yP = pg.inp(S_P), pg.inp(S_P + 1)
    Q = ((pg.inp(S_Q), pg.inp(S_Q + 1)), (pg.inp(S_Q + 2), pg.inp(S_Q + 3)))
    T2, (l0, l2, l3) = (miller_add_relaxed if relaxed else W.miller_add)(t, Tt, Q, xP, yP)
    l0, l2, l3 = t.f2mat(l0), t.f2mat(l2), t.f2mat(l3)
    pg.output(W.fp12_flat(t.f12mulline(f, l0, l2, l3)) + [c for x in T2 for c in x])
    progs["G_ADD"] = pg
    out_state = list(range(S_F, S_F + 12)) + list(range(S_T, S_T + 6))
    codes = {k: encode_grouped(v, out_state) for k, v in progs.items()}
    return progs, codes


def consts_list():
    c = [0] * W.N_CONST
    c[W.C_B3], c[W.C_B3 + 1] = 12, 12
    c[W.C_INV2] = pow(2, P - 2, P)
    return c


def check(codes):
    """a whole Miller loop through the grouped programs vs the oracle pairing"""
    sys.path.insert(0, ROOT)
    from oracle import bls_oracle as o
    consts = consts_list()
    for seed in (0x1234567, 0xBEEF):
        Pp = o.sk_to_pk(seed)
        Qq = o.hash_to_g2(bytes([seed & 0xFF]) * 32)
        st = [1] + [0] * 11 + [Qq[0][0], Qq[0][1], Qq[1][0], Qq[1][1], 1, 0] + [Pp[0], Pp[1]] + \
             [Qq[0][0], Qq[0][1], Qq[1][0], Qq[1][1]]
        xabs = 0xD201000000010000
        for i in range(62, -1, -1):
            st = run_grouped(codes["G_DBL"][0], st, consts)
            if (xabs >> i) & 1:
                st = run_grouped(codes["G_ADD"][0], st, consts)
        f = st[:12]
        c = [(f[0], f[1]), (f[6], f[7]), (f[2], f[3]), (f[8], f[9]), (f[4], f[5]), (f[10], f[11])]
        ml = o.f12_conj(o.f12_from_f2_coeffs(c))
        assert o.final_exponentiation(ml) == o.pairing(Pp, Qq), "grouped Miller programs"


def render():
    progs, codes = build()
    check(codes)
    image = []
    lines = ["// Generated by tools/gen_group_programs.py -- do not edit.",
             "// Grouped (G lanes per instance) Miller-step programs; see the generator's docstring.",
             "#pragma once", "#include <stdint.h>", "",
             f"#define LBG_N_STATE {N_STATE}",
             f"#define LBG_S_F {S_F}", f"#define LBG_S_T {S_T}", f"#define LBG_S_P {S_P}", f"#define LBG_S_Q {S_Q}"]
    nslot = 0
    maxp = maxl = 1
    for name in ("G_DBL", "G_ADD"):
        code = codes[name][0]
        pos = 8
        for _ in range(code[0]):
            kind, n, npa, nna, npb, nnb, rs, _z = code[pos:pos + 8]
            pos += 8 + n * rs
            if kind == 0:
                maxp = max(maxp, npa, nna, npb, nnb)
            else:
                maxl = max(maxl, npa, nna)
    lines.append(f"#define LBG_MAXP {maxp}  // most added / subtracted terms of a product operand")
    lines.append(f"#define LBG_MAXL {maxl}  // ... of a linear task")
    for name in ("G_DBL", "G_ADD"):
        code, ns = codes[name]
        pg = progs[name]
        nslot = max(nslot, ns)
        np_ = sum(1 for _ in pg.prods)
        lines.append(f"// {name}: {np_} products, {len(pg.lins)} linear tasks, {code[0]} phases, {ns} slots, "
                     f"{len(code)} int16, offset {len(image)}, modelled cost {cost(code)} VALU per wave")
        lines.append(f"#define LB{name} {len(image)}")
        image += code
    lines.append(f"#define LBG_NSLOT {nslot}")
    lines.append(f"#define LBG_IMAGE {len(image)}")
    body = ", ".join(str(v) for v in image)
    lines.append(f"static __device__ const int16_t __attribute__((aligned(16))) LBG_PROGS[{len(image)}] = {{{body}}};")
    return progs, codes, "\n".join(lines) + "\n"


def main():
    progs, codes, text = render()
    with open(OUT_PATH, "w") as fh:
        fh.write(text)
    for name, (code, ns) in codes.items():
        print(f"{name}: {code[0]} phases, {ns} slots, {len(code)} int16")
    print("wrote", OUT_PATH)


if __name__ == "__main__":
    main()
