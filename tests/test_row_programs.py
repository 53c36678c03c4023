"""CPU checks of the row engine (lodestar_amd/csrc/lb_row.h) and the split build:
  * the exact model of the row Montgomery product and of the reduced limb sums
    (tools/gen_row_programs.py, the same operations as the device code) against big integers,
    including the bounds the device code relies on (int32 limbs, int64 columns);
  * every row program (MUL12, SQR12, CSQR12, FROB, FROB2, DBL_STEP, ADD_STEP) interpreted with that
    arithmetic against the oracle's tower / the wave programs' values, and the committed
    lb_row_progs.h equal to a fresh render;
  * lb_kdecl.h (the kernel declarations of the split build) in step with the kernel sources."""
import os
import random
import subprocess
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_row_product_model_against_big_integers():
    import gen_row_programs as R
    rnd = random.Random(3)
    for it in range(300):
        bits = rnd.choice([381, 383, 386])  # slot values, operand sums (<= 32 p), beyond
        a = rnd.randrange(-(1 << bits), 1 << bits)
        b = rnd.randrange(-(1 << bits), 1 << bits)
        r = R.rp_mul(R.limbs(a), R.limbs(b))
        v = R.val(r)
        assert (v - a * b * pow(R.RP, -1, R.P)) % R.P == 0
        assert all(-2 <= x < (1 << 28) + 3 for x in r[:13])
        if bits <= 386:
            assert abs(v) < 2 * R.P   # the slot invariant
    # reduced limb sums: any signed combination of slot values lands in [0, p) up to far below p
    for it in range(300):
        terms = [(rnd.randrange(-7, 8), R.limbs(rnd.randrange(-2 * R.P, 2 * R.P))) for _ in range(rnd.randrange(1, 24))]
        tot = sum(c * R.val(l) for c, l in terms)
        v = R.val(R.lin(terms))
        assert (v - tot) % R.P == 0 and -R.P // (1 << 20) <= v < R.P + R.P // (1 << 20)


def test_row_programs_render_and_header_in_step():
    import gen_row_programs as R
    _, _, text = R.render(check=True)
    with open(R.OUT_PATH) as f:
        assert f.read() == text, "lb_row_progs.h is stale: python tools/gen_row_programs.py"


def test_kernel_declarations_in_step():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_kdecls.py"), "check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_written_out_pdbl_and_csqr_on_the_row_model():
    """lb_row.h r_pdbl_fast / r_csqr_fast (the op lists' projective doubling and cyclotomic
    squaring without the interpreter) replayed with the row engine's exact arithmetic (carry-only
    operand sums where the device skips the reduction, quotient-estimate reductions elsewhere),
    chained as the ladders chain them, against the oracle."""
    import gen_row_programs as R
    import gen_pdbl_fast as D
    from oracle import bls_oracle as o
    assert D.check()
    with open(os.path.join(ROOT, "lodestar_amd", "csrc", "lb_pdbl_tab.h")) as f:
        assert f.read() == D.emit(), "lb_pdbl_tab.h is stale: python tools/gen_pdbl_fast.py"
    L1, L2, L3 = D.tables()

    def pdbl(s):  # s: 6 slots (limb lists) X.c0 X.c1 Y.c0 Y.c1 Z.c0 Z.c1
        Pv = [R.rp_mul(R.lin([(c, s[e]) for e, c in enumerate(a) if c], reduce=False),
                       R.lin([(c, s[e]) for e, c in enumerate(b) if c], reduce=False)) for a, b in L1]
        Qv = [R.rp_mul(R.lin([(c, Pv[e]) for e, c in enumerate(a) if c]),
                       R.lin([(c, Pv[e]) for e, c in enumerate(b) if c])) for a, b in L2]
        return [R.lin([(c, Qv[e]) for e, c in enumerate(c3) if c]) for c3 in L3]

    rnd = random.Random(9)
    A = o.hash_to_g2(bytes(range(32)))
    z = (rnd.randrange(1, o.P), rnd.randrange(o.P))
    P = (o.f2_mul(A[0], z), o.f2_mul(A[1], z), z)
    s = [R.to_row(v) for c in P for v in c]
    want = A
    for _ in range(70):  # a ladder's run of doublings on the carried slots
        s = pdbl(s)
        want = o.g2_add(want, want)
        assert all(-2 <= x < (1 << 28) + 3 for l in s for x in l[:13])
    X, Y, Z = [(R.from_row(s[2 * c]), R.from_row(s[2 * c + 1])) for c in range(3)]
    zi = o.f2_inv(Z)
    assert (o.f2_mul(X, zi), o.f2_mul(Y, zi)) == want

    # cyclotomic squaring: the pair / form tables of r_csqr_fast, written out here again
    def csqr(s):
        Pv = [None] * 18
        for row in range(18):
            q, j = divmod(row, 6)
            xs, ys = (0, 8) if q == 0 else ((6, 4) if q == 1 else (2, 10))
            x0, x1, y0, y1 = s[xs], s[xs + 1], s[ys], s[ys + 1]
            cx = [(1, 1, 0, 0), (1, 0, 0, 0), (0, 0, 1, 1), (0, 0, 1, 0), (1, 1, 1, 1), (1, 0, 1, 0)][j]
            cy = [(1, -1, 0, 0), (0, 1, 0, 0), (0, 0, 1, -1), (0, 0, 0, 1), (1, -1, 1, -1), (0, 1, 0, 1)][j]
            v = (x0, x1, y0, y1)
            Pv[row] = R.rp_mul(R.lin([(c, v[e]) for e, c in enumerate(cx) if c], reduce=False),
                               R.lin([(c, v[e]) for e, c in enumerate(cy) if c], reduce=False))
        forms = [(3, 0, 3, -6, 0, 0, -2), (0, 6, 3, 6, 0, 0, -2), (-3, 0, -3, 0, 3, 0, 2),
                 (0, -6, 0, -6, 0, 6, 2), (-3, 6, -3, 6, 3, -6, 2), (-3, -6, -3, -6, 3, 6, 2)]
        out = []
        for row in range(12):
            q = 0 if row in (0, 1, 8, 9) else (1 if row in (2, 3, 10, 11) else 2)
            f = (row & 1) if row < 6 else (4 + (row & 1) if row < 8 else 2 + (row & 1))
            c = forms[f]
            out.append(R.lin([(c[e], Pv[6 * q + e]) for e in range(6) if c[e]] + [(c[6], s[row])]))
        return out

    # an element of the cyclotomic subgroup: f^((p^6 - 1)(p^2 + 1)) of a Miller value
    f = o.miller_loop(o.G1, A)
    g = o.f12_mul(o.f12_conj(f), o.f12_inv(f))
    g = o.f12_mul(o.f12_pow(g, o.P * o.P), g)
    flat = lambda a: [c for h in a for x in h for c in x]
    s = [R.to_row(v) for v in flat(g)]
    want = g
    for _ in range(6):
        s = csqr(s)
        want = o.f12_sqr(want)
    assert [R.from_row(l) for l in s] == flat(want)


def test_written_out_mul12_on_the_row_model():
    """lb_row.h r_mul12_fast (tools/gen_mul12_fast.py tables: 54 Karatsuba products, carry-only
    operand sums, reduced outputs) on the row engine's exact arithmetic, chained, against the
    oracle's Fp12 product; the committed lb_mul12_tab.h equal to a fresh render."""
    import gen_row_programs as R
    import gen_mul12_fast as M
    from oracle import bls_oracle as o
    assert M.check()
    with open(os.path.join(ROOT, "lodestar_amd", "csrc", "lb_mul12_tab.h")) as f:
        assert f.read() == M.emit(), "lb_mul12_tab.h is stale: python tools/gen_mul12_fast.py"
    prods, flat = M.tables()

    def mul(sa, sb):
        vin = sa + sb
        pv = [R.rp_mul(R.lin([(c, vin[k]) for k, c in x.items()], reduce=False),
                       R.lin([(c, vin[k]) for k, c in y.items()], reduce=False)) for x, y in prods]
        return [R.lin([(c, pv[k]) for k, c in f.items()]) for f in flat]

    rnd = random.Random(12)
    tw = lambda v: tuple(tuple((v[6 * h + 2 * j], v[6 * h + 2 * j + 1]) for j in range(3)) for h in range(2))
    flatf = lambda a: [c for h in a for x in h for c in x]
    a = [rnd.randrange(o.P) for _ in range(12)]
    acc, want = [R.to_row(v) for v in a], tw(a)
    for _ in range(5):
        b = [rnd.randrange(o.P) for _ in range(12)]
        acc = mul(acc, [R.to_row(v) for v in b])
        want = o.f12_mul(want, tw(b))
        assert all(-2 <= x < (1 << 28) + 3 for l in acc for x in l[:13])
    assert [R.from_row(l) for l in acc] == flatf(want)


def test_compiled_miller_steps_on_the_row_model():
    """lb_row.h rc_miller_step's compiled DBL_STEP / ADD_STEP (tools/gen_row_compiled.py: the
    interpreter's phases decoded into per-row records, one task per row) replayed on the row
    arithmetic against the interpreter's own replay; lb_row_compiled.h equal to a fresh render."""
    import gen_row_compiled as C
    assert C.check()
    with open(os.path.join(ROOT, "lodestar_amd", "csrc", "lb_row_compiled.h")) as f:
        assert f.read() == C.emit(), "lb_row_compiled.h is stale: python tools/gen_row_compiled.py"
