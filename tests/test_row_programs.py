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
