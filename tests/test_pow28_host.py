"""The limb-resident exponentiation chain (lb_field.h fp_pow_const_28) equals the reference chain
(fp_pow_const_i<false>) on random inputs, 0 and 1, for the sqrt exponents (p+1)/4 and (p-3)/4.
Host build of the device header: no GPU needed."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_pow28_matches_reference_chain(tmp_path):
    exe = tmp_path / "pow28_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "lodestar_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "pow28_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches: 0 / 300" in out.stdout
