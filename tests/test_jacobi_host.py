"""The posdivsteps Jacobi symbol hash_to_G2's SSWU uses (lb_field.h fp_is_square_sg, wired in as
lb_kernels.h fp_is_square_i) equals the binary Jacobi algorithm (fp_is_square) bit for bit, and
settles within its jump budget.  Host build of the device header: no GPU needed."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_posdivsteps_jacobi_matches_binary(tmp_path):
    exe = tmp_path / "jacobi_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "lodestar_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "jacobi_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches: 0 / 12000 unsettled 0" in out.stdout
