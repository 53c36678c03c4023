"""The Node.js host side (N-API addon + JS IBlsVerifier, lodestar_amd/js) - run with the system node."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

NODE = shutil.which("node")
SCRIPT = os.path.join(ROOT, "tests", "js", "test_verifier.js")
ADDON = os.path.join(ROOT, "lodestar_amd", "napi", "lodestar_bls.node")


def _run(mode):
    if NODE is None:
        pytest.skip("node not installed")
    if not os.path.exists(ADDON):
        from lodestar_amd.build import build_napi
        build_napi(verbose=False)
    r = subprocess.run([NODE, SCRIPT, mode], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_js_policy_and_addon_cpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu variant")
    assert "js cpu ok" in _run("cpu")


@pytest.mark.gpu
def test_js_verifier_gpu():
    assert "js gpu ok" in _run("gpu")


KZG_SCRIPT = os.path.join(ROOT, "tests", "js", "test_kzg.js")


def _run_kzg(mode):
    if NODE is None:
        pytest.skip("node not installed")
    r = subprocess.run([NODE, KZG_SCRIPT, mode], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    import json
    lines = r.stdout.strip().splitlines()
    assert lines[-1] == f"js kzg {mode} ok", r.stdout
    return json.loads(lines[-2])


def test_js_kzg_field_work_matches_python():
    """lodestar_amd/js/kzg.js's BigInt field work equals lodestar_amd/kzg.py's (same transcript,
    same inverse NTT, same evaluation)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu variant")
    if not os.path.exists(ADDON):
        from lodestar_amd.build import build_napi
        build_napi(verbose=False)
    from lodestar_amd import kzg as K
    got = _run_kzg("cpu")
    R = K.BLS_MODULUS
    vals = []
    for i in range(4096):
        x = K.ROOTS_BRP[i]
        vals.append((5 + 3 * x + 11 * pow(x, 4095, R)) % R)
    rp, x = K.compute_challenges([vals], [b"\x11" * 48])
    assert int(got["r0"]) == rp[0] and int(got["x"]) == x
    assert int(got["y"]) == K.evaluate_coefficients(K.evaluations_to_coefficients(vals), 12345)


@pytest.mark.gpu
def test_js_kzg_gpu_matches_python(engine):
    """the JS ckzg surface's commitments and proof are byte-identical to lodestar_amd/kzg.py's"""
    from lodestar_amd import kzg as K
    got = _run_kzg("gpu")
    k = K.Kzg(engine)

    def blob(off):
        b = bytearray(K.BYTES_PER_BLOB)
        for i in range(4096):
            b[32 * i: 32 * i + 4] = (i + off).to_bytes(4, "big")
        return bytes(b)
    blobs = [blob(0), blob(7)]
    assert got["commitments"] == [k.blob_to_kzg_commitment(b).hex() for b in blobs]
    assert got["proof"] == k.compute_aggregate_kzg_proof(blobs).hex()
