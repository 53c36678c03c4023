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


SR_SCRIPT = os.path.join(ROOT, "tests", "js", "test_signing_roots.js")


def _ops_file(tmp_path):
    import json
    from conftest import load_json
    from test_signing_roots import _operations_block
    p = tmp_path / "ops_block.json"
    p.write_text(json.dumps(_operations_block(load_json("k3_devnet.json"))))
    return str(p)


def _python_ops_roots(ops_path):
    import json
    from conftest import load_json
    from lodestar_amd import signing_roots as SR
    from test_signing_roots import cpu_merkleize, k3_state
    blk = json.loads(open(ops_path).read())
    sets = SR.resolve(SR.block_signature_sets(blk, k3_state(load_json("k3_devnet.json"))), cpu_merkleize)
    return [{"name": s.name, "root": s.signing_root.hex(), "keys": [bytes(k).hex() for k in s.pubkeys]} for s in sets]


def test_js_signing_roots_cpu(tmp_path):
    """lodestar_amd/js/signing_roots.js (getBlockSignatureSets for the TS host): the K3 devnet roots,
    and an operations block (slashing, exit, BLS change) equal to the Python walk's"""
    if NODE is None:
        pytest.skip("node not installed")
    import json
    ops = _ops_file(tmp_path)
    r = subprocess.run([NODE, SR_SCRIPT, "cpu", ops], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.strip().splitlines()
    assert lines[-1] == "js signing roots cpu ok"
    assert json.loads(lines[-2]) == _python_ops_roots(ops)


@pytest.mark.gpu
def test_js_signing_roots_gpu(tmp_path):
    """the same walk through addon.merkleize (lb_merkleize), plus its timings"""
    if NODE is None:
        pytest.skip("node not installed")
    import json
    ops = _ops_file(tmp_path)
    r = subprocess.run([NODE, SR_SCRIPT, "gpu", ops], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.strip().splitlines()
    assert lines[-1] == "js signing roots gpu ok"
    out = json.loads(lines[-2])
    assert out["ops"] == _python_ops_roots(ops)
    print("signing-root timings:", {k: v for k, v in out.items() if k != "ops"})


def _fork_cases_file(tmp_path):
    import json
    from conftest import load_json
    from test_signing_roots import MAINNET_GVR, fork_cases
    cases = [{"name": n, "block": b, "state": kind, "forks": (None if forks in (None, "mainnet") else forks),
              "err": err} for n, b, kind, forks, err in fork_cases(load_json("k3_devnet.json"))]
    p = tmp_path / "fork_cases.json"
    p.write_text(json.dumps({"mainnet_gvr": MAINNET_GVR, "cases": cases}))
    return str(p)


def _js_fork_cases(tmp_path, gpu):
    import json
    r = subprocess.run([NODE, SR_SCRIPT, "forks", _fork_cases_file(tmp_path)] + (["gpu"] if gpu else []),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.strip().splitlines()
    assert lines[-1] == "js fork cases ok"
    return json.loads(lines[-2])


def test_js_fork_cases_cpu(tmp_path):
    """the JS walk's fork dispatch (phase0 backfill blocks, altair, bellatrix), empty sync
    participation (infinity: no set; otherwise the reference's error) and attester slashings equal
    the Python walk's, which tests/test_signing_roots.py checks against oracle/ssz.py"""
    if NODE is None:
        pytest.skip("node not installed")
    from conftest import load_json
    from test_signing_roots import cpu_merkleize, python_fork_case_roots
    assert _js_fork_cases(tmp_path, False) == python_fork_case_roots(load_json("k3_devnet.json"), cpu_merkleize)


@pytest.mark.gpu
def test_js_fork_cases_gpu(tmp_path):
    if NODE is None:
        pytest.skip("node not installed")
    from conftest import load_json
    from test_signing_roots import cpu_merkleize, python_fork_case_roots
    assert _js_fork_cases(tmp_path, True) == python_fork_case_roots(load_json("k3_devnet.json"), cpu_merkleize)
