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
