"""The C-ABI library builds for gfx950, loads on CPU and exports every entry point that
include/lodestar_bls.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

from conftest import ROOT


def header_functions():
    src = open(os.path.join(ROOT, "include", "lodestar_bls.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lb_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_header_symbols():
    from lodestar_amd import _native as N
    lib = N.load()
    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
        assert n in N.SIGNATURES, f"{n} missing from the ctypes table"


def test_error_names_match_reference_strings():
    from lodestar_amd import _native as N
    assert N.error_name(N.LB_INVALID_SIZE) == "BLST_INVALID_SIZE"          # multithread.test.ts:97
    assert N.error_name(N.LB_EMPTY_SIGNATURE_SET) == "Empty signature set"  # maybeBatch.ts:30
    assert N.error_name(N.LB_POINT_NOT_IN_GROUP) == "BLST_POINT_NOT_IN_GROUP"


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        return
    from lodestar_amd import _native as N
    h = ctypes.c_void_p()
    st = N.load().lb_engine_create(0, ctypes.byref(h))
    assert st == N.LB_ERR_NO_DEVICE


def test_gfx950_code_object_present():
    from lodestar_amd import _native as N
    data = open(N.LIB_PATH, "rb").read()
    assert b"gfx950" in data
