"""ctypes binding of the C ABI in include/lodestar_bls.h (liblodestar_bls.so, built in-tree).

There is no fallback: if the HIP library is missing or no gfx950 device is present, the
calls fail loudly (NativeUnavailable / BlsError with LB_ERR_NO_DEVICE).
"""
from __future__ import annotations

import ctypes
import os

# LODESTAR_BLS_LIB points at an alternative build of the same library (A/B of compile options).
LIB_PATH = os.environ.get("LODESTAR_BLS_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                               "liblodestar_bls.so")

# status codes (include/lodestar_bls.h)
LB_OK = 0
LB_BAD_ENCODING = 1
LB_POINT_NOT_ON_CURVE = 2
LB_POINT_NOT_IN_GROUP = 3
LB_AGGR_TYPE_MISMATCH = 4
LB_VERIFY_FAIL = 5
LB_PK_IS_INFINITY = 6
LB_BAD_SCALAR = 7
LB_INVALID_SIZE = 10
LB_EMPTY_AGGREGATE_ARRAY = 11
LB_EMPTY_SIGNATURE_SET = 12
LB_ERR_ARGUMENT = 100
LB_ERR_DEVICE = 101
LB_ERR_NO_DEVICE = 102


class NativeUnavailable(RuntimeError):
    pass


_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_i32p = ctypes.POINTER(ctypes.c_int32)
_vp = ctypes.c_void_p

# name -> (restype, argtypes); must cover every function declared in include/lodestar_bls.h
SIGNATURES = {
    "lb_error_name": (ctypes.c_char_p, [ctypes.c_int32]),
    "lb_abi_version": (ctypes.c_int32, []),
    "lb_engine_create": (ctypes.c_int32, [ctypes.c_int32, ctypes.POINTER(_vp)]),
    "lb_engine_create_ex": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_uint32, ctypes.POINTER(_vp)]),
    "lb_engine_destroy": (None, [_vp]),
    "lb_engine_cu_count": (ctypes.c_int32, [_vp]),
    "lb_batch_create": (ctypes.c_int32, [_vp, ctypes.c_uint32, _u32p, _u32p, _u8p, _u8p, _u8p, _u32p,
                                         ctypes.POINTER(_vp)]),
    "lb_batch_destroy": (None, [_vp]),
    "lb_batch_num_sets": (ctypes.c_uint32, [_vp]),
    "lb_batch_num_jobs": (ctypes.c_uint32, [_vp]),
    "lb_batch_verify": (ctypes.c_int32, [_vp, _vp, _u64p, _i32p]),
    "lb_batch_partial": (ctypes.c_int32, [_vp, _vp, _u64p, _u8p, _i32p]),
    "lb_batch_search_after_partial": (ctypes.c_int32, [_vp, _vp, _i32p]),
    "lb_fp12_product_is_one": (ctypes.c_int32, [_vp, _u8p, ctypes.c_uint32, _i32p]),
    "lb_verify_jobs": (ctypes.c_int32, [_vp, ctypes.c_uint32, _u32p, _u32p, _u8p, _u8p, _u8p, _u32p, _u64p,
                                        _i32p]),
    "lb_verify_jobs_indexed": (ctypes.c_int32, [_vp, ctypes.c_uint32, _u32p, _u32p, _u32p, _u8p, _u8p, _u32p,
                                                _u64p, _i32p]),
    "lb_host_alloc": (_vp, [ctypes.c_size_t]),
    "lb_host_free": (None, [_vp]),
    "lb_aggregate_pubkeys": (ctypes.c_int32, [_vp, ctypes.c_uint32, _u32p, _u8p, _u8p, _i32p]),
    "lb_aggregate_signatures": (ctypes.c_int32, [_vp, ctypes.c_uint32, _u32p, _u8p, _u32p, ctypes.c_int32, _u8p,
                                                 _i32p]),
    "lb_g1_decompress": (ctypes.c_int32, [_vp, ctypes.c_uint32, _u8p, _u8p, _i32p, ctypes.c_int32]),
    "lb_merkleize": (ctypes.c_int32, [_vp, ctypes.c_uint32, _u32p, _u8p, _u32p, _u64p, _u8p]),
    "lb_kzg_load_setup": (ctypes.c_int32, [_vp, _u8p, ctypes.c_uint32, _u8p, ctypes.c_uint32, _i32p]),
    "lb_g1_lincomb": (ctypes.c_int32, [_vp, ctypes.c_uint32, _u8p, _u8p, _u8p]),
    "lb_kzg_verify_proof": (ctypes.c_int32, [_vp, _u8p, _u8p, _u8p, _u8p, _i32p]),
    "lb_sk_to_pk": (ctypes.c_int32, [_vp, ctypes.c_uint32, _u8p, _u8p, _u8p]),
    "lb_sign": (ctypes.c_int32, [_vp, ctypes.c_uint32, _u8p, _u8p, _u8p]),
    "lb_pubkey_table_append": (ctypes.c_int32, [_vp, ctypes.c_uint32, _u8p, ctypes.c_uint32, ctypes.c_int32, _i32p,
                                                _u32p]),
    "lb_pubkey_table_size": (ctypes.c_uint32, [_vp]),
    "lb_batch_create_indexed": (ctypes.c_int32, [_vp, ctypes.c_uint32, _u32p, _u32p, _u32p, _u8p, _u8p, _u32p,
                                                 ctypes.POINTER(_vp)]),
    "lb_engine_set_profiling": (ctypes.c_int32, [_vp, ctypes.c_int32]),
    "lb_engine_last_profile": (ctypes.c_int32, [_vp, ctypes.POINTER(ctypes.c_char_p),
                                                ctypes.POINTER(ctypes.c_float), ctypes.c_int32, _i32p]),
}

_lib = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load liblodestar_bls.so (raises NativeUnavailable if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise NativeUnavailable(
            f"{path} not found: build it with `python -m lodestar_amd.build` (hipcc, gfx950)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def error_name(code: int) -> str:
    return load().lb_error_name(int(code)).decode()
