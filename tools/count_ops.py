#!/usr/bin/env python3
"""Algorithmic work per pipeline stage, for bench.py's roofline.

Replays each kernel's arithmetic on the CPU build of the same headers with every Fp
multiplication counted (tests/harness/lb_count.cpp, -DLB_COUNT_OPS), averages the
data-dependent stages (64-bit blinding scalars) over random scalars, and writes
profiles/roofline_counts.json.  One Fp multiplication = 12x12-limb CIOS Montgomery =
288 v_mad_u64_u32 + 12 v_mul_lo_u32 = 300 32-bit integer multiply(-accumulate)s.
The peak is the measured chip-wide v_mad_u64_u32 rate (tools/ubench_int.hip,
profiles/r1_ubench_int.json)."""
import ctypes
import json
import os
import random
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import bls_oracle as o  # noqa: E402

SO = os.path.join(ROOT, "build", "lb_count.so")


def main():
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "lodestar_amd", "csrc"),
                    os.path.join(ROOT, "tests", "harness", "lb_count.cpp"), "-o", SO], check=True)
    L = ctypes.CDLL(SO)
    for f in ("cnt_decode", "cnt_hash_map", "cnt_hash_finish", "cnt_pk_blind", "cnt_miller", "cnt_fp12_mul",
              "cnt_g2_add", "cnt_node_check", "cnt_g1_blind", "cnt_g2_blind", "cnt_pk_key", "cnt_fe"):
        getattr(L, f).restype = ctypes.c_ulonglong
    L.cnt_g1_blind.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
    L.cnt_g2_blind.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
    L.cnt_pk_key.argtypes = [ctypes.c_char_p, ctypes.c_int]
    L.cnt_pk_blind.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_char_p]
    rnd = random.Random(5)
    sks = [o.interop_secret_key(i) for i in range(4)]
    msgs = [bytes([rnd.randrange(256) for _ in range(32)]) for _ in range(4)]
    sigs = [o.g2_compress(o.sign(sks[i], msgs[i])) for i in range(4)]
    pks = [o.g1_serialize(o.sk_to_pk(s)) for s in sks]
    avg = lambda xs: sum(xs) / len(xs)  # noqa: E731
    c = {}
    c["decode_sigs"] = avg([L.cnt_decode(s) for s in sigs])
    c["hash_map"] = avg([L.cnt_hash_map(m, w) for m in msgs for w in (0, 1)])
    c["hash_finish"] = avg([L.cnt_hash_finish(m) for m in msgs])
    blind1 = avg([L.cnt_pk_blind(pks[0], 1, rnd.getrandbits(64) | 1, sigs[0]) for _ in range(16)])
    pk3 = b"".join(pks[:3])
    blind3 = avg([L.cnt_pk_blind(pk3, 3, rnd.getrandbits(64) | 1, sigs[0]) for _ in range(16)])
    pk4 = b"".join(pks[:4])
    blind4 = avg([L.cnt_pk_blind(pk4, 4, rnd.getrandbits(64) | 1, sigs[0]) for _ in range(16)])
    c["miller"] = avg([L.cnt_miller(pks[i], msgs[i]) for i in range(2)])
    fp12m = L.cnt_fp12_mul()
    g2add = L.cnt_g2_add(sigs[0])
    node = L.cnt_node_check(sigs[0])
    g1b = avg([L.cnt_g1_blind(pks[0], rnd.getrandbits(64) | 1) for _ in range(16)])
    g2b = avg([L.cnt_g2_blind(sigs[0], rnd.getrandbits(64) | 1) for _ in range(16)])
    per_key = (L.cnt_pk_key(b"".join(pks[:4]), 4) - L.cnt_pk_key(pks[0], 1)) / 3
    fe = L.cnt_fe()
    out = {
        "mac_per_fp_mul": 300,
        "peak_tmac_s": json.load(open(os.path.join(ROOT, "profiles", "r1_ubench_int.json")))["v_mad_u64_u32_Tops"],
        "peak_source": "tools/ubench_int.hip v_mad_u64_u32 chip-wide rate, profiles/r1_ubench_int.json",
        "fp_mul_per_item": {
            "decode_sigs": c["decode_sigs"],          # per set
            "hash_map": c["hash_map"],                # per field element (2 per set)
            "hash_finish": c["hash_finish"],          # per set
            "pk_blind_k1": blind1,                    # per set with one pubkey
            "pk_blind_per_extra_key": (blind4 - blind3),  # each additional aggregated pubkey
            "pk_blind_k_base": blind3 - 2 * (blind4 - blind3),
            "miller": c["miller"],                    # per set
            "fp12_mul": fp12m, "g2_add": g2add,       # job_leaves / tree_up building blocks
            "node_check": node,                       # per checked tree node (ML + FE)
            "pk_key": per_key,                        # k_pk_chunks: decode + add per pubkey
            "g1_blind": g1b,                          # k_pk_blind per set (r*PK + affine)
            "g2_blind": g2b,                          # k_sig_blind per set (r*sig)
            "final_exp": fe,                          # k_root_check
            "ml_S": c["miller"] + (node - fe - c["miller"] - fp12m),  # k_ml_S: ML + G2 affine
        },
        "items_per_set": {"decode_sigs": 1, "hash_map": 2, "hash_finish": 1, "pk_blind": 1, "miller": 1},
    }
    out["fp_mul_per_set_k1_estimate"] = (c["decode_sigs"] + 2 * c["hash_map"] + c["hash_finish"] + blind1
                                         + c["miller"] + fp12m + g2add)
    path = os.path.join(ROOT, "profiles", "roofline_counts.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
