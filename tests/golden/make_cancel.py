#!/usr/bin/env python3
"""Generates tests/golden/cancel_pair.json from the CPU oracle: two single-set jobs whose
signatures carry opposite offsets, sig_A = sk_A H(m_A) + D and sig_B = sk_B H(m_B) - D.

Each set is invalid on its own (oracle core_verify -> false), but the UNBLINDED product
e(PK_A, H(m_A)) e(PK_B, H(m_B)) e(-G1, sig_A + sig_B) is one.  A multi-GPU exchange whose 1-set
shards sent unblinded partials would accept both (round-5 ADVICE on lb_batch_partial); blinded
partials (independent random r_A, r_B) reject them.  Run from the repo root:
    python3 tests/golden/make_cancel.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import bls_oracle as o  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    sk_a, sk_b = o.interop_secret_key(3), o.interop_secret_key(4)
    m_a, m_b = bytes([0xA1]) * 32, bytes([0xB2]) * 32
    d = o.g2_mul(o.hash_to_g2(b"cancel-offset"), 7)
    sig_a = o.g2_add(o.sign(sk_a, m_a), d)
    sig_b = o.g2_add(o.sign(sk_b, m_b), o.g2_neg(d))
    sets = []
    for sk, m, s in ((sk_a, m_a, sig_a), (sk_b, m_b, sig_b)):
        sets.append({"pubkey": o.g1_serialize(o.sk_to_pk(sk)).hex(), "signing_root": m.hex(),
                     "signature": o.g2_compress(s).hex()})
    out = {"generator": "tests/golden/make_cancel.py", "sets": sets,
           "note": "each set alone verifies false; the unblinded product of the two is one"}
    with open(os.path.join(OUT, "cancel_pair.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
