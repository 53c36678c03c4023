"""Pins the CPU oracle (oracle/bls_oracle.py) against the reference's own known-answer data
(SURVEY.md §8(c) K1, K2, K4).  CPU only."""
import hashlib

from conftest import load_json
from oracle import bls_oracle as o


def test_k1_interop_pubkeys():
    k = load_json("reference_kats.json")["K1_interop_pubkeys"]
    for i, pk in enumerate(k["pubkeys"][:6]):
        assert o.g1_compress(o.sk_to_pk(o.interop_secret_key(i))).hex() == pk


def test_k2_deposit_signature_sign_and_verify():
    k = load_json("reference_kats.json")["K2_deposit_signature"]
    sk = o.interop_secret_key(0)
    pk0 = o.g1_compress(o.sk_to_pk(sk))
    assert pk0.hex() == k["pubkey"]
    root = o.deposit_message_root(pk0, bytes.fromhex(k["withdrawal_credentials"]), k["amount"])
    dom = o.compute_domain(bytes.fromhex(k["domain_type"]), bytes.fromhex(k["fork_version"]), bytes(32))
    msg = o.compute_signing_root(root, dom)
    assert msg.hex() == k["signing_root"]
    sig = o.sign(sk, msg)
    assert o.g2_compress(sig).hex() == k["signature"]
    assert o.core_verify(o.sk_to_pk(sk), msg, o.signature_from_bytes(bytes.fromhex(k["signature"])))


def test_k4_sets_batch_verify():
    sets = load_json("reference_kats.json")["K4_multithread_sets"]["sets"]
    job = [([bytes.fromhex(s["pubkey96"])], bytes.fromhex(s["signing_root"]), bytes.fromhex(s["signature"]))
           for s in sets]
    assert o.verify_job(job, scalars=[3, 5, 7]) is True
    bad = list(job)
    bad[1] = (bad[1][0], bad[2][1], bad[1][2])
    assert o.verify_job(bad, scalars=[3, 5, 7]) is False


def test_expand_message_xmd_rfc9380_vector():
    # RFC 9380 App. K.1 (expand_message_xmd, SHA-256), msg = "", len_in_bytes = 0x20
    dst = b"QUUX-V01-CS02-with-expander-SHA256-128"
    out = o.expand_message_xmd(b"", dst, 0x20)
    assert out.hex() == "68a985b87eb6b46952128911f2a4412bbc302a9d759667f87f7a21d803f07235"


def test_interop_sk_formula():
    d = hashlib.sha256((0).to_bytes(32, "little")).digest()
    assert o.interop_secret_key(0) == int.from_bytes(d, "little") % o.R
