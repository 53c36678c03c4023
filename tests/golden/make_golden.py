#!/usr/bin/env python3
"""Generates tests/golden/*.json from the CPU oracle (oracle/bls_oracle.py) and from data files
held by the reference's own tests.  Run from the repo root in the CPU container:
    python3 tests/golden/make_golden.py
Fixtures are data only (hex inputs + expected outputs); the GPU box reads them, never the
reference tree.

  reference_kats.json  K1: interop pubkeys 0..15 (packages/state-transition/test-cache/
                       interop-pubkeys.json) with their secret-key formula (interop.ts:19-23);
                       K2: interop deposit signature (beacon-node/test/e2e/interop/
                       genesisState.test.ts:9-50); K4: multithread.test.ts:24-38 sets.
  jobs.json            jobs (lists of sets) with the expected per-job result of the reference
                       semantics (oracle.verify_job): true / false / error name.
  aggregates.json      getAggregatedPubkey + toBytes(uncompressed) expectations.
"""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import bls_oracle as o  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
rnd = random.Random(0x4C4F4445)


def h(b):
    return b.hex()


def pk96(sk):
    return o.g1_serialize(o.sk_to_pk(sk))


def sig_of(sk, msg):
    return o.g2_compress(o.sign(sk, msg))


def kats():
    with open(os.path.join(REF, "packages/state-transition/test-cache/interop-pubkeys.json")) as f:
        pks = json.load(f)[:16]
    k2 = {
        "sk_index": 0,
        "withdrawal_credentials": "00fad2a6bfb0e7f1f0f45460944fbd8dfa7f37da06a4d13b3983cc90bb46963b",
        "amount": 32000000000,
        "domain_type": "03000000",
        "fork_version": "00000001",
        "signature": "a95af8ff0f8c06af4d29aef05ce865f85f82df42b606008ec5b1bcb42b17ae47f4b78cdce1db31ce32d18f4"
                     "2a6b296b4014a2164981780e56b5a40d7723c27b8423173e58fa36f075078b177634f66351412b867c103f532"
                     "aedd50bcd9b98446",
    }
    sk0 = o.interop_secret_key(0)
    pk0 = o.g1_compress(o.sk_to_pk(sk0))
    root = o.deposit_message_root(pk0, bytes.fromhex(k2["withdrawal_credentials"]), k2["amount"])
    dom = o.compute_domain(bytes.fromhex(k2["domain_type"]), bytes.fromhex(k2["fork_version"]), bytes(32))
    k2["signing_root"] = h(o.compute_signing_root(root, dom))
    k2["pubkey"] = h(pk0)
    k2["pubkey96"] = h(o.g1_serialize(o.sk_to_pk(sk0)))
    k4 = []
    for i in range(3):
        sk = int.from_bytes(bytes([i + 1]) * 32, "big")
        msg = bytes([i + 1]) * 32
        k4.append({"sk": "%064x" % sk, "pubkey96": h(pk96(sk)), "signing_root": h(msg), "signature": h(sig_of(sk, msg))})
    return {
        "K1_interop_pubkeys": {"source": "packages/state-transition/test-cache/interop-pubkeys.json",
                               "formula": "sk_i = LE(sha256(LE32(i))) mod r (state-transition/src/util/interop.ts:19-23)",
                               "pubkeys": [p[2:] for p in pks]},
        "K2_deposit_signature": dict(source="packages/beacon-node/test/e2e/interop/genesisState.test.ts:9-50", **k2),
        "K4_multithread_sets": {"source": "packages/beacon-node/test/e2e/chain/bls/multithread.test.ts:24-38",
                                "sets": k4},
    }


def g2_point_off_subgroup():
    while True:
        x = (rnd.randrange(o.P), rnd.randrange(o.P))
        y = o.f2_sqrt(o.f2_add(o.f2_mul(o.f2_sqr(x), x), o.B2))
        if y is not None and not o.g2_in_subgroup((x, y)):
            return o.g2_compress((x, y))


def g2_x_off_curve():
    while True:
        x = (rnd.randrange(o.P), rnd.randrange(o.P))
        if o.f2_sqrt(o.f2_add(o.f2_mul(o.f2_sqr(x), x), o.B2)) is None:
            b = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
            b[0] |= 0x80
            return bytes(b)


def jobs():
    keys = [o.interop_secret_key(i) for i in range(8)]
    pks = [pk96(k) for k in keys]
    msgs = [bytes([0xA0 + i]) * 32 for i in range(8)]
    sigs = [sig_of(k, m) for k, m in zip(keys, msgs)]

    def single(i, msg=None, sig=None):
        return ([pks[i]], msgs[i] if msg is None else msg, sigs[i] if sig is None else sig)

    agg_msg = b"\x5a" * 32
    agg_keys = [0, 1, 2, 3]
    agg_sig = o.g2_compress(o.g2_mul(o.hash_to_g2(agg_msg), sum(keys[i] for i in agg_keys) % o.R))
    agg_set = ([pks[i] for i in agg_keys], agg_msg, agg_sig)
    dup_sig = o.g2_compress(o.g2_mul(o.hash_to_g2(agg_msg), (2 * keys[5] + keys[6]) % o.R))
    dup_set = ([pks[5], pks[5], pks[6]], agg_msg, dup_sig)
    neg_pk = o.g1_serialize(o.g1_neg(o.sk_to_pk(keys[0])))
    inf_agg = ([pks[0], neg_pk], agg_msg, sigs[0])
    sig_other = sigs[1]
    bad_flag = bytes([sigs[0][0] & 0x7F]) + sigs[0][1:]
    big_x = bytearray(o.P.to_bytes(48, "big") + bytes(48))
    big_x[0] |= 0x80
    inf_sig = bytes([0xC0]) + bytes(95)
    bad_inf = bytes([0xC0]) + bytes(94) + b"\x01"
    bad_pk = bytes([pks[2][0] | 0x80]) + pks[2][1:]
    pk_off_curve = pks[2][:95] + bytes([pks[2][95] ^ 1])
    cases = [
        ("single_valid_0", [single(0)]),
        ("single_valid_1", [single(1)]),
        ("two_valid", [single(2), single(3)]),
        ("aggregate_valid", [agg_set]),
        ("aggregate_duplicate_keys", [dup_set]),
        ("mixed_valid_with_aggregate", [single(4), agg_set, single(5)]),
        ("wrong_message", [single(0, msg=msgs[1])]),
        ("wrong_signature", [single(0, sig=sig_other)]),
        ("batch_one_wrong", [single(0), single(1, sig=sigs[2]), single(3)]),
        ("aggregate_missing_key", [([pks[i] for i in agg_keys[:3]], agg_msg, agg_sig)]),
        ("invalid_size_32_zero", [single(0, sig=bytes(32))]),
        ("invalid_size_in_batch", [single(1), single(0, sig=bytes(95))]),
        ("bad_encoding_flag", [single(0, sig=bad_flag)]),
        ("bad_encoding_x_ge_p", [single(0, sig=bytes(big_x))]),
        ("bad_encoding_infinity_nonzero", [single(0, sig=bad_inf)]),
        ("not_on_curve", [single(0, sig=g2_x_off_curve())]),
        ("not_in_group", [single(1, sig=g2_point_off_subgroup())]),
        ("infinity_signature_single", [single(0, sig=inf_sig)]),
        ("infinity_signature_in_batch", [single(1), single(0, sig=inf_sig)]),
        ("aggregate_pubkey_infinity", [inf_agg]),
        ("aggregate_empty", [([], agg_msg, agg_sig)]),
        ("pubkey_bad_encoding", [([bad_pk], msgs[2], sigs[2])]),
        ("pubkey_not_on_curve", [([pk_off_curve], msgs[2], sigs[2])]),
        ("error_precedence_sig_before_pkinf", [inf_agg, single(0, sig=bad_flag)]),
        ("empty_job", []),
        ("k4_like_batch", [single(6), single(7), single(6), single(7)]),
    ]
    out = []
    for name, sets in cases:
        try:
            exp = o.verify_job(sets, scalars=[rnd.getrandbits(64) | 1 for _ in sets])
            expected = bool(exp)
        except o.BlsError as e:
            expected = str(e)
        print(f"  {name}: {expected}", flush=True)
        out.append({"name": name, "expected": expected,
                    "sets": [{"pubkeys": [h(p) for p in s[0]], "signing_root": h(s[1]), "signature": h(s[2])}
                             for s in sets]})
    return {"cases": out}


def aggregates():
    keys = [o.interop_secret_key(i) for i in range(6)]
    pts = [o.sk_to_pk(k) for k in keys]
    neg0 = o.g1_neg(pts[0])
    groups = [[0], [0, 1], [0, 1, 2, 3, 4, 5], [2, 2], [3, 3, 3, 4], ["n0", 0], [0, "n0", 1]]
    out = []
    for g in groups:
        P = [neg0 if x == "n0" else pts[x] for x in g]
        acc = None
        for p in P:
            acc = o.g1_add(acc, p)
        out.append({"pubkeys": [h(o.g1_serialize(p)) for p in P], "expected96": h(o.g1_serialize(acc)),
                    "status": "BLST_SUCCESS"})
    out.append({"pubkeys": [], "expected96": h(bytes([0x40]) + bytes(95)), "status": "EMPTY_AGGREGATE_ARRAY"})
    comp = [{"in48": h(o.g1_compress(p)), "out96": h(o.g1_serialize(p))} for p in pts]
    return {"aggregate": out, "g1_decompress": comp, "signature_aggregate": signature_aggregates()}


def signature_aggregates():
    """bls.Signature.aggregate over decoded signatures (the opPools' aggregation,
    chain/opPools/aggregatedAttestationPool.ts:321): ZCash compressed G2 sum, infinity = 0xc0.
    Decoding follows Signature.fromBytes(.., validate); the first bad signature's error rejects
    the group, an empty group rejects with EMPTY_AGGREGATE_ARRAY."""
    keys = [o.interop_secret_key(i) for i in range(4)]
    msgs = [bytes([0x20 + i]) * 32 for i in range(4)]
    pts = [o.sign(k, m) for k, m in zip(keys, msgs)]
    comp = [o.g2_compress(p) for p in pts]
    neg0 = o.g2_compress(o.g2_neg(pts[0]))
    inf = bytes([0xC0]) + bytes(95)
    groups = [[0], [0, 1], [0, 1, 2, 3], [0, 0], [0, "n0"], ["inf", 1], [2, "inf", 3]]
    out = []
    for g in groups:
        sigs = [neg0 if x == "n0" else inf if x == "inf" else comp[x] for x in g]
        acc = None
        for b in sigs:
            acc = o.g2_add(acc, o.signature_from_bytes(b, True))
        out.append({"signatures": [h(b) for b in sigs], "expected96": h(o.g2_compress(acc)), "status": "BLST_SUCCESS"})
    bad = bytearray(comp[1])
    bad[0] &= 0x7F
    out.append({"signatures": [h(comp[0]), h(bytes(bad))], "expected96": None, "status": "BLST_BAD_ENCODING"})
    out.append({"signatures": [h(comp[0]), h(g2_point_off_subgroup())], "expected96": None,
                "status": "BLST_POINT_NOT_IN_GROUP"})
    out.append({"signatures": [], "expected96": None, "status": "EMPTY_AGGREGATE_ARRAY"})
    return out


if __name__ == "__main__":
    if "--aggregates-only" in sys.argv:
        with open(os.path.join(OUT, "aggregates.json"), "w") as f:
            json.dump(aggregates(), f, indent=1)
        sys.exit(0)
    print("kats", flush=True)
    with open(os.path.join(OUT, "reference_kats.json"), "w") as f:
        json.dump(kats(), f, indent=1)
    print("aggregates", flush=True)
    with open(os.path.join(OUT, "aggregates.json"), "w") as f:
        json.dump(aggregates(), f, indent=1)
    print("jobs", flush=True)
    with open(os.path.join(OUT, "jobs.json"), "w") as f:
        json.dump(jobs(), f, indent=1)
