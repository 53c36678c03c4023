"""Signing-root production: the host walk of lodestar_amd/signing_roots.py
(getBlockSignatureSets for a capella block) against the K3 devnet fixture, whose roots come from
oracle/ssz.py and whose body root is pinned by the reference's postState (tests/golden/make_k3.py).
CPU: the walk with a hashlib merkleizer.  GPU: the same walk with lb_merkleize, then the four
real devnet signature sets verified on the GPU."""
import hashlib

import numpy as np
import pytest

from conftest import load_json
from lodestar_amd import signing_roots as SR

ZH = [bytes(32)]
for _ in range(64):
    ZH.append(hashlib.sha256(ZH[-1] + ZH[-1]).digest())


def cpu_merkleize(trees):
    out = []
    for t in trees:
        layer = SR.leaves(t)
        for d in range(t.depth):
            if len(layer) % 2:
                layer.append(ZH[d])
            layer = [hashlib.sha256(layer[i] + layer[i + 1]).digest() for i in range(0, len(layer), 2)]
        r = layer[0] if layer else ZH[t.depth]
        if t.mix is not None:
            r = hashlib.sha256(r + t.mix.to_bytes(32, "little")).digest()
        out.append(r)
    return out


def k3_state(k3, pubkey=lambda b: b):
    sv = k3["state_view"]
    keys = [bytes.fromhex(k) for k in sv["validator_pubkeys48"]]
    return SR.StateView(
        genesis_validators_root=bytes.fromhex(k3["genesis_validators_root"]),
        fork_previous_version=bytes.fromhex(k3["fork"]["previous_version"]),
        fork_current_version=bytes.fromhex(k3["fork"]["current_version"]),
        fork_epoch=k3["fork"]["epoch"], genesis_fork_version=bytes.fromhex(k3["fork"]["previous_version"]),
        pubkey=lambda i: pubkey(keys[i]),
        beacon_committee=lambda slot, index: sv["committees"][f"{slot}:{index}"],
        sync_committee=lambda: [pubkey(keys[i]) for i in sv["sync_committee_indices"]])


def test_k3_block_signing_roots_cpu_walk():
    k3 = load_json("k3_devnet.json")
    sets = SR.resolve(SR.block_signature_sets(k3["signed_block"], k3_state(k3)), cpu_merkleize)
    gold = k3["sets"]
    assert [s.name for s in sets] == ["proposer", "randao", "attestation", "sync_aggregate"]
    for s, g in zip(sets, gold):
        assert s.signing_root.hex() == g["signing_root"], s.name
        assert s.signature.hex() == g["signature"]
        assert len(s.pubkeys) == len(g["pubkeys"])
    block = SR.beacon_block_capella(k3["signed_block"]["message"])
    assert SR.evaluate([block], cpu_merkleize)[0].hex() == k3["block_root"]
    body = SR.beacon_block_body_capella(k3["signed_block"]["message"]["body"])
    assert SR.evaluate([body], cpu_merkleize)[0].hex() == k3["body_root"]


def test_k3_sets_verify_in_oracle():
    """The oracle accepts the devnet's own signatures (pins it with real-network vectors)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import bls_oracle as o
    for s in load_json("k3_devnet.json")["sets"]:
        assert o.verify_job([([bytes.fromhex(p) for p in s["pubkeys"]], bytes.fromhex(s["signing_root"]),
                              bytes.fromhex(s["signature"]))]) is True, s["name"]


@pytest.mark.gpu
def test_k3_signing_roots_gpu_and_verify(engine):
    from lodestar_amd.engine import SetInput
    k3 = load_json("k3_devnet.json")
    m = SR.GpuMerkleizer(engine)
    pk96 = {}

    def pub(b48):
        if b48 not in pk96:
            out, st = engine.g1_decompress([b48])
            assert st == [0]
            pk96[b48] = out[0]
        return pk96[b48]
    sets = SR.resolve(SR.block_signature_sets(k3["signed_block"], k3_state(k3, pub)), m)
    assert [s.signing_root.hex() for s in sets] == [g["signing_root"] for g in k3["sets"]]
    assert m.launches <= 12  # one launch per tree level, however many trees
    block = SR.beacon_block_capella(k3["signed_block"]["message"])
    assert SR.evaluate([block], m)[0].hex() == k3["block_root"]
    # the devnet's own signatures, verified on the GPU: each set alone, and all four as one job
    jobs = [[SetInput(s.pubkeys, s.signing_root, s.signature)] for s in sets]
    assert engine.verify_jobs(jobs) == [1, 1, 1, 1]
    assert engine.verify_jobs([[j[0] for j in jobs]]) == [1]
    bad = SetInput(sets[3].pubkeys[1:], sets[3].signing_root, sets[3].signature)  # one participant short
    assert engine.verify_jobs([[bad]]) == [0]
