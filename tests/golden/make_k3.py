#!/usr/bin/env python3
"""Builds tests/golden/k3_devnet.json from the reference's capella devnet fixture (SURVEY.md §8(c)
K3): packages/state-transition/test/unit/data/withdrawal-devnet-slot-10497/{preState.ssz,
block.json, postState.ssz}.  Runs in the build container only (it reads /root/reference); the
GPU box gets the JSON.

The four signature sets getBlockSignatureSets produces for that block
(state-transition/src/signatureSets/index.ts:64-111) -- proposer, randao, one attestation
(aggregate, committee from the swap-or-not shuffle), the sync aggregate (388 participants over
the 80 validators' keys) -- with their signing roots computed by oracle/ssz.py, the pubkeys
decompressed from the state by the oracle, and every set verified by the oracle.  The block
body root is cross-checked against postState.latest_block_header.body_root, which pins the SSZ
merkleization of the capella body (execution payload with withdrawals included).  The signatures
are the devnet's own, so these are real-network vectors, not oracle output.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import bls_oracle as o  # noqa: E402
from oracle import ssz  # noqa: E402

DATA = "/root/reference/packages/state-transition/test/unit/data/withdrawal-devnet-slot-10497"


def main():
    with open(os.path.join(DATA, "block.json")) as f:
        signed = json.load(f)["data"]
    with open(os.path.join(DATA, "preState.ssz"), "rb") as f:
        pre = ssz.CapellaState(f.read())
    with open(os.path.join(DATA, "postState.ssz"), "rb") as f:
        post = ssz.CapellaState(f.read())
    m = signed["message"]
    body = m["body"]
    slot = int(m["slot"])
    epoch = slot // ssz.SLOTS_PER_EPOCH
    body_root = ssz.beacon_block_body_capella(body)
    assert body_root == post.latest_block_header[80:112], "body root != postState.latest_block_header.body_root"
    block_root = ssz.beacon_block_capella(m)
    pk = lambda v: o.g1_serialize(o.g1_decompress(pre.validators[v]["pubkey"]))  # noqa: E731
    sets = []
    # proposer (single): signing root of the block, DOMAIN_BEACON_PROPOSER
    sets.append(("proposer", [pk(int(m["proposer_index"]))],
                 ssz.signing_root(block_root, pre.domain(ssz.DOMAIN_BEACON_PROPOSER, epoch)), signed["signature"],
                 "single"))
    # randao (single): signing root of the epoch, DOMAIN_RANDAO
    sets.append(("randao", [pk(int(m["proposer_index"]))],
                 ssz.signing_root(ssz.uint64(epoch), pre.domain(ssz.DOMAIN_RANDAO, epoch)), body["randao_reveal"],
                 "single"))
    # attestations (aggregate): attesting indices from the committee and the aggregation bits
    for a in body["attestations"]:
        d = a["data"]
        committee = pre.beacon_committee(int(d["slot"]), int(d["index"]))
        bits = ssz.bits_from_hex_bitlist(a["aggregation_bits"])
        assert len(bits) == len(committee)
        idx = sorted(v for v, b in zip(committee, bits) if b)
        sets.append((f"attestation_slot{d['slot']}_index{d['index']}", [pk(v) for v in idx],
                     ssz.signing_root(ssz.attestation_data(d),
                                      pre.domain(ssz.DOMAIN_BEACON_ATTESTER, int(d["target"]["epoch"]))),
                     a["signature"], "aggregate"))
    # sync aggregate: participants of the current sync committee sign the previous slot's block root
    sa = body["sync_aggregate"]
    bits = ssz.bits_from_hex_bitvector(sa["sync_committee_bits"], ssz.SYNC_COMMITTEE_SIZE)
    keys = [o.g1_serialize(o.g1_decompress(k)) for k, b in zip(pre.current_sync_committee, bits) if b]
    prev = slot - 1
    sets.append(("sync_aggregate", keys,
                 ssz.signing_root(ssz.hx(m["parent_root"]),
                                  pre.domain(ssz.DOMAIN_SYNC_COMMITTEE, prev // ssz.SLOTS_PER_EPOCH)),
                 sa["sync_committee_signature"], "aggregate"))
    out = []
    for name, pks, root, sig, kind in sets:
        sig_b = ssz.hx(sig)
        ok = o.verify_job([(pks, root, sig_b)])
        assert ok is True, (name, ok)
        out.append({"name": name, "type": kind, "pubkeys": [p.hex() for p in pks], "signing_root": root.hex(),
                    "signature": sig_b.hex(), "expected": True})
        print(name, len(pks), "keys, oracle verifies", flush=True)
    # what getBlockSignatureSets reads from the state, for the signing-root tests on the GPU box
    pk_index = {v["pubkey"]: i for i, v in enumerate(pre.validators)}
    committees = {}
    for a in body["attestations"]:
        d = a["data"]
        committees[f"{d['slot']}:{d['index']}"] = pre.beacon_committee(int(d["slot"]), int(d["index"]))
    state_view = {"validator_pubkeys48": [v["pubkey"].hex() for v in pre.validators],
                  "committees": committees,
                  "sync_committee_indices": [pk_index[k] for k in pre.current_sync_committee]}
    doc = {
        "source": "packages/state-transition/test/unit/data/withdrawal-devnet-slot-10497 (capella devnet, "
                  "signatures from the network)",
        "signed_block": signed, "state_view": state_view,
        "slot": slot, "genesis_validators_root": pre.genesis_validators_root.hex(),
        "fork": {"previous_version": pre.fork_previous.hex(), "current_version": pre.fork_current.hex(),
                 "epoch": pre.fork_epoch},
        "block_root": block_root.hex(), "body_root": body_root.hex(),
        "validators": len(pre.validators), "sync_participants": sum(bits),
        "sets": out,
    }
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "k3_devnet.json"), "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
