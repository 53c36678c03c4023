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
        fork_epoch=k3["fork"]["epoch"],
        pubkey=lambda i: pubkey(keys[i]), key_from_bytes=pubkey,
        beacon_committee=lambda slot, index: sv["committees"][f"{slot}:{index}"],
        sync_committee=lambda: [pubkey(keys[i]) for i in sv["sync_committee_indices"]])


def test_k3_block_signing_roots_cpu_walk():
    k3 = load_json("k3_devnet.json")
    sets = SR.resolve(SR.block_signature_sets(k3["signed_block"], k3_state(k3)), cpu_merkleize)
    gold = {g["name"].split("_slot")[0]: g for g in k3["sets"]}
    # getBlockSignatureSets order (signatureSets/index.ts:64-111)
    assert [s.name for s in sets] == ["randao", "attestation", "proposer", "sync_aggregate"]
    for s in sets:
        g = gold[s.name]
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
    gold = {g["name"].split("_slot")[0]: g["signing_root"] for g in k3["sets"]}
    assert [s.signing_root.hex() for s in sets] == [gold[s.name] for s in sets]
    assert m.launches <= 12  # one launch per tree level, however many trees
    block = SR.beacon_block_capella(k3["signed_block"]["message"])
    assert SR.evaluate([block], m)[0].hex() == k3["block_root"]
    # the devnet's own signatures, verified on the GPU: each set alone, and all four as one job
    jobs = [[SetInput(s.pubkeys, s.signing_root, s.signature)] for s in sets]
    assert engine.verify_jobs(jobs) == [1, 1, 1, 1]
    assert engine.verify_jobs([[j[0] for j in jobs]]) == [1]
    sync = [s for s in sets if s.name == "sync_aggregate"][0]
    bad = SetInput(sync.pubkeys[1:], sync.signing_root, sync.signature)  # one participant short
    assert engine.verify_jobs([[bad]]) == [0]


def _operations_block(k3):
    """The K3 block with operations the devnet block lacks: a proposer slashing whose two headers
    name DIFFERENT proposers (the reference takes signedHeader1's key for both,
    proposerSlashings.ts:14-16), a voluntary exit and a BLS-to-execution change.  Signatures are
    placeholders: only the set list and its signing roots are compared."""
    import copy
    blk = copy.deepcopy(k3["signed_block"])
    b = blk["message"]["body"]
    slot = int(blk["message"]["slot"])

    def header(pi, salt):
        return {"message": {"slot": str(slot - 40), "proposer_index": str(pi), "parent_root": "0x" + salt * 32,
                            "state_root": "0x" + "22" * 32, "body_root": "0x" + "33" * 32},
                "signature": "0x" + salt * 96}
    b["proposer_slashings"] = [{"signed_header_1": header(3, "a1"), "signed_header_2": header(5, "a2")}]
    b["voluntary_exits"] = [{"message": {"epoch": "1", "validator_index": "7"}, "signature": "0x" + "b1" * 96}]
    key48 = k3["state_view"]["validator_pubkeys48"][9]
    b["bls_to_execution_changes"] = [{"message": {"validator_index": "9", "from_bls_pubkey": "0x" + key48,
                                                  "to_execution_address": "0x" + "c1" * 20},
                                      "signature": "0x" + "c2" * 96}]
    return blk


def test_operations_sets_match_oracle():
    """order, keys and domains of the operation sets against oracle/ssz.py: the BLS
    change's domain uses the state's fork (config.getDomain(state.slot, ..), blsToExecutionChange.ts:23),
    not the genesis fork version; slashings use header 1's proposer for both sets"""
    import oracle.ssz as S
    k3 = load_json("k3_devnet.json")
    blk = _operations_block(k3)
    st = k3_state(k3)
    sets = SR.resolve(SR.block_signature_sets(blk, st), cpu_merkleize)
    assert [s.name for s in sets] == ["randao", "proposer_slashing", "proposer_slashing", "attestation",
                                      "voluntary_exit", "proposer", "sync_aggregate", "bls_to_execution_change"]
    keys = [bytes.fromhex(k) for k in k3["state_view"]["validator_pubkeys48"]]
    m = blk["message"]
    b = m["body"]
    epoch = int(m["slot"]) // S.SLOTS_PER_EPOCH
    gvr = bytes.fromhex(k3["genesis_validators_root"])
    prev_v, cur_v = bytes.fromhex(k3["fork"]["previous_version"]), bytes.fromhex(k3["fork"]["current_version"])

    def dom(t, ep):
        return S.compute_domain(t, prev_v if ep < k3["fork"]["epoch"] else cur_v, gvr)
    ps = b["proposer_slashings"][0]
    exp = {
        1: (keys[3], S.signing_root(S.block_header(ps["signed_header_1"]["message"]), dom(S.DOMAIN_BEACON_PROPOSER, epoch - 2))),
        2: (keys[3], S.signing_root(S.block_header(ps["signed_header_2"]["message"]), dom(S.DOMAIN_BEACON_PROPOSER, epoch - 2))),
        4: (keys[7], S.signing_root(S.voluntary_exit(b["voluntary_exits"][0]["message"]), dom(S.DOMAIN_VOLUNTARY_EXIT, 1))),
        5: (keys[int(m["proposer_index"])], S.signing_root(S.beacon_block_capella(m), dom(S.DOMAIN_BEACON_PROPOSER, epoch))),
        7: (keys[9], S.signing_root(S.bls_to_execution_change(b["bls_to_execution_changes"][0]["message"]),
                                    dom(S.DOMAIN_BLS_TO_EXECUTION_CHANGE, epoch))),
    }
    for k, (key, root) in exp.items():
        assert sets[k].pubkeys == [key], sets[k].name
        assert sets[k].signing_root == root, sets[k].name
    # the state's fork at this epoch is the current one, so the genesis-version domain would differ
    assert epoch >= k3["fork"]["epoch"] and prev_v != cur_v
    wrong = S.signing_root(S.bls_to_execution_change(b["bls_to_execution_changes"][0]["message"]),
                           S.compute_domain(S.DOMAIN_BLS_TO_EXECUTION_CHANGE, prev_v, gvr))
    assert sets[7].signing_root != wrong


@pytest.mark.gpu
def test_operations_sets_gpu_roots(engine):
    """the same operations block through lb_merkleize: roots equal the hashlib walk's"""
    k3 = load_json("k3_devnet.json")
    blk = _operations_block(k3)
    cpu = SR.resolve(SR.block_signature_sets(blk, k3_state(k3)), cpu_merkleize)
    gpu = SR.resolve(SR.block_signature_sets(blk, k3_state(k3)), SR.GpuMerkleizer(engine))
    assert [s.signing_root for s in gpu] == [s.signing_root for s in cpu]


# ------------------------------------------------------------------ forks, sync participation, slashings
MAINNET_GVR = "4b363db94e286120d76eb905340fdd4e54bfe9f06bf33ff6cf5ad27f511bfe95"  # verify.test.ts:19-22
INFINITY_SIG = "0xc0" + "00" * 95


def mainnet_phase0_state(fork_seq=None):
    """The backfill test's config: mainnet fork schedule, genesis fork version 0x00000000 and the
    mainnet genesis validators root.  Keys are unknown to the fixture, so index2pubkey returns the
    index itself (4 bytes): only set lists and signing roots are compared."""
    v0 = bytes(4)
    return SR.StateView(genesis_validators_root=bytes.fromhex(MAINNET_GVR), fork_previous_version=v0,
                        fork_current_version=v0, fork_epoch=0, pubkey=lambda i: i.to_bytes(4, "big"),
                        beacon_committee=lambda slot, index: list(range(2048)),
                        sync_committee=lambda: [i.to_bytes(4, "big") for i in range(512)],
                        fork_seq=fork_seq or SR.fork_schedule(*SR.MAINNET_FORK_EPOCHS))


def _indexed(indices, salt, d):
    return {"attesting_indices": [str(i) for i in indices], "data": d, "signature": "0x" + salt * 96}


def fork_cases(k3):
    """(name, signed block, state kind, fork epochs or None (capella), expected error) -- shared with
    the JS walk (tests/js/test_signing_roots.js forks mode)."""
    import copy
    cases = []
    ops = _operations_block(k3)
    d = ops["message"]["body"]["attestations"][0]["data"]
    ops["message"]["body"]["attester_slashings"] = [
        {"attestation_1": _indexed([1, 4, 9], "d1", d), "attestation_2": _indexed([4, 9, 20, 33, 61], "d2", d)}]
    cases.append(("capella_attester_slashing", ops, "k3", None, None))
    for name, sig, err in (("sync_empty_infinity", INFINITY_SIG, None),
                           ("sync_empty_not_infinity", k3["signed_block"]["message"]["body"]["sync_aggregate"]
                            ["sync_committee_signature"], "Empty sync committee signature is not infinity")):
        blk = copy.deepcopy(k3["signed_block"])
        blk["message"]["body"]["sync_aggregate"] = {"sync_committee_bits": "0x" + "00" * 64,
                                                    "sync_committee_signature": sig}
        cases.append((name, blk, "k3", None, err))
    altair = copy.deepcopy(k3["signed_block"])
    for k in ("execution_payload", "bls_to_execution_changes"):
        del altair["message"]["body"][k]
    cases.append(("altair", altair, "k3", {"altair": 0}, None))
    bell = copy.deepcopy(_operations_block(k3))       # carries a BLS change: not a set before capella
    del bell["message"]["body"]["execution_payload"]["withdrawals"]
    cases.append(("bellatrix", bell, "k3", {"altair": 0, "bellatrix": 0}, None))
    for b in load_json("backfill_phase0.json")["blocks"]:
        cases.append((f"phase0_slot{b['message']['slot']}", b, "mainnet", "mainnet", None))
    return cases


def _case_state(k3, kind, forks):
    if kind == "mainnet":
        return mainnet_phase0_state()
    st = k3_state(k3, pubkey=lambda b: b)
    if forks is not None:
        st.fork_seq = SR.fork_schedule(forks.get("altair", SR.FAR_FUTURE), forks.get("bellatrix", SR.FAR_FUTURE),
                                       forks.get("capella", SR.FAR_FUTURE))
    return st


def python_fork_case_roots(k3, merkleize):
    out = []
    for name, blk, kind, forks, err in fork_cases(k3):
        try:
            sets = SR.resolve(SR.block_signature_sets(blk, _case_state(k3, kind, forks)), merkleize)
            out.append({"case": name, "sets": [{"name": s.name, "root": s.signing_root.hex(),
                                                "keys": [bytes(k).hex() for k in s.pubkeys]} for s in sets]})
        except ValueError as e:
            out.append({"case": name, "error": str(e)})
    return out


def test_backfill_phase0_block_roots_cpu():
    """phase0 BeaconBlock walk pinned by the reference's mainnet blocks: hash_tree_root(message)
    of each block is the next block's parent_root (sync/backfill/verify.ts:24-40); the walk's sets
    are randao, attestations, proposer (no sync aggregate before altair, index.ts:46-58), the
    proposer root under the mainnet GVR of verify.test.ts:19-22"""
    import oracle.ssz as S
    blocks = load_json("backfill_phase0.json")["blocks"]
    st = mainnet_phase0_state()
    roots = SR.evaluate([SR.beacon_block(b["message"], st.fork_seq(int(b["message"]["slot"]))) for b in blocks],
                        cpu_merkleize)
    for i in range(3):
        assert "0x" + roots[i].hex() == blocks[i + 1]["message"]["parent_root"]
    dom = S.compute_domain(S.DOMAIN_BEACON_PROPOSER, bytes(4), bytes.fromhex(MAINNET_GVR))
    for b, r in zip(blocks, roots):
        sets = SR.resolve(SR.block_signature_sets(b, st), cpu_merkleize)
        assert [s.name for s in sets] == ["randao"] + ["attestation"] * len(b["message"]["body"]["attestations"]) + \
            ["proposer"]
        assert sets[-1].signing_root == S.signing_root(r, dom)
        assert sets[-1].signature.hex() == b["signature"][2:]
        assert sets[-1].pubkeys == [int(b["message"]["proposer_index"]).to_bytes(4, "big")]


def test_fork_cases_match_oracle():
    """every fork case against oracle/ssz.py: the proposer root over the fork's BeaconBlock, the
    sync-aggregate rule (processSyncCommittee.ts:93-101), the attester slashings' IndexedAttestation
    (packed uint64 indices), no BLS-change set before capella"""
    import oracle.ssz as S
    k3 = load_json("k3_devnet.json")
    got = {c["case"]: c for c in python_fork_case_roots(k3, cpu_merkleize)}
    forkid = {None: S.FORK_CAPELLA, "mainnet": S.FORK_PHASE0}
    for name, blk, kind, forks, err in fork_cases(k3):
        g = got[name]
        if err:
            assert g == {"case": name, "error": err}
            continue
        f = forkid.get(forks) if not isinstance(forks, dict) else (
            S.FORK_BELLATRIX if "bellatrix" in forks else S.FORK_ALTAIR)
        names = [s["name"] for s in g["sets"]]
        assert ("sync_aggregate" in names) == (f >= S.FORK_ALTAIR and name != "sync_empty_infinity"), name
        assert ("bls_to_execution_change" in names) == (f >= S.FORK_CAPELLA and name == "capella_attester_slashing")
        st = _case_state(k3, kind, forks)
        m = blk["message"]
        dom = st.domain(S.DOMAIN_BEACON_PROPOSER, int(m["slot"]) // 32)
        prop = [s for s in g["sets"] if s["name"] == "proposer"][0]
        assert prop["root"] == S.signing_root(S.beacon_block(m, f), dom).hex(), name
    # the slashing block: both IndexedAttestations inside the body root, their sets' keys in order
    g = got["capella_attester_slashing"]
    sl = [s for s in g["sets"] if s["name"] == "attester_slashing"]
    keys = [bytes.fromhex(k) for k in k3["state_view"]["validator_pubkeys48"]]
    assert [s["keys"] for s in sl] == [[keys[i].hex() for i in (1, 4, 9)], [keys[i].hex() for i in (4, 9, 20, 33, 61)]]
    # a one-chunk-per-index (unpacked) list would give another body root
    ia = fork_cases(k3)[0][1]["message"]["body"]["attester_slashings"][0]["attestation_2"]
    unpacked = S.mix_in_length(S.merkleize([S.uint64(int(i)) for i in ia["attesting_indices"]], 2048), 5)
    assert unpacked != S.list_of_uint64([int(i) for i in ia["attesting_indices"]], 2048)


@pytest.mark.gpu
def test_fork_cases_gpu_roots(engine):
    """the fork cases through lb_merkleize equal the hashlib walk's; the backfill chain's parent
    roots reproduced on the GPU"""
    k3 = load_json("k3_devnet.json")
    assert python_fork_case_roots(k3, SR.GpuMerkleizer(engine)) == python_fork_case_roots(k3, cpu_merkleize)
    blocks = load_json("backfill_phase0.json")["blocks"]
    roots = SR.evaluate([SR.beacon_block(b["message"], SR.FORK_PHASE0) for b in blocks], SR.GpuMerkleizer(engine))
    assert ["0x" + r.hex() for r in roots[:3]] == [b["message"]["parent_root"] for b in blocks[1:]]
