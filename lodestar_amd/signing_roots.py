"""Signing-root production on the GPU: the signature sets of a block.

Mirrors getBlockSignatureSets (packages/state-transition/src/signatureSets/index.ts:26-72) for
phase0, altair, bellatrix and capella blocks, dispatched on the fork of the block's slot like
the reference (config.getForkSeq(slot), index.ts:46-70): proposer (signatureSets/proposer.ts,
the fork's BeaconBlock type), randao (randao.ts), proposer and attester slashings
(proposerSlashings.ts, attesterSlashings.ts), attestations (indexedAttestation.ts), voluntary
exits (voluntaryExits.ts), the sync aggregate from altair on (block/processSyncCommittee.ts:58-111,
including its "Empty sync committee signature is not infinity" rejection) and BLS-to-execution
changes from capella on (blsToExecutionChange.ts).  Each set's signing root is
computeSigningRoot(type, value, domain) = hash_tree_root(SigningData{hash_tree_root(value),
domain}) (src/util/signingRoot.ts:7-13).

The SSZ containers are walked here, on the host, into merkle TREES (chunk lists, depth = the
type's limit, optional length mix-in); every tree of one dependency level is hashed in ONE GPU
launch (lb_merkleize, lodestar_amd/csrc/lb_ssz.h), so a 32-block range-sync segment costs a
handful of launches however many attestations it carries.  Domains come from the fork data like
the reference's cached getDomain (packages/config/src/genesisConfig/index.ts:27-54): four
SHA-256 calls per fork, computed once on the host.
"""
from __future__ import annotations

import ctypes
import hashlib
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Union

import numpy as np

SLOTS_PER_EPOCH = 32
SYNC_COMMITTEE_SIZE = 512
MAX_VALIDATORS_PER_COMMITTEE = 2048
NO_MIX = 0xFFFFFFFFFFFFFFFF

DOMAIN_BEACON_PROPOSER = bytes.fromhex("00000000")
DOMAIN_BEACON_ATTESTER = bytes.fromhex("01000000")
DOMAIN_RANDAO = bytes.fromhex("02000000")
DOMAIN_VOLUNTARY_EXIT = bytes.fromhex("04000000")
DOMAIN_SYNC_COMMITTEE = bytes.fromhex("07000000")
DOMAIN_BLS_TO_EXECUTION_CHANGE = bytes.fromhex("0a000000")

# ForkSeq (packages/params/src/forkName.ts)
FORK_PHASE0, FORK_ALTAIR, FORK_BELLATRIX, FORK_CAPELLA = range(4)
FAR_FUTURE = 2 ** 64 - 1
# mainnet fork epochs (config/src/chainConfig/presets/mainnet.ts:34-42; capella unscheduled there)
MAINNET_FORK_EPOCHS = (74240, 144896, FAR_FUTURE)
# G2_POINT_AT_INFINITY (params/src/index.ts): the compressed infinity flag byte, then zeros
G2_POINT_AT_INFINITY = bytes([0xC0]) + bytes(95)


def fork_schedule(altair_epoch: int, bellatrix_epoch: int = FAR_FUTURE,
                  capella_epoch: int = FAR_FUTURE) -> Callable[[int], int]:
    """slot -> ForkSeq, as config.getForkSeq(slot) for the given fork epochs."""
    def seq(slot: int) -> int:
        ep = int(slot) // SLOTS_PER_EPOCH
        return (FORK_CAPELLA if ep >= capella_epoch else FORK_BELLATRIX if ep >= bellatrix_epoch
                else FORK_ALTAIR if ep >= altair_epoch else FORK_PHASE0)
    return seq


# ------------------------------------------------------------------ merkle trees
class Tree:
    """hash_tree_root of `parts` (32-byte chunks or Trees) padded to 2^depth leaves, optionally
    mixed with a length."""
    __slots__ = ("parts", "depth", "mix", "root", "height")

    def __init__(self, parts: Sequence[Union[bytes, "Tree"]], depth: int, mix: Optional[int] = None):
        assert len(parts) <= (1 << depth)
        self.parts = list(parts)
        self.depth = depth
        self.mix = mix
        self.root: Optional[bytes] = None
        self.height = 1 + max((p.height for p in self.parts if isinstance(p, Tree)), default=0)


Node = Union[bytes, Tree]


def _ceil_log2(n: int) -> int:
    return max(n - 1, 0).bit_length()


def evaluate(nodes: Sequence[Node], merkleize: Callable[[List[Tree]], List[bytes]]) -> List[bytes]:
    """Roots of `nodes`: all trees of one height go to `merkleize` together (one GPU launch)."""
    by_h: Dict[int, List[Tree]] = {}
    seen = set()

    def walk(t):
        if isinstance(t, Tree) and id(t) not in seen:
            seen.add(id(t))
            by_h.setdefault(t.height, []).append(t)
            for p in t.parts:
                walk(p)
    for n in nodes:
        walk(n)
    for h in sorted(by_h):
        trees = by_h[h]
        for t, r in zip(trees, merkleize(trees)):
            t.root = r
    return [n if isinstance(n, bytes) else n.root for n in nodes]


def leaves(t: Tree) -> List[bytes]:
    return [p if isinstance(p, bytes) else p.root for p in t.parts]


class GpuMerkleizer:
    """Trees of one level -> lb_merkleize on the engine's GPU."""

    def __init__(self, engine):
        self.engine = engine
        self.launches = 0

    def __call__(self, trees: List[Tree]) -> List[bytes]:
        off = np.zeros(len(trees) + 1, dtype=np.uint32)
        chunks = []
        for k, t in enumerate(trees):
            ls = leaves(t)
            chunks.extend(ls)
            off[k + 1] = off[k] + len(ls)
        depth = np.asarray([t.depth for t in trees], dtype=np.uint32)
        mix = np.asarray([NO_MIX if t.mix is None else t.mix for t in trees], dtype=np.uint64)
        buf = np.frombuffer(b"".join(chunks), dtype=np.uint8).copy() if chunks else np.zeros(32, np.uint8)
        out = np.zeros(32 * max(len(trees), 1), dtype=np.uint8)
        P = lambda a, t: a.ctypes.data_as(ctypes.POINTER(t))  # noqa: E731
        from .engine import _check
        _check(self.engine.lib.lb_merkleize(self.engine.h, len(trees), P(off, ctypes.c_uint32), P(buf, ctypes.c_uint8),
                                            P(depth, ctypes.c_uint32), P(mix, ctypes.c_uint64),
                                            P(out, ctypes.c_uint8)))
        self.launches += 1
        ob = out.tobytes()
        return [ob[32 * k:32 * k + 32] for k in range(len(trees))]


# ------------------------------------------------------------------ SSZ types -> trees
def hx(s: str) -> bytes:
    return bytes.fromhex(s[2:] if s.startswith("0x") else s)


def pack(b: bytes) -> List[bytes]:
    b = bytes(b)
    if len(b) % 32:
        b += bytes(32 - len(b) % 32)
    return [b[i:i + 32] for i in range(0, len(b), 32)]


def uint64(x) -> bytes:
    return int(x).to_bytes(8, "little") + bytes(24)


def uint256(x) -> bytes:
    return int(x).to_bytes(32, "little")


def bytes_n(b: bytes) -> Node:
    """ByteVector[N]: one chunk (N <= 32) or a tree over its chunks."""
    ch = pack(b)
    return ch[0] if len(ch) == 1 else Tree(ch, _ceil_log2(len(ch)))


def uint64_list(values: Sequence[int], limit: int) -> Tree:
    """List[uint64, limit]: basic values packed 4 per 32-byte chunk, limit ceil(8*limit/32) chunks."""
    raw = b"".join(int(v).to_bytes(8, "little") for v in values)
    return Tree(pack(raw), _ceil_log2((8 * limit + 31) // 32), mix=len(values))


def byte_list(b: bytes, limit: int) -> Tree:
    return Tree(pack(b), _ceil_log2((limit + 31) // 32), mix=len(b))


def _bits_to_bytes(bits: Sequence[int]) -> bytes:
    v = 0
    for i, x in enumerate(bits):
        v |= (x & 1) << i
    return v.to_bytes((len(bits) + 7) // 8, "little") if bits else b""


def bitlist(bits: Sequence[int], limit: int) -> Tree:
    return Tree(pack(_bits_to_bytes(bits)), _ceil_log2((limit + 255) // 256), mix=len(bits))


def bitvector(bits: Sequence[int]) -> Node:
    ch = pack(_bits_to_bytes(bits))
    return Tree(ch, _ceil_log2((len(bits) + 255) // 256)) if len(ch) > 1 else ch[0]


def container(fields: Sequence[Node]) -> Tree:
    return Tree(fields, _ceil_log2(len(fields)))


def list_of(items: Sequence[Node], limit: int) -> Tree:
    return Tree(items, _ceil_log2(limit), mix=len(items))


def bits_from_bitlist_hex(h: str) -> List[int]:
    v = int.from_bytes(hx(h), "little")
    return [(v >> i) & 1 for i in range(v.bit_length() - 1)]


def bits_from_bitvector_hex(h: str, n: int) -> List[int]:
    v = int.from_bytes(hx(h), "little")
    return [(v >> i) & 1 for i in range(n)]


def checkpoint(c) -> Tree:
    return container([uint64(c["epoch"]), hx(c["root"])])


def attestation_data(d) -> Tree:
    return container([uint64(d["slot"]), uint64(d["index"]), hx(d["beacon_block_root"]), checkpoint(d["source"]),
                      checkpoint(d["target"])])


def indexed_attestation(a) -> Tree:
    return container([uint64_list([int(i) for i in a["attesting_indices"]], MAX_VALIDATORS_PER_COMMITTEE),
                      attestation_data(a["data"]), bytes_n(hx(a["signature"]))])


def attestation(a) -> Tree:
    return container([bitlist(bits_from_bitlist_hex(a["aggregation_bits"]), 2048), attestation_data(a["data"]),
                      bytes_n(hx(a["signature"]))])


def block_header(h) -> Tree:
    return container([uint64(h["slot"]), uint64(h["proposer_index"]), hx(h["parent_root"]), hx(h["state_root"]),
                      hx(h["body_root"])])


def signed_header(s) -> Tree:
    return container([block_header(s["message"]), bytes_n(hx(s["signature"]))])


def voluntary_exit(e) -> Tree:
    return container([uint64(e["epoch"]), uint64(e["validator_index"])])


def bls_to_execution_change(c) -> Tree:
    return container([uint64(c["validator_index"]), bytes_n(hx(c["from_bls_pubkey"])),
                      bytes_n(hx(c["to_execution_address"]))])


def withdrawal(w) -> Tree:
    return container([uint64(w["index"]), uint64(w["validator_index"]), bytes_n(hx(w["address"])), uint64(w["amount"])])


def _execution_payload_fields(p) -> List[Node]:
    return [hx(p["parent_hash"]), bytes_n(hx(p["fee_recipient"])), hx(p["state_root"]), hx(p["receipts_root"]),
            bytes_n(hx(p["logs_bloom"])), hx(p["prev_randao"]), uint64(p["block_number"]), uint64(p["gas_limit"]),
            uint64(p["gas_used"]), uint64(p["timestamp"]), byte_list(hx(p["extra_data"]), 32),
            uint256(int(p["base_fee_per_gas"])), hx(p["block_hash"]),
            list_of([byte_list(hx(t), 2 ** 30) for t in p["transactions"]], 2 ** 20)]


def execution_payload_bellatrix(p) -> Tree:
    return container(_execution_payload_fields(p))


def execution_payload_capella(p) -> Tree:
    return container(_execution_payload_fields(p) + [list_of([withdrawal(w) for w in p["withdrawals"]], 16)])


def beacon_block_body(b, fork: int) -> Tree:
    """BeaconBlockBody of `fork` (types/src/{phase0,altair,bellatrix,capella}/sszTypes.ts): phase0's
    8 fields, + sync_aggregate (altair), + execution_payload (bellatrix), capella's payload with
    withdrawals + bls_to_execution_changes."""
    fields: List[Node] = [
        bytes_n(hx(b["randao_reveal"])),
        container([hx(b["eth1_data"]["deposit_root"]), uint64(b["eth1_data"]["deposit_count"]),
                   hx(b["eth1_data"]["block_hash"])]),
        hx(b["graffiti"]),
        list_of([container([signed_header(s["signed_header_1"]), signed_header(s["signed_header_2"])])
                 for s in b["proposer_slashings"]], 16),
        list_of([container([indexed_attestation(s["attestation_1"]), indexed_attestation(s["attestation_2"])])
                 for s in b["attester_slashings"]], 2),
        list_of([attestation(a) for a in b["attestations"]], 128),
        list_of([_deposit(d) for d in b["deposits"]], 16),
        list_of([container([voluntary_exit(e["message"]), bytes_n(hx(e["signature"]))])
                 for e in b["voluntary_exits"]], 16)]
    if fork >= FORK_ALTAIR:
        sa = b["sync_aggregate"]
        fields.append(container([bitvector(bits_from_bitvector_hex(sa["sync_committee_bits"], SYNC_COMMITTEE_SIZE)),
                                 bytes_n(hx(sa["sync_committee_signature"]))]))
    if fork == FORK_BELLATRIX:
        fields.append(execution_payload_bellatrix(b["execution_payload"]))
    if fork >= FORK_CAPELLA:
        fields.append(execution_payload_capella(b["execution_payload"]))
        fields.append(list_of([container([bls_to_execution_change(c["message"]), bytes_n(hx(c["signature"]))])
                               for c in b["bls_to_execution_changes"]], 16))
    return container(fields)


def _deposit(d) -> Tree:
    data = d["data"]
    return container([Tree([hx(p) for p in d["proof"]], 6),  # Vector[Bytes32, 33] -> 64 leaves
                      container([bytes_n(hx(data["pubkey"])), hx(data["withdrawal_credentials"]),
                                 uint64(data["amount"]), bytes_n(hx(data["signature"]))])])


def beacon_block(m, fork: int) -> Tree:
    """BeaconBlock of `fork` (config.getForkTypes(slot).BeaconBlock, proposer.ts:22-24)."""
    return container([uint64(m["slot"]), uint64(m["proposer_index"]), hx(m["parent_root"]), hx(m["state_root"]),
                      beacon_block_body(m["body"], fork)])


def beacon_block_body_capella(b) -> Tree:
    return beacon_block_body(b, FORK_CAPELLA)


def beacon_block_capella(m) -> Tree:
    return beacon_block(m, FORK_CAPELLA)


def signing_tree(obj: Node, domain: bytes) -> Tree:
    """computeSigningRoot: SigningData{object_root, domain} (src/util/signingRoot.ts:7-13)."""
    return container([obj, domain])


def compute_domain(domain_type: bytes, fork_version: bytes, genesis_validators_root: bytes) -> bytes:
    fork_data_root = hashlib.sha256(fork_version + bytes(28) + genesis_validators_root).digest()
    return domain_type + fork_data_root[:28]


# ------------------------------------------------------------------ block signature sets
@dataclass
class StateView:
    """What getBlockSignatureSets reads from the (cached) beacon state."""
    genesis_validators_root: bytes
    fork_previous_version: bytes
    fork_current_version: bytes
    fork_epoch: int
    pubkey: Callable[[int], object]                     # index2pubkey (epochContext.index2pubkey)
    beacon_committee: Callable[[int, int], List[int]]   # epochContext.getBeaconCommittee(slot, index)
    sync_committee: Callable[[], List[object]]          # current sync committee pubkeys (512)
    slot: Optional[int] = None                          # state.slot (None: the block's slot)
    # bls.PublicKey.fromBytes(bytes48, affine, true) for keys carried in the block itself
    # (BLS-to-execution changes, blsToExecutionChange.ts:30)
    key_from_bytes: Callable[[bytes], object] = lambda b: b
    # config.getForkSeq(slot): capella for every slot unless a schedule is given (fork_schedule)
    fork_seq: Callable[[int], int] = lambda slot: FORK_CAPELLA

    def domain(self, domain_type: bytes, epoch: int) -> bytes:
        """config.getDomain(state.slot, type, messageSlot) (config/src/genesisConfig/index.ts:27-54):
        the state's previous fork version for messages before its fork epoch, else the current one"""
        v = self.fork_previous_version if epoch < self.fork_epoch else self.fork_current_version
        return compute_domain(domain_type, v, self.genesis_validators_root)


@dataclass
class BlockSet:
    name: str
    type: str                # "single" | "aggregate"
    pubkeys: List[object]
    signing_root: object     # Tree / bytes until evaluated, then bytes
    signature: bytes


def block_signature_sets(signed_block, state: StateView, skip_proposer_signature: bool = False) -> List[BlockSet]:
    """getBlockSignatureSets (signatureSets/index.ts:26-72) for one SignedBeaconBlock of any fork
    up to capella (JSON as served by the beacon API), in the reference's order: randao, proposer
    slashings, attester slashings, attestations, voluntary exits, proposer, then by the fork of the
    block's slot the sync aggregate (altair on) and BLS-to-execution changes (capella on).  Signing
    roots are left as trees: evaluate() hashes the trees of many blocks together.  Raises
    ValueError("Empty sync committee signature is not infinity") like processSyncCommittee.ts:93-101."""
    m = signed_block["message"]
    b = m["body"]
    slot = int(m["slot"])
    fork = state.fork_seq(slot)
    epoch = slot // SLOTS_PER_EPOCH
    state_epoch = (slot if state.slot is None else int(state.slot)) // SLOTS_PER_EPOCH
    out: List[BlockSet] = []
    # randao.ts:26
    out.append(BlockSet("randao", "single", [state.pubkey(int(m["proposer_index"]))],
                        signing_tree(uint64(epoch), state.domain(DOMAIN_RANDAO, epoch)), hx(b["randao_reveal"])))
    # proposerSlashings.ts:14-37: both headers are checked against signedHeader1's proposer
    for s in b["proposer_slashings"]:
        pk = state.pubkey(int(s["signed_header_1"]["message"]["proposer_index"]))
        for h in (s["signed_header_1"], s["signed_header_2"]):
            ep = int(h["message"]["slot"]) // SLOTS_PER_EPOCH
            out.append(BlockSet("proposer_slashing", "single", [pk],
                                signing_tree(block_header(h["message"]), state.domain(DOMAIN_BEACON_PROPOSER, ep)),
                                hx(h["signature"])))
    # attesterSlashings.ts:32
    for s in b["attester_slashings"]:
        for ia in (s["attestation_1"], s["attestation_2"]):
            ep = int(ia["data"]["target"]["epoch"])
            out.append(BlockSet("attester_slashing", "aggregate", [state.pubkey(int(i)) for i in ia["attesting_indices"]],
                                signing_tree(attestation_data(ia["data"]), state.domain(DOMAIN_BEACON_ATTESTER, ep)),
                                hx(ia["signature"])))
    # indexedAttestation.ts:6-37
    for a in b["attestations"]:
        d = a["data"]
        committee = state.beacon_committee(int(d["slot"]), int(d["index"]))
        bits = bits_from_bitlist_hex(a["aggregation_bits"])
        idx = sorted(v for v, bit in zip(committee, bits) if bit)
        out.append(BlockSet("attestation", "aggregate", [state.pubkey(v) for v in idx],
                            signing_tree(attestation_data(d), state.domain(DOMAIN_BEACON_ATTESTER,
                                                                           int(d["target"]["epoch"]))),
                            hx(a["signature"])))
    # voluntaryExits.ts:28
    for e in b["voluntary_exits"]:
        out.append(BlockSet("voluntary_exit", "single", [state.pubkey(int(e["message"]["validator_index"]))],
                            signing_tree(voluntary_exit(e["message"]),
                                         state.domain(DOMAIN_VOLUNTARY_EXIT, int(e["message"]["epoch"]))),
                            hx(e["signature"])))
    # proposer.ts:20 (index.ts:86-88: after the operations)
    if not skip_proposer_signature:
        out.append(BlockSet("proposer", "single", [state.pubkey(int(m["proposer_index"]))],
                            signing_tree(beacon_block(m, fork), state.domain(DOMAIN_BEACON_PROPOSER, epoch)),
                            hx(signed_block["signature"])))
    if fork >= FORK_ALTAIR:
        s = sync_committee_set(m, state)
        if s is not None:
            out.append(s)
    if fork < FORK_CAPELLA:
        return out
    # blsToExecutionChange.ts:23: getDomain(state.slot, DOMAIN_BLS_TO_EXECUTION_CHANGE), i.e. the
    # fork of the state's own epoch; the key is the message's from_bls_pubkey (48 B compressed)
    for c in b["bls_to_execution_changes"]:
        dom = state.domain(DOMAIN_BLS_TO_EXECUTION_CHANGE, state_epoch)
        out.append(BlockSet("bls_to_execution_change", "single", [state.key_from_bytes(hx(c["message"]["from_bls_pubkey"]))],
                            signing_tree(bls_to_execution_change(c["message"]), dom), hx(c["signature"])))
    return out


def sync_committee_set(m, state: StateView) -> Optional[BlockSet]:
    """getSyncCommitteeSignatureSet (block/processSyncCommittee.ts:58-111): the participants' keys
    over the parent root; no participant -> None if the signature is G2_POINT_AT_INFINITY, else the
    reference's error (the block is rejected)."""
    sa = m["body"]["sync_aggregate"]
    sig = hx(sa["sync_committee_signature"])
    bits = bits_from_bitvector_hex(sa["sync_committee_bits"], SYNC_COMMITTEE_SIZE)
    keys = [k for k, bit in zip(state.sync_committee(), bits) if bit]
    if not keys:
        if sig == G2_POINT_AT_INFINITY:
            return None
        raise ValueError("Empty sync committee signature is not infinity")
    prev = max(int(m["slot"]), 1) - 1
    return BlockSet("sync_aggregate", "aggregate", keys,
                    signing_tree(hx(m["parent_root"]), state.domain(DOMAIN_SYNC_COMMITTEE, prev // SLOTS_PER_EPOCH)),
                    sig)


def resolve(sets: Sequence[BlockSet], merkleize) -> List[BlockSet]:
    """Hashes every pending signing root of `sets` (any number of blocks) level by level."""
    roots = evaluate([s.signing_root for s in sets], merkleize)
    for s, r in zip(sets, roots):
        s.signing_root = r
    return list(sets)
