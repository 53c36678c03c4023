"""SSZ hash_tree_root for the containers behind the hot path's signing roots -- TEST
INFRASTRUCTURE (golden-vector generation and the CPU checker of the GPU merkleization), never on
the product path.

A from-scratch restatement of the consensus-spec SSZ merkleization (the reference computes these
with @chainsafe/ssz through @lodestar/types: ssz.phase0.SigningData.hashTreeRoot in
packages/state-transition/src/util/signingRoot.ts:7-13, BeaconBlock / AttestationData roots in
src/signatureSets/*.ts) and of the domain / committee helpers the block's signature sets need:
compute_domain / getDomain (packages/config/src/genesisConfig/index.ts:27-54), the swap-or-not
shuffle (state-transition/src/util/shuffle.ts), get_beacon_committee (epochContext).  Block
containers for phase0 / altair / bellatrix / capella (packages/types/src/{phase0,altair,bellatrix,
capella}/sszTypes.ts), pinned by the capella devnet fixture K3 and the first four mainnet phase0
blocks of beacon-node/test/unit/sync/backfill/blocks.json.  Mainnet preset
constants.
"""
from __future__ import annotations

import hashlib
from typing import List, Sequence

SLOTS_PER_EPOCH = 32
SHUFFLE_ROUND_COUNT = 90
TARGET_COMMITTEE_SIZE = 128
MAX_COMMITTEES_PER_SLOT = 64
EPOCHS_PER_HISTORICAL_VECTOR = 65536
SLOTS_PER_HISTORICAL_ROOT = 8192
EPOCHS_PER_SLASHINGS_VECTOR = 8192
MIN_SEED_LOOKAHEAD = 1
SYNC_COMMITTEE_SIZE = 512
MAX_VALIDATORS_PER_COMMITTEE = 2048
FAR_FUTURE_EPOCH = 2 ** 64 - 1

DOMAIN_BEACON_PROPOSER = bytes.fromhex("00000000")
DOMAIN_BEACON_ATTESTER = bytes.fromhex("01000000")
DOMAIN_RANDAO = bytes.fromhex("02000000")
DOMAIN_VOLUNTARY_EXIT = bytes.fromhex("04000000")
DOMAIN_SYNC_COMMITTEE = bytes.fromhex("07000000")
DOMAIN_BLS_TO_EXECUTION_CHANGE = bytes.fromhex("0a000000")

ZERO = bytes(32)


def sha256(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


_ZH = [ZERO]
for _ in range(64):
    _ZH.append(sha256(_ZH[-1] + _ZH[-1]))


def merkleize(chunks: Sequence[bytes], limit: int = None) -> bytes:
    """Root of the chunks padded with zero chunks to next_pow2(limit or len) leaves."""
    n = len(chunks)
    cap = max(limit if limit is not None else n, 1)
    depth = (cap - 1).bit_length()
    assert n <= (1 << depth)
    layer = list(chunks)
    for d in range(depth):
        if len(layer) % 2:
            layer.append(_ZH[d])
        layer = [sha256(layer[i] + layer[i + 1]) for i in range(0, len(layer), 2)]
    return layer[0] if layer else _ZH[depth]


def mix_in_length(root: bytes, n: int) -> bytes:
    return sha256(root + n.to_bytes(32, "little"))


def pack(b: bytes) -> List[bytes]:
    b = bytes(b)
    if len(b) % 32:
        b += bytes(32 - len(b) % 32)
    return [b[i:i + 32] for i in range(0, len(b), 32)]


def uint64(x: int) -> bytes:
    return int(x).to_bytes(8, "little") + bytes(24)


def uint256(x: int) -> bytes:
    return int(x).to_bytes(32, "little")


def bytes_n(b: bytes) -> bytes:
    """ByteVector[N] (N <= 32: one chunk; longer: merkleized chunks)."""
    return merkleize(pack(b))


def byte_list(b: bytes, limit: int) -> bytes:
    return mix_in_length(merkleize(pack(b), (limit + 31) // 32), len(b))


def bitlist(bits: Sequence[int], limit: int) -> bytes:
    v = 0
    for i, x in enumerate(bits):
        v |= (x & 1) << i
    raw = v.to_bytes((len(bits) + 7) // 8, "little") if bits else b""
    return mix_in_length(merkleize(pack(raw), (limit + 255) // 256), len(bits))


def bitvector(bits: Sequence[int]) -> bytes:
    v = 0
    for i, x in enumerate(bits):
        v |= (x & 1) << i
    return merkleize(pack(v.to_bytes((len(bits) + 7) // 8, "little")), (len(bits) + 255) // 256)


def container(field_roots: Sequence[bytes]) -> bytes:
    return merkleize(field_roots)


def list_of(roots: Sequence[bytes], limit: int) -> bytes:
    return mix_in_length(merkleize(roots, limit), len(roots))


def list_of_uint64(values: Sequence[int], limit: int) -> bytes:
    """List[uint64, limit]: basic values packed 4 per chunk, limit ceil(limit*8/32) chunks."""
    raw = b"".join(int(v).to_bytes(8, "little") for v in values)
    return mix_in_length(merkleize(pack(raw), (limit * 8 + 31) // 32), len(values))


def bits_from_hex_bitlist(h: str) -> List[int]:
    """SSZ Bitlist serialisation (length marker bit) -> list of bits."""
    b = bytes.fromhex(h[2:] if h.startswith("0x") else h)
    v = int.from_bytes(b, "little")
    n = v.bit_length() - 1
    return [(v >> i) & 1 for i in range(n)]


def bits_from_hex_bitvector(h: str, n: int) -> List[int]:
    b = bytes.fromhex(h[2:] if h.startswith("0x") else h)
    v = int.from_bytes(b, "little")
    return [(v >> i) & 1 for i in range(n)]


def hx(s: str) -> bytes:
    return bytes.fromhex(s[2:] if s.startswith("0x") else s)


# ------------------------------------------------------------------ containers (JSON in, root out)
def checkpoint(c) -> bytes:
    return container([uint64(int(c["epoch"])), hx(c["root"])])


def attestation_data(d) -> bytes:
    return container([uint64(int(d["slot"])), uint64(int(d["index"])), hx(d["beacon_block_root"]),
                      checkpoint(d["source"]), checkpoint(d["target"])])


def attestation(a) -> bytes:
    return container([bitlist(bits_from_hex_bitlist(a["aggregation_bits"]), 2048), attestation_data(a["data"]),
                      bytes_n(hx(a["signature"]))])


def eth1_data(e) -> bytes:
    return container([hx(e["deposit_root"]), uint64(int(e["deposit_count"])), hx(e["block_hash"])])


def withdrawal(w) -> bytes:
    return container([uint64(int(w["index"])), uint64(int(w["validator_index"])), bytes_n(hx(w["address"])),
                      uint64(int(w["amount"]))])


def execution_payload_capella(p) -> bytes:
    txs = [byte_list(hx(t), 2 ** 30) for t in p["transactions"]]
    return container([
        hx(p["parent_hash"]), bytes_n(hx(p["fee_recipient"])), hx(p["state_root"]), hx(p["receipts_root"]),
        bytes_n(hx(p["logs_bloom"])), hx(p["prev_randao"]), uint64(int(p["block_number"])),
        uint64(int(p["gas_limit"])), uint64(int(p["gas_used"])), uint64(int(p["timestamp"])),
        byte_list(hx(p["extra_data"]), 32), uint256(int(p["base_fee_per_gas"])), hx(p["block_hash"]),
        list_of(txs, 2 ** 20), list_of([withdrawal(w) for w in p["withdrawals"]], 16)])


def block_header(h) -> bytes:
    """phase0 BeaconBlockHeader"""
    return container([uint64(int(h["slot"])), uint64(int(h["proposer_index"])), hx(h["parent_root"]),
                      hx(h["state_root"]), hx(h["body_root"])])


def signed_block_header(s) -> bytes:
    return container([block_header(s["message"]), bytes_n(hx(s["signature"]))])


def voluntary_exit(e) -> bytes:
    return container([uint64(int(e["epoch"])), uint64(int(e["validator_index"]))])


def bls_to_execution_change(c) -> bytes:
    """capella BLSToExecutionChange"""
    return container([uint64(int(c["validator_index"])), bytes_n(hx(c["from_bls_pubkey"])),
                      bytes_n(hx(c["to_execution_address"]))])


def execution_payload_bellatrix(p) -> bytes:
    txs = [byte_list(hx(t), 2 ** 30) for t in p["transactions"]]
    return container([
        hx(p["parent_hash"]), bytes_n(hx(p["fee_recipient"])), hx(p["state_root"]), hx(p["receipts_root"]),
        bytes_n(hx(p["logs_bloom"])), hx(p["prev_randao"]), uint64(int(p["block_number"])),
        uint64(int(p["gas_limit"])), uint64(int(p["gas_used"])), uint64(int(p["timestamp"])),
        byte_list(hx(p["extra_data"]), 32), uint256(int(p["base_fee_per_gas"])), hx(p["block_hash"]),
        list_of(txs, 2 ** 20)])


def indexed_attestation(a) -> bytes:
    """phase0 IndexedAttestation: attesting_indices is List[ValidatorIndex, 2048] of packed uint64"""
    return container([list_of_uint64([int(i) for i in a["attesting_indices"]], MAX_VALIDATORS_PER_COMMITTEE),
                      attestation_data(a["data"]), bytes_n(hx(a["signature"]))])


def attester_slashing(s) -> bytes:
    return container([indexed_attestation(s["attestation_1"]), indexed_attestation(s["attestation_2"])])


def deposit(d) -> bytes:
    """phase0 Deposit: proof Vector[Bytes32, 33] + DepositData"""
    data = d["data"]
    return container([merkleize([hx(x) for x in d["proof"]], 33),
                      container([bytes_n(hx(data["pubkey"])), hx(data["withdrawal_credentials"]),
                                 uint64(int(data["amount"])), bytes_n(hx(data["signature"]))])])


def sync_aggregate(sa) -> bytes:
    return container([bitvector(bits_from_hex_bitvector(sa["sync_committee_bits"], SYNC_COMMITTEE_SIZE)),
                      bytes_n(hx(sa["sync_committee_signature"]))])


FORK_PHASE0, FORK_ALTAIR, FORK_BELLATRIX, FORK_CAPELLA = range(4)


def beacon_block_body(b, fork: int) -> bytes:
    """BeaconBlockBody of `fork` (phase0: 8 fields, altair +sync_aggregate, bellatrix
    +execution_payload, capella: capella payload +bls_to_execution_changes)."""
    fields = [
        bytes_n(hx(b["randao_reveal"])), eth1_data(b["eth1_data"]), hx(b["graffiti"]),
        list_of([container([signed_block_header(s["signed_header_1"]), signed_block_header(s["signed_header_2"])])
                 for s in b["proposer_slashings"]], 16),
        list_of([attester_slashing(s) for s in b["attester_slashings"]], 2),
        list_of([attestation(a) for a in b["attestations"]], 128),
        list_of([deposit(d) for d in b["deposits"]], 16),
        list_of([container([voluntary_exit(e["message"]), bytes_n(hx(e["signature"]))])
                 for e in b["voluntary_exits"]], 16)]
    if fork >= FORK_ALTAIR:
        fields.append(sync_aggregate(b["sync_aggregate"]))
    if fork == FORK_BELLATRIX:
        fields.append(execution_payload_bellatrix(b["execution_payload"]))
    if fork >= FORK_CAPELLA:
        fields.append(execution_payload_capella(b["execution_payload"]))
        fields.append(list_of([container([bls_to_execution_change(c["message"]), bytes_n(hx(c["signature"]))])
                               for c in b["bls_to_execution_changes"]], 16))
    return container(fields)


def beacon_block(m, fork: int) -> bytes:
    return container([uint64(int(m["slot"])), uint64(int(m["proposer_index"])), hx(m["parent_root"]),
                      hx(m["state_root"]), beacon_block_body(m["body"], fork)])


def beacon_block_body_capella(b) -> bytes:
    return beacon_block_body(b, FORK_CAPELLA)


def beacon_block_capella(m) -> bytes:
    return beacon_block(m, FORK_CAPELLA)


def signing_root(object_root: bytes, domain: bytes) -> bytes:
    """compute_signing_root = hash_tree_root(SigningData{object_root, domain})
    (state-transition/src/util/signingRoot.ts:7-13)."""
    return sha256(object_root + domain)


def compute_domain(domain_type: bytes, fork_version: bytes, genesis_validators_root: bytes) -> bytes:
    fork_data_root = sha256(fork_version + bytes(28) + genesis_validators_root)
    return domain_type + fork_data_root[:28]


# ------------------------------------------------------------------ BeaconState (capella) reader
class CapellaState:
    """The fields of a serialized capella BeaconState the signature sets need."""

    def __init__(self, raw: bytes):
        o = 0

        def take(n):
            nonlocal o
            v = raw[o:o + n]
            o += n
            return v
        self.genesis_time = int.from_bytes(take(8), "little")
        self.genesis_validators_root = take(32)
        self.slot = int.from_bytes(take(8), "little")
        self.fork_previous = take(4)
        self.fork_current = take(4)
        self.fork_epoch = int.from_bytes(take(8), "little")
        self.latest_block_header = take(112)        # slot, proposer, parent, state, body roots
        self.block_roots = take(32 * SLOTS_PER_HISTORICAL_ROOT)
        take(32 * SLOTS_PER_HISTORICAL_ROOT)        # state_roots
        take(4)                                     # historical_roots (offset)
        take(72)                                    # eth1_data
        take(4)                                     # eth1_data_votes (offset)
        take(8)                                     # eth1_deposit_index
        off_validators = int.from_bytes(take(4), "little")
        off_balances = int.from_bytes(take(4), "little")
        self.randao_mixes = take(32 * EPOCHS_PER_HISTORICAL_VECTOR)
        take(8 * EPOCHS_PER_SLASHINGS_VECTOR)       # slashings
        take(4)
        take(4)                                     # epoch participation (offsets)
        take(1)                                     # justification_bits
        take(40 * 3)                                # checkpoints
        take(4)                                     # inactivity_scores (offset)
        self.current_sync_committee = [take(48) for _ in range(SYNC_COMMITTEE_SIZE)]
        take(48)
        vraw = raw[off_validators:off_balances]
        assert len(vraw) % 121 == 0
        self.validators = []
        for k in range(len(vraw) // 121):
            v = vraw[121 * k:121 * (k + 1)]
            self.validators.append({
                "pubkey": v[0:48],
                "activation_epoch": int.from_bytes(v[97:105], "little"),
                "exit_epoch": int.from_bytes(v[105:113], "little"),
            })

    def fork_version(self, epoch: int) -> bytes:
        return self.fork_previous if epoch < self.fork_epoch else self.fork_current

    def domain(self, domain_type: bytes, epoch: int) -> bytes:
        return compute_domain(domain_type, self.fork_version(epoch), self.genesis_validators_root)

    def randao_mix(self, epoch: int) -> bytes:
        i = epoch % EPOCHS_PER_HISTORICAL_VECTOR
        return self.randao_mixes[32 * i:32 * (i + 1)]

    def active_indices(self, epoch: int) -> List[int]:
        return [i for i, v in enumerate(self.validators) if v["activation_epoch"] <= epoch < v["exit_epoch"]]

    def seed(self, epoch: int, domain_type: bytes) -> bytes:
        mix = self.randao_mix(epoch + EPOCHS_PER_HISTORICAL_VECTOR - MIN_SEED_LOOKAHEAD - 1)
        return sha256(domain_type + epoch.to_bytes(8, "little") + mix)

    def beacon_committee(self, slot: int, index: int) -> List[int]:
        epoch = slot // SLOTS_PER_EPOCH
        active = self.active_indices(epoch)
        per_slot = max(1, min(MAX_COMMITTEES_PER_SLOT, len(active) // SLOTS_PER_EPOCH // TARGET_COMMITTEE_SIZE))
        count = per_slot * SLOTS_PER_EPOCH
        k = (slot % SLOTS_PER_EPOCH) * per_slot + index
        seed = self.seed(epoch, DOMAIN_BEACON_ATTESTER)
        n = len(active)
        start, end = n * k // count, n * (k + 1) // count
        return [active[shuffled_index(i, n, seed)] for i in range(start, end)]


def shuffled_index(index: int, count: int, seed: bytes) -> int:
    """compute_shuffled_index (swap-or-not, SHUFFLE_ROUND_COUNT rounds)."""
    for r in range(SHUFFLE_ROUND_COUNT):
        pivot = int.from_bytes(sha256(seed + bytes([r]))[:8], "little") % count
        flip = (pivot + count - index) % count
        pos = max(index, flip)
        src = sha256(seed + bytes([r]) + (pos // 256).to_bytes(4, "little"))
        if (src[(pos % 256) // 8] >> (pos % 8)) & 1:
            index = flip
    return index
