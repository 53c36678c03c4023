"use strict";
/**
 * Signing-root production for the TypeScript host (SURVEY.md §8(f) row 2): the signature sets of
 * a phase0 / altair / bellatrix / capella block with their signing roots hashed on the GPU.
 *
 * Mirrors getBlockSignatureSets (packages/state-transition/src/signatureSets/index.ts:26-72):
 * randao (randao.ts), proposer slashings (proposerSlashings.ts), attester slashings
 * (attesterSlashings.ts), attestations (indexedAttestation.ts), voluntary exits
 * (voluntaryExits.ts), proposer (proposer.ts, the BeaconBlock type of the block's fork), then by
 * config.getForkSeq(slot) the sync aggregate from altair on (block/processSyncCommittee.ts:58-111,
 * which throws "Empty sync committee signature is not infinity" for an empty participation with
 * another signature) and BLS-to-execution changes from capella on (blsToExecutionChange.ts).  Each root is computeSigningRoot(type, value, domain) =
 * hash_tree_root(SigningData{hash_tree_root(value), domain}) (src/util/signingRoot.ts:7-13).
 *
 * The SSZ containers (beacon-API JSON, the same objects lodestar_amd/signing_roots.py walks) are
 * turned into merkle trees on the host; every tree of one height -- across all the blocks of a
 * call -- is hashed in ONE lb_merkleize launch (addon.merkleize), so a 32-block range-sync
 * segment costs a handful of launches.  Domains follow config.getDomain (config/src/genesisConfig/
 * index.ts:27-54): previous fork version before the state's fork epoch, else the current one.
 */
const crypto = require("crypto");
const path = require("path");

const addon = require(path.join(__dirname, "..", "napi", "lodestar_bls.node"));

const SLOTS_PER_EPOCH = 32;
const SYNC_COMMITTEE_SIZE = 512;
const NO_MIX = 0xffffffffffffffffn;
const DOMAIN_BEACON_PROPOSER = Uint8Array.from([0, 0, 0, 0]);
const DOMAIN_BEACON_ATTESTER = Uint8Array.from([1, 0, 0, 0]);
const DOMAIN_RANDAO = Uint8Array.from([2, 0, 0, 0]);
const DOMAIN_VOLUNTARY_EXIT = Uint8Array.from([4, 0, 0, 0]);
const DOMAIN_SYNC_COMMITTEE = Uint8Array.from([7, 0, 0, 0]);
const DOMAIN_BLS_TO_EXECUTION_CHANGE = Uint8Array.from([10, 0, 0, 0]);
const MAX_VALIDATORS_PER_COMMITTEE = 2048;
/** ForkSeq (packages/params/src/forkName.ts) */
const ForkSeq = {phase0: 0, altair: 1, bellatrix: 2, capella: 3};
/** mainnet fork epochs (config/src/chainConfig/presets/mainnet.ts:34-42; capella unscheduled there) */
const MAINNET_FORK_EPOCHS = {altair: 74240, bellatrix: 144896, capella: Infinity};
/** G2_POINT_AT_INFINITY (params/src/index.ts) */
const G2_POINT_AT_INFINITY = (() => {
  const b = new Uint8Array(96);
  b[0] = 0xc0;
  return b;
})();

/** slot -> ForkSeq for the given fork epochs (config.getForkSeq) */
function forkSchedule(epochs) {
  const e = Object.assign({altair: Infinity, bellatrix: Infinity, capella: Infinity}, epochs);
  return (slot) => {
    const ep = Math.floor(Number(slot) / SLOTS_PER_EPOCH);
    return ep >= e.capella ? ForkSeq.capella : ep >= e.bellatrix ? ForkSeq.bellatrix : ep >= e.altair ? ForkSeq.altair : ForkSeq.phase0;
  };
}

/** hash_tree_root of `parts` (32-byte chunks or Trees) padded to 2^depth leaves, mix = length or null */
class Tree {
  constructor(parts, depth, mix) {
    if (parts.length > 2 ** depth) throw Error("tree overflow");
    this.parts = parts;
    this.depth = depth;
    this.mix = mix === undefined ? null : mix;
    this.root = null;
    let h = 0;
    for (const p of parts) if (p instanceof Tree && p.height > h) h = p.height;
    this.height = 1 + h;
  }
}

const ceilLog2 = (n) => (n <= 1 ? 0 : Math.ceil(Math.log2(n)));

function hx(s) {
  return Uint8Array.from(Buffer.from(s.startsWith("0x") ? s.slice(2) : s, "hex"));
}

function pack(b) {
  const n = Math.max(1, Math.ceil(b.length / 32));
  const out = [];
  for (let i = 0; i < n; i++) {
    const c = new Uint8Array(32);
    c.set(b.subarray(32 * i, Math.min(b.length, 32 * i + 32)));
    out.push(c);
  }
  return b.length === 0 ? [new Uint8Array(32)] : out;
}

function uint64(x) {
  const c = new Uint8Array(32);
  let v = BigInt(x);
  for (let i = 0; i < 8; i++) {
    c[i] = Number(v & 0xffn);
    v >>= 8n;
  }
  return c;
}

function uint256(x) {
  const c = new Uint8Array(32);
  let v = BigInt(x);
  for (let i = 0; i < 32; i++) {
    c[i] = Number(v & 0xffn);
    v >>= 8n;
  }
  return c;
}

function bytesN(b) {
  const ch = pack(b);
  return ch.length === 1 ? ch[0] : new Tree(ch, ceilLog2(ch.length));
}

/** List[uint64, limit]: values packed 4 per 32-byte chunk, limit ceil(8*limit/32) chunks */
function uint64List(values, limit) {
  const raw = new Uint8Array(8 * values.length);
  values.forEach((x, i) => {
    let v = BigInt(x);
    for (let j = 0; j < 8; j++) {
      raw[8 * i + j] = Number(v & 0xffn);
      v >>= 8n;
    }
  });
  return new Tree(raw.length ? pack(raw) : [], ceilLog2(Math.ceil((8 * limit) / 32)), values.length);
}

function byteList(b, limit) {
  return new Tree(b.length ? pack(b) : [], ceilLog2(Math.ceil(limit / 32)), b.length);
}

function bitsToBytes(bits) {
  const out = new Uint8Array(Math.ceil(bits.length / 8));
  bits.forEach((x, i) => {
    if (x) out[i >> 3] |= 1 << (i & 7);
  });
  return out;
}

function bitlist(bits, limit) {
  const b = bitsToBytes(bits);
  return new Tree(b.length ? pack(b) : [], ceilLog2(Math.ceil(limit / 256)), bits.length);
}

function bitvector(bits) {
  const ch = pack(bitsToBytes(bits));
  return ch.length > 1 ? new Tree(ch, ceilLog2(Math.ceil(bits.length / 256))) : ch[0];
}

const container = (fields) => new Tree(fields, ceilLog2(fields.length));
const listOf = (items, limit) => new Tree(items, ceilLog2(limit), items.length);

function bitsFromBitlistHex(h) {
  const b = hx(h);
  let last = -1;
  for (let i = b.length * 8 - 1; i >= 0; i--)
    if ((b[i >> 3] >> (i & 7)) & 1) {
      last = i;
      break;
    }
  const out = [];
  for (let i = 0; i < last; i++) out.push((b[i >> 3] >> (i & 7)) & 1);
  return out;
}

function bitsFromBitvectorHex(h, n) {
  const b = hx(h);
  const out = [];
  for (let i = 0; i < n; i++) out.push(i >> 3 < b.length ? (b[i >> 3] >> (i & 7)) & 1 : 0);
  return out;
}

const checkpoint = (c) => container([uint64(c.epoch), hx(c.root)]);
const attestationData = (d) =>
  container([uint64(d.slot), uint64(d.index), hx(d.beacon_block_root), checkpoint(d.source), checkpoint(d.target)]);
const indexedAttestation = (a) =>
  container([uint64List(a.attesting_indices, MAX_VALIDATORS_PER_COMMITTEE), attestationData(a.data), bytesN(hx(a.signature))]);
const attestation = (a) =>
  container([bitlist(bitsFromBitlistHex(a.aggregation_bits), 2048), attestationData(a.data), bytesN(hx(a.signature))]);
const blockHeader = (h) =>
  container([uint64(h.slot), uint64(h.proposer_index), hx(h.parent_root), hx(h.state_root), hx(h.body_root)]);
const signedHeader = (s) => container([blockHeader(s.message), bytesN(hx(s.signature))]);
const voluntaryExit = (e) => container([uint64(e.epoch), uint64(e.validator_index)]);
const blsToExecutionChange = (c) =>
  container([uint64(c.validator_index), bytesN(hx(c.from_bls_pubkey)), bytesN(hx(c.to_execution_address))]);
const withdrawal = (w) => container([uint64(w.index), uint64(w.validator_index), bytesN(hx(w.address)), uint64(w.amount)]);

const executionPayloadFields = (p) => [
  hx(p.parent_hash), bytesN(hx(p.fee_recipient)), hx(p.state_root), hx(p.receipts_root), bytesN(hx(p.logs_bloom)),
  hx(p.prev_randao), uint64(p.block_number), uint64(p.gas_limit), uint64(p.gas_used), uint64(p.timestamp),
  byteList(hx(p.extra_data), 32), uint256(p.base_fee_per_gas), hx(p.block_hash),
  listOf(p.transactions.map((t) => byteList(hx(t), 2 ** 30)), 2 ** 20),
];
const executionPayloadBellatrix = (p) => container(executionPayloadFields(p));
const executionPayloadCapella = (p) => container([...executionPayloadFields(p), listOf(p.withdrawals.map(withdrawal), 16)]);

function deposit(d) {
  const data = d.data;
  return container([new Tree(d.proof.map(hx), 6),
    container([bytesN(hx(data.pubkey)), hx(data.withdrawal_credentials), uint64(data.amount), bytesN(hx(data.signature))])]);
}

/**
 * BeaconBlockBody of `fork` (types/src/{phase0,altair,bellatrix,capella}/sszTypes.ts): phase0's 8
 * fields, + sync_aggregate (altair), + execution_payload (bellatrix), capella's payload with
 * withdrawals + bls_to_execution_changes
 */
function beaconBlockBody(b, fork) {
  const fields = [
    bytesN(hx(b.randao_reveal)),
    container([hx(b.eth1_data.deposit_root), uint64(b.eth1_data.deposit_count), hx(b.eth1_data.block_hash)]),
    hx(b.graffiti),
    listOf(b.proposer_slashings.map((s) => container([signedHeader(s.signed_header_1), signedHeader(s.signed_header_2)])), 16),
    listOf(b.attester_slashings.map((s) => container([indexedAttestation(s.attestation_1), indexedAttestation(s.attestation_2)])), 2),
    listOf(b.attestations.map(attestation), 128),
    listOf(b.deposits.map(deposit), 16),
    listOf(b.voluntary_exits.map((e) => container([voluntaryExit(e.message), bytesN(hx(e.signature))])), 16),
  ];
  if (fork >= ForkSeq.altair) {
    const sa = b.sync_aggregate;
    fields.push(container([bitvector(bitsFromBitvectorHex(sa.sync_committee_bits, SYNC_COMMITTEE_SIZE)), bytesN(hx(sa.sync_committee_signature))]));
  }
  if (fork === ForkSeq.bellatrix) fields.push(executionPayloadBellatrix(b.execution_payload));
  if (fork >= ForkSeq.capella) {
    fields.push(executionPayloadCapella(b.execution_payload));
    fields.push(listOf(b.bls_to_execution_changes.map((c) => container([blsToExecutionChange(c.message), bytesN(hx(c.signature))])), 16));
  }
  return container(fields);
}

/** BeaconBlock of `fork` (config.getForkTypes(slot).BeaconBlock, proposer.ts:22-24) */
const beaconBlock = (m, fork) =>
  container([uint64(m.slot), uint64(m.proposer_index), hx(m.parent_root), hx(m.state_root), beaconBlockBody(m.body, fork)]);
const beaconBlockBodyCapella = (b) => beaconBlockBody(b, ForkSeq.capella);
const beaconBlockCapella = (m) => beaconBlock(m, ForkSeq.capella);

const signingTree = (obj, domain) => container([obj, domain]);

function computeDomain(domainType, forkVersion, genesisValidatorsRoot) {
  const data = new Uint8Array(64);
  data.set(forkVersion, 0);
  data.set(genesisValidatorsRoot, 32);
  const root = crypto.createHash("sha256").update(data).digest();
  const out = new Uint8Array(32);
  out.set(domainType, 0);
  out.set(root.subarray(0, 28), 4);
  return out;
}

/**
 * What getBlockSignatureSets reads from the cached state: the fork, the genesis validators root,
 * index2pubkey, beacon committees and the current sync committee.
 * @typedef {{genesisValidatorsRoot: Uint8Array, forkPreviousVersion: Uint8Array, forkCurrentVersion: Uint8Array,
 *   forkEpoch: number, slot?: number, pubkey: (i: number) => any, beaconCommittee: (slot: number, index: number) => number[],
 *   syncCommittee: () => any[], keyFromBytes?: (b48: Uint8Array) => any, forkSeq?: (slot: number) => number}} StateView
 * (forkSeq: config.getForkSeq; capella for every slot when absent, see forkSchedule)
 */
function domainOf(state, domainType, epoch) {
  const key = `${Buffer.from(domainType).toString("hex")}:${epoch < state.forkEpoch ? "p" : "c"}`;
  state._domains = state._domains || new Map();
  let d = state._domains.get(key);
  if (!d) {
    d = computeDomain(domainType, epoch < state.forkEpoch ? state.forkPreviousVersion : state.forkCurrentVersion,
      state.genesisValidatorsRoot);
    state._domains.set(key, d);
  }
  return d;
}

/**
 * getSyncCommitteeSignatureSet (block/processSyncCommittee.ts:58-111): null for an empty
 * participation with the infinity signature, the reference's Error for any other signature
 */
function getSyncCommitteeSignatureSet(state, m) {
  const sa = m.body.sync_aggregate;
  const sig = hx(sa.sync_committee_signature);
  const sbits = bitsFromBitvectorHex(sa.sync_committee_bits, SYNC_COMMITTEE_SIZE);
  const keys = state.syncCommittee().filter((_, k) => sbits[k]);
  if (keys.length === 0) {
    if (Buffer.from(sig).equals(Buffer.from(G2_POINT_AT_INFINITY))) return null;
    throw Error("Empty sync committee signature is not infinity");
  }
  const prev = Math.max(Number(m.slot), 1) - 1;
  return {name: "sync_aggregate", type: "aggregate", pubkeys: keys,
    signingRoot: signingTree(hx(m.parent_root), domainOf(state, DOMAIN_SYNC_COMMITTEE, Math.floor(prev / SLOTS_PER_EPOCH))),
    signature: sig};
}

/**
 * getBlockSignatureSets for one SignedBeaconBlock of any fork up to capella (beacon-API JSON).
 * Signing roots are left as Trees; resolve() hashes the trees of many blocks together.
 * @returns {{name: string, type: "single"|"aggregate", pubkey?: any, pubkeys?: any[], signingRoot: Tree|Uint8Array, signature: Uint8Array}[]}
 */
function getBlockSignatureSets(state, signedBlock, opts) {
  const m = signedBlock.message;
  const b = m.body;
  const slot = Number(m.slot);
  const epoch = Math.floor(slot / SLOTS_PER_EPOCH);
  const stateEpoch = Math.floor((state.slot === undefined ? slot : Number(state.slot)) / SLOTS_PER_EPOCH);
  const keyFromBytes = state.keyFromBytes || ((k) => k);
  const fork = state.forkSeq ? state.forkSeq(slot) : ForkSeq.capella;
  const single = (name, pk, root, sig) => ({name, type: "single", pubkey: pk, signingRoot: root, signature: sig});
  const sets = [];
  sets.push(single("randao", state.pubkey(Number(m.proposer_index)), signingTree(uint64(epoch), domainOf(state, DOMAIN_RANDAO, epoch)),
    hx(b.randao_reveal)));
  for (const s of b.proposer_slashings) {
    const pk = state.pubkey(Number(s.signed_header_1.message.proposer_index));
    for (const h of [s.signed_header_1, s.signed_header_2]) {
      const ep = Math.floor(Number(h.message.slot) / SLOTS_PER_EPOCH);
      sets.push(single("proposer_slashing", pk, signingTree(blockHeader(h.message), domainOf(state, DOMAIN_BEACON_PROPOSER, ep)),
        hx(h.signature)));
    }
  }
  for (const s of b.attester_slashings)
    for (const ia of [s.attestation_1, s.attestation_2])
      sets.push({name: "attester_slashing", type: "aggregate", pubkeys: ia.attesting_indices.map((i) => state.pubkey(Number(i))),
        signingRoot: signingTree(attestationData(ia.data), domainOf(state, DOMAIN_BEACON_ATTESTER, Number(ia.data.target.epoch))),
        signature: hx(ia.signature)});
  for (const a of b.attestations) {
    const d = a.data;
    const committee = state.beaconCommittee(Number(d.slot), Number(d.index));
    const bits = bitsFromBitlistHex(a.aggregation_bits);
    const idx = committee.filter((_, k) => bits[k]).sort((x, y) => x - y);
    sets.push({name: "attestation", type: "aggregate", pubkeys: idx.map((v) => state.pubkey(v)),
      signingRoot: signingTree(attestationData(d), domainOf(state, DOMAIN_BEACON_ATTESTER, Number(d.target.epoch))),
      signature: hx(a.signature)});
  }
  for (const e of b.voluntary_exits)
    sets.push(single("voluntary_exit", state.pubkey(Number(e.message.validator_index)),
      signingTree(voluntaryExit(e.message), domainOf(state, DOMAIN_VOLUNTARY_EXIT, Number(e.message.epoch))), hx(e.signature)));
  if (!(opts && opts.skipProposerSignature))
    sets.push(single("proposer", state.pubkey(Number(m.proposer_index)),
      signingTree(beaconBlock(m, fork), domainOf(state, DOMAIN_BEACON_PROPOSER, epoch)), hx(signedBlock.signature)));
  if (fork >= ForkSeq.altair) {
    const sync = getSyncCommitteeSignatureSet(state, m);
    if (sync) sets.push(sync);
  }
  if (fork < ForkSeq.capella) return sets;
  for (const c of b.bls_to_execution_changes)
    sets.push(single("bls_to_execution_change", keyFromBytes(hx(c.message.from_bls_pubkey)),
      signingTree(blsToExecutionChange(c.message), domainOf(state, DOMAIN_BLS_TO_EXECUTION_CHANGE, stateEpoch)), hx(c.signature)));
  return sets;
}

/** roots of `nodes` (Trees or 32-byte chunks): all trees of one height in one merkleize() call */
function evaluate(nodes, merkleize) {
  const byH = new Map();
  const seen = new Set();
  const walk = (t) => {
    if (!(t instanceof Tree) || seen.has(t)) return;
    seen.add(t);
    if (!byH.has(t.height)) byH.set(t.height, []);
    byH.get(t.height).push(t);
    for (const p of t.parts) walk(p);
  };
  for (const n of nodes) walk(n);
  for (const h of [...byH.keys()].sort((x, y) => x - y)) {
    const trees = byH.get(h);
    const roots = merkleize(trees);
    trees.forEach((t, k) => {
      t.root = roots[k];
    });
  }
  return nodes.map((n) => (n instanceof Tree ? n.root : n));
}

/** trees of one level -> addon.merkleize on `engine` (one GPU launch) */
function gpuMerkleizer(engine) {
  const fn = (trees) => {
    const off = new Uint32Array(trees.length + 1);
    let total = 0;
    trees.forEach((t, k) => {
      total += t.parts.length;
      off[k + 1] = total;
    });
    const chunks = new Uint8Array(32 * total);
    const depths = new Uint32Array(trees.length);
    const mix = new BigUint64Array(trees.length);
    let c = 0;
    trees.forEach((t, k) => {
      for (const p of t.parts) chunks.set(p instanceof Tree ? p.root : p, 32 * c++);
      depths[k] = t.depth;
      mix[k] = t.mix === null ? NO_MIX : BigInt(t.mix);
    });
    fn.launches++;
    const out = addon.merkleize(engine, off, chunks, depths, mix);
    return trees.map((_, k) => out.subarray(32 * k, 32 * k + 32));
  };
  fn.launches = 0;
  return fn;
}

/** hashes every pending signing root of `sets` (any number of blocks) level by level */
function resolve(sets, merkleize) {
  const roots = evaluate(sets.map((s) => s.signingRoot), merkleize);
  sets.forEach((s, k) => {
    s.signingRoot = roots[k];
  });
  return sets;
}

module.exports = {
  Tree,
  ForkSeq,
  MAINNET_FORK_EPOCHS,
  G2_POINT_AT_INFINITY,
  forkSchedule,
  getBlockSignatureSets,
  getSyncCommitteeSignatureSet,
  beaconBlock,
  beaconBlockBody,
  evaluate,
  resolve,
  gpuMerkleizer,
  beaconBlockCapella,
  beaconBlockBodyCapella,
  computeDomain,
};
