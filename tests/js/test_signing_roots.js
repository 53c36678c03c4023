"use strict";
// lodestar_amd/js/signing_roots.js (getBlockSignatureSets for the TS host, SURVEY.md §8(f) row 2).
//   node tests/js/test_signing_roots.js cpu [ops.json]  -> K3 devnet roots with a hashlib-style
//        merkleizer (Node crypto); with ops.json, prints the roots of that block for the Python test
//   node tests/js/test_signing_roots.js forks cases.json [gpu]  -> the fork / sync-participation /
//        attester-slashing cases of tests/test_signing_roots.py fork_cases, roots or errors
//   node tests/js/test_signing_roots.js gpu [ops.json]  -> the same through addon.merkleize (one
//        launch per tree level), plus timings: the K3 block, a synthetic 128-attestation block, and a
//        32-block range-sync segment (the reference's set construction takes ~45 ms per 100-signature
//        block, chain/blocks/verifyBlocksSignatures.ts:41-43)
const assert = require("assert");
const crypto = require("crypto");
const fs = require("fs");
const path = require("path");
const SR = require(path.join(__dirname, "..", "..", "lodestar_amd", "js", "signing_roots.js"));

const k3 = JSON.parse(fs.readFileSync(path.join(__dirname, "..", "golden", "k3_devnet.json"), "utf8"));
const hexb = (h) => Uint8Array.from(Buffer.from(h, "hex"));
const hex = (u) => Buffer.from(u).toString("hex");

const ZH = [new Uint8Array(32)];
for (let i = 0; i < 64; i++) ZH.push(crypto.createHash("sha256").update(ZH[i]).update(ZH[i]).digest());
function cpuMerkleize(trees) {
  return trees.map((t) => {
    let layer = t.parts.map((p) => (p instanceof SR.Tree ? p.root : p));
    for (let d = 0; d < t.depth; d++) {
      if (layer.length % 2) layer.push(ZH[d]);
      const nx = [];
      for (let i = 0; i < layer.length; i += 2) nx.push(crypto.createHash("sha256").update(layer[i]).update(layer[i + 1]).digest());
      layer = nx;
    }
    let r = layer.length ? layer[0] : ZH[t.depth];
    if (t.mix !== null) {
      const m = Buffer.alloc(32);
      m.writeBigUInt64LE(BigInt(t.mix), 0);
      r = crypto.createHash("sha256").update(r).update(m).digest();
    }
    return Uint8Array.from(r);
  });
}

function stateView(k3, nKeys) {
  const keys = k3.state_view.validator_pubkeys48.map(hexb);
  return {
    genesisValidatorsRoot: hexb(k3.genesis_validators_root),
    forkPreviousVersion: hexb(k3.fork.previous_version), forkCurrentVersion: hexb(k3.fork.current_version),
    forkEpoch: k3.fork.epoch,
    pubkey: (i) => keys[i % (nKeys || keys.length)],
    beaconCommittee: (slot, index) => k3.state_view.committees[`${slot}:${index}`] ||
      Array.from({length: 256}, (_, k) => (index * 256 + k) % keys.length),
    syncCommittee: () => k3.state_view.sync_committee_indices.map((i) => keys[i]),
    keyFromBytes: (b) => b,
  };
}

function checkK3(merkleize) {
  const sets = SR.resolve(SR.getBlockSignatureSets(stateView(k3), k3.signed_block), merkleize);
  const gold = {};
  for (const g of k3.sets) gold[g.name.split("_slot")[0]] = g;
  assert.deepStrictEqual(sets.map((s) => s.name), ["randao", "attestation", "proposer", "sync_aggregate"]);
  for (const s of sets) {
    assert.strictEqual(hex(s.signingRoot), gold[s.name].signing_root, s.name);
    assert.strictEqual(hex(s.signature), gold[s.name].signature, s.name);
  }
  assert.strictEqual(hex(SR.evaluate([SR.beaconBlockCapella(k3.signed_block.message)], merkleize)[0]), k3.block_root);
  assert.strictEqual(hex(SR.evaluate([SR.beaconBlockBodyCapella(k3.signed_block.message.body)], merkleize)[0]), k3.body_root);
}

/** K3's block with 128 attestations of committee 256 (the C2 block shape) */
function bigBlock(salt) {
  const blk = JSON.parse(JSON.stringify(k3.signed_block));
  const a0 = blk.message.body.attestations[0];
  const bits = "0x" + "ff".repeat(32) + "01";  // 256 participants + the length bit
  blk.message.body.attestations = Array.from({length: 128}, (_, i) => {
    const a = JSON.parse(JSON.stringify(a0));
    a.data.index = String(1 + i);
    a.data.beacon_block_root = "0x" + crypto.createHash("sha256").update(`${salt}:${i}`).digest("hex");
    a.aggregation_bits = bits;
    return a;
  });
  return blk;
}

function opsRoots(file, merkleize) {
  const blk = JSON.parse(fs.readFileSync(file, "utf8"));
  const sets = SR.resolve(SR.getBlockSignatureSets(stateView(k3), blk), merkleize);
  return sets.map((s) => ({name: s.name, root: hex(s.signingRoot),
    keys: (s.type === "single" ? [s.pubkey] : s.pubkeys).map(hex)}));
}

/** fork cases written by tests/test_signing_roots.py (fork_cases): roots or the thrown error */
function forkCaseRoots(file, merkleize) {
  const cases = JSON.parse(fs.readFileSync(file, "utf8"));
  const mainnet = {
    genesisValidatorsRoot: hexb(cases.mainnet_gvr), forkPreviousVersion: new Uint8Array(4), forkCurrentVersion: new Uint8Array(4),
    forkEpoch: 0, pubkey: (i) => Uint8Array.from(Buffer.from(i.toString(16).padStart(8, "0"), "hex")),
    beaconCommittee: () => Array.from({length: 2048}, (_, k) => k),
    syncCommittee: () => Array.from({length: 512}, (_, k) => k),
    forkSeq: SR.forkSchedule(SR.MAINNET_FORK_EPOCHS),
  };
  return cases.cases.map((c) => {
    let st = mainnet;
    if (c.state === "k3") {
      st = stateView(k3);
      if (c.forks) st.forkSeq = SR.forkSchedule(c.forks);
    }
    try {
      const sets = SR.resolve(SR.getBlockSignatureSets(st, c.block), merkleize);
      return {case: c.name, sets: sets.map((s) => ({name: s.name, root: hex(s.signingRoot),
        keys: (s.type === "single" ? [s.pubkey] : s.pubkeys).map(hex)}))};
    } catch (e) {
      return {case: c.name, error: e.message};
    }
  });
}

function time(fn, reps) {
  const ts = [];
  for (let r = 0; r < reps; r++) {
    const t0 = process.hrtime.bigint();
    fn();
    ts.push(Number(process.hrtime.bigint() - t0) / 1e6);
  }
  ts.sort((a, b) => a - b);
  return Number(ts[Math.floor(ts.length / 2)].toFixed(3));
}

const mode = process.argv[2];
const ops = process.argv[3];
if (mode === "forks") {
  // node tests/js/test_signing_roots.js forks cases.json [gpu]
  let m = cpuMerkleize;
  let eng = null;
  const addon = process.argv[4] === "gpu" ? require(path.join(__dirname, "..", "..", "lodestar_amd", "napi", "lodestar_bls.node")) : null;
  if (addon) {
    eng = addon.createEngine(0);
    m = SR.gpuMerkleizer(eng);
  }
  console.log(JSON.stringify(forkCaseRoots(ops, m)));
  if (addon) addon.destroyEngine(eng);
  console.log("js fork cases ok");
} else if (mode === "cpu") {
  checkK3(cpuMerkleize);
  if (ops) console.log(JSON.stringify(opsRoots(ops, cpuMerkleize)));
  console.log("js signing roots cpu ok");
} else {
  const addon = require(path.join(__dirname, "..", "..", "lodestar_amd", "napi", "lodestar_bls.node"));
  const eng = addon.createEngine(0);
  const gm = SR.gpuMerkleizer(eng);
  checkK3(gm);
  const out = {};
  if (ops) out.ops = opsRoots(ops, gm);
  // one 128-attestation block: GPU roots equal the CPU walk's
  const st = stateView(k3);
  const blk = bigBlock("b");
  const g = SR.resolve(SR.getBlockSignatureSets(st, blk), SR.gpuMerkleizer(eng)).map((s) => hex(s.signingRoot));
  const c = SR.resolve(SR.getBlockSignatureSets(st, blk), cpuMerkleize).map((s) => hex(s.signingRoot));
  assert.deepStrictEqual(g, c);
  const seg = Array.from({length: 32}, (_, i) => bigBlock("s" + i));
  out.k3_block_ms = time(() => SR.resolve(SR.getBlockSignatureSets(st, k3.signed_block), SR.gpuMerkleizer(eng)), 20);
  out.block128_ms = time(() => SR.resolve(SR.getBlockSignatureSets(st, blk), SR.gpuMerkleizer(eng)), 10);
  out.block128_cpu_merkleize_ms = time(() => SR.resolve(SR.getBlockSignatureSets(st, blk), cpuMerkleize), 5);
  let launches = 0;
  out.segment32_ms = time(() => {
    const m = SR.gpuMerkleizer(eng);
    SR.resolve(seg.flatMap((b) => SR.getBlockSignatureSets(st, b)), m);
    launches = m.launches;
  }, 5);
  out.segment32_launches = launches;
  out.reference_ms_per_block = 45;
  addon.destroyEngine(eng);
  console.log(JSON.stringify(out));
  console.log("js signing roots gpu ok");
}
