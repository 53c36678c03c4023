"use strict";
// Node-side tests of the JS IBlsVerifier drop-in (lodestar_amd/js/index.js).
//   node tests/js/test_verifier.js cpu   -> policy + addon load, no GPU
//   node tests/js/test_verifier.js gpu   -> golden fixtures and the reference's multithread.test.ts cases
const assert = require("assert");
const fs = require("fs");
const path = require("path");
const m = require(path.join(__dirname, "..", "..", "lodestar_amd", "js", "index.js"));

const golden = (name) => JSON.parse(fs.readFileSync(path.join(__dirname, "..", "golden", name), "utf8"));
const hex = (h) => Uint8Array.from(Buffer.from(h, "hex"));

function cpuTests() {
  // packages/beacon-node/test/unit/chain/bls/utils.test.ts:6-34
  const expected = [
    [[0]], [[0, 1]], [[0, 1, 2]], [[0, 1, 2, 3]], [[0, 1, 2, 3, 4]],
    [[0, 1, 2], [3, 4, 5]], [[0, 1, 2, 3], [4, 5, 6]], [[0, 1, 2, 3], [4, 5, 6, 7]],
  ];
  expected.forEach((exp, i) => {
    const arr = Array.from({length: i + 1}, (_, k) => k);
    assert.deepStrictEqual(m.chunkifyMaximizeChunkSize(arr, 3), exp);
  });
  assert.strictEqual(m.addon.errorName(10), "BLST_INVALID_SIZE");
  assert.throws(() => new m.BlsGpuVerifier(), /LB_ERR_NO_DEVICE/);
  // packing: 32-byte signature flagged by size
  const set = {type: "single", pubkey: new Uint8Array(96), signingRoot: new Uint8Array(32), signature: new Uint8Array(32)};
  const packed = m.packJobs([[set]]);
  assert.strictEqual(packed[5][0], 32);
  console.log("js cpu ok");
}

function setsFromCase(c) {
  return c.sets.map((s) =>
    s.pubkeys.length === 1 && c.name.indexOf("aggregate") < 0
      ? {type: "single", pubkey: hex(s.pubkeys[0]), signingRoot: hex(s.signing_root), signature: hex(s.signature)}
      : {type: "aggregate", pubkeys: s.pubkeys.map(hex), signingRoot: hex(s.signing_root), signature: hex(s.signature)}
  );
}

async function outcome(p) {
  try {
    return await p;
  } catch (e) {
    return e.message;
  }
}

async function gpuTests() {
  const pool = new m.BlsGpuVerifier();
  // golden jobs (each case = one verifySignatureSets call), concurrently, batchable and not
  const cases = golden("jobs.json").cases;
  for (const batchable of [false, true]) {
    const got = await Promise.all(cases.map((c) => outcome(pool.verifySignatureSets(setsFromCase(c), {batchable}))));
    cases.forEach((c, k) => assert.strictEqual(got[k], c.expected, `${c.name} batchable=${batchable}`));
  }
  // verifyOnMainThread path
  for (const c of cases.slice(0, 10)) {
    assert.strictEqual(await outcome(pool.verifySignatureSets(setsFromCase(c), {verifyOnMainThread: true})), c.expected, c.name);
  }
  // packages/beacon-node/test/e2e/chain/bls/multithread.test.ts:60-103
  const k4 = golden("reference_kats.json").K4_multithread_sets.sets.map((s) => ({
    type: "single", pubkey: hex(s.pubkey96), signingRoot: hex(s.signing_root), signature: hex(s.signature),
  }));
  for (const [sleep, opts] of [[false, {}], [true, {}], [true, {batchable: true}]]) {
    const ps = [];
    for (let i = 0; i < 8; i++) {
      ps.push(pool.verifySignatureSets(k4, opts));
      if (sleep) await new Promise((r) => setTimeout(r, 5));
    }
    assert.deepStrictEqual(await Promise.all(ps), Array(8).fill(true));
  }
  const invalid = {...k4[0], signature: new Uint8Array(32)};
  const bad = outcome(pool.verifySignatureSets([invalid], {batchable: true}));
  const goods = [];
  for (let i = 0; i < 8; i++) goods.push(pool.verifySignatureSets(k4, {batchable: true}));
  assert.strictEqual(await bad, "BLST_INVALID_SIZE");
  assert.deepStrictEqual(await Promise.all(goods), Array(8).fill(true));
  // a malformed set rejects only its own call, before anything is queued (ADVICE r1)
  const shortRoot = {...k4[0], signingRoot: new Uint8Array(31)};
  const mixed = await Promise.all([
    outcome(pool.verifySignatureSets([shortRoot], {batchable: true})),
    outcome(pool.verifySignatureSets(k4, {batchable: true})),
  ]);
  assert.deepStrictEqual(mixed, ["signing root must be 32 bytes", true]);
  // resident pubkey table: registered handles ship 4-byte indices; mixing them with raw keys
  // falls back to bytes for that package
  const keys = golden("reference_kats.json").K4_multithread_sets.sets.map((s) => hex(s.pubkey96));
  const handles = pool.registerPubkeys(keys);
  assert.strictEqual(handles.length, keys.length);
  const k4idx = k4.map((s, i) => ({...s, pubkey: handles[i]}));
  const packedIdx = m.packJobs([k4idx]);
  assert.ok(packedIdx[2] instanceof Uint32Array);
  const idxRes = await Promise.all([
    pool.verifySignatureSets(k4idx, {batchable: true}),
    pool.verifySignatureSets([k4idx[0], k4[1]], {batchable: true}),
    pool.verifySignatureSets(k4idx, {verifyOnMainThread: true}),
    outcome(pool.verifySignatureSets([{...k4idx[0], signingRoot: k4[1].signingRoot}], {batchable: true})),
  ]);
  assert.deepStrictEqual(idxRes, [true, true, true, false]);
  // compressed keys register too (decompressed on the GPU)
  const k1 = golden("reference_kats.json").K1_interop_pubkeys.pubkeys.slice(0, 4).map(hex);
  const h1 = pool.registerPubkeys(k1, true);
  assert.strictEqual(h1[0].toBytes().length, 96);
  // addon argument checks: lengths must match the offsets (TypeError, nothing queued)
  const eng = m.addon.createEngine(0);
  const jo = Uint32Array.from([0, 1]);
  const po = Uint32Array.from([0, 1]);
  assert.throws(() => m.addon.verifyJobs(eng, jo, po, new Uint8Array(95), new Uint8Array(32), new Uint8Array(96)), TypeError);
  assert.throws(() => m.addon.verifyJobs(eng, jo, po, new Uint8Array(96), new Uint8Array(31), new Uint8Array(96)), TypeError);
  assert.throws(() => m.addon.verifyJobs(eng, jo, po, new Uint8Array(96), new Uint8Array(32), new Uint8Array(95)), TypeError);
  assert.throws(() => m.addon.verifyJobs(eng, jo, Uint32Array.from([0]), new Uint8Array(96), new Uint8Array(32), new Uint8Array(96)), TypeError);
  assert.throws(() => m.addon.verifyJobs(eng, Uint32Array.from([0, 2, 1]), po, new Uint8Array(96), new Uint8Array(32), new Uint8Array(96)), TypeError);
  assert.throws(() => m.addon.verifyJobs(eng, jo, po, new Uint8Array(96), new Uint8Array(32), new Uint8Array(96), new Uint32Array(0)), TypeError);
  // destroyEngine while a request is in flight: deferred until it settles
  const single = m.packJobs([[k4[0]]]);
  const inflight = m.addon.verifyJobs(eng, ...single);
  m.addon.destroyEngine(eng);
  assert.deepStrictEqual(Array.from(await inflight), [1]);
  assert.throws(() => m.addon.verifyJobs(eng, ...single), /engine destroyed/);
  // direct callers: verifySignatureSet (state transition), isValidBlsAggregate (light client),
  // aggregateSignatures (op pools)
  const byName = Object.fromEntries(cases.map((c) => [c.name, c]));
  assert.strictEqual(pool.verifySignatureSet(setsFromCase(byName.single_valid_0)[0]), true);
  assert.strictEqual(pool.verifySignatureSet(setsFromCase(byName.aggregate_valid)[0]), true);
  assert.strictEqual(pool.verifySignatureSet(setsFromCase(byName.wrong_message)[0]), false);
  assert.throws(() => pool.verifySignatureSet(setsFromCase(byName.invalid_size_32_zero)[0]), /BLST_INVALID_SIZE/);
  const av = setsFromCase(byName.aggregate_valid)[0];
  assert.strictEqual(m.isValidBlsAggregate(pool, av.pubkeys, av.signingRoot, av.signature), true);
  assert.throws(() => m.isValidBlsAggregate(pool, [], av.signingRoot, av.signature),
    /^Error: Error aggregating pubkeys: EMPTY_AGGREGATE_ARRAY$/);
  for (const g of golden("aggregates.json").signature_aggregate) {
    const sigs = g.signatures.map(hex);
    if (g.status === "BLST_SUCCESS") assert.strictEqual(Buffer.from(pool.aggregateSignatures(sigs)).toString("hex"), g.expected96);
    else assert.throws(() => pool.aggregateSignatures(sigs), new RegExp(g.status));
  }
  // close(): queued jobs abort
  const pending = outcome(pool.verifySignatureSets(k4, {batchable: true}));
  await pool.close();
  assert.strictEqual(await pending, "QUEUE_ABORTED");
  console.log("js gpu ok");
}

(process.argv[2] === "gpu" ? gpuTests() : Promise.resolve(cpuTests())).catch((e) => {
  console.error(e);
  process.exit(1);
});
