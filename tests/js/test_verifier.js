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
  // QueueError as beacon-node/src/util/queue/errors.ts:3-14 (message = type.code)
  const qe = new m.QueueError({code: m.QueueErrorCode.QUEUE_ABORTED});
  assert.strictEqual(qe.type.code, "QUEUE_ERROR_QUEUE_ABORTED");
  assert.strictEqual(qe.message, "QUEUE_ERROR_QUEUE_ABORTED");
  // @chainsafe/bls PublicKey objects: toBytes(PointFormat.uncompressed) is what gets shipped; a key
  // whose toBytes ignores the format (48-byte default) is decompressed in one batch per call
  const b96 = Uint8Array.from({length: 96}, (_, i) => i);
  const b48 = Uint8Array.from({length: 48}, (_, i) => 200 - i);
  const formats = [];
  const pkU = {toBytes: (f) => (formats.push(f), f === "uncompressed" ? b96 : b48)};
  const pkC = {toBytes: () => b48};
  const calls = [];
  const stub = (flat) => {
    calls.push(flat.length);
    return {out: new Uint8Array(2 * flat.length).fill(7), status: new Int32Array(flat.length / 48)};
  };
  const sets = [
    {type: "single", pubkey: pkU, signingRoot: new Uint8Array(32), signature: new Uint8Array(96)},
    {type: "aggregate", pubkeys: [pkC, pkU, b48], signingRoot: new Uint8Array(32), signature: new Uint8Array(96)},
  ];
  const norm = m.normalizeSets(sets, stub);
  assert.deepStrictEqual(calls, [96]);  // pkC + the raw 48-byte key, one batch
  assert.strictEqual(formats[0], "uncompressed");
  assert.strictEqual(norm[0], sets[0]);  // untouched: its key is already 96 bytes
  assert.strictEqual(norm[1].pubkeys[0][0], 7);
  assert.strictEqual(norm[1].pubkeys[1], pkU);
  assert.strictEqual(sets[1].pubkeys[0], pkC);  // the caller's sets are not modified
  m.normalizeSets(sets, stub);  // the key objects' 96-byte forms are cached
  assert.deepStrictEqual(calls, [96, 48]);
  assert.strictEqual(formats.length, 1);
  assert.throws(() => m.normalizeSets([{...sets[0], pubkey: {toBytes: () => new Uint8Array(47)}}], stub), /48 or 96/);
  assert.throws(() => m.normalizeSets([{...sets[1], pubkeys: [b48]}],
    (flat) => ({out: new Uint8Array(96), status: Int32Array.from([1])})), /BLST_BAD_ENCODING/);
  assert.strictEqual(m.getAggregatedPubkeysCount(sets), 3);
  console.log("js cpu ok");
}

function setsFromCase(c) {
  return c.sets.map((s) =>
    s.pubkeys.length === 1 && c.name.indexOf("aggregate") < 0
      ? {type: "single", pubkey: hex(s.pubkeys[0]), signingRoot: hex(s.signing_root), signature: hex(s.signature)}
      : {type: "aggregate", pubkeys: s.pubkeys.map(hex), signingRoot: hex(s.signing_root), signature: hex(s.signature)}
  );
}

// a @chainsafe/bls-shaped PublicKey: toBytes() defaults to the 48-byte compressed encoding
// (PointFormat.compressed); toBytes("uncompressed") gives the 96 bytes the reference pool ships
const P_FIELD = BigInt("0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab");
function compress96(b96) {
  const out = Uint8Array.from(b96.subarray(0, 48));
  if (b96[0] & 0x40) {
    out.fill(0);
    out[0] = 0xc0;
    return out;
  }
  const y = BigInt("0x" + Buffer.from(b96.subarray(48, 96)).toString("hex"));
  out[0] |= 0x80 | (2n * y > P_FIELD ? 0x20 : 0);
  return out;
}
class MockPublicKey {
  constructor(b96, ignoreFormat) {
    this.b96 = b96;
    this.b48 = compress96(b96);
    this.ignoreFormat = ignoreFormat;
  }
  toBytes(format) {
    return format === "uncompressed" && !this.ignoreFormat ? this.b96 : this.b48;
  }
}
function mockSets(c, ignoreFormat) {
  return setsFromCase(c).map((s) =>
    s.type === "single" ? {...s, pubkey: new MockPublicKey(s.pubkey, ignoreFormat)}
      : {...s, pubkeys: s.pubkeys.map((k) => new MockPublicKey(k, ignoreFormat))});
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
  // the reference's own key objects (@chainsafe/bls PublicKey): serialised with
  // toBytes("uncompressed"), or decompressed on the GPU when toBytes only gives 48 bytes.  Keys that
  // do not decode cannot exist as PublicKey objects (pubkey_* cases are byte-level only).
  const keyCases = cases.filter((c) => !c.name.startsWith("pubkey_"));
  for (const ignoreFormat of [false, true]) {
    for (const batchable of [false, true]) {
      const got = await Promise.all(keyCases.map((c) => outcome(pool.verifySignatureSets(mockSets(c, ignoreFormat), {batchable}))));
      keyCases.forEach((c, k) => assert.strictEqual(got[k], c.expected, `${c.name} mock keys ignoreFormat=${ignoreFormat}`));
    }
    for (const c of keyCases.slice(0, 12))
      assert.strictEqual(await outcome(pool.verifySignatureSets(mockSets(c, ignoreFormat), {verifyOnMainThread: true})),
        c.expected, `${c.name} main thread mock keys`);
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
  // verifyOnMainThread runs on its own engine: it does not wait for a pool batch in flight
  const big = [];
  for (let r = 0; r < 40; r++) big.push(...k4);
  const inflightBatch = pool.verifySignatureSets(big);
  assert.strictEqual(pool.verifySignatureSets([k4[0]], {verifyOnMainThread: true}) instanceof Promise, true);
  assert.strictEqual(await inflightBatch, true);
  assert.ok(pool.stats.batchRetries >= 1);  // the false / rejected golden jobs above
  // close(): queued jobs abort with QueueError(QUEUE_ABORTED) (util/queue/errors.ts:3-6)
  const pendingP = pool.verifySignatureSets(k4, {batchable: true});
  let qerr = null;
  pendingP.catch((e) => { qerr = e; });
  await pool.close();
  await pendingP.catch(() => {});
  assert.ok(qerr instanceof m.QueueError);
  assert.strictEqual(qerr.type.code, m.QueueErrorCode.QUEUE_ABORTED);
  assert.strictEqual(qerr.message, "QUEUE_ERROR_QUEUE_ABORTED");
  await assert.rejects(pool.verifySignatureSets(k4), (e) => e.type.code === "QUEUE_ERROR_QUEUE_ABORTED");
  console.log("js gpu ok");
}

(process.argv[2] === "gpu" ? gpuTests() : Promise.resolve(cpuTests())).catch((e) => {
  console.error(e);
  process.exit(1);
});
