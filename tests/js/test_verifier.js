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
