"use strict";
// KZG through the JS c-kzg surface (lodestar_amd/js/kzg.js).  Mode "cpu": the BigInt field work
// (inverse NTT, challenges) printed as JSON for tests/test_js.py to compare with the Python host
// and the oracle.  Mode "gpu": kzg.test.ts's round trip (two blobs -> commitments -> aggregate
// proof -> verifies), tampering, and the bytes printed for comparison with lodestar_amd/kzg.py.
const path = require("path");
const assert = require("assert");
const kzg = require(path.join(__dirname, "..", "..", "lodestar_amd", "js", "kzg.js"));
const I = kzg._internal;

function sequentialBlob(off) {
  const b = new Uint8Array(4096 * 32);
  const dv = new DataView(b.buffer);
  for (let i = 0; i < 4096; i++) dv.setUint32(i * 32, (i + off) >>> 0);
  return b;
}
const hex = (u) => Buffer.from(u).toString("hex");

const mode = process.argv[2];
if (mode === "cpu") {
  // p(X) = 5 + 3 X + 11 X^4095 evaluated at the bit-reversed roots, then recovered
  const vals = I.ROOTS.map((_, i) => {
    const x = I.ROOTS[I.BRP[i]];
    let xe = 1n;
    for (let k = 0; k < 4095; k++) xe = (xe * x) % I.R;
    return (5n + 3n * x + 11n * xe) % I.R;
  });
  const c = I.evaluationsToCoefficients(vals);
  assert.strictEqual(c[0], 5n);
  assert.strictEqual(c[1], 3n);
  assert.strictEqual(c[4095], 11n);
  for (let k = 2; k < 4095; k++) assert.strictEqual(c[k], 0n);
  const ch = I.computeChallenges([vals.slice(0, 4096)], [new Uint8Array(48).fill(0x11)]);
  console.log(JSON.stringify({r0: ch.rPowers[0].toString(), x: ch.x.toString(), y: I.evaluate(c, 12345n).toString()}));
  console.log("js kzg cpu ok");
} else {
  kzg.loadTrustedSetup(path.join(__dirname, "..", "..", "lodestar_amd", "trusted_setup.bin"));
  const blobs = [sequentialBlob(0), sequentialBlob(7)];
  const comms = blobs.map((b) => kzg.blobToKzgCommitment(b));
  const proof = kzg.computeAggregateKzgProof(blobs);
  assert.strictEqual(kzg.verifyAggregateKzgProof(blobs, comms, proof), true);
  const bad = Uint8Array.from(blobs[1]);
  bad[31] ^= 1;
  assert.strictEqual(kzg.verifyAggregateKzgProof([blobs[0], bad], comms, proof), false);
  assert.strictEqual(kzg.verifyAggregateKzgProof(blobs, comms.slice().reverse(), proof), false);
  // zero blobs (a blobless block, chain.ts:402): the proof is the point at infinity
  const inf = kzg.computeAggregateKzgProof([]);
  assert.strictEqual(hex(inf), "c0" + "00".repeat(47));
  assert.strictEqual(kzg.verifyAggregateKzgProof([], [], inf), true);
  assert.strictEqual(kzg.verifyAggregateKzgProof([], [], proof), false);
  console.log(JSON.stringify({commitments: comms.map(hex), proof: hex(proof)}));
  console.log("js kzg gpu ok");
}
