"use strict";
/**
 * The `c-kzg` module surface Lodestar binds (packages/beacon-node/src/util/kzg.ts:15-65):
 *   loadTrustedSetup(filePath), blobToKzgCommitment(blob), computeAggregateKzgProof(blobs),
 *   verifyAggregateKzgProof(blobs, expectedKzgCommitments, kzgAggregatedProof)
 * so `ckzg = require("@lodestar/bls-mi355x/kzg")` replaces `await import("c-kzg")` (initCKZG).
 *
 * The scalar-field work runs here in BigInt (inverse NTT of the blob's evaluations to monomial
 * coefficients, the Fiat-Shamir transcript of the EIP-4844 spec's compute_challenges, Horner
 * evaluation, the quotient by synthetic division); the group work runs on the GPU through the
 * addon (kzgLoadSetup / g1Lincomb / kzgVerifyProof -> include/lodestar_bls.h lb_kzg_*), as in
 * lodestar_amd/kzg.py, which it mirrors line for line.  The setup file is the text format
 * kzg.ts writes (trustedSetupJsonToTxt: "4096", "65", then hex points) or Lodestar's
 * trusted_setup.bin.  Field elements are big-endian (blobsSidecar.ts:138-150).  Parity with
 * c-kzg's bytes is unpinned (DESIGN.md §5.1); calls are synchronous, as c-kzg's are.
 */
const crypto = require("crypto");
const fs = require("fs");
const path = require("path");

const addon = require(path.join(__dirname, "..", "napi", "lodestar_bls.node"));

const R = 52435875175126190479447740508185965837690552500527637822603658699938581184513n;
const N = 4096;
const BYTES_PER_BLOB = 32 * N;
const DOMAIN = Buffer.from("FSBLOBVERIFY_V1_", "ascii");

function powmod(b, e) {
  let r = 1n;
  b %= R;
  while (e > 0n) {
    if (e & 1n) r = (r * b) % R;
    b = (b * b) % R;
    e >>= 1n;
  }
  return r;
}
const mod = (a) => ((a % R) + R) % R;

const BRP = (() => {
  const bits = Math.log2(N);
  const out = new Array(N);
  for (let i = 0; i < N; i++) {
    let r = 0;
    for (let b = 0; b < bits; b++) if (i & (1 << b)) r |= 1 << (bits - 1 - b);
    out[i] = r;
  }
  return out;
})();
const ROOTS = (() => {
  const w = powmod(7n, (R - 1n) / BigInt(N));
  const out = new Array(N);
  let x = 1n;
  for (let i = 0; i < N; i++) {
    out[i] = x;
    x = (x * w) % R;
  }
  return out;
})();

function ntt(a, roots) {
  const n = a.length;
  const v = new Array(n);
  for (let i = 0; i < n; i++) v[i] = a[BRP[i]];
  for (let m = 1; m < n; m *= 2) {
    const step = n / (2 * m);
    for (let s = 0; s < n; s += 2 * m) {
      for (let j = 0; j < m; j++) {
        const u = v[s + j];
        const t = (v[s + j + m] * roots[j * step]) % R;
        v[s + j] = (u + t) % R;
        v[s + j + m] = mod(u - t);
      }
    }
  }
  return v;
}

function bytesToBig(b) {
  return BigInt("0x" + (Buffer.from(b).toString("hex") || "0"));
}
function bigToBytes(x, n, little) {
  const hex = x.toString(16).padStart(2 * n, "0");
  const buf = Buffer.from(hex, "hex");
  return little ? Buffer.from(buf.reverse()) : buf;
}

function blobToPolynomial(blob) {
  if (!(blob instanceof Uint8Array) || blob.length !== BYTES_PER_BLOB) throw Error("blob length != 131072");
  const out = new Array(N);
  for (let i = 0; i < N; i++) {
    const v = bytesToBig(blob.subarray(32 * i, 32 * i + 32));
    if (v >= R) throw Error("blob field element >= BLS_MODULUS");
    out[i] = v;
  }
  return out;
}
function evaluationsToCoefficients(poly) {
  const nat = new Array(N);
  for (let i = 0; i < N; i++) nat[BRP[i]] = poly[i];
  const inv = new Array(N);
  for (let k = 0; k < N; k++) inv[k] = ROOTS[(N - k) % N];
  const invN = powmod(BigInt(N), R - 2n);
  return ntt(nat, inv).map((c) => (c * invN) % R);
}
function evaluate(coeffs, z) {
  let y = 0n;
  for (let k = coeffs.length - 1; k >= 0; k--) y = (y * z + coeffs[k]) % R;
  return y;
}
function quotient(coeffs, z) {
  const q = new Array(coeffs.length - 1);
  let acc = 0n;
  for (let k = coeffs.length - 1; k > 0; k--) {
    acc = (acc * z + coeffs[k]) % R;
    q[k - 1] = acc;
  }
  return q;
}
function hashToBlsField(data) {
  return bytesToBig(crypto.createHash("sha256").update(data).digest()) % R;
}
function computeChallenges(polys, commitments) {
  const parts = [DOMAIN, bigToBytes(BigInt(N), 8, false), bigToBytes(BigInt(polys.length), 8, false)];
  for (const p of polys) for (const v of p) parts.push(bigToBytes(v, 32, false));
  for (const c of commitments) parts.push(Buffer.from(c));
  const h = crypto.createHash("sha256").update(Buffer.concat(parts)).digest();
  const r = hashToBlsField(Buffer.concat([h, Buffer.from([0])]));
  const powers = [];
  let x = 1n;
  for (let i = 0; i < commitments.length; i++) {
    powers.push(x);
    x = (x * r) % R;
  }
  return {rPowers: powers, x: hashToBlsField(Buffer.concat([h, Buffer.from([1])]))};
}
function scalarsLE(vals) {
  const out = new Uint8Array(32 * vals.length);
  vals.forEach((v, i) => out.set(bigToBytes(v, 32, true), 32 * i));
  return out;
}

let engine = null;
function requireSetup() {
  if (!engine) throw Error("c-kzg library not loaded");
}

function parseSetup(filePath) {
  const raw = fs.readFileSync(filePath);
  let g1 = [];
  let g2 = [];
  if (raw.length === 8 + 4096 * 48 + 65 * 96) {
    for (let i = 0; i < 4096; i++) g1.push(raw.subarray(8 + 48 * i, 8 + 48 * (i + 1)));
    const base = 8 + 4096 * 48;
    for (let i = 0; i < 65; i++) g2.push(raw.subarray(base + 96 * i, base + 96 * (i + 1)));
  } else {
    const lines = raw.toString("utf8").split(/\s+/).filter((l) => l.length);
    const n1 = parseInt(lines[0], 10);
    const n2 = parseInt(lines[1], 10);
    g1 = lines.slice(2, 2 + n1).map((h) => Buffer.from(h, "hex"));
    g2 = lines.slice(2 + n1, 2 + n1 + n2).map((h) => Buffer.from(h, "hex"));
  }
  return {g1: Buffer.concat(g1), g2: Buffer.concat(g2)};
}

function loadTrustedSetup(filePath, device = 0) {
  const {g1, g2} = parseSetup(filePath);
  const e = engine || addon.createEngine(device);
  addon.kzgLoadSetup(e, new Uint8Array(g1), new Uint8Array(g2));
  engine = e;
}

function commitCoefficients(coeffs) {
  return addon.g1Lincomb(engine, scalarsLE(coeffs));
}
function blobToKzgCommitment(blob) {
  requireSetup();
  return commitCoefficients(evaluationsToCoefficients(blobToPolynomial(blob)));
}
function aggregate(blobs, commitments) {
  const polys = blobs.map(blobToPolynomial);
  const {rPowers, x} = computeChallenges(polys, commitments);
  const agg = new Array(N);
  for (let i = 0; i < N; i++) {
    let s = 0n;
    for (let j = 0; j < polys.length; j++) s += rPowers[j] * polys[j][i];
    agg[i] = s % R;
  }
  return {agg, rPowers, x};
}
// compressed point at infinity: the proof of zero blobs (the zero polynomial)
const G1_INFINITY48 = Uint8Array.from([0xc0, ...new Array(47).fill(0)]);

function computeAggregateKzgProof(blobs) {
  requireSetup();
  // chain.ts:402 calls this for every produced block, blobless ones included
  if (!blobs.length) return G1_INFINITY48.slice();
  const commitments = blobs.map(blobToKzgCommitment);
  const {agg, x} = aggregate(blobs, commitments);
  return commitCoefficients(quotient(evaluationsToCoefficients(agg), x));
}
function verifyAggregateKzgProof(blobs, expectedKzgCommitments, kzgAggregatedProof) {
  requireSetup();
  if (blobs.length !== expectedKzgCommitments.length) throw Error("blobs / commitments length mismatch");
  if (!blobs.length) {
    // aggregated commitment = infinity, y = 0: true iff the proof is infinity (still decoded)
    const {x} = computeChallenges([], []);
    return addon.kzgVerifyProof(engine, G1_INFINITY48, bigToBytes(x, 32, true), bigToBytes(0n, 32, true), kzgAggregatedProof);
  }
  const {agg, rPowers, x} = aggregate(blobs, expectedKzgCommitments);
  const pts = new Uint8Array(48 * expectedKzgCommitments.length);
  expectedKzgCommitments.forEach((c, i) => pts.set(c, 48 * i));
  const c = addon.g1Lincomb(engine, scalarsLE(rPowers), pts);
  const y = evaluate(evaluationsToCoefficients(agg), x);
  return addon.kzgVerifyProof(engine, c, bigToBytes(x, 32, true), bigToBytes(y, 32, true), kzgAggregatedProof);
}

module.exports = {
  loadTrustedSetup,
  blobToKzgCommitment,
  computeAggregateKzgProof,
  verifyAggregateKzgProof,
  G1_INFINITY48,
  // host field work, exported for tests
  _internal: {evaluationsToCoefficients, evaluate, quotient, computeChallenges, ROOTS, BRP, R},
};
