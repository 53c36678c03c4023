"use strict";
/**
 * MI355X drop-in for Lodestar's IBlsVerifier (packages/beacon-node/src/chain/bls/interface.ts:20-46).
 *
 * Same contract and observable policy as BlsMultiThreadWorkerPool (multithread/index.ts:98-424):
 *   - a call is split into jobs of >= 128 sets (chunkifyMaximizeChunkSize, multithread/utils.ts:4-19);
 *   - batchable jobs are buffered until > 32 sigs or 100 ms (:48, :57, :257-275);
 *   - non-batchable jobs run on the next tick (:280-283);
 *   - verifyOnMainThread verifies synchronously on the caller's thread (:138-151);
 *   - each job resolves true / false or rejects with the blst error string, independently of the
 *     other jobs in the same GPU batch (multithread.test.ts:86-103);
 *   - close() rejects queued jobs with QUEUE_ABORTED (:176-197).
 * Instead of worker threads, one runner hands every queued job to the GPU as ONE batch through the
 * N-API addon (../napi/lb_napi.c -> include/lodestar_bls.h); the event loop is never blocked.
 *
 * Public keys: a `PublicKey` here is anything with `toBytes()` returning the 96-byte uncompressed
 * encoding (what the reference main thread sends to workers: getAggregatedPubkey(s).toBytes(
 * PointFormat.uncompressed), multithread/index.ts:160), or a 96-byte Uint8Array.
 */
const path = require("path");

const addon = require(path.join(__dirname, "..", "napi", "lodestar_bls.node"));

const MAX_SIGNATURE_SETS_PER_JOB = 128;
const MAX_BUFFERED_SIGS = 32;
const MAX_BUFFER_WAIT_MS = 100;

const SignatureSetType = {single: "single", aggregate: "aggregate"};

class QueueError extends Error {
  constructor(code) {
    super(code);
    this.type = {code: code};
  }
}

/** multithread/utils.ts:4-19 */
function chunkifyMaximizeChunkSize(arr, minPerChunk) {
  const chunkCount = Math.floor(arr.length / minPerChunk);
  if (chunkCount <= 1) return [arr];
  const perChunk = Math.ceil(arr.length / chunkCount);
  const out = [];
  for (let i = 0; i < arr.length; i += perChunk) out.push(arr.slice(i, i + perChunk));
  return out;
}

function pkBytes(pk) {
  const b = pk instanceof Uint8Array ? pk : pk.toBytes();
  if (b.length !== 96) throw Error("pubkey must be 96-byte uncompressed");
  return b;
}

/** jobs: ISignatureSet[][] -> flat typed arrays of the C ABI */
function packJobs(jobs) {
  let nSets = 0;
  let nPks = 0;
  for (const job of jobs)
    for (const s of job) {
      nSets++;
      nPks += s.type === SignatureSetType.single ? 1 : s.pubkeys.length;
    }
  const jobOff = new Uint32Array(jobs.length + 1);
  const pkOff = new Uint32Array(nSets + 1);
  const pks = new Uint8Array(nPks * 96);
  const roots = new Uint8Array(nSets * 32);
  const sigs = new Uint8Array(nSets * 96);
  const sizes = new Uint32Array(nSets);
  let odd = false;
  let si = 0;
  let pi = 0;
  jobs.forEach((job, j) => {
    for (const s of job) {
      const list = s.type === SignatureSetType.single ? [s.pubkey] : s.pubkeys;
      for (const pk of list) pks.set(pkBytes(pk), 96 * pi++);
      pkOff[si + 1] = pi;
      const root = s.signingRoot instanceof Uint8Array ? s.signingRoot : Uint8Array.from(s.signingRoot);
      if (root.length !== 32) throw Error("signing root must be 32 bytes");
      roots.set(root, 32 * si);
      sizes[si] = s.signature.length;
      if (s.signature.length === 96) sigs.set(s.signature, 96 * si);
      else odd = true;
      si++;
    }
    jobOff[j + 1] = si;
  });
  return [jobOff, pkOff, pks, roots, sigs, odd ? sizes : null];
}

function codeToResult(code) {
  if (code < 0) throw Error(addon.errorName(-code));
  return code === 1;
}

class BlsGpuVerifier {
  /**
   * @param {{device?: number, blsVerifyAllMultiThread?: boolean}} [opts]
   */
  constructor(opts) {
    opts = opts || {};
    this.engine = addon.createEngine(opts.device === undefined ? 0 : opts.device);
    this.blsVerifyAllMultiThread = Boolean(opts.blsVerifyAllMultiThread);
    this.jobs = [];
    this.buffered = null;
    this.running = null;
    this.closed = false;
  }

  /**
   * @param {Array} sets ISignatureSet[]
   * @param {{batchable?: boolean, verifyOnMainThread?: boolean}} [opts]
   * @returns {Promise<boolean>}
   */
  async verifySignatureSets(sets, opts) {
    opts = opts || {};
    if (this.closed) throw new QueueError("QUEUE_ABORTED");
    if (opts.verifyOnMainThread && !this.blsVerifyAllMultiThread) {
      const res = addon.verifyJobsSync(this.engine, ...packJobs([sets]));
      return codeToResult(res[0]);
    }
    const results = await Promise.all(
      chunkifyMaximizeChunkSize(sets, MAX_SIGNATURE_SETS_PER_JOB).map((chunk) => this.queueJob(chunk, opts))
    );
    if (results.length === 0) throw Error("Empty results array");
    return results.every((v) => v === true);
  }

  async close() {
    this.closed = true;
    if (this.buffered) {
      clearTimeout(this.buffered.timeout);
      for (const job of this.buffered.jobs) job.reject(new QueueError("QUEUE_ABORTED"));
      this.buffered = null;
    }
    for (const job of this.jobs.splice(0)) job.reject(new QueueError("QUEUE_ABORTED"));
    if (this.running) await this.running;
    addon.destroyEngine(this.engine);
  }

  queueJob(sets, opts) {
    return new Promise((resolve, reject) => {
      const job = {sets, resolve, reject};
      if (opts.batchable) {
        if (!this.buffered) {
          this.buffered = {jobs: [], sigCount: 0, timeout: setTimeout(() => this.flushBuffer(), MAX_BUFFER_WAIT_MS)};
        }
        this.buffered.jobs.push(job);
        this.buffered.sigCount += sets.length;
        if (this.buffered.sigCount > MAX_BUFFERED_SIGS) this.flushBuffer();
      } else {
        this.jobs.push(job);
        setTimeout(() => this.runJobs(), 0);
      }
    });
  }

  flushBuffer() {
    if (!this.buffered) return;
    clearTimeout(this.buffered.timeout);
    this.jobs.push(...this.buffered.jobs);
    this.buffered = null;
    setTimeout(() => this.runJobs(), 0);
  }

  runJobs() {
    if (this.running || this.jobs.length === 0) return;
    this.running = (async () => {
      while (this.jobs.length > 0) {
        const pkg = this.jobs.splice(0);
        let codes;
        try {
          codes = await addon.verifyJobs(this.engine, ...packJobs(pkg.map((j) => j.sets)));
        } catch (e) {
          for (const j of pkg) j.reject(e);
          continue;
        }
        pkg.forEach((j, k) => {
          if (codes[k] < 0) j.reject(Error(addon.errorName(-codes[k])));
          else j.resolve(codes[k] === 1);
        });
      }
      this.running = null;
    })();
  }
}

module.exports = {
  BlsGpuVerifier,
  QueueError,
  SignatureSetType,
  chunkifyMaximizeChunkSize,
  packJobs,
  addon,
  MAX_SIGNATURE_SETS_PER_JOB,
  MAX_BUFFERED_SIGS,
  MAX_BUFFER_WAIT_MS,
};
