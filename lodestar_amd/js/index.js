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
 * Instead of worker threads, `engines` GPU engines (default 2; each one batch in flight with its own
 * HIP streams and device workspace) take packages from one queue: an idle engine drains EVERY
 * queued job into one device batch through the N-API addon (../napi/lb_napi.c ->
 * include/lodestar_bls.h), like the reference's idle worker taking the next package
 * (multithread/index.ts:290-330).  The event loop is never blocked.
 *
 * Public keys: a `PublicKey` here is
 *   - a handle returned by registerPubkeys() (the epoch cache's index2pubkey entries,
 *     state-transition/src/cache/pubkeyCache.ts:56-77): it carries its index into the
 *     GPU-resident key table, and packages whose keys all have one ship 4-byte indices;
 *   - or anything with `toBytes()` returning the 96-byte uncompressed encoding (what the reference
 *     main thread sends to workers: getAggregatedPubkey(s).toBytes(PointFormat.uncompressed),
 *     multithread/index.ts:160), or a 96-byte Uint8Array.
 * Malformed inputs (root not 32 bytes, pubkey not 96 bytes, signature not a Uint8Array) reject
 * only the call that carries them, before anything is queued.
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
  if (!(b instanceof Uint8Array) || b.length !== 96) throw Error("pubkey must be 96-byte uncompressed");
  return b;
}

function setPubkeys(s) {
  if (s.type === SignatureSetType.single) return [s.pubkey];
  if (s.type === SignatureSetType.aggregate) return s.pubkeys;
  throw Error("Unknown signature set type");
}

/** Checks one call's sets before queueing: a malformed set rejects only its own call. */
function validateSets(sets) {
  for (const s of sets) {
    const pks = setPubkeys(s);
    if (!Array.isArray(pks)) throw Error("aggregate set needs a pubkeys array");
    for (const pk of pks) if (!(pk instanceof GpuPublicKey)) pkBytes(pk);
    const root = s.signingRoot;
    if (!root || root.length !== 32) throw Error("signing root must be 32 bytes");
    if (!(s.signature instanceof Uint8Array)) throw Error("signature must be a Uint8Array");
  }
}

/** A public key registered in the GPU-resident table (index2pubkey entry). */
class GpuPublicKey {
  constructor(index, bytes96) {
    this.index = index;
    this.bytes = bytes96;
  }
  toBytes() {
    return this.bytes;
  }
}

/** jobs: ISignatureSet[][] -> flat typed arrays of the C ABI (indices when every key has one) */
function packJobs(jobs) {
  let nSets = 0;
  let nPks = 0;
  let indexed = true;
  for (const job of jobs)
    for (const s of job) {
      nSets++;
      const list = setPubkeys(s);
      nPks += list.length;
      if (indexed) for (const pk of list) if (!(pk instanceof GpuPublicKey)) indexed = false;
    }
  const jobOff = new Uint32Array(jobs.length + 1);
  const pkOff = new Uint32Array(nSets + 1);
  const pks = indexed ? new Uint32Array(nPks) : new Uint8Array(nPks * 96);
  const roots = new Uint8Array(nSets * 32);
  const sigs = new Uint8Array(nSets * 96);
  const sizes = new Uint32Array(nSets);
  let odd = false;
  let si = 0;
  let pi = 0;
  jobs.forEach((job, j) => {
    for (const s of job) {
      const list = setPubkeys(s);
      if (indexed) for (const pk of list) pks[pi++] = pk.index;
      else for (const pk of list) pks.set(pkBytes(pk), 96 * pi++);
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
   * @param {{device?: number, engines?: number, blsVerifyAllMultiThread?: boolean}} [opts]
   */
  constructor(opts) {
    opts = opts || {};
    const n = opts.engines === undefined ? 2 : opts.engines;
    if (!(n >= 1)) throw Error("engines must be >= 1");
    this.engines = [];
    for (let k = 0; k < n; k++) this.engines.push(addon.createEngine(opts.device === undefined ? 0 : opts.device));
    this.idle = this.engines.slice();
    this.blsVerifyAllMultiThread = Boolean(opts.blsVerifyAllMultiThread);
    this.jobs = [];
    this.buffered = null;
    this.running = new Set();
    this.closed = false;
    this.stats = {batches: 0, jobs: 0, sets: 0, batchRetries: 0, jobsInvalid: 0, jobsError: 0};
  }

  /**
   * Loads keys (each 48-byte compressed or 96-byte uncompressed) into every engine's resident
   * table once, like the epoch cache's index2pubkey (pubkeyCache.ts:56-77).  Returns handles
   * usable as ISignatureSet pubkeys.  Keys are decoded on the GPU; a bad key throws its blst error.
   * @param {Uint8Array[]} keys
   * @returns {GpuPublicKey[]}
   */
  registerPubkeys(keys, validate) {
    if (keys.length === 0) return [];
    const size = keys[0].length;
    if (size !== 48 && size !== 96) throw Error("keys must be 48 or 96 bytes");
    let flat = new Uint8Array(keys.length * size);
    keys.forEach((k, i) => {
      if (k.length !== size) throw Error("keys must all have the same size");
      flat.set(k, i * size);
    });
    if (size === 48) {
      // decompressed once on the GPU: handles keep the 96-byte form for byte-carrying packages
      const d = addon.g1Decompress(this.engines[0], flat);
      for (const st of d.status) if (st !== 0) throw Error(addon.errorName(st));
      flat = d.out;
    }
    let first = -1;
    for (const e of this.engines) {
      const r = addon.registerPubkeys(e, flat, 96, Boolean(validate));
      for (const st of r.status) if (st !== 0) throw Error(addon.errorName(st));
      if (first >= 0 && r.first !== first) throw Error("engine pubkey tables out of step");
      first = r.first;
    }
    return keys.map((k, i) => new GpuPublicKey(first + i, flat.subarray(96 * i, 96 * i + 96)));
  }

  /**
   * state-transition verifySignatureSet (src/util/signatureSets.ts:24-38): synchronous; `single`
   * -> Signature.verify, `aggregate` -> Signature.verifyAggregate; throws the blst error on
   * malformed input.
   * @returns {boolean}
   */
  verifySignatureSet(set) {
    validateSets([set]);
    return codeToResult(addon.verifyJobsSync(this.engines[0], ...packJobs([[set]]))[0]);
  }

  /**
   * bls.Signature.aggregate(signatures).toBytes() for block production (chain/opPools/*).
   * @param {Uint8Array[]} signatures 96-byte compressed
   * @returns {Uint8Array} 96-byte compressed aggregate
   */
  aggregateSignatures(signatures, validate) {
    const flat = new Uint8Array(96 * signatures.length);
    const sizes = new Uint32Array(signatures.length);
    let odd = false;
    signatures.forEach((sg, i) => {
      sizes[i] = sg.length;
      if (sg.length === 96) flat.set(sg, 96 * i);
      else odd = true;
    });
    const r = addon.aggregateSignatures(this.engines[0], Uint32Array.from([0, signatures.length]), flat,
      odd ? sizes : null, validate === undefined ? true : Boolean(validate));
    if (r.status[0] !== 0) throw Error(addon.errorName(r.status[0]));
    return r.out;
  }

  /**
   * @param {Array} sets ISignatureSet[]
   * @param {{batchable?: boolean, verifyOnMainThread?: boolean}} [opts]
   * @returns {Promise<boolean>}
   */
  verifySignatureSets(sets, opts) {
    // not `async`: a gossip call (one job of <= 128 sets) returns its job's own promise, so a call
    // costs one promise instead of four (the per-call promise machinery dominated the JS side)
    opts = opts || {};
    try {
      if (this.closed) throw new QueueError("QUEUE_ABORTED");
      validateSets(sets);
      if (opts.verifyOnMainThread && !this.blsVerifyAllMultiThread) {
        const res = addon.verifyJobsSync(this.engines[0], ...packJobs([sets]));
        return Promise.resolve(codeToResult(res[0]));
      }
    } catch (e) {
      return Promise.reject(e);
    }
    // (an empty call is one empty job, which rejects with "Empty signature set" as in the reference)
    if (sets.length < 2 * MAX_SIGNATURE_SETS_PER_JOB) return this.queueJob(sets, opts);
    return Promise.all(
      chunkifyMaximizeChunkSize(sets, MAX_SIGNATURE_SETS_PER_JOB).map((chunk) => this.queueJob(chunk, opts))
    ).then((results) => results.every((v) => v === true));
  }

  async close() {
    this.closed = true;
    if (this.buffered) {
      clearTimeout(this.buffered.timeout);
      for (const job of this.buffered.jobs) job.reject(new QueueError("QUEUE_ABORTED"));
      this.buffered = null;
    }
    for (const job of this.jobs.splice(0)) job.reject(new QueueError("QUEUE_ABORTED"));
    await Promise.all([...this.running]);
    for (const e of this.engines) addon.destroyEngine(e);
    this.engines = [];
    this.idle = [];
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

  /** every idle engine takes the whole queue as one package (multithread/index.ts:290-330) */
  runJobs() {
    while (this.idle.length > 0 && this.jobs.length > 0 && !this.closedEngines()) {
      const engine = this.idle.pop();
      const pkg = this.jobs.splice(0);
      const p = this.runPackage(engine, pkg).finally(() => {
        this.running.delete(p);
        if (this.engines.includes(engine)) this.idle.push(engine);
        if (this.jobs.length > 0) this.runJobs();
      });
      this.running.add(p);
    }
  }

  closedEngines() {
    return this.engines.length === 0;
  }

  async runPackage(engine, pkg) {
    let codes;
    try {
      codes = await addon.verifyJobs(engine, ...packJobs(pkg.map((j) => j.sets)));
    } catch (e) {
      // device failure: every job of the package rejects (multithread/index.ts:368-375)
      for (const j of pkg) j.reject(e);
      return;
    }
    this.stats.batches++;
    this.stats.jobs += pkg.length;
    pkg.forEach((j, k) => {
      this.stats.sets += j.sets.length;
      if (codes[k] < 0) {
        this.stats.jobsError++;
        j.reject(Error(addon.errorName(-codes[k])));
      } else {
        if (codes[k] === 0) this.stats.jobsInvalid++;
        j.resolve(codes[k] === 1);
      }
    });
  }
}

/**
 * light-client/src/validation.ts:154-184 isValidBlsAggregate: aggregate the participants' keys,
 * decode the signature, verify -- with the reference's stage-prefixed error messages.
 */
function isValidBlsAggregate(verifier, publicKeys, message, signature) {
  try {
    return verifier.verifySignatureSet({type: SignatureSetType.aggregate, pubkeys: publicKeys, signingRoot: message,
                                        signature});
  } catch (e) {
    const stage = e.message === "EMPTY_AGGREGATE_ARRAY" ? "Error aggregating pubkeys"
      : e.message === "BLST_PK_IS_INFINITY" ? "Error verifying signature" : "Error deserializing signature";
    e.message = `${stage}: ${e.message}`;
    throw e;
  }
}

module.exports = {
  BlsGpuVerifier,
  isValidBlsAggregate,
  GpuPublicKey,
  QueueError,
  SignatureSetType,
  chunkifyMaximizeChunkSize,
  packJobs,
  addon,
  MAX_SIGNATURE_SETS_PER_JOB,
  MAX_BUFFERED_SIGS,
  MAX_BUFFER_WAIT_MS,
};
