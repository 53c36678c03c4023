"use strict";
/**
 * MI355X drop-in for Lodestar's IBlsVerifier (packages/beacon-node/src/chain/bls/interface.ts:20-46).
 *
 * Same contract and observable policy as BlsMultiThreadWorkerPool (multithread/index.ts:98-424):
 *   - a call is split into jobs of >= 128 sets (chunkifyMaximizeChunkSize, multithread/utils.ts:4-19);
 *   - batchable jobs are buffered until > 32 sigs or 100 ms (:48, :57, :257-275);
 *   - non-batchable jobs run on the next tick (:280-283);
 *   - verifyOnMainThread goes straight to its own latency engine, past the buffer and the queue
 *     (:138-151); the reference runs it synchronously and blocks the event loop for the whole
 *     verification, here only the marshalling runs on the loop and the Promise<boolean> settles
 *     when the device is done (the contract is the same Promise);
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
 *   - or a `@chainsafe/bls` `PublicKey` (anything with `toBytes(format)`): it is serialised with
 *     `toBytes("uncompressed")`, exactly as the reference main thread does before posting to a
 *     worker (getAggregatedPubkey(s).toBytes(PointFormat.uncompressed), multithread/index.ts:126,160).
 *     An object whose toBytes ignores the format and returns the 48-byte compressed default is
 *     decompressed on the GPU.  The 96 bytes are cached per key object (WeakMap), so a long-lived
 *     index2pubkey entry is serialised once, not once per call;
 *   - or a 96-byte (uncompressed) or 48-byte (compressed) Uint8Array.
 * Malformed inputs (root not 32 bytes, pubkey of another length, signature not a Uint8Array)
 * reject only the call that carries them, before anything is queued.
 *
 * Main-thread entry points (verifyOnMainThread, and the synchronous verifySignatureSet,
 * aggregateSignatures, key decompression) run on their own engine, outside the async pool, so a main-thread call never
 * waits behind a gossip batch holding a pool engine (the reference runs them on the main thread
 * while workers are busy, multithread/index.ts:138-151).
 */
const path = require("path");

const addon = require(path.join(__dirname, "..", "napi", "lodestar_bls.node"));

const MAX_SIGNATURE_SETS_PER_JOB = 128;
const MAX_BUFFERED_SIGS = 32;
const MAX_BUFFER_WAIT_MS = 100;

const SignatureSetType = {single: "single", aggregate: "aggregate"};

/** beacon-node/src/util/queue/errors.ts:3-14 (a LodestarError: message = type.code, utils/src/errors.ts:6-8) */
const QueueErrorCode = {
  QUEUE_ABORTED: "QUEUE_ERROR_QUEUE_ABORTED",
  QUEUE_MAX_LENGTH: "QUEUE_ERROR_QUEUE_MAX_LENGTH",
};

class QueueError extends Error {
  constructor(type) {
    super(type.code);
    this.type = type;
  }
  getMetadata() {
    return this.type;
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

/** PointFormat of @chainsafe/bls (its toBytes default is compressed, 48 bytes) */
const PointFormat = {compressed: "compressed", uncompressed: "uncompressed"};

// 96-byte uncompressed encodings of PublicKey objects seen before (index2pubkey entries live for
// the epoch cache's lifetime; the reference pays toBytes(uncompressed) on every call)
const pkCache = new WeakMap();

/** The 96- or 48-byte encoding of one key (48 only if its toBytes ignores the format argument). */
function pkRawBytes(pk) {
  if (pk instanceof Uint8Array) return pk;
  if (pk === null || typeof pk !== "object" || typeof pk.toBytes !== "function") throw Error("pubkey must be a PublicKey or Uint8Array");
  const hit = pkCache.get(pk);
  if (hit) return hit;
  const b = pk.toBytes(PointFormat.uncompressed);
  if (!(b instanceof Uint8Array) || (b.length !== 96 && b.length !== 48)) throw Error("pubkey must be 48 or 96 bytes");
  if (b.length === 96) pkCache.set(pk, b);
  return b;
}

/** 96-byte encoding of a key already normalised by normalizeKeys (packJobs only) */
function pkBytes(pk) {
  const b = pkRawBytes(pk);
  if (b.length !== 96) throw Error("pubkey must be 96-byte uncompressed");
  return b;
}

function setPubkeys(s) {
  if (s.type === SignatureSetType.single) return [s.pubkey];
  if (s.type === SignatureSetType.aggregate) return s.pubkeys;
  throw Error("Unknown signature set type");
}

/**
 * Checks one call's sets before queueing (a malformed set rejects only its own call) and returns
 * the sets with every 48-byte key replaced by its 96-byte form: compressed keys of the call are
 * decompressed on the GPU in one batch by `decompress(flat48) -> {out, status}`; a key that does not
 * decode rejects the call with its blst error.
 */
function normalizeSets(sets, decompress) {
  let short = null;  // [setIndex, keyIndex | -1, bytes48]
  sets.forEach((s, si) => {
    const pks = setPubkeys(s);
    if (!Array.isArray(pks)) throw Error("aggregate set needs a pubkeys array");
    pks.forEach((pk, ki) => {
      if (pk instanceof GpuPublicKey) return;
      const b = pkRawBytes(pk);
      if (b.length === 48) (short = short || []).push([si, s.type === SignatureSetType.single ? -1 : ki, b, pk]);
    });
    const root = s.signingRoot;
    if (!root || root.length !== 32) throw Error("signing root must be 32 bytes");
    if (!(s.signature instanceof Uint8Array)) throw Error("signature must be a Uint8Array");
  });
  if (short === null) return sets;
  const flat = new Uint8Array(48 * short.length);
  short.forEach(([, , b], k) => flat.set(b, 48 * k));
  const d = decompress(flat);
  d.status.forEach((st) => {
    if (st !== 0) throw Error(addon.errorName(st));
  });
  const out = sets.slice();
  short.forEach(([si, ki, , pk], k) => {
    const b96 = d.out.subarray(96 * k, 96 * k + 96);
    if (!(pk instanceof Uint8Array)) pkCache.set(pk, b96);
    if (out[si] === sets[si]) out[si] = ki < 0 ? {...sets[si]} : {...sets[si], pubkeys: sets[si].pubkeys.slice()};
    if (ki < 0) out[si].pubkey = b96;
    else out[si].pubkeys[ki] = b96;
  });
  return out;
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
   * @param {{device?: number, engines?: number, blsVerifyAllMultiThread?: boolean, latencyPartition?: boolean}} [opts]
   * @param {{logger?: object, metrics?: object|null}} [modules] as the reference pool's
   *   (multithread/index.ts:98-134): `metrics.blsThreadPool.*` / `metrics.bls.*` receive the same
   *   updates (lodestar.ts:433-523) when given
   */
  constructor(opts, modules) {
    opts = opts || {};
    modules = modules || {};
    const n = opts.engines === undefined ? 2 : opts.engines;
    if (!(n >= 1)) throw Error("engines must be >= 1");
    const device = opts.device === undefined ? 0 : opts.device;
    this.engines = [];
    try {
      // synchronous calls get their own engine, created first as the device's latency engine
      // (LB_ENGINE_LATENCY: its own reserved CUs, the pool's engines on the rest), so a
      // verifyOnMainThread call is neither queued behind a pool batch's engine mutex nor behind
      // the pool's kernels on the device
      try {
        this.syncEngine = addon.createEngine(device, opts.latencyPartition === false ? 0 : 1);
      } catch (e) {
        this.syncEngine = addon.createEngine(device);
      }
      for (let k = 0; k < n; k++) this.engines.push(addon.createEngine(device));
    } catch (e) {
      for (const en of this.engines) addon.destroyEngine(en);
      if (this.syncEngine) addon.destroyEngine(this.syncEngine);
      throw e;
    }
    this.idle = this.engines.slice();
    this.blsVerifyAllMultiThread = Boolean(opts.blsVerifyAllMultiThread);
    this.logger = modules.logger || null;
    this.metrics = modules.metrics || null;
    this.jobs = [];
    this.buffered = null;
    this.running = new Set();
    this.closed = false;
    this.stats = {batches: 0, jobs: 0, sets: 0, batchRetries: 0, batchSigsSuccess: 0, jobsInvalid: 0, jobsError: 0,
      jobWaitMs: 0, deviceMs: 0, mainThreadMs: 0};
    this.decompress = (flat48) => addon.g1Decompress(this.syncEngine, flat48);
  }

  /** every engine, the synchronous one included (they share one key-table layout) */
  allEngines() {
    return this.syncEngine ? [this.syncEngine, ...this.engines] : this.engines;
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
      const d = this.decompress(flat);
      for (const st of d.status) if (st !== 0) throw Error(addon.errorName(st));
      flat = d.out;
    }
    let first = -1;
    for (const e of this.allEngines()) {
      const r = addon.registerPubkeys(e, flat, 96, Boolean(validate));
      for (const st of r.status) if (st !== 0) throw Error(addon.errorName(st));
      if (first >= 0 && r.first !== first) throw Error("engine pubkey tables out of step");
      first = r.first;
    }
    return keys.map((k, i) => new GpuPublicKey(first + i, flat.subarray(96 * i, 96 * i + 96)));
  }

  /**
   * The reference's main-thread path (multithread/index.ts:138-151) without blocking the event
   * loop: one job on the latency engine through the addon's engine thread.  Malformed input
   * rejects the returned promise (the reference throws from the same call).
   */
  verifyMainThread(sets) {
    const t0 = Date.now();
    return addon.verifyJobs(this.syncEngine, ...packJobs([normalizeSets(sets, this.decompress)])).then((res) => {
      const dt = Date.now() - t0;
      this.stats.mainThreadMs += dt;
      if (this.metrics) this.metrics.blsThreadPool.mainThreadDurationInThreadPool.observe(dt / 1000);
      return codeToResult(res[0]);
    });
  }

  /** one job verified synchronously on the caller's thread (state-transition verifySignatureSet) */
  verifySync(sets) {
    const t0 = Date.now();
    const res = addon.verifyJobsSync(this.syncEngine, ...packJobs([normalizeSets(sets, this.decompress)]));
    const dt = Date.now() - t0;
    this.stats.mainThreadMs += dt;
    if (this.metrics) this.metrics.blsThreadPool.mainThreadDurationInThreadPool.observe(dt / 1000);
    return codeToResult(res[0]);
  }

  /**
   * state-transition verifySignatureSet (src/util/signatureSets.ts:24-38): synchronous; `single`
   * -> Signature.verify, `aggregate` -> Signature.verifyAggregate; throws the blst error on
   * malformed input.
   * @returns {boolean}
   */
  verifySignatureSet(set) {
    return this.verifySync([set]);
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
    const r = addon.aggregateSignatures(this.syncEngine, Uint32Array.from([0, signatures.length]), flat,
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
      if (this.closed) throw new QueueError({code: QueueErrorCode.QUEUE_ABORTED});
      if (this.metrics) this.metrics.bls.aggregatedPubkeys.inc(getAggregatedPubkeysCount(sets));
      if (opts.verifyOnMainThread && !this.blsVerifyAllMultiThread) return this.verifyMainThread(sets);
      sets = normalizeSets(sets, this.decompress);
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
      // (the reference only clears the timer and leaves these promises pending forever,
      // multithread/index.ts:176-180; here they reject like the queued jobs)
      clearTimeout(this.buffered.timeout);
      for (const job of this.buffered.jobs) job.reject(new QueueError({code: QueueErrorCode.QUEUE_ABORTED}));
      this.buffered = null;
    }
    for (const job of this.jobs.splice(0)) job.reject(new QueueError({code: QueueErrorCode.QUEUE_ABORTED}));
    await Promise.all([...this.running]);
    for (const e of this.allEngines()) addon.destroyEngine(e);
    this.engines = [];
    this.syncEngine = null;
    this.idle = [];
  }

  queueJob(sets, opts) {
    return new Promise((resolve, reject) => {
      const job = {sets, resolve, reject, addedTimeMs: Date.now()};
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
      if (this.metrics) this.metrics.blsThreadPool.queueLength.set(this.jobs.length);
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
    const m = this.metrics;
    const start = Date.now();
    let startedSigSets = 0;
    for (const j of pkg) {
      const wait = start - j.addedTimeMs;
      this.stats.jobWaitMs += wait;
      if (m) m.blsThreadPool.jobWaitTime.observe(wait / 1000);
      startedSigSets += j.sets.length;
    }
    if (m) {
      m.blsThreadPool.totalJobsGroupsStarted.inc(1);
      m.blsThreadPool.totalJobsStarted.inc(pkg.length);
      m.blsThreadPool.totalSigSetsStarted.inc(startedSigSets);
    }
    let codes;
    try {
      codes = await addon.verifyJobs(engine, ...packJobs(pkg.map((j) => j.sets)));
    } catch (e) {
      // device failure: every job of the package rejects (multithread/index.ts:368-375)
      if (!this.closed && this.logger) this.logger.error("BlsGpuVerifier error", {}, e);
      for (const j of pkg) j.reject(e);
      return;
    }
    const sec = (Date.now() - start) / 1000;
    this.stats.deviceMs += sec * 1000;
    this.stats.batches++;
    this.stats.jobs += pkg.length;
    let success = 0;
    let error = 0;
    let failed = false;
    pkg.forEach((j, k) => {
      this.stats.sets += j.sets.length;
      if (codes[k] < 0) {
        this.stats.jobsError++;
        error += j.sets.length;
        j.reject(Error(addon.errorName(-codes[k])));
      } else {
        if (codes[k] === 0) {
          this.stats.jobsInvalid++;
          failed = true;
        }
        success += j.sets.length;
        j.resolve(codes[k] === 1);
      }
    });
    // a package with a false job failed its batch equation and ran the invalid-set search (the
    // reference's batch retry, worker.ts:76-98); otherwise every live set was batch-verified
    const retries = failed ? 1 : 0;
    const batchSigs = failed ? 0 : success;
    this.stats.batchRetries += retries;
    this.stats.batchSigsSuccess += batchSigs;
    if (m) {
      m.blsThreadPool.timePerSigSet.observe(startedSigSets ? sec / startedSigSets : 0);
      m.blsThreadPool.jobsWorkerTime.inc({workerId: this.engines.indexOf(engine)}, sec);
      m.blsThreadPool.successJobsSignatureSetsCount.inc(success);
      m.blsThreadPool.errorJobsSignatureSetsCount.inc(error);
      m.blsThreadPool.batchRetries.inc(retries);
      m.blsThreadPool.batchSigsSuccess.inc(batchSigs);
    }
  }
}

/** chain/bls/utils.ts:18-26 */
function getAggregatedPubkeysCount(sets) {
  let n = 0;
  for (const s of sets) if (s.type === SignatureSetType.aggregate) n += s.pubkeys.length;
  return n;
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
  QueueErrorCode,
  PointFormat,
  SignatureSetType,
  normalizeSets,
  getAggregatedPubkeysCount,
  chunkifyMaximizeChunkSize,
  packJobs,
  addon,
  MAX_SIGNATURE_SETS_PER_JOB,
  MAX_BUFFERED_SIGS,
  MAX_BUFFER_WAIT_MS,
};
