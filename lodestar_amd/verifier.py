"""Host-side mirror of Lodestar's IBlsVerifier over the MI355X engine.

Reference interface and policy (paths under the reference repo):
  * IBlsVerifier / VerifySignatureOpts     packages/beacon-node/src/chain/bls/interface.ts:3-46
  * BlsMultiThreadWorkerPool policy        packages/beacon-node/src/chain/bls/multithread/index.ts:98-424
      - calls split into jobs of >=128 sets (chunkifyMaximizeChunkSize, :39,156; utils.ts:4-19)
      - batchable jobs buffered until >32 sigs or 100 ms (:48,57,257-275)
      - non-batchable jobs run on the next tick (:280-283)
      - verifyOnMainThread runs synchronously on the caller's thread (:138-151)
      - close() rejects queued jobs with QueueError(QUEUE_ABORTED) (:176-197)
  * per-job results (worker.ts:32-108): job j resolves true/false or rejects with its error,
    independently of every other job in the same batch (multithread.test.ts:86-103).

The worker threads are replaced by one GPU runner thread per engine (`n_engines` batches in
flight on the device, default 2): an idle runner drains every queued job into ONE device batch
(one final exponentiation for all valid jobs, a search for the failing sets when it fails),
instead of the reference's packages of ~128 sets per CPU worker and per-job re-verification.
Malformed inputs (root not 32 bytes, pubkey not a PublicKey, signature not bytes) raise in the
caller's own call before anything is queued, so they never touch other callers' jobs.
"""
from __future__ import annotations

import asyncio
import threading
import time
from dataclasses import dataclass, field
from enum import Enum
from typing import List, Optional, Sequence, Union

from .engine import BlsError, Engine, SetInput

MAX_SIGNATURE_SETS_PER_JOB = 128   # multithread/index.ts:39
MAX_BUFFERED_SIGS = 32             # multithread/index.ts:48
MAX_BUFFER_WAIT_MS = 100           # multithread/index.ts:57


class QueueErrorCode(str, Enum):
    """beacon-node/src/util/queue/errors.ts:3-6"""
    QUEUE_ABORTED = "QUEUE_ERROR_QUEUE_ABORTED"
    QUEUE_MAX_LENGTH = "QUEUE_ERROR_QUEUE_MAX_LENGTH"


class QueueError(Exception):
    """util/queue QueueError (a LodestarError: `type` = {code}, message = type.code,
    utils/src/errors.ts:6-8); code QUEUE_ABORTED after close()."""

    def __init__(self, type_: Optional[dict] = None):
        self.type = dict(type_ or {"code": QueueErrorCode.QUEUE_ABORTED.value})
        self.code = self.type["code"]
        super().__init__(self.code)


def chunkify_maximize_chunk_size(arr: Sequence, min_per_chunk: int) -> List[list]:
    """multithread/utils.ts:4-19: split into floor(n/min) chunks of ceil(n/count) items."""
    arr = list(arr)
    chunk_count = len(arr) // min_per_chunk
    if chunk_count <= 1:
        return [arr]
    per_chunk = -(-len(arr) // chunk_count)
    return [arr[i:i + per_chunk] for i in range(0, len(arr), per_chunk)]


class PublicKey:
    """A G1 public key held as its 96-byte uncompressed encoding (what the reference's main
    thread sends to workers: getAggregatedPubkey(s).toBytes(uncompressed))."""

    __slots__ = ("raw", "index")

    def __init__(self, raw96: bytes, index: Optional[int] = None):
        if len(raw96) != 96:
            raise ValueError("PublicKey expects 96-byte uncompressed bytes")
        self.raw = bytes(raw96)
        self.index = index  # position in the engine's resident pubkey table, if registered

    @staticmethod
    def many_from_compressed(engine: Engine, pks48: Sequence[bytes], validate: bool = False) -> List["PublicKey"]:
        out, st = engine.g1_decompress(pks48, validate)
        for s in st:
            if s:
                raise BlsError(s)
        return [PublicKey(o) for o in out]

    def to_bytes(self) -> bytes:
        return self.raw


class SignatureSetType(str, Enum):
    single = "single"
    aggregate = "aggregate"


@dataclass
class SingleSignatureSet:
    pubkey: PublicKey
    signing_root: bytes
    signature: bytes
    type: SignatureSetType = SignatureSetType.single


@dataclass
class AggregatedSignatureSet:
    pubkeys: List[PublicKey]
    signing_root: bytes
    signature: bytes
    type: SignatureSetType = SignatureSetType.aggregate


ISignatureSet = Union[SingleSignatureSet, AggregatedSignatureSet]


@dataclass
class VerifySignatureOpts:
    batchable: bool = False
    verify_on_main_thread: bool = False


def _pk_list(s: ISignatureSet) -> List[PublicKey]:
    if s.type == SignatureSetType.single:
        return [s.pubkey]
    if s.type == SignatureSetType.aggregate:
        return list(s.pubkeys)
    raise ValueError("Unknown signature set type")


def _to_input(s: ISignatureSet) -> SetInput:
    """Validates one set on the caller's side (ValueError) and reduces it to the C ABI's input."""
    pks = _pk_list(s)
    for p in pks:
        if not isinstance(p, PublicKey):
            raise ValueError("pubkeys must be PublicKey objects")
    if not isinstance(s.signature, (bytes, bytearray, memoryview)):
        raise ValueError("signature must be bytes")
    root = bytes(s.signing_root)
    if len(root) != 32:
        raise ValueError("signing root must be 32 bytes")
    return SetInput(pubkeys=[p.raw for p in pks], signing_root=root, signature=bytes(s.signature))


def _result(code: int) -> bool:
    if code < 0:
        raise BlsError(-code)
    return code == 1


@dataclass
class _Job:
    sets: List[SetInput]
    idx: Optional[List[List[int]]]  # per set: pubkey table indices (None if any key is unregistered)
    opts: VerifySignatureOpts
    future: asyncio.Future
    loop: asyncio.AbstractEventLoop
    added: float = field(default_factory=time.monotonic)


@dataclass
class PoolStats:
    batches: int = 0
    jobs: int = 0
    sets: int = 0
    jobs_invalid: int = 0
    jobs_error: int = 0


class BlsGpuVerifier:
    """IBlsVerifier backed by MI355X engines (drop-in for BlsMultiThreadWorkerPool)."""

    def __init__(self, engine: Optional[Engine] = None, device: int = 0, bls_verify_all_multi_thread: bool = False,
                 n_engines: int = 2):
        if engine is not None:
            self.engines = [engine]
            self._own_engines = False
        else:
            if n_engines < 1:
                raise ValueError("n_engines must be >= 1")
            self.engines = [Engine(device) for _ in range(n_engines)]
            self._own_engines = True
        # synchronous callers (verify_on_main_thread, verify_signature_set, aggregate_signatures,
        # key decompression) use an engine outside the runners' pool when the pool owns its
        # engines, so they never wait behind a batch in flight (multithread/index.ts:138-151)
        self.engine = Engine(device) if self._own_engines else self.engines[0]
        self.bls_verify_all_multi_thread = bls_verify_all_multi_thread
        self.stats = PoolStats()
        self._lock = threading.Condition()
        self._jobs: List[_Job] = []
        self._buffered: List[_Job] = []
        self._buffered_sigs = 0
        self._buffer_timer: Optional[asyncio.TimerHandle] = None
        self._closed = False
        self._runners = [threading.Thread(target=self._run, args=(e,), name=f"lodestar-bls-gpu-{k}", daemon=True)
                         for k, e in enumerate(self.engines)]
        for t in self._runners:
            t.start()

    # ---------------------------------------------------------------- IBlsVerifier
    async def verify_signature_sets(self, sets: Sequence[ISignatureSet],
                                    opts: Optional[VerifySignatureOpts] = None) -> bool:
        opts = opts or VerifySignatureOpts()
        if self._closed:
            raise QueueError({"code": QueueErrorCode.QUEUE_ABORTED.value})
        inputs = [_to_input(s) for s in sets]
        idx = []
        for s in sets:
            pks = _pk_list(s)
            idx.append([p.index for p in pks] if all(p.index is not None for p in pks) else None)
        if opts.verify_on_main_thread and not self.bls_verify_all_multi_thread:
            # synchronous, blocks the caller like the reference (multithread/index.ts:138-151)
            return _result(self.engine.verify_jobs([inputs])[0])
        loop = asyncio.get_running_loop()
        futs = []
        chunks = chunkify_maximize_chunk_size(list(range(len(inputs))), MAX_SIGNATURE_SETS_PER_JOB)
        for chunk in chunks:
            cidx = [idx[i] for i in chunk]
            job = _Job(sets=[inputs[i] for i in chunk], idx=None if (not cidx or any(x is None for x in cidx)) else cidx,
                       opts=opts, future=loop.create_future(), loop=loop)
            futs.append(job.future)
            self._queue(job)
        results = await asyncio.gather(*futs)
        return all(r is True for r in results)

    async def close(self) -> None:
        with self._lock:
            self._closed = True
            if self._buffer_timer is not None:
                self._buffer_timer.cancel()
                self._buffer_timer = None
            pending = self._jobs + self._buffered
            self._jobs, self._buffered, self._buffered_sigs = [], [], 0
            self._lock.notify_all()
        for j in pending:
            j.loop.call_soon_threadsafe(_set_exc, j.future, QueueError({"code": QueueErrorCode.QUEUE_ABORTED.value}))
        for t in self._runners:
            await asyncio.get_running_loop().run_in_executor(None, t.join)
        if self._own_engines:
            for e in [self.engine] + self.engines:
                e.close()

    # ---------------------------------------------------------------- direct (non-pool) callers
    def verify_signature_set(self, s: ISignatureSet) -> bool:
        """state-transition verifySignatureSet (src/util/signatureSets.ts:24-38): synchronous, the
        signature subgroup-checked, `single` -> Signature.verify, `aggregate` ->
        Signature.verifyAggregate (fastAggregateVerify).  Raises BlsError on malformed input."""
        return _result(self.engine.verify_jobs([[_to_input(s)]])[0])

    def aggregate_signatures(self, signatures: Sequence[bytes], validate: bool = True) -> bytes:
        """bls.Signature.aggregate(sigs).toBytes() (chain/opPools/*: block production), on the GPU."""
        out, st = self.engine.aggregate_signatures([list(signatures)], validate)
        if st[0]:
            raise BlsError(st[0])
        return out[0]

    def register_pubkeys(self, pks: Sequence[bytes], validate: bool = False) -> List[PublicKey]:
        """Load keys (48-byte compressed or 96-byte uncompressed) into the GPU-resident table once,
        like the epoch cache's index2pubkey (pubkeyCache.ts:56-77); returned PublicKeys carry their
        table index, so sets built from them ship 4-byte indices instead of 96-byte keys."""
        pks = list(pks)
        if pks and len(pks[0]) == 48:
            raws, st = self.engine.g1_decompress(pks)
            for s in st:
                if s:
                    raise BlsError(s)
        else:
            raws = pks
        first = None
        engines = self.engines if self.engine in self.engines else [self.engine] + self.engines
        for e in engines:  # every engine holds the same table (same indices)
            f, st = e.pubkey_table_append(raws, validate)
            for s in st:
                if s:
                    raise BlsError(s)
            if first is not None and f != first:
                raise RuntimeError("engine pubkey tables out of step")
            first = f
        return [PublicKey(r, first + k) for k, r in enumerate(raws)]

    # ---------------------------------------------------------------- queueing policy
    def _queue(self, job: _Job):
        if job.opts.batchable:
            self._buffered.append(job)
            self._buffered_sigs += len(job.sets)
            if self._buffered_sigs > MAX_BUFFERED_SIGS:
                self._flush_buffer()
            elif self._buffer_timer is None:
                self._buffer_timer = job.loop.call_later(MAX_BUFFER_WAIT_MS / 1000.0, self._flush_buffer)
        else:
            with self._lock:
                self._jobs.append(job)
                self._lock.notify_all()

    def _flush_buffer(self):
        if self._buffer_timer is not None:
            self._buffer_timer.cancel()
            self._buffer_timer = None
        with self._lock:
            self._jobs.extend(self._buffered)
            self._buffered, self._buffered_sigs = [], 0
            self._lock.notify_all()

    # ---------------------------------------------------------------- GPU runner
    def _run(self, engine: Engine):
        while True:
            with self._lock:
                while not self._jobs and not self._closed:
                    self._lock.wait()
                if self._closed and not self._jobs:
                    return
                jobs, self._jobs = self._jobs, []
            try:
                if all(j.idx is not None for j in jobs):
                    codes = engine.verify_jobs_indexed([j.sets for j in jobs], [j.idx for j in jobs])
                else:
                    codes = engine.verify_jobs([j.sets for j in jobs])
                err = None
            except Exception as e:  # device failure: every job of the package rejects (index.ts:368-375)
                codes, err = None, e
            with self._lock:
                self.stats.batches += 1
                self.stats.jobs += len(jobs)
                self.stats.sets += sum(len(j.sets) for j in jobs)
            for k, j in enumerate(jobs):
                if err is not None:
                    j.loop.call_soon_threadsafe(_set_exc, j.future, err)
                elif codes[k] < 0:
                    self.stats.jobs_error += 1
                    j.loop.call_soon_threadsafe(_set_exc, j.future, BlsError(-codes[k]))
                else:
                    if codes[k] == 0:
                        self.stats.jobs_invalid += 1
                    j.loop.call_soon_threadsafe(_set_res, j.future, codes[k] == 1)


def _set_res(f: asyncio.Future, v):
    if not f.done():
        f.set_result(v)


def _set_exc(f: asyncio.Future, e):
    if not f.done():
        f.set_exception(e)


_PK_STAGE = {"EMPTY_AGGREGATE_ARRAY"}
_VERIFY_STAGE = {"BLST_PK_IS_INFINITY"}


def is_valid_bls_aggregate(verifier: BlsGpuVerifier, public_keys: Sequence[PublicKey], message: bytes,
                           signature: bytes) -> bool:
    """light-client/src/validation.ts:154-184 isValidBlsAggregate: PublicKey.aggregate, then
    Signature.fromBytes(.., true), then verify, with the reference's stage-prefixed error messages.
    Used for sync-committee aggregates of light-client updates."""
    try:
        return verifier.verify_signature_set(AggregatedSignatureSet(list(public_keys), bytes(message), bytes(signature)))
    except BlsError as e:
        stage = ("Error aggregating pubkeys" if e.name in _PK_STAGE else
                 "Error verifying signature" if e.name in _VERIFY_STAGE else "Error deserializing signature")
        raise BlsError(e.code, f"{stage}: {e.name}") from None
