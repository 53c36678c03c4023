"""Pythonic wrapper of one lb_engine (one GPU).  Marshals jobs of signature sets into the flat
arrays of the C ABI (include/lodestar_bls.h) and maps per-job codes back.

A *job* is what the reference ships to a worker as one BlsWorkReq
(packages/beacon-node/src/chain/bls/multithread/types.ts:14-17) and gets one result for
(worker.ts:32-108): 1 valid / 0 invalid / error.  A *set* is one ISignatureSet reduced to
(pubkeys, signing_root, signature) (state-transition/src/util/signatureSets.ts:5-22).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N


class BlsError(Exception):
    """A job rejected with a blst-style error (message = the reference's error string,
    e.g. "BLST_INVALID_SIZE", multithread.test.ts:97)."""

    def __init__(self, code: int, message: Optional[str] = None):
        self.code = int(code)
        self.name = N.error_name(code)
        super().__init__(message if message is not None else self.name)


@dataclass
class SetInput:
    pubkeys: Sequence[bytes]   # 96-byte uncompressed affine G1 each (1 for a `single` set)
    signing_root: bytes        # 32 bytes
    signature: bytes           # 96 bytes compressed G2 (other lengths -> BLST_INVALID_SIZE)


@dataclass
class PackedJobs:
    job_off: np.ndarray    # uint32 [n_jobs+1]
    pk_off: np.ndarray     # uint32 [n_sets+1]
    pubkeys: Optional[np.ndarray]    # uint8  [n_pks*96]  (None when pk_indices is used)
    msgs: np.ndarray       # uint8  [n_sets*32]
    sigs: np.ndarray       # uint8  [n_sets*96]
    sig_sizes: Optional[np.ndarray]  # uint32 [n_sets] or None
    pk_indices: Optional[np.ndarray] = None  # uint32 [n_pks]: indices into the engine's pubkey table

    @property
    def n_jobs(self):
        return len(self.job_off) - 1

    @property
    def n_sets(self):
        return len(self.pk_off) - 1


def pack_jobs(jobs: Sequence[Sequence[SetInput]]) -> PackedJobs:
    job_off = [0]
    pk_off = [0]
    pks, msgs, sigs, sizes = [], [], [], []
    odd = False
    for job in jobs:
        for s in job:
            for pk in s.pubkeys:
                if len(pk) != 96:
                    raise ValueError("pubkeys must be 96-byte uncompressed (PointFormat.uncompressed)")
                pks.append(bytes(pk))
            pk_off.append(pk_off[-1] + len(s.pubkeys))
            if len(s.signing_root) != 32:
                raise ValueError("signing roots are 32 bytes")
            msgs.append(bytes(s.signing_root))
            sig = bytes(s.signature)
            sizes.append(len(sig))
            if len(sig) != 96:
                odd = True
                sig = (sig + bytes(96))[:96]
            sigs.append(sig)
        job_off.append(job_off[-1] + len(job))
    return PackedJobs(
        job_off=np.asarray(job_off, dtype=np.uint32),
        pk_off=np.asarray(pk_off, dtype=np.uint32),
        pubkeys=np.frombuffer(b"".join(pks), dtype=np.uint8).copy() if pks else np.zeros(0, np.uint8),
        msgs=np.frombuffer(b"".join(msgs), dtype=np.uint8).copy() if msgs else np.zeros(0, np.uint8),
        sigs=np.frombuffer(b"".join(sigs), dtype=np.uint8).copy() if sigs else np.zeros(0, np.uint8),
        sig_sizes=np.asarray(sizes, dtype=np.uint32) if odd else None,
    )


def _p(a: Optional[np.ndarray], t):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.POINTER(t))


def _check(st: int):
    if st != N.LB_OK:
        raise BlsError(st)


class Batch:
    """A batch of jobs resident in device memory (lb_batch)."""

    def __init__(self, engine: "Engine", packed: PackedJobs):
        self.engine = engine
        self.packed = packed
        h = ctypes.c_void_p()
        if packed.pk_indices is not None:
            idx = np.ascontiguousarray(packed.pk_indices, dtype=np.uint32)
            if idx.size == 0:
                idx = np.zeros(1, dtype=np.uint32)
            _check(engine.lib.lb_batch_create_indexed(
                engine.h, packed.n_jobs, _p(packed.job_off, ctypes.c_uint32), _p(packed.pk_off, ctypes.c_uint32),
                _p(idx, ctypes.c_uint32), _p(packed.msgs, ctypes.c_uint8), _p(packed.sigs, ctypes.c_uint8),
                _p(packed.sig_sizes, ctypes.c_uint32), ctypes.byref(h)))
        else:
            _check(engine.lib.lb_batch_create(
                engine.h, packed.n_jobs, _p(packed.job_off, ctypes.c_uint32), _p(packed.pk_off, ctypes.c_uint32),
                _p(packed.pubkeys, ctypes.c_uint8), _p(packed.msgs, ctypes.c_uint8), _p(packed.sigs, ctypes.c_uint8),
                _p(packed.sig_sizes, ctypes.c_uint32), ctypes.byref(h)))
        self.h = h

    @property
    def n_jobs(self):
        return self.packed.n_jobs

    @property
    def n_sets(self):
        return self.packed.n_sets

    def verify(self, scalars: Optional[np.ndarray] = None) -> np.ndarray:
        out = np.zeros(max(self.n_jobs, 1), dtype=np.int32)
        sc = None if scalars is None else np.ascontiguousarray(scalars, dtype=np.uint64)
        _check(self.engine.lib.lb_batch_verify(self.engine.h, self.h, _p(sc, ctypes.c_uint64),
                                               _p(out, ctypes.c_int32)))
        return out[: self.n_jobs]

    def partial(self, scalars: Optional[np.ndarray] = None) -> Tuple[bytes, np.ndarray]:
        out = np.zeros(max(self.n_jobs, 1), dtype=np.int32)
        buf = (ctypes.c_uint8 * 576)()
        sc = None if scalars is None else np.ascontiguousarray(scalars, dtype=np.uint64)
        _check(self.engine.lib.lb_batch_partial(self.engine.h, self.h, _p(sc, ctypes.c_uint64),
                                                ctypes.cast(buf, ctypes.POINTER(ctypes.c_uint8)),
                                                _p(out, ctypes.c_int32)))
        return bytes(buf), out[: self.n_jobs]

    def search_after_partial(self, fallback: bool = True) -> np.ndarray:
        """Per-job codes from the state the last partial() of this batch left in the engine (the
        shard's own root check, then the invalid-set search): lb_batch_search_after_partial.
        When another call ran on the engine since (LB_ERR_ARGUMENT: the state is gone, e.g. a
        second thread shares the engine), the shard is re-verified in full (lb_batch_verify), as
        include/lodestar_bls.h prescribes; fallback=False raises instead."""
        out = np.zeros(max(self.n_jobs, 1), dtype=np.int32)
        st = self.engine.lib.lb_batch_search_after_partial(self.engine.h, self.h, _p(out, ctypes.c_int32))
        if st == N.LB_ERR_ARGUMENT and fallback:
            return self.verify()
        _check(st)
        return out[: self.n_jobs]

    def free(self):
        if self.h:
            self.engine.lib.lb_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Engine:
    """One lb_engine bound to one gfx950 device."""

    LATENCY = 1  # lb_engine_create_ex flag LB_ENGINE_LATENCY (include/lodestar_bls.h)

    def __init__(self, device: int = 0, flags: int = 0):
        self.lib = N.load()
        h = ctypes.c_void_p()
        _check(self.lib.lb_engine_create_ex(int(device), ctypes.c_uint32(flags), ctypes.byref(h)))
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            self.lib.lb_engine_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def cu_count(self) -> int:
        """CUs this engine's streams may use (lb_engine_cu_count)."""
        return int(self.lib.lb_engine_cu_count(self.h))

    # ---------------------------------------------------------------- verification
    def upload(self, jobs_or_packed) -> Batch:
        packed = jobs_or_packed if isinstance(jobs_or_packed, PackedJobs) else pack_jobs(jobs_or_packed)
        return Batch(self, packed)

    def verify_jobs(self, jobs, scalars: Optional[np.ndarray] = None) -> List[int]:
        """Per-job 1 / 0 / -code."""
        return self.verify_jobs_packed(pack_jobs(jobs), scalars)

    def verify_jobs_packed(self, packed: PackedJobs, scalars: Optional[np.ndarray] = None) -> List[int]:
        """Upload + verify through the engine-owned workspace (lb_verify_jobs[_indexed]): the
        drop-in path, no per-call device allocation."""
        out = np.zeros(max(packed.n_jobs, 1), dtype=np.int32)
        sc = None if scalars is None else np.ascontiguousarray(scalars, dtype=np.uint64)
        if packed.pk_indices is not None:
            idx = np.ascontiguousarray(packed.pk_indices, dtype=np.uint32)
            st = self.lib.lb_verify_jobs_indexed(
                self.h, packed.n_jobs, _p(packed.job_off, ctypes.c_uint32), _p(packed.pk_off, ctypes.c_uint32),
                _p(idx if idx.size else None, ctypes.c_uint32), _p(packed.msgs, ctypes.c_uint8),
                _p(packed.sigs, ctypes.c_uint8), _p(packed.sig_sizes, ctypes.c_uint32), _p(sc, ctypes.c_uint64),
                _p(out, ctypes.c_int32))
        else:
            st = self.lib.lb_verify_jobs(
                self.h, packed.n_jobs, _p(packed.job_off, ctypes.c_uint32), _p(packed.pk_off, ctypes.c_uint32),
                _p(packed.pubkeys, ctypes.c_uint8), _p(packed.msgs, ctypes.c_uint8), _p(packed.sigs, ctypes.c_uint8),
                _p(packed.sig_sizes, ctypes.c_uint32), _p(sc, ctypes.c_uint64), _p(out, ctypes.c_int32))
        _check(st)
        return [int(x) for x in out[: packed.n_jobs]]

    def verify_jobs_indexed(self, jobs, indices, scalars: Optional[np.ndarray] = None) -> List[int]:
        """Jobs whose pubkeys are table indices: indices[j][s] = list of table indices of set s."""
        packed = pack_jobs([[SetInput([], s.signing_root, s.signature) for s in job] for job in jobs])
        counts = [len(ix) for jix in indices for ix in jix]
        packed.pk_off = np.zeros(len(counts) + 1, dtype=np.uint32)
        packed.pk_off[1:] = np.cumsum(counts, dtype=np.uint64).astype(np.uint32)
        packed.pubkeys = None
        packed.pk_indices = np.asarray([i for jix in indices for ix in jix for i in ix], dtype=np.uint32)
        return self.verify_jobs_packed(packed, scalars)

    def product_is_one(self, partials: Sequence[bytes]) -> bool:
        buf = np.frombuffer(b"".join(partials), dtype=np.uint8).copy() if partials else np.zeros(1, np.uint8)
        ok = ctypes.c_int32(0)
        _check(self.lib.lb_fp12_product_is_one(self.h, _p(buf, ctypes.c_uint8), len(partials), ctypes.byref(ok)))
        return bool(ok.value)

    # ---------------------------------------------------------------- pubkeys
    def pubkey_table_append(self, keys: Sequence[bytes], validate: bool = False) -> Tuple[int, List[int]]:
        """Decode keys (all 48-byte compressed or all 96-byte uncompressed) into the resident table.
        Returns (index of the first appended key, per-key status)."""
        n = len(keys)
        if n == 0:
            return self.pubkey_table_size(), []
        if isinstance(keys, np.ndarray) and keys.ndim == 2:  # n x 48 / n x 96 uint8 rows
            size = int(keys.shape[1])
            if size not in (48, 96):
                raise ValueError("keys must all be 48 or all be 96 bytes")
            buf = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1).copy()
        else:
            size = len(keys[0])
            if any(len(k) != size for k in keys) or size not in (48, 96):
                raise ValueError("keys must all be 48 or all be 96 bytes")
            buf = np.frombuffer(b"".join(bytes(k) for k in keys), dtype=np.uint8).copy()
        st = np.zeros(n, dtype=np.int32)
        first = ctypes.c_uint32(0)
        _check(self.lib.lb_pubkey_table_append(self.h, n, _p(buf, ctypes.c_uint8), size, 1 if validate else 0,
                                               _p(st, ctypes.c_int32), ctypes.byref(first)))
        return int(first.value), [int(x) for x in st]

    def pubkey_table_size(self) -> int:
        return int(self.lib.lb_pubkey_table_size(self.h))

    def aggregate_pubkeys(self, sets_pubkeys: Sequence[Sequence[bytes]]) -> Tuple[List[bytes], List[int]]:
        off = [0]
        flat = []
        for pks in sets_pubkeys:
            flat.extend(bytes(p) for p in pks)
            off.append(off[-1] + len(pks))
        n = len(sets_pubkeys)
        offa = np.asarray(off, dtype=np.uint32)
        pka = np.frombuffer(b"".join(flat), dtype=np.uint8).copy() if flat else np.zeros(1, np.uint8)
        out = np.zeros(max(n, 1) * 96, dtype=np.uint8)
        st = np.zeros(max(n, 1), dtype=np.int32)
        _check(self.lib.lb_aggregate_pubkeys(self.h, n, _p(offa, ctypes.c_uint32), _p(pka, ctypes.c_uint8),
                                             _p(out, ctypes.c_uint8), _p(st, ctypes.c_int32)))
        ob = out.tobytes()
        return [ob[96 * i: 96 * i + 96] for i in range(n)], [int(x) for x in st[:n]]

    def aggregate_signatures(self, groups: Sequence[Sequence[bytes]], validate: bool = True
                             ) -> Tuple[List[bytes], List[int]]:
        """bls.Signature.aggregate per group (lb_aggregate_signatures): 96-byte compressed sums
        and per-group status (0 = ok, else the blst error code)."""
        off = [0]
        flat, sizes, odd = [], [], False
        for g in groups:
            for sg in g:
                sg = bytes(sg)
                sizes.append(len(sg))
                if len(sg) != 96:
                    odd = True
                    sg = (sg + bytes(96))[:96]
                flat.append(sg)
            off.append(off[-1] + len(g))
        n = len(groups)
        offa = np.asarray(off, dtype=np.uint32)
        buf = np.frombuffer(b"".join(flat), dtype=np.uint8).copy() if flat else np.zeros(1, np.uint8)
        sz = np.asarray(sizes, dtype=np.uint32) if odd else None
        out = np.zeros(max(n, 1) * 96, dtype=np.uint8)
        st = np.zeros(max(n, 1), dtype=np.int32)
        _check(self.lib.lb_aggregate_signatures(self.h, n, _p(offa, ctypes.c_uint32), _p(buf, ctypes.c_uint8),
                                                _p(sz, ctypes.c_uint32), 1 if validate else 0,
                                                _p(out, ctypes.c_uint8), _p(st, ctypes.c_int32)))
        ob = out.tobytes()
        return [ob[96 * i: 96 * i + 96] for i in range(n)], [int(x) for x in st[:n]]

    def g1_decompress(self, pks48: Sequence[bytes], validate: bool = False) -> Tuple[List[bytes], List[int]]:
        n = len(pks48)
        if n == 0:
            return [], []
        inp = np.frombuffer(b"".join(bytes(p) for p in pks48), dtype=np.uint8).copy()
        out = np.zeros(n * 96, dtype=np.uint8)
        st = np.zeros(n, dtype=np.int32)
        _check(self.lib.lb_g1_decompress(self.h, n, _p(inp, ctypes.c_uint8), _p(out, ctypes.c_uint8),
                                         _p(st, ctypes.c_int32), 1 if validate else 0))
        ob = out.tobytes()
        return [ob[96 * i: 96 * i + 96] for i in range(n)], [int(x) for x in st]

    # ---------------------------------------------------------------- synthetic data
    def sk_to_pk(self, sks: Sequence[int]) -> Tuple[np.ndarray, np.ndarray]:
        """-> (n x 48 compressed, n x 96 uncompressed) uint8 arrays."""
        n = len(sks)
        sk = np.frombuffer(b"".join(int(s).to_bytes(32, "big") for s in sks), dtype=np.uint8).copy()
        o48 = np.zeros(n * 48, dtype=np.uint8)
        o96 = np.zeros(n * 96, dtype=np.uint8)
        _check(self.lib.lb_sk_to_pk(self.h, n, _p(sk, ctypes.c_uint8), _p(o48, ctypes.c_uint8),
                                    _p(o96, ctypes.c_uint8)))
        return o48.reshape(n, 48), o96.reshape(n, 96)

    def sign(self, sks: Sequence[int], msgs: np.ndarray) -> np.ndarray:
        """sks[i] signs msgs[i] (32 B) -> n x 96 compressed signatures."""
        n = len(sks)
        sk = np.frombuffer(b"".join(int(s).to_bytes(32, "big") for s in sks), dtype=np.uint8).copy()
        m = np.ascontiguousarray(msgs, dtype=np.uint8).reshape(-1)
        assert m.size == 32 * n
        out = np.zeros(n * 96, dtype=np.uint8)
        _check(self.lib.lb_sign(self.h, n, _p(sk, ctypes.c_uint8), _p(m, ctypes.c_uint8), _p(out, ctypes.c_uint8)))
        return out.reshape(n, 96)

    # ---------------------------------------------------------------- profiling
    def set_profiling(self, on: bool):
        _check(self.lib.lb_engine_set_profiling(self.h, 1 if on else 0))

    def last_profile(self) -> dict:
        names = (ctypes.c_char_p * 32)()
        ms = (ctypes.c_float * 32)()
        n = ctypes.c_int32(0)
        _check(self.lib.lb_engine_last_profile(self.h, names, ms, 32, ctypes.byref(n)))
        return {names[i].decode(): float(ms[i]) for i in range(n.value)}
