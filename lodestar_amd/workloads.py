"""Synthetic mainnet-shaped signature-set workloads (BASELINE.json configs).

Keys follow the reference's perf convention: validator v uses interop key v mod 100
(packages/state-transition/test/perf/util.ts:49-71; interop sk formula
packages/state-transition/src/util/interop.ts:19-23).  Signing roots are
sha256(seed || type || key): sets that sign the same object on mainnet share a key (a committee's
unaggregated attestations and its aggregates sign one AttestationData; every aggregator of a slot
signs the same selection-proof slot; the sync committee signs one block root), every other set
gets its own root.  Signatures are produced on the GPU with the engine's
synthetic-data kernels (SecretKey.sign); an aggregate signature is (sum sk_i mod r) * H(m).

Shapes (jobs = verifySignatureSets calls after chunkifyMaximizeChunkSize(sets, 128)):
  c1  128 single-pubkey sets, one job (BASELINE configs[0])
  c2  one block: proposer + randao + 128 attestation aggregates (k=256) + sync aggregate
      (k=358), one non-batchable call of 131 sets (configs[1])
  c3  gossip flood per slot: 16384 attestation calls (1 set, k=1, batchable) + 1024
      aggregate-and-proof calls (2 singles + 1 aggregate k=256)  = 17408 jobs, 19456 sets
      (configs[2]).  Roots: 64 committees, each voting for the majority head (95 %) or one
      alternative (5 %) -> <= 128 attestation roots; 1 selection-proof root per slot; 1024
      distinct AggregateAndProof roots; aggregates carry their committee's majority root.
      c3_distinct: the same shape with all 19456 roots distinct (the no-sharing bound).
  c4  sync committee: 512 single sync-committee messages + 64 contribution calls (2 singles +
      k=128) + block sync aggregate (k=512) + 4 light-client update aggregates (k=512), with
      invalid sets at >= 1/1000 split between well-formed wrong-message signatures (-> false)
      and malformed bytes (32-byte signature -> BLST_INVALID_SIZE, cleared compression flag
      -> BLST_BAD_ENCODING), SURVEY.md §8(d) (configs[3])
  c5  range sync: 32 blocks of c2 shape, one call per block (configs[4]); c5_64: 64 blocks
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from .engine import Engine, PackedJobs

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
SEED = 0x4C4F4445
N_KEYS = 100
# the distinct-key variant: a mainnet-sized index2pubkey table (~10^6 validators,
# pubkeyCache.ts:56-77), every validator id of the workloads ([0, 2^20)) its own key
N_KEYS_MAINNET = 1 << 20


def interop_sk(i: int) -> int:
    d = hashlib.sha256(i.to_bytes(32, "little")).digest()
    return int.from_bytes(d, "little") % R


@dataclass
class SetSpec:
    validators: List[int]   # pubkey indices (validator ids)
    kind: int               # domain-ish tag for the signing root
    invalid: bool = False   # sign a different message (well-formed, wrong)
    root: Optional[int] = None  # sets with equal (kind, root) sign the same message; None = own root
    malformed: Optional[str] = None  # "short32": 32-byte signature; "flag": compression flag cleared


@dataclass
class Workload:
    name: str
    packed: PackedJobs      # carries both 96-byte keys and pk_indices into the key pool
    n_invalid_jobs: int
    expected: np.ndarray    # per job 1 / 0 / -code (the C ABI's out_job convention)
    pool96: Optional[np.ndarray] = None  # the key pool (row k = key of index k)


class KeyPool:
    def __init__(self, engine: Engine, n: int = N_KEYS):
        self.sks = [interop_sk(i) for i in range(n)]
        step = 1 << 16
        parts = [engine.sk_to_pk(self.sks[a:a + step])[1] for a in range(0, n, step)]
        self.pk96 = parts[0] if len(parts) == 1 else np.concatenate(parts)

    def sk(self, v: int) -> int:
        return self.sks[v % len(self.sks)]

    def pk(self, v: int) -> np.ndarray:
        return self.pk96[v % len(self.sks)]


def build(engine: Engine, jobs: Sequence[Sequence[SetSpec]], name: str, keys: Optional[KeyPool] = None,
          seed: int = SEED) -> Workload:
    keys = keys or KeyPool(engine)
    flat = [s for job in jobs for s in job]
    n = len(flat)
    msgs = np.zeros((n, 32), dtype=np.uint8)
    sks = []
    for i, s in enumerate(flat):
        tag = (b"\x01" + s.root.to_bytes(8, "little")) if s.root is not None else (b"\x00" + i.to_bytes(8, "little"))
        msgs[i] = np.frombuffer(hashlib.sha256(seed.to_bytes(8, "little") + s.kind.to_bytes(2, "little")
                                               + tag).digest(), np.uint8)
        sks.append(sum(keys.sk(v) for v in s.validators) % R or 1)
    sign_msgs = msgs.copy()
    for i, s in enumerate(flat):
        if s.invalid:
            sign_msgs[i, 0] ^= 0xFF
    sigs = np.zeros((n, 96), dtype=np.uint8)
    step = 8192
    for a in range(0, n, step):
        sigs[a:a + step] = engine.sign(sks[a:a + step], sign_msgs[a:a + step])
    sizes = None
    for i, s in enumerate(flat):
        if s.malformed == "flag":
            sigs[i, 0] &= 0x7F                      # compression flag cleared -> BLST_BAD_ENCODING
        elif s.malformed == "short32":
            if sizes is None:
                sizes = np.full(n, 96, dtype=np.uint32)
            sizes[i] = 32                           # 32-byte signature -> BLST_INVALID_SIZE
            sigs[i] = 0
    job_off = np.zeros(len(jobs) + 1, dtype=np.uint32)
    job_off[1:] = np.cumsum([len(j) for j in jobs])
    pk_off = np.zeros(n + 1, dtype=np.uint32)
    pk_off[1:] = np.cumsum([len(s.validators) for s in flat])
    vidx = np.fromiter((v % len(keys.sks) for s in flat for v in s.validators), dtype=np.int64)
    pubkeys = np.ascontiguousarray(keys.pk96[vidx].reshape(-1))
    expected = np.array([expected_code(j) for j in jobs], dtype=np.int32)
    packed = PackedJobs(job_off=job_off, pk_off=pk_off, pubkeys=pubkeys, msgs=msgs.reshape(-1).copy(),
                        sigs=sigs.reshape(-1).copy(), sig_sizes=sizes, pk_indices=vidx.astype(np.uint32))
    return Workload(name=name, packed=packed, n_invalid_jobs=int((expected != 1).sum()), expected=expected,
                    pool96=keys.pk96)


LB_BAD_ENCODING = 1
LB_INVALID_SIZE = 10


def expected_code(job: Sequence[SetSpec]) -> int:
    """Reference verdict of one job of valid keys: the first malformed signature in set order
    rejects the job (maybeBatch.ts:18-25 decodes every signature before verifying); otherwise any
    wrong-message set makes it false."""
    for s in job:
        if s.malformed == "short32":
            return -LB_INVALID_SIZE
        if s.malformed == "flag":
            return -LB_BAD_ENCODING
    return 0 if any(s.invalid for s in job) else 1


def _block(rng, base_v: int, sync_k: int = 358, att_k: int = 256, n_att: int = 128) -> List[SetSpec]:
    sets = [SetSpec([base_v], 1), SetSpec([base_v], 2)]
    for a in range(n_att):
        sets.append(SetSpec([int(x) for x in rng.integers(0, 1 << 20, att_k)], 3))
    sets.append(SetSpec([int(x) for x in rng.integers(0, 1 << 20, sync_k)], 4))
    return sets


def c1_specs(rng):
    return [[SetSpec([i], 0) for i in range(128)]]


def c2_specs(rng):
    return [_block(rng, 7)]


def c3_specs(rng, n_att: int = 16384, n_agg: int = 1024, agg_k: int = 256, committees: int = 64,
             minority: float = 0.05, shared: bool = True, slots: int = 1):
    """`slots` consecutive slots' gossip in one batch (each slot: its own committees and
    selection-proof root)."""
    if slots > 1:
        return [j for s in range(slots) for j in _shift_roots(
            c3_specs(rng, n_att, n_agg, agg_k, committees, minority, shared), s)]

    def att_root(c, alt):
        return 2 * c + alt if shared else None

    jobs = [[SetSpec([int(rng.integers(0, 1 << 20))], 3,
                     root=att_root(int(rng.integers(0, committees)), int(rng.random() < minority)))]
            for _ in range(n_att)]
    for a in range(n_agg):
        v = int(rng.integers(0, 1 << 20))
        jobs.append([SetSpec([v], 5, root=0 if shared else None), SetSpec([v], 6),
                     SetSpec([int(x) for x in rng.integers(0, 1 << 20, agg_k)], 3,
                             root=att_root(a % committees, 0))])
    return jobs


def _shift_roots(jobs, slot):
    for j in jobs:
        for st in j:
            if st.root is not None:
                st.root += slot << 32
    return jobs


def c3_distinct_specs(rng, **kw):
    return c3_specs(rng, shared=False, **kw)


def c3_invalid_specs(rng, slots: int = 1, **kw):
    """c3 with one planted wrong-message attestation per slot (value_one_invalid_per_batch)."""
    jobs = c3_specs(rng, slots=slots, **kw)
    per = len(jobs) // slots
    for s in range(slots):
        jobs[s * per + int(rng.integers(0, 16384))][0].invalid = True
    return jobs


def c3_mixed_specs(rng, **kw):
    """one slot of c3 with the §8(d) invalid mix planted (wrong-message + malformed bytes)."""
    jobs = c3_specs(rng, **kw)
    plant_invalid(rng, jobs, 1e-3, min_each=4)
    return jobs


def c4_specs(rng, invalid_rate: float = 1e-3):
    # sync-committee messages and contributions sign this slot's block root; selection proofs
    # sign (slot, subcommittee); the block's sync aggregate signs the previous block root
    jobs = [[SetSpec([int(rng.integers(0, 512))], 7, root=0)] for _ in range(512)]
    for c in range(64):
        v = int(rng.integers(0, 512))
        jobs.append([SetSpec([v], 8, root=c % 4), SetSpec([v], 9),
                     SetSpec([int(x) for x in rng.integers(0, 512, 128)], 7, root=0)])
    jobs.append([SetSpec([int(x) for x in rng.integers(0, 512, 512)], 7, root=1)])
    for _ in range(4):
        jobs.append([SetSpec([int(x) for x in rng.integers(0, 512, 512)], 10)])
    plant_invalid(rng, jobs, invalid_rate)
    return jobs


def plant_invalid(rng, jobs, rate: float, min_each: int = 1):
    """SURVEY.md §8(d) invalid mix: ceil(rate * sets) bad sets, at least `min_each` of each kind,
    split between well-formed wrong-message signatures and malformed bytes (32-byte signature,
    cleared compression flag)."""
    flat = [s for j in jobs for s in j]
    n_bad = max(3 * min_each, int(np.ceil(len(flat) * rate)))
    picks = rng.choice(len(flat), n_bad, replace=False)
    for k, i in enumerate(picks):
        kind = k % 3
        if kind == 0:
            flat[int(i)].invalid = True
        else:
            flat[int(i)].malformed = "short32" if kind == 1 else "flag"


def c5_specs(rng, n_blocks: int = 32):
    return [_block(rng, 11 + b) for b in range(n_blocks)]


def c5_64_specs(rng):
    """range sync at the reference's own sizing: a 64-block batch (~8 000 sets per 64 blocks,
    multithread/index.ts:34)"""
    return c5_specs(rng, n_blocks=64)


SPECS = {"c1": c1_specs, "c2": c2_specs, "c3": c3_specs, "c3_distinct": c3_distinct_specs,
         "c3_invalid": c3_invalid_specs, "c3_mixed": c3_mixed_specs, "c4": c4_specs, "c5": c5_specs,
         "c5_64": c5_64_specs}


def make(engine: Engine, name: str, keys: Optional[KeyPool] = None, seed: int = SEED, **kw) -> Workload:
    """`keys`: the key pool validator v draws from (v mod its size); default the reference perf
    convention's 100 keys, KeyPool(engine, N_KEYS_MAINNET) for the distinct-key variant."""
    rng = np.random.default_rng(seed)
    return build(engine, SPECS[name](rng, **kw), name, keys=keys, seed=seed)


def indexed_for(engine: Engine, wl: Workload) -> PackedJobs:
    """Register the workload's key pool in `engine`'s resident table and return the batch with
    4-byte table indices instead of 96-byte keys (the index2pubkey path)."""
    base, st = engine.pubkey_table_append(np.asarray(wl.pool96, dtype=np.uint8))
    if any(st):
        raise RuntimeError("pubkey table append failed")
    p = wl.packed
    return PackedJobs(job_off=p.job_off, pk_off=p.pk_off, pubkeys=None, msgs=p.msgs, sigs=p.sigs,
                      sig_sizes=p.sig_sizes, pk_indices=(p.pk_indices + np.uint32(base)).astype(np.uint32))


def slice_jobs(p: PackedJobs, j0: int, j1: int) -> PackedJobs:
    """Jobs [j0, j1) of a packed batch as their own batch (a rank's shard, distributed.shard_jobs)."""
    s0, s1 = int(p.job_off[j0]), int(p.job_off[j1])
    k0, k1 = int(p.pk_off[s0]), int(p.pk_off[s1])
    return PackedJobs(job_off=(p.job_off[j0:j1 + 1] - s0).astype(np.uint32),
                      pk_off=(p.pk_off[s0:s1 + 1] - k0).astype(np.uint32),
                      pubkeys=None if p.pubkeys is None else p.pubkeys[96 * k0:96 * k1].copy(),
                      msgs=p.msgs[32 * s0:32 * s1].copy(), sigs=p.sigs[96 * s0:96 * s1].copy(),
                      sig_sizes=None if p.sig_sizes is None else p.sig_sizes[s0:s1].copy(),
                      pk_indices=None if p.pk_indices is None else p.pk_indices[k0:k1].copy())
