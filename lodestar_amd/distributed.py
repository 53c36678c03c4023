"""Multi-GPU verification protocol: one process per GPU, jobs sharded across
ranks; each rank reduces its shard to one 576-byte Fp12 partial product
    f_r = prod_{i in shard} ML(r_i PK_i, H(m_i)) * ML(-G1, sum_i r_i sig_i),
the partials are all-gathered (RCCL over xGMI with the "nccl" backend; gloo on CPU in tests),
and one final exponentiation of their product decides the whole segment.  RCCL has no Fp12
reduction op, so it is a gather + an on-device product, never an all-reduce.  On a 0 verdict
every rank localises its own invalid jobs from the state its partial left on its GPU
(lb_batch_search_after_partial: the shard's own final exponentiation, then the invalid-set
search), without re-running the pipeline."""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple

import numpy as np


def shard_jobs(n_jobs: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced job range of `rank` (whole jobs stay on one GPU so per-job fallback is local)."""
    per = n_jobs // world
    extra = n_jobs % world
    lo = rank * per + min(rank, extra)
    hi = lo + per + (1 if rank < extra else 0)
    return lo, hi


# Per-set and per-key device work in Fp multiplications (DESIGN.md §5 kernel table,
# profiles/roofline_counts.json): signature decode + subgroup check 2 111, r*PK 601, the bucket MSM
# ~232 per set; 16 per aggregated key (k_pk_chunks' mixed additions).  SURVEY.md §8(e) prices a
# key at ~11; the measured per-key figure is used.
SET_COST = 2111 + 601 + 232
KEY_COST = 16


def job_costs(job_off: Sequence[int], pk_off: Sequence[int]) -> np.ndarray:
    """Device work of each job: SET_COST per set + KEY_COST per pubkey."""
    job_off = np.asarray(job_off, dtype=np.int64)
    pk_off = np.asarray(pk_off, dtype=np.int64)
    sets = np.diff(job_off)
    keys = pk_off[job_off[1:]] - pk_off[job_off[:-1]]
    return SET_COST * sets + KEY_COST * keys


def shard_jobs_by_cost(job_off: Sequence[int], pk_off: Sequence[int], world: int, rank: int) -> Tuple[int, int]:
    """Contiguous job range of `rank`, balanced by device work (whole jobs per GPU,
    balanced by cost), so a segment mixing 1-set gossip jobs and 256-key block jobs does not load
    one rank with all the keys.  Rank r takes the jobs whose cost midpoint falls in
    [r T / world, (r + 1) T / world), T the segment's total cost."""
    c = job_costs(job_off, pk_off)
    if c.size == 0:
        return 0, 0
    pre = np.concatenate([[0], np.cumsum(c)])
    mid = (pre[:-1] + pre[1:]) / 2.0
    tot = float(pre[-1])
    lo = int(np.searchsorted(mid, rank * tot / world, side="left"))
    hi = int(np.searchsorted(mid, (rank + 1) * tot / world, side="left")) if rank + 1 < world else int(c.size)
    return lo, hi


def verify_sharded(partial: Callable[[], Tuple[bytes, Sequence[int]]],
                   product_is_one: Callable[[List[bytes]], bool],
                   local_verify: Callable[[], Sequence[int]],
                   group=None, device=None) -> Tuple[List[int], bool]:
    """Returns (per-job codes of this rank's shard, global verdict).  local_verify runs after a
    failing global verdict: Batch.search_after_partial (continues from this rank's partial) or
    any full re-verification of the shard."""
    import torch
    import torch.distributed as dist

    f, status = partial()
    t = torch.frombuffer(bytearray(f), dtype=torch.uint8)
    if device is not None:
        t = t.to(device)
    world = dist.get_world_size(group)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    ok = product_is_one([p.cpu().numpy().tobytes() for p in parts])
    if ok:
        return [int(s) for s in status], True
    return [int(c) for c in local_verify()], False
