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
