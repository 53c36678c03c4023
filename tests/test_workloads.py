"""Workload shapes (CPU only: the specs, not the signed batches)."""
import numpy as np

from lodestar_amd import workloads as W


def _roots(jobs):
    flat = [s for j in jobs for s in j]
    keyed = {(s.kind, s.root) for s in flat if s.root is not None}
    return len(keyed) + sum(1 for s in flat if s.root is None), len(flat)


def test_c3_shape_and_shared_roots():
    jobs = W.c3_specs(np.random.default_rng(W.SEED))
    n_roots, n_sets = _roots(jobs)
    assert len(jobs) == 17408 and n_sets == 19456
    # <= 128 attestation roots (64 committees x majority/minority head), 1 selection-proof root,
    # 1024 distinct AggregateAndProof roots
    assert 1024 + 1 + 64 <= n_roots <= 1024 + 1 + 128


def test_c3_distinct_has_no_shared_roots():
    jobs = W.c3_distinct_specs(np.random.default_rng(W.SEED))
    n_roots, n_sets = _roots(jobs)
    assert n_roots == n_sets == 19456


def test_c4_sync_committee_roots():
    jobs = W.c4_specs(np.random.default_rng(W.SEED))
    n_roots, n_sets = _roots(jobs)
    # block root (messages + contributions), 4 selection-proof roots, previous block root,
    # 64 contribution-and-proof roots, 4 light-client update roots
    assert n_roots == 1 + 4 + 1 + 64 + 4
    assert sum(s.invalid for j in jobs for s in j) >= 1
