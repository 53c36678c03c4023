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


def test_c4_invalid_mix_follows_survey():
    """>= 1/1000 invalid sets, split between well-formed wrong-message
    signatures (-> false) and malformed bytes (32-byte signature, cleared flag -> reject)."""
    jobs = W.c4_specs(np.random.default_rng(W.SEED))
    flat = [s for j in jobs for s in j]
    wrong = sum(s.invalid for s in flat)
    short = sum(s.malformed == "short32" for s in flat)
    flag = sum(s.malformed == "flag" for s in flat)
    assert wrong >= 1 and short >= 1 and flag >= 1
    assert wrong + short + flag >= len(flat) / 1000


def test_expected_code_precedence():
    S = W.SetSpec
    assert W.expected_code([S([1], 0)]) == 1
    assert W.expected_code([S([1], 0, invalid=True)]) == 0
    # a malformed signature rejects the job even when another set is merely wrong
    assert W.expected_code([S([1], 0, invalid=True), S([2], 0, malformed="flag")]) == -W.LB_BAD_ENCODING
    assert W.expected_code([S([1], 0, malformed="short32"), S([2], 0, malformed="flag")]) == -W.LB_INVALID_SIZE


def test_c3_invalid_and_mixed_shapes():
    jobs = W.c3_invalid_specs(np.random.default_rng(W.SEED), slots=2)
    assert len(jobs) == 2 * 17408
    assert sum(s.invalid for j in jobs for s in j) == 2
    mixed = W.c3_mixed_specs(np.random.default_rng(W.SEED))
    flat = [s for j in mixed for s in j]
    assert sum(s.invalid for s in flat) >= 4
    assert sum(s.malformed == "short32" for s in flat) >= 4 and sum(s.malformed == "flag" for s in flat) >= 4


def test_c5_block_counts():
    """range sync: 32 blocks (BASELINE configs[4]) and the reference's own 64-block sizing
    (multithread/index.ts:34: ~8 000 sets per 64 blocks), one non-batchable call per block"""
    rng = np.random.default_rng(1)
    for name, nb in (("c5", 32), ("c5_64", 64)):
        jobs = W.SPECS[name](rng)
        assert len(jobs) == nb
        n = sum(len(j) for j in jobs)
        assert 125 * nb <= n <= 135 * nb  # ~131 sets per C2-shaped block
