"""The CPU baseline pool (oracle/cpu_pool.cpp, benchmark infrastructure) gives the reference's
per-job results on the golden fixtures — so the cpu_baseline bench leg times correct work."""
import numpy as np

from conftest import load_json
from lodestar_amd.engine import SetInput, pack_jobs


def test_cpu_pool_matches_golden():
    from oracle.cpu_pool import run_jobs
    from lodestar_amd import _native as N
    cases = [c for c in load_json("jobs.json")["cases"] if all(len(bytes.fromhex(s["signature"])) == 96
                                                               for s in c["sets"])]
    jobs = [[SetInput([bytes.fromhex(p) for p in s["pubkeys"]], bytes.fromhex(s["signing_root"]),
                      bytes.fromhex(s["signature"])) for s in c["sets"]] for c in cases]
    packed = pack_jobs(jobs)
    out, _ = run_jobs(packed, 0, packed.n_jobs, 4)
    got = [N.error_name(-c) if c < 0 else bool(c) for c in out]
    assert got == [c["expected"] for c in cases]


def test_cpu_pool_reference_policy_matches_golden():
    """The policy path (128-set packages, 16-job batch chunks, per-job retry on a failing chunk,
    Signature.verify for 1-set jobs; worker.ts:17-98) gives the same per-job results, batchable or
    not: a failing chunk is retried job by job, so one bad job never taints the others."""
    from oracle.cpu_pool import run_policy
    from lodestar_amd import _native as N
    cases = [c for c in load_json("jobs.json")["cases"] if all(len(bytes.fromhex(s["signature"])) == 96
                                                               for s in c["sets"])]
    # repeat the cases so chunks of >= 16 jobs form and hold valid and invalid jobs together
    cases = cases * 3
    jobs = [[SetInput([bytes.fromhex(p) for p in s["pubkeys"]], bytes.fromhex(s["signing_root"]),
                      bytes.fromhex(s["signature"])) for s in c["sets"]] for c in cases]
    packed = pack_jobs(jobs)
    for batchable in (True, False):
        out, _ = run_policy(packed, 0, packed.n_jobs, 4, batchable)
        got = [N.error_name(-c) if c < 0 else bool(c) for c in out]
        assert got == [c["expected"] for c in cases], batchable
