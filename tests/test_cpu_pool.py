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
