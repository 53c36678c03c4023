"""Host policy of the IBlsVerifier mirror (no GPU): chunking (K6), buffering, per-job error
isolation and close(), against a stub engine."""
import asyncio

import pytest

from lodestar_amd import verifier as V
from lodestar_amd.engine import BlsError


def test_chunkify_maximize_chunk_size_k6():
    # packages/beacon-node/test/unit/chain/bls/utils.test.ts:6-34 (minPerChunk = 3)
    expected = [
        [[0]], [[0, 1]], [[0, 1, 2]], [[0, 1, 2, 3]], [[0, 1, 2, 3, 4]],
        [[0, 1, 2], [3, 4, 5]], [[0, 1, 2, 3], [4, 5, 6]], [[0, 1, 2, 3], [4, 5, 6, 7]],
    ]
    for i, exp in enumerate(expected):
        assert V.chunkify_maximize_chunk_size(list(range(i + 1)), 3) == exp


def test_chunkify_jobs_of_128():
    assert [len(c) for c in V.chunkify_maximize_chunk_size(list(range(255)), 128)] == [255]
    assert [len(c) for c in V.chunkify_maximize_chunk_size(list(range(256)), 128)] == [128, 128]
    assert [len(c) for c in V.chunkify_maximize_chunk_size(list(range(1000)), 128)] == [143] * 6 + [142]
    assert V.chunkify_maximize_chunk_size([], 128) == [[]]


class StubEngine:
    """valid iff the signature is 96 bytes and not all-zero; 'size' errors like blst."""

    def __init__(self):
        self.calls = []

    def verify_jobs(self, jobs, scalars=None):
        self.calls.append([len(j) for j in jobs])
        out = []
        for job in jobs:
            if not job:
                out.append(-12)
            elif any(len(s.signature) != 96 for s in job):
                out.append(-10)
            else:
                out.append(0 if any(s.signature == bytes(96) for s in job) else 1)
        return out

    def close(self):
        pass


def mk_sets(n, sig=b"\x01" * 96):
    pk = V.PublicKey(b"\x02" * 96)
    return [V.SingleSignatureSet(pubkey=pk, signing_root=bytes(32), signature=sig) for _ in range(n)]


def run(coro):
    return asyncio.get_event_loop().run_until_complete(coro) if False else asyncio.run(coro)


def test_batchable_buffering_and_error_isolation():
    async def main():
        eng = StubEngine()
        pool = V.BlsGpuVerifier(engine=eng)
        bad = pool.verify_signature_sets(mk_sets(1, sig=bytes(32)), V.VerifySignatureOpts(batchable=True))
        goods = [pool.verify_signature_sets(mk_sets(3), V.VerifySignatureOpts(batchable=True)) for _ in range(8)]
        res = await asyncio.gather(bad, *goods, return_exceptions=True)
        await pool.close()
        return eng, res
    eng, res = run(main())
    assert isinstance(res[0], BlsError) and str(res[0]) == "BLST_INVALID_SIZE"
    assert res[1:] == [True] * 8
    # 25 buffered sigs: the >32 threshold is crossed at the 11th set -> flushed as one package
    assert sum(sum(c) for c in eng.calls) == 25


def test_non_batchable_runs_without_waiting_and_invalid_is_false():
    async def main():
        pool = V.BlsGpuVerifier(engine=StubEngine())
        a = await pool.verify_signature_sets(mk_sets(2))
        b = await pool.verify_signature_sets(mk_sets(1, sig=bytes(96)))
        await pool.close()
        return a, b
    assert run(main()) == (True, False)


def test_empty_call_rejects():
    async def main():
        pool = V.BlsGpuVerifier(engine=StubEngine())
        try:
            with pytest.raises(BlsError, match="Empty signature set"):
                await pool.verify_signature_sets([])
        finally:
            await pool.close()
    run(main())


def test_close_aborts_queued():
    async def main():
        pool = V.BlsGpuVerifier(engine=StubEngine())
        fut = asyncio.ensure_future(pool.verify_signature_sets(mk_sets(1), V.VerifySignatureOpts(batchable=True)))
        await asyncio.sleep(0)
        await pool.close()
        with pytest.raises(V.QueueError, match="^QUEUE_ERROR_QUEUE_ABORTED$") as ei:
            await fut
        # util/queue/errors.ts:3-6: callers compare e.type.code with QueueErrorCode.QUEUE_ABORTED
        assert ei.value.type == {"code": V.QueueErrorCode.QUEUE_ABORTED.value} == {"code": "QUEUE_ERROR_QUEUE_ABORTED"}
        with pytest.raises(V.QueueError) as ei:
            await pool.verify_signature_sets(mk_sets(1))
        assert ei.value.type["code"] == "QUEUE_ERROR_QUEUE_ABORTED"
    run(main())
