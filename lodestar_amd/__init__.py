"""MI355X-native BLS12-381 signature-set verifier: drop-in for Lodestar's IBlsVerifier
(packages/beacon-node/src/chain/bls).  The compute path is liblodestar_bls.so (HIP, gfx950)
behind the C ABI in include/lodestar_bls.h; this package is the host-side mirror."""
from .engine import BlsError, Engine, SetInput, pack_jobs  # noqa: F401
from .verifier import (  # noqa: F401
    AggregatedSignatureSet,
    BlsGpuVerifier,
    PublicKey,
    QueueError,
    QueueErrorCode,
    SignatureSetType,
    SingleSignatureSet,
    VerifySignatureOpts,
    chunkify_maximize_chunk_size,
)
