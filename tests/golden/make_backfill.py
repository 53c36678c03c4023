"""Extracts the first four mainnet phase0 blocks the reference's backfill test holds
(packages/beacon-node/test/unit/sync/backfill/blocks.json, read by verify.test.ts:53-60) and the
mainnet genesis validators root that test configures (verify.test.ts:19-22) into
tests/golden/backfill_phase0.json.  Data only: the signed blocks as beacon-API JSON.

Each block's parent_root is hash_tree_root of the previous block's message (verifyBlockSequence,
sync/backfill/verify.ts:24-40), which pins the phase0 BeaconBlock walk of signing_roots.py.

    python tests/golden/make_backfill.py /root/reference
"""
import json
import os
import sys

ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
src = os.path.join(ref, "packages/beacon-node/test/unit/sync/backfill/blocks.json")
blocks = json.load(open(src))
out = {
    "source": "packages/beacon-node/test/unit/sync/backfill/blocks.json (first 4 mainnet blocks)",
    "genesis_validators_root": "4b363db94e286120d76eb905340fdd4e54bfe9f06bf33ff6cf5ad27f511bfe95",
    "genesis_fork_version": "00000000",
    "blocks": blocks,
}
dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "backfill_phase0.json")
with open(dst, "w") as f:
    json.dump(out, f, indent=1)
print("wrote", dst, len(blocks), "blocks")
