"""KZG commitments for EIP-4844 blobs on the GPU.

Mirrors the c-kzg surface Lodestar binds in packages/beacon-node/src/util/kzg.ts:15-65
(`loadTrustedSetup`, `blobToKzgCommitment`, `computeAggregateKzgProof`, `verifyAggregateKzgProof`;
callers chain/validation/blobsSidecar.ts:75-120 and chain/produceBlock/validateBlobsAndKzgCommitments.ts)
following the EIP-4844 polynomial-commitments spec of the reference's pinned consensus-spec
version (v1.3.0-alpha.2, test/spec/specTestVersioning.ts:18).

Split: the scalar-field work is host code here (the inverse FFT from the blob's evaluations to
monomial coefficients, Fiat-Shamir challenges, evaluation, quotient); the group work runs on the
GPU through the C ABI -- 4096-term G1 linear combinations of the resident trusted setup
(`lb_g1_lincomb`) and the proof check as one two-pair pairing product (`lb_kzg_verify_proof`).

The setup is Lodestar's own `trusted_setup.bin` (kzg.ts:36-48: two u32 counts, 4096 compressed
[tau^i] G1, 65 compressed [tau^i] G2), i.e. MONOMIAL form (setup_G1[0] is the G1 generator).
Committing in monomial form, sum a_j [tau^j] G1 with a = IFFT of the blob's evaluations, gives
exactly the spec's g1_lincomb(bit_reversal_permutation(KZG_SETUP_LAGRANGE), blob).

Parity: c-kzg is an un-vendored npm dependency with no fixtures in the reference (kzg.test.ts only
checks that its own proofs verify), so byte parity with c-kzg is UNPINNED.  Field elements are
read big-endian, as Lodestar's own range check reads them (blobsSidecar.ts:138-150); the
transcript follows the spec's compute_challenges with the same byte order.  Tests pin the
mathematics against the independent oracle restatement (oracle/kzg.py).
"""
from __future__ import annotations

import ctypes
import hashlib
import os
from typing import List, Sequence, Tuple

import numpy as np

BLS_MODULUS = 52435875175126190479447740508185965837690552500527637822603658699938581184513
FIELD_ELEMENTS_PER_BLOB = 4096
BYTES_PER_FIELD_ELEMENT = 32
BYTES_PER_BLOB = FIELD_ELEMENTS_PER_BLOB * BYTES_PER_FIELD_ELEMENT
FIAT_SHAMIR_PROTOCOL_DOMAIN = b"FSBLOBVERIFY_V1_"
PRIMITIVE_ROOT_OF_UNITY = 7
ENDIANNESS = "big"
TRUSTED_SETUP_BIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "trusted_setup.bin")

G1_COUNT, G1_BYTES, G2_COUNT, G2_BYTES = FIELD_ELEMENTS_PER_BLOB, 48, 65, 96


def read_trusted_setup_bin(data: bytes) -> Tuple[List[bytes], List[bytes]]:
    """kzg.ts trustedSetupBinToJson: skip the two u32 counts, then 4096 x 48 B G1, 65 x 96 B G2."""
    total = 8 + G1_COUNT * G1_BYTES + G2_COUNT * G2_BYTES
    if len(data) < total:
        raise ValueError(f"trusted_setup size {len(data)} < {total}")
    g1 = [bytes(data[8 + i * 48: 8 + (i + 1) * 48]) for i in range(G1_COUNT)]
    base = 8 + G1_COUNT * G1_BYTES
    g2 = [bytes(data[base + i * 96: base + (i + 1) * 96]) for i in range(G2_COUNT)]
    return g1, g2


# ------------------------------------------------------------------ scalar field (host)
def _roots_of_unity(n: int) -> List[int]:
    w = pow(PRIMITIVE_ROOT_OF_UNITY, (BLS_MODULUS - 1) // n, BLS_MODULUS)
    out, x = [], 1
    for _ in range(n):
        out.append(x)
        x = x * w % BLS_MODULUS
    return out


def _brp_index(n: int) -> List[int]:
    bits = n.bit_length() - 1
    return [int(format(i, f"0{bits}b")[::-1], 2) for i in range(n)]


ROOTS = _roots_of_unity(FIELD_ELEMENTS_PER_BLOB)
BRP = _brp_index(FIELD_ELEMENTS_PER_BLOB)
ROOTS_BRP = [ROOTS[BRP[i]] for i in range(FIELD_ELEMENTS_PER_BLOB)]


def _ntt(a: List[int], roots: List[int]) -> List[int]:
    """in-order radix-2 transform: out[k] = sum_j a[j] roots[j k mod n]"""
    n = len(a)
    idx = BRP if n == FIELD_ELEMENTS_PER_BLOB else _brp_index(n)
    a = [a[idx[i]] for i in range(n)]
    m = 1
    while m < n:
        step = n // (2 * m)
        for s in range(0, n, 2 * m):
            for j in range(m):
                w = roots[j * step]
                u, v = a[s + j], a[s + j + m] * w % BLS_MODULUS
                a[s + j] = (u + v) % BLS_MODULUS
                a[s + j + m] = (u - v) % BLS_MODULUS
        m *= 2
    return a


def blob_to_polynomial(blob: bytes) -> List[int]:
    """the blob's 4096 field elements (its evaluations at the bit-reversed roots of unity)"""
    if len(blob) != BYTES_PER_BLOB:
        raise ValueError(f"blob length {len(blob)} != {BYTES_PER_BLOB}")
    out = []
    for i in range(FIELD_ELEMENTS_PER_BLOB):
        v = int.from_bytes(blob[32 * i: 32 * i + 32], ENDIANNESS)
        if v >= BLS_MODULUS:
            raise ValueError("blob field element >= BLS_MODULUS")
        out.append(v)
    return out


def evaluations_to_coefficients(poly: Sequence[int]) -> List[int]:
    """monomial coefficients of the polynomial with p(ROOTS_BRP[i]) = poly[i] (inverse NTT)"""
    n = len(poly)
    nat = [0] * n
    for i, v in enumerate(poly):
        nat[BRP[i]] = v
    inv_roots = [ROOTS[(-k) % n] for k in range(n)]
    inv_n = pow(n, BLS_MODULUS - 2, BLS_MODULUS)
    return [c * inv_n % BLS_MODULUS for c in _ntt(nat, inv_roots)]


def evaluate_coefficients(coeffs: Sequence[int], z: int) -> int:
    y = 0
    for c in reversed(coeffs):
        y = (y * z + c) % BLS_MODULUS
    return y


def quotient_coefficients(coeffs: Sequence[int], z: int) -> List[int]:
    """(p(X) - p(z)) / (X - z) by synthetic division"""
    n = len(coeffs)
    q = [0] * (n - 1)
    acc = 0
    for k in range(n - 1, 0, -1):
        acc = (acc * z + coeffs[k]) % BLS_MODULUS
        q[k - 1] = acc
    return q


def hash_to_bls_field(data: bytes) -> int:
    return int.from_bytes(hashlib.sha256(data).digest(), ENDIANNESS) % BLS_MODULUS


def compute_challenges(polys: Sequence[Sequence[int]], commitments: Sequence[bytes]) -> Tuple[List[int], int]:
    """spec compute_challenges: transcript = domain || degree (8 B) || count (8 B) || every field
    element (32 B) || every commitment (48 B); r = H(h || 0x00), x = H(h || 0x01)"""
    data = bytearray(FIAT_SHAMIR_PROTOCOL_DOMAIN)
    data += FIELD_ELEMENTS_PER_BLOB.to_bytes(8, ENDIANNESS)
    data += len(polys).to_bytes(8, ENDIANNESS)
    for p in polys:
        for v in p:
            data += int(v).to_bytes(BYTES_PER_FIELD_ELEMENT, ENDIANNESS)
    for c in commitments:
        data += bytes(c)
    h = hashlib.sha256(bytes(data)).digest()
    r = hash_to_bls_field(h + b"\x00")
    powers, x = [], 1
    for _ in range(len(commitments)):
        powers.append(x)
        x = x * r % BLS_MODULUS
    return powers, hash_to_bls_field(h + b"\x01")


def _scalars_le(vals: Sequence[int]) -> np.ndarray:
    out = np.zeros((len(vals), 32), np.uint8)
    for i, v in enumerate(vals):
        out[i] = np.frombuffer(int(v).to_bytes(32, "little"), np.uint8)
    return out


# ------------------------------------------------------------------ GPU-backed KZG
G1_INFINITY48 = b"\xc0" + b"\x00" * 47  # compressed point at infinity


class KzgError(Exception):
    pass


class Kzg:
    """ckzg for one engine: `load_trusted_setup` once, then commitments / aggregate proofs."""

    def __init__(self, engine, setup: bytes = None):
        from lodestar_amd import _native as N
        self.engine = engine
        self.lib = N.load()
        self._N = N
        if setup is None:
            with open(TRUSTED_SETUP_BIN, "rb") as f:
                setup = f.read()
        self.load_trusted_setup(setup)

    def _check(self, st: int, what: str):
        if st != 0:
            raise KzgError(f"{what}: {self._N.error_name(st)}")

    def load_trusted_setup(self, setup_bin: bytes) -> None:
        g1, g2 = read_trusted_setup_bin(setup_bin)
        g1b = np.frombuffer(b"".join(g1), np.uint8)
        g2b = np.frombuffer(b"".join(g2), np.uint8)
        status = np.zeros(len(g1), np.int32)
        u8 = ctypes.POINTER(ctypes.c_uint8)
        st = self.lib.lb_kzg_load_setup(self.engine.h, g1b.ctypes.data_as(u8), len(g1), g2b.ctypes.data_as(u8),
                                        len(g2), status.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        self._check(st, "loadTrustedSetup")

    def g1_lincomb(self, scalars: Sequence[int], points48: Sequence[bytes] = None) -> bytes:
        """sum s_i P_i with P_i the setup's [tau^i] G1 (points48 None) or the given points"""
        n = len(scalars)
        sc = _scalars_le(scalars)
        out = (ctypes.c_uint8 * 48)()
        u8 = ctypes.POINTER(ctypes.c_uint8)
        pts = None
        if points48 is not None:
            if len(points48) != n or any(len(p) != 48 for p in points48):
                raise KzgError("g1_lincomb: points must be 48-byte compressed, one per scalar")
            pts = np.frombuffer(b"".join(bytes(p) for p in points48), np.uint8)
        st = self.lib.lb_g1_lincomb(self.engine.h, n, None if pts is None else pts.ctypes.data_as(u8),
                                    sc.ctypes.data_as(u8), ctypes.cast(out, u8))
        self._check(st, "g1_lincomb")
        return bytes(out)

    def commit_coefficients(self, coeffs: Sequence[int]) -> bytes:
        return self.g1_lincomb(coeffs)

    def blob_to_kzg_commitment(self, blob: bytes) -> bytes:
        return self.commit_coefficients(evaluations_to_coefficients(blob_to_polynomial(blob)))

    def _aggregate(self, blobs: Sequence[bytes], commitments: Sequence[bytes]):
        polys = [blob_to_polynomial(b) for b in blobs]
        r_powers, x = compute_challenges(polys, commitments)
        agg = [sum(r_powers[j] * polys[j][i] for j in range(len(polys))) % BLS_MODULUS
               for i in range(FIELD_ELEMENTS_PER_BLOB)]
        return agg, r_powers, x

    def compute_kzg_proof_coefficients(self, coeffs: Sequence[int], z: int) -> Tuple[bytes, int]:
        return self.commit_coefficients(quotient_coefficients(coeffs, z)), evaluate_coefficients(coeffs, z)

    def compute_aggregate_kzg_proof(self, blobs: Sequence[bytes]) -> bytes:
        """c-kzg compute_aggregate_kzg_proof; called for every produced block (chain.ts:402), blobless
        ones included: zero blobs aggregate to the zero polynomial, whose proof is the point at
        infinity (the spec's compute_kzg_proof of the zero polynomial)."""
        if not blobs:
            return G1_INFINITY48
        commitments = [self.blob_to_kzg_commitment(b) for b in blobs]
        agg, _, x = self._aggregate(blobs, commitments)
        proof, _ = self.compute_kzg_proof_coefficients(evaluations_to_coefficients(agg), x)
        return proof

    def verify_kzg_proof(self, commitment: bytes, z: int, y: int, proof: bytes) -> bool:
        if len(commitment) != 48 or len(proof) != 48:
            raise KzgError("verify_kzg_proof: 48-byte commitment and proof")
        ok = ctypes.c_int32(0)
        u8 = ctypes.POINTER(ctypes.c_uint8)
        zb = (ctypes.c_uint8 * 32).from_buffer_copy(int(z).to_bytes(32, "little"))
        yb = (ctypes.c_uint8 * 32).from_buffer_copy(int(y).to_bytes(32, "little"))
        cb = (ctypes.c_uint8 * 48).from_buffer_copy(bytes(commitment))
        pb = (ctypes.c_uint8 * 48).from_buffer_copy(bytes(proof))
        st = self.lib.lb_kzg_verify_proof(self.engine.h, ctypes.cast(cb, u8), ctypes.cast(zb, u8),
                                          ctypes.cast(yb, u8), ctypes.cast(pb, u8), ctypes.byref(ok))
        self._check(st, "verify_kzg_proof")
        if ok.value < 0:
            raise KzgError(f"verify_kzg_proof: {self._N.error_name(-ok.value)}")
        return ok.value == 1

    def verify_aggregate_kzg_proof(self, blobs: Sequence[bytes], commitments: Sequence[bytes], proof: bytes) -> bool:
        if len(blobs) != len(commitments):
            raise KzgError("verifyAggregateKzgProof: blobs / commitments length mismatch")
        if not blobs:
            # aggregated commitment = infinity, y = 0: e(pi, [tau - z] G2) == 1 iff pi is infinity
            # (the check still decodes pi: a malformed proof raises)
            return self.verify_kzg_proof(G1_INFINITY48, compute_challenges([], [])[1], 0, proof)
        agg, r_powers, x = self._aggregate(blobs, commitments)
        c = self.g1_lincomb(r_powers, list(commitments))
        y = evaluate_coefficients(evaluations_to_coefficients(agg), x)
        return self.verify_kzg_proof(c, x, y, proof)

    # the ckzg names kzg.ts binds
    blobToKzgCommitment = blob_to_kzg_commitment
    computeAggregateKzgProof = compute_aggregate_kzg_proof
    verifyAggregateKzgProof = verify_aggregate_kzg_proof
    loadTrustedSetup = load_trusted_setup
