"""KZG (reference packages/beacon-node/src/util/kzg.ts:15-65 and its test
test/unit/util/kzg.test.ts).  c-kzg is un-vendored and the reference holds no KZG vectors, so
parity with c-kzg's bytes is unpinned; these tests pin the mathematics against the independent
oracle (oracle/kzg.py: the spec's evaluation-form formulas over oracle/bls_oracle.py).

CPU: the host scalar-field work (inverse NTT, evaluation, quotient, transcript) against the
oracle, and the trusted-setup format.  GPU: commitments of sparse polynomials against the oracle's
group arithmetic, G1 linear combinations of given points, the reference test's round trip
(two blobs -> commitments -> aggregate proof -> verifies), tampering, and the GPU's proof checked
by the oracle's pairing."""
import random

import pytest

from lodestar_amd import kzg as K
from oracle import bls_oracle as o
from oracle import kzg as OK

R = o.R


def _setup():
    with open(K.TRUSTED_SETUP_BIN, "rb") as f:
        return K.read_trusted_setup_bin(f.read())


def _blob_of(vals):
    return b"".join(int(v).to_bytes(32, "big") for v in vals)


def _sparse_blob(coeffs):
    return [sum(a * pow(x, j, R) for j, a in coeffs.items()) % R for x in K.ROOTS_BRP]


def _sequential_blob(off=0):
    """kzg.test.ts generateRandomBlob: element i = big-endian u32 i at the start of its 32 bytes"""
    b = bytearray(K.BYTES_PER_BLOB)
    for i in range(K.FIELD_ELEMENTS_PER_BLOB):
        b[32 * i: 32 * i + 4] = ((i + off) & 0xFFFFFFFF).to_bytes(4, "big")
    return bytes(b)


def test_trusted_setup_is_monomial_form():
    g1, g2 = _setup()
    assert len(g1) == 4096 and len(g2) == 65
    assert g1[0] == o.g1_compress(o.G1)                        # [tau^0] G1 = G1
    t1 = o.g1_decompress(g1[1])
    assert o.pairing(t1, o.g2_decompress(g2[0])) == o.pairing(o.G1, o.g2_decompress(g2[1]))  # same tau


def test_host_field_work_matches_oracle():
    rnd = random.Random(3)
    coeffs = {0: rnd.randrange(R), 1: rnd.randrange(R), 9: rnd.randrange(R), 4095: rnd.randrange(R)}
    vals = _sparse_blob(coeffs)
    c = K.evaluations_to_coefficients(vals)
    assert all(c[j] == coeffs.get(j, 0) for j in range(4096))
    z = rnd.randrange(R)
    y = OK.evaluate_polynomial_in_evaluation_form(vals, z, K.ROOTS_BRP)
    assert K.evaluate_coefficients(c, z) == y
    q = K.quotient_coefficients(c, z)
    t = rnd.randrange(R)
    assert K.evaluate_coefficients(q, t) * (t - z) % R == (K.evaluate_coefficients(c, t) - y) % R
    assert K.blob_to_polynomial(_blob_of(vals)) == vals
    with pytest.raises(ValueError):
        K.blob_to_polynomial(_blob_of([R] + [0] * 4095))
    polys = [vals, list(range(4096))]
    comms = [b"\x11" * 48, b"\x22" * 48]
    assert K.compute_challenges(polys, comms) == OK.compute_challenges(polys, comms)


@pytest.fixture(scope="module")
def kzg(engine):
    return K.Kzg(engine)


@pytest.mark.gpu
def test_commitment_of_sparse_polynomials_matches_oracle(kzg):
    g1, _ = _setup()
    rnd = random.Random(5)
    for coeffs in ({0: 1}, {1: 1}, {0: rnd.randrange(R), 3: rnd.randrange(R), 4095: rnd.randrange(R)}):
        got = kzg.blob_to_kzg_commitment(_blob_of(_sparse_blob(coeffs)))
        assert got == o.g1_compress(OK.commit_monomials(g1, coeffs)), coeffs
    assert kzg.blob_to_kzg_commitment(bytes(K.BYTES_PER_BLOB)) == bytes([0xC0]) + bytes(47)  # zero poly: infinity


@pytest.mark.gpu
def test_g1_lincomb_of_given_points(kzg):
    rnd = random.Random(9)
    pts = [o.g1_mul(o.G1, rnd.randrange(1, R)) for _ in range(70)]   # 70 terms: two reduction levels
    sc = [rnd.randrange(R) for _ in pts]
    exp = None
    for p, s in zip(pts, sc):
        exp = o.g1_add(exp, o.g1_mul(p, s))
    assert kzg.g1_lincomb(sc, [o.g1_compress(p) for p in pts]) == o.g1_compress(exp)


@pytest.mark.gpu
def test_aggregate_proof_round_trip_and_tampering(kzg):
    """kzg.test.ts 'computes the correct commitments and aggregate proofs from blobs'"""
    _, g2 = _setup()
    blobs = [_sequential_blob(0), _sequential_blob(7)]
    comms = [kzg.blobToKzgCommitment(b) for b in blobs]
    proof = kzg.computeAggregateKzgProof(blobs)
    assert kzg.verifyAggregateKzgProof(blobs, comms, proof) is True
    # the GPU's proof checked by the oracle's pairing, at the point the transcript picks
    agg, r_powers, x = kzg._aggregate(blobs, comms)
    y = OK.evaluate_polynomial_in_evaluation_form(agg, x, K.ROOTS_BRP)
    c_agg = kzg.g1_lincomb(r_powers, comms)
    assert OK.verify_kzg_proof_impl(c_agg, x, y, proof, g2)
    assert not OK.verify_kzg_proof_impl(c_agg, x, (y + 1) % R, proof, g2)
    # tampering: a changed blob, swapped commitments, another proof
    bad = bytearray(blobs[1])
    bad[31] ^= 1
    assert kzg.verifyAggregateKzgProof([blobs[0], bytes(bad)], comms, proof) is False
    assert kzg.verifyAggregateKzgProof(blobs, comms[::-1], proof) is False
    assert kzg.verifyAggregateKzgProof(blobs, comms, kzg.computeAggregateKzgProof(blobs[:1])) is False
    # one blob
    assert kzg.verifyAggregateKzgProof(blobs[:1], comms[:1], kzg.computeAggregateKzgProof(blobs[:1])) is True
    # zero blobs (every blobless block, chain.ts:402): the proof is the point at infinity and
    # verifies against no commitments; any other proof does not
    inf = bytes([0xC0]) + bytes(47)
    assert kzg.computeAggregateKzgProof([]) == inf
    assert kzg.verifyAggregateKzgProof([], [], inf) is True
    assert kzg.verifyAggregateKzgProof([], [], proof) is False
    with pytest.raises(K.KzgError):
        kzg.verifyAggregateKzgProof(blobs[:1], [], proof)


def _off_subgroup_g1():
    """an on-curve G1 point outside the order-r subgroup (cofactor component)"""
    x = 5
    while True:
        y = o.fp_sqrt((x * x * x + o.B1) % o.P)
        if y is not None and o.g1_mul((x, y), R) is not None:
            return (x, y)
        x += 1


@pytest.mark.gpu
def test_points_outside_g1_are_rejected(kzg):
    """c-kzg validate_kzg_g1: commitments, proofs and lincomb points must lie in G1"""
    bad = o.g1_compress(_off_subgroup_g1())
    good = o.g1_compress(o.G1)
    with pytest.raises(K.KzgError, match="BLST_POINT_NOT_IN_GROUP"):
        kzg.g1_lincomb([1, 2], [good, bad])
    with pytest.raises(K.KzgError, match="BLST_POINT_NOT_IN_GROUP"):
        kzg.verify_kzg_proof(bad, 3, 4, good)
    with pytest.raises(K.KzgError, match="BLST_POINT_NOT_IN_GROUP"):
        kzg.verify_kzg_proof(good, 3, 4, bad)
    assert kzg.verify_kzg_proof(good, 3, 4, good) is False  # in-group points still decide normally
