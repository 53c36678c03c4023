"""CPU oracle for the KZG path (test infrastructure only: tests/ and bench.py's baseline may
import it; the product, lodestar_amd/kzg.py + the HIP kernels, never does).

Restates the EIP-4844 polynomial-commitments functions of the reference's pinned spec version
(v1.3.0-alpha.2, packages/beacon-node/test/spec/specTestVersioning.ts:18) the way the spec writes
them -- evaluation form with the barycentric formula over the bit-reversed roots of unity, the
pairing check verify_kzg_proof_impl -- over oracle/bls_oracle.py's group arithmetic and pairing.
This is a different route from the product's (monomial coefficients by an inverse NTT on the
host, commitments as GPU multi-scalar multiplications of the monomial setup), so agreement checks
both.  c-kzg itself is un-vendored and the reference holds no KZG vectors: parity with c-kzg's
bytes is UNPINNED (see lodestar_amd/kzg.py); field elements are big-endian as in Lodestar's
blobsSidecar.ts:138-150.
"""
import hashlib

from oracle import bls_oracle as o

BLS_MODULUS = o.R
N = 4096
DOMAIN = b"FSBLOBVERIFY_V1_"


def roots_brp(n=N):
    w = pow(7, (BLS_MODULUS - 1) // n, BLS_MODULUS)
    roots = [pow(w, i, BLS_MODULUS) for i in range(n)]
    bits = n.bit_length() - 1
    return [roots[int(format(i, f"0{bits}b")[::-1], 2)] for i in range(n)]


def evaluate_polynomial_in_evaluation_form(poly, z, rb=None):
    """spec: barycentric evaluation of the polynomial given by its values at the bit-reversed roots"""
    rb = rb or roots_brp(len(poly))
    width = len(poly)
    inv_width = pow(width, BLS_MODULUS - 2, BLS_MODULUS)
    acc = 0
    for i in range(width):
        acc += poly[i] * rb[i] * pow((z - rb[i]) % BLS_MODULUS, BLS_MODULUS - 2, BLS_MODULUS)
    return acc % BLS_MODULUS * (pow(z, width, BLS_MODULUS) - 1) * inv_width % BLS_MODULUS


def hash_to_bls_field(data):
    return int.from_bytes(hashlib.sha256(data).digest(), "big") % BLS_MODULUS


def compute_challenges(polys, commitments):
    data = DOMAIN + N.to_bytes(8, "big") + len(polys).to_bytes(8, "big")
    data += b"".join(v.to_bytes(32, "big") for p in polys for v in p)
    data += b"".join(commitments)
    h = hashlib.sha256(data).digest()
    r = hash_to_bls_field(h + b"\x00")
    return [pow(r, i, BLS_MODULUS) for i in range(len(commitments))], hash_to_bls_field(h + b"\x01")


def commit_monomials(setup_g1, coeffs):
    """sum a_j [tau^j] G1 for a sparse {j: a_j}"""
    acc = None
    for j, a in coeffs.items():
        acc = o.g1_add(acc, o.g1_mul(o.g1_decompress(setup_g1[j]), a))
    return acc


def verify_kzg_proof_impl(commitment48, z, y, proof48, setup_g2):
    """e(C - [y] G1, -G2) e(proof, [tau] G2 - [z] G2) == 1"""
    g2 = o.g2_decompress(setup_g2[0])
    tau_g2 = o.g2_decompress(setup_g2[1])
    x_minus_z = o.g2_add(tau_g2, o.g2_mul(g2, (BLS_MODULUS - z) % BLS_MODULUS))
    p_minus_y = o.g1_add(o.g1_decompress(commitment48), o.g1_mul(o.G1, (BLS_MODULUS - y) % BLS_MODULUS))
    pi = o.g1_decompress(proof48)
    f = o.F12_ONE
    if p_minus_y is not None:
        f = o.f12_mul(f, o.miller_loop(p_minus_y, o.g2_neg(g2)))
    if pi is not None:
        f = o.f12_mul(f, o.miller_loop(pi, x_minus_z))
    return o.final_exponentiation(f) == o.F12_ONE
