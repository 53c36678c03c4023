// KZG commitments over BLS12-381 (the c-kzg calls behind packages/beacon-node/src/util/kzg.ts:15-65:
// blobToKzgCommitment, computeAggregateKzgProof, verifyAggregateKzgProof).
// The GPU does the group work: G1 linear combinations of the resident trusted setup (a 4 096-term
// multi-scalar multiplication per commitment or proof) or of given points (the aggregated
// commitment), and the proof check as one two-pair pairing product.  The scalar-field work
// (inverse FFT, Fiat-Shamir challenges, evaluations, quotients) is host code
// (lodestar_amd/kzg.py).
//
// Setup layout: the monomial-form points [tau^i] G1 (what Lodestar's trusted_setup.bin holds; a
// commitment to p(X) = sum a_i X^i is sum a_i [tau^i] G1, the same point as the spec's Lagrange
// form sum p(w_i) L_i(tau) G1) as a g1a SoA table; [tau^0] G2 and [tau^1] G2 as two g2a.
#pragma once
#include "lb_kernels.h"

// [r] P == O for an affine G1 point (r = the BLS12-381 subgroup order): the G1 subgroup check of
// points that come from the wire (KZG commitments and proofs of gossip blob sidecars; c-kzg's
// validate_kzg_g1 rejects the same points)
__device__ __forceinline__ bool g1_in_subgroup_r(const g1a& a) {
  const uint32_t rr[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                          0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
  return jac_is_inf(jac_mul_u256(a, rr));
}

// one point per thread: P_i (table entry i, or 48 compressed bytes) times scalar i (32 bytes,
// little endian, < r) -> Jacobian SoA terms.  Given points are curve- and subgroup-checked.
#if LB_KG(7)
__global__ void __launch_bounds__(LB_TPB, LB_MINW) k_g1_terms(uint32_t n, const uint8_t* __restrict__ pts48,
                                                     const uint32_t* __restrict__ table, uint32_t table_cap,
                                                     const uint32_t* __restrict__ scalars,
                                                     uint32_t* __restrict__ terms, int32_t* __restrict__ status) {
  const uint32_t i = lb_tid();
  if (i >= n) return;
  g1a p;
  bool inf = false;
  int st = LB_OK;
  if (pts48) {
    uint8_t b[48];
    ld_bytes<48>(b, pts48 + (size_t)48 * i);
    st = g1_decompress48(b, p, inf);
    if (st == LB_OK && !inf && !g1_in_subgroup_r(p)) st = LB_POINT_NOT_IN_GROUP;
  } else {
    p = soa_ld<g1a>(table, table_cap, i);
  }
  uint32_t k[8];
  LB_UNROLL for (int w = 0; w < 8; w++) k[w] = scalars[(size_t)8 * i + w];
  g1j t = jac_infinity<fp>();
  if (st == LB_OK && !inf) t = jac_mul_u256(p, k);
  soa_st(terms, n, i, t);
  status[i] = st;
}
#endif  // LB_KG

// out[b] = sum of in[64 b .. 64 b + 63] (SoA, strides n_in / n_out), one wave per block
#if LB_KG(7)
__global__ void __launch_bounds__(64) k_g1_sum64(uint32_t n_in, const uint32_t* __restrict__ in, uint32_t n_out,
                                                 uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  g1j v = i < n_in ? soa_ld<g1j>(in, n_in, i) : jac_infinity<fp>();
  for (int l = 5; l >= 0; l--) {
    const unsigned d = 1u << l;
    const g1j o{fp_shfl_down(v.x, d), fp_shfl_down(v.y, d), fp_shfl_down(v.z, d)};
    if (threadIdx.x < d) v = jac_add_i(v, o);
  }
  if (threadIdx.x == 0) soa_st(out, n_out, blockIdx.x, v);
}
#endif  // LB_KG

// element 0 of a g1j SoA (stride n) -> 48 compressed bytes
#if LB_KG(7)
__global__ void __launch_bounds__(64) k_g1_out48(const uint32_t* __restrict__ in, uint32_t n, uint8_t* __restrict__ out48) {
  if (threadIdx.x != 0) return;
  const g1j v = soa_ld<g1j>(in, n, 0);
  g1a a;
  const bool fin = jac_to_aff(a, v);
  uint8_t b[48];
  g1_compress48(b, a, !fin);
  for (int k = 0; k < 48; k++) out48[k] = b[k];
}
#endif  // LB_KG

// decode the trusted setup into the resident tables (G1 points: curve + subgroup checks)
#if LB_KG(7)
__global__ void __launch_bounds__(LB_TPB, LB_MINW) k_kzg_setup_g1(uint32_t n, const uint8_t* __restrict__ in48,
                                                         uint32_t* __restrict__ table, uint32_t cap,
                                                         int32_t* __restrict__ status) {
  const uint32_t i = lb_tid();
  if (i >= n) return;
  uint8_t b[48];
  ld_bytes<48>(b, in48 + (size_t)48 * i);
  g1a a;
  bool inf;
  int st = g1_decompress48(b, a, inf);
  if (st == LB_OK && inf) st = LB_PK_IS_INFINITY;
  if (st == LB_OK) {
    const uint32_t rr[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                            0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
    if (!jac_is_inf(jac_mul_u256(a, rr))) st = LB_POINT_NOT_IN_GROUP;
  }
  if (st != LB_OK) {
    a.x = fp_zero();
    a.y = fp_zero();
  }
  soa_st(table, cap, i, a);
  status[i] = st;
}
#endif  // LB_KG
#if LB_KG(7)
__global__ void __launch_bounds__(64) k_kzg_setup_g2(const uint8_t* __restrict__ in96, uint32_t* __restrict__ g2,
                                                     int32_t* __restrict__ status) {
  const uint32_t i = threadIdx.x;
  if (i >= 2) return;
  uint8_t b[96];
  ld_bytes<96>(b, in96 + (size_t)96 * i);
  g2a a;
  bool inf;
  int st = g2_decompress96(b, a, inf);
  if (st == LB_OK && (inf || !g2_in_subgroup(jac_from_aff(a)))) st = LB_POINT_NOT_IN_GROUP;
  uint32_t* w = reinterpret_cast<uint32_t*>(&a);
  for (int k = 0; k < 48; k++) g2[48 * i + k] = w[k];
  status[i] = st;
}
#endif  // LB_KG

// verify_kzg_proof_impl: e(C - [y] G1, -G2) e(pi, [tau] G2 - [z] G2) == 1, rewritten with the
// scalar moved to G1 (bilinearity): e(Q, -G2) e(pi, [tau] G2) == 1 with Q = C - [y] G1 + [z] pi.
// Lanes 0 and 1 compute [y] G1 and [z] pi side by side, lanes 2 and 3 the subgroup checks of C
// and pi (c-kzg rejects commitments and proofs outside G1); the two Miller loops and the final
// exponentiation run on the wave engine.  io[0..47] C, [48..95] pi, scalars y, z (8 LE words
// each); g2 = [tau^0] G2, [tau^1] G2 (g2a).  *ok = 1 / 0, or -code for a bad point encoding.
#if LB_KG(5)
__global__ void __launch_bounds__(64) k_kzg_check(const uint8_t* __restrict__ io, const uint32_t* __restrict__ yz,
                                                  const uint32_t* __restrict__ g2, int32_t* __restrict__ ok) {
  LBW_SHARED_ML(S);
  __shared__ g1j sh[2];
  __shared__ int st_sh, qinf_sh, pinf_sh, grp_sh[2];
  const int lane = threadIdx.x;
  w_init_consts(S, LBW_PROGS_ALL);
  g1a c, pi;
  bool cinf = false, pinf = false;
  int st = LB_OK;
  {
    uint8_t b[48];
    for (int k = 0; k < 48; k++) b[k] = io[k];
    st = g1_decompress48(b, c, cinf);
    if (st == LB_OK) {
      for (int k = 0; k < 48; k++) b[k] = io[48 + k];
      st = g1_decompress48(b, pi, pinf);
    }
  }
  if (lane < 2) {
    uint32_t k[8];
    for (int w = 0; w < 8; w++) k[w] = yz[8 * lane + w];
    const g1a base = lane == 0 ? g1a{fp_load(LB_G1X), fp_load(LB_G1Y)} : pi;
    const bool binf = lane == 1 && pinf;
    sh[lane] = (st == LB_OK && !binf) ? jac_mul_u256(base, k) : jac_infinity<fp>();
  } else if (lane < 4) {
    const bool isc = lane == 2;
    const bool skip = st != LB_OK || (isc ? cinf : pinf);
    grp_sh[lane - 2] = skip || g1_in_subgroup_r(isc ? c : pi) ? 1 : 0;
  }
  __syncthreads();
  if (st == LB_OK && !(grp_sh[0] && grp_sh[1])) st = LB_POINT_NOT_IN_GROUP;
  if (lane == 0) {
    g1j q = cinf ? jac_infinity<fp>() : jac_from_aff(c);
    q = jac_add_i(q, jac_neg(sh[0]));
    q = jac_add_i(q, sh[1]);
    g1a qa;
    const bool qfin = jac_to_aff(qa, q);
    st_sh = st;
    qinf_sh = qfin ? 0 : 1;
    pinf_sh = pinf ? 1 : 0;
    w_st(S, LBW_PT + 0, qa.x);
    w_st(S, LBW_PT + 1, qa.y);
    const g2a* G = reinterpret_cast<const g2a*>(g2);
    const g2a g0 = G[0];
    w_st(S, LBW_PT + 2, g0.x.c0);
    w_st(S, LBW_PT + 3, g0.x.c1);
    w_st(S, LBW_PT + 4, fp_neg(g0.y.c0));  // -G2
    w_st(S, LBW_PT + 5, fp_neg(g0.y.c1));
  }
  __syncthreads();
  const int st_u = st_sh, qinf = qinf_sh, pinf_u = pinf_sh;
  __syncthreads();
  if (st_u != LB_OK) {
    if (lane == 0) *ok = -st_u;
    return;
  }
  if (qinf)
    w_set_one(S, LBW_A(0));
  else
    w_miller(S, LBW_A(0));
  if (lane == 0) {
    const g2a* G = reinterpret_cast<const g2a*>(g2);
    const g2a g1t = G[1];
    w_st(S, LBW_PT + 0, pi.x);
    w_st(S, LBW_PT + 1, pi.y);
    w_st(S, LBW_PT + 2, g1t.x.c0);
    w_st(S, LBW_PT + 3, g1t.x.c1);
    w_st(S, LBW_PT + 4, g1t.y.c0);
    w_st(S, LBW_PT + 5, g1t.y.c1);
  }
  __syncthreads();
  if (pinf_u)
    w_set_one(S, LBW_A(7));
  else
    w_miller(S, LBW_A(7));
  w_mul(S, LBW_A(0), LBW_A(0), LBW_A(7));
  w_final_exp(S, LBW_A(0), LBW_A(0));
  const bool one = w_is_one(S, LBW_A(0));
  if (lane == 0) *ok = one ? 1 : 0;
}
#endif  // LB_KG
