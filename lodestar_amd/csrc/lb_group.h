// 8-lane groups: one G2 point operation spread over the 8 lanes of a group, for the per-root
// chain of small batches (a slot of gossip, a block, one set), where one lane per root leaves
// the chip idle and the batch waits on a lone lane's serial Fp products (~1.4 us each).
//
// Every lane of a group holds the whole point (replicated state).  A formula is cut into levels
// of independent Fp products; at each level lane q of the group computes product q (one inline
// Montgomery product), and every lane collects the group's products with cross-lane reads
// (ds_bpermute).  Additions, subtractions and the selection of each lane's operands are done
// redundantly by all lanes: they cost ~1/20 of a product.  A doubling (dbl-2009-l, 16 Fp
// products) takes 3 product levels instead of 16 serial products; an addition (add-2007-bl, 43)
// takes 6.  Results are the same field elements as the lone-lane forms (canonical Fp values), so
// the group kernels are drop-in replacements (tests/test_gpu_parity.py runs both paths).
#pragma once
#include "lb_curve.h"

typedef __attribute__((address_space(3))) uint32_t lds_u32;  // (as lb_wave.h)

__device__ __forceinline__ int g8_q() { return threadIdx.x & 7; }
__device__ __forceinline__ int g8_base() { return (threadIdx.x & 63) & ~7; }

// product of lane `src` (absolute lane id within the wave)
__device__ __forceinline__ fp g8_get(const fp& m, int src) {
  fp r;
  LB_UNROLL for (int w = 0; w < 12; w++) r.v[w] = __shfl(m.v[w], src, 64);
  return r;
}
__device__ __forceinline__ fp g8_sel(bool c, const fp& a, const fp& b) {
  fp r;
  LB_UNROLL for (int w = 0; w < 12; w++) r.v[w] = c ? a.v[w] : b.v[w];
  return r;
}
// operand of lane q among up to 8 candidates (q >= count: the last one, a harmless duplicate)
__device__ __forceinline__ fp g8_pick(int q, const fp& c0, const fp& c1, const fp& c2, const fp& c3, const fp& c4,
                                      const fp& c5, const fp& c6, const fp& c7) {
  fp r = c7;
  r = g8_sel(q == 6, c6, r);
  r = g8_sel(q == 5, c5, r);
  r = g8_sel(q == 4, c4, r);
  r = g8_sel(q == 3, c3, r);
  r = g8_sel(q == 2, c2, r);
  r = g8_sel(q == 1, c1, r);
  return g8_sel(q == 0, c0, r);
}
// one product level: lane q multiplies its picked operands (inline product, no call: values
// live across an out-of-line call would go to scratch)
__device__ __forceinline__ fp g8_mul(const fp& a, const fp& b) {
  __builtin_amdgcn_sched_barrier(0);
  fp r = fp_mul28(a, b);
  __builtin_amdgcn_sched_barrier(0);
  return r;
}
// Fp2 helpers on collected products: complex squaring (t0 = (a0+a1)(a0-a1), t1 = a0 a1) and
// Karatsuba (t0 = a0 b0, t1 = a1 b1, t2 = (a0+a1)(b0+b1))
__device__ __forceinline__ fp2 g8_sqr_out(const fp& t0, const fp& t1) { return fp2{t0, fp_dbl(t1)}; }
__device__ __forceinline__ fp2 g8_mul_out(const fp& t0, const fp& t1, const fp& t2) {
  return fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}

// p = 2 p (dbl-2009-l, as jac_dbl_i); infinity (z = 0) stays infinity
__device__ __forceinline__ void g8_dbl(g2j& p) {
  const int q = g8_q(), bs = g8_base();
  // level 1: A = X^2, B = Y^2, Y Z
  {
    const fp sx = fp_add(p.x.c0, p.x.c1), dx = fp_sub(p.x.c0, p.x.c1);
    const fp sy = fp_add(p.y.c0, p.y.c1), dy = fp_sub(p.y.c0, p.y.c1), sz = fp_add(p.z.c0, p.z.c1);
    const fp a = g8_pick(q, sx, p.x.c0, sy, p.y.c0, p.y.c0, p.y.c1, sy, sy);
    const fp b = g8_pick(q, dx, p.x.c1, dy, p.y.c1, p.z.c0, p.z.c1, sz, sz);
    const fp m = g8_mul(a, b);
    const fp2 A = g8_sqr_out(g8_get(m, bs), g8_get(m, bs + 1));
    const fp2 B = g8_sqr_out(g8_get(m, bs + 2), g8_get(m, bs + 3));
    p.z = fp2_dbl(g8_mul_out(g8_get(m, bs + 4), g8_get(m, bs + 5), g8_get(m, bs + 6)));
    // level 2: C = B^2, (X + B)^2, F = E^2 with E = 3 A
    const fp2 E = fp2_mul3(A);
    const fp2 T = fp2_add(p.x, B);
    const fp a2 = g8_pick(q, fp_add(B.c0, B.c1), B.c0, fp_add(T.c0, T.c1), T.c0, fp_add(E.c0, E.c1), E.c0, E.c0, E.c0);
    const fp b2 = g8_pick(q, fp_sub(B.c0, B.c1), B.c1, fp_sub(T.c0, T.c1), T.c1, fp_sub(E.c0, E.c1), E.c1, E.c1, E.c1);
    const fp m2 = g8_mul(a2, b2);
    const fp2 C = g8_sqr_out(g8_get(m2, bs), g8_get(m2, bs + 1));
    const fp2 XB2 = g8_sqr_out(g8_get(m2, bs + 2), g8_get(m2, bs + 3));
    const fp2 F = g8_sqr_out(g8_get(m2, bs + 4), g8_get(m2, bs + 5));
    const fp2 D = fp2_dbl(fp2_sub(fp2_sub(XB2, A), C));
    p.x = fp2_sub(F, fp2_dbl(D));
    // level 3: E (D - X3)
    const fp2 W = fp2_sub(D, p.x);
    const fp a3 = g8_pick(q, E.c0, E.c1, fp_add(E.c0, E.c1), E.c0, E.c0, E.c0, E.c0, E.c0);
    const fp b3 = g8_pick(q, W.c0, W.c1, fp_add(W.c0, W.c1), W.c0, W.c0, W.c0, W.c0, W.c0);
    const fp m3 = g8_mul(a3, b3);
    p.y = fp2_sub(g8_mul_out(g8_get(m3, bs), g8_get(m3, bs + 1), g8_get(m3, bs + 2)), fp2_mul8(C));
  }
}

// p = p + r for Jacobian p, r (add-2007-bl with the exceptional cases, as jac_add_i):
// 43 Fp products in 6 levels of <= 8.  Branches are uniform within a group (replicated values).
__device__ __forceinline__ void g8_add(g2j& p, const g2j& r) {
  if (jac_is_inf(r)) return;
  if (jac_is_inf(p)) {
    p = r;
    return;
  }
  const int q = g8_q(), bs = g8_base();
  // 1: Z1Z1 (2), Z2Z2 (2), Y1 Z2 (3)
  const fp s1z = fp_add(p.z.c0, p.z.c1), s2z = fp_add(r.z.c0, r.z.c1);
  fp m = g8_mul(g8_pick(q, s1z, p.z.c0, s2z, r.z.c0, p.y.c0, p.y.c1, fp_add(p.y.c0, p.y.c1), s1z),
                g8_pick(q, fp_sub(p.z.c0, p.z.c1), p.z.c1, fp_sub(r.z.c0, r.z.c1), r.z.c1, r.z.c0, r.z.c1, s2z, s1z));
  const fp2 Z1Z1 = g8_sqr_out(g8_get(m, bs), g8_get(m, bs + 1));
  const fp2 Z2Z2 = g8_sqr_out(g8_get(m, bs + 2), g8_get(m, bs + 3));
  const fp2 Y1Z2 = g8_mul_out(g8_get(m, bs + 4), g8_get(m, bs + 5), g8_get(m, bs + 6));
  // 2: Y2 Z1 (3), U1 = X1 Z2Z2 (3), (Z1 + Z2)^2 (2)
  const fp2 ZS = fp2_add(p.z, r.z);
  m = g8_mul(g8_pick(q, r.y.c0, r.y.c1, fp_add(r.y.c0, r.y.c1), p.x.c0, p.x.c1, fp_add(p.x.c0, p.x.c1),
                     fp_add(ZS.c0, ZS.c1), ZS.c0),
             g8_pick(q, p.z.c0, p.z.c1, s1z, Z2Z2.c0, Z2Z2.c1, fp_add(Z2Z2.c0, Z2Z2.c1), fp_sub(ZS.c0, ZS.c1),
                     ZS.c1));
  const fp2 Y2Z1 = g8_mul_out(g8_get(m, bs), g8_get(m, bs + 1), g8_get(m, bs + 2));
  const fp2 U1 = g8_mul_out(g8_get(m, bs + 3), g8_get(m, bs + 4), g8_get(m, bs + 5));
  const fp2 ZZ = g8_sqr_out(g8_get(m, bs + 6), g8_get(m, bs + 7));
  // 3: U2 = X2 Z1Z1 (3), S1 = Y1Z2 Z2Z2 (3)
  m = g8_mul(g8_pick(q, r.x.c0, r.x.c1, fp_add(r.x.c0, r.x.c1), Y1Z2.c0, Y1Z2.c1, fp_add(Y1Z2.c0, Y1Z2.c1),
                     Y1Z2.c0, Y1Z2.c0),
             g8_pick(q, Z1Z1.c0, Z1Z1.c1, fp_add(Z1Z1.c0, Z1Z1.c1), Z2Z2.c0, Z2Z2.c1, fp_add(Z2Z2.c0, Z2Z2.c1),
                     Z2Z2.c0, Z2Z2.c0));
  const fp2 U2 = g8_mul_out(g8_get(m, bs), g8_get(m, bs + 1), g8_get(m, bs + 2));
  const fp2 S1 = g8_mul_out(g8_get(m, bs + 3), g8_get(m, bs + 4), g8_get(m, bs + 5));
  const fp2 H = fp2_sub(U2, U1);
  // 4: S2 = Y2Z1 Z1Z1 (3), I = (2H)^2 (2), Z3 = (ZZ - Z1Z1 - Z2Z2) H (3)
  const fp2 H2 = fp2_dbl(H);
  const fp2 ZH = fp2_sub(fp2_sub(ZZ, Z1Z1), Z2Z2);
  m = g8_mul(g8_pick(q, Y2Z1.c0, Y2Z1.c1, fp_add(Y2Z1.c0, Y2Z1.c1), fp_add(H2.c0, H2.c1), H2.c0, ZH.c0, ZH.c1,
                     fp_add(ZH.c0, ZH.c1)),
             g8_pick(q, Z1Z1.c0, Z1Z1.c1, fp_add(Z1Z1.c0, Z1Z1.c1), fp_sub(H2.c0, H2.c1), H2.c1, H.c0, H.c1,
                     fp_add(H.c0, H.c1)));
  const fp2 S2 = g8_mul_out(g8_get(m, bs), g8_get(m, bs + 1), g8_get(m, bs + 2));
  const fp2 I = g8_sqr_out(g8_get(m, bs + 3), g8_get(m, bs + 4));
  const fp2 Z3 = g8_mul_out(g8_get(m, bs + 5), g8_get(m, bs + 6), g8_get(m, bs + 7));
  const fp2 rr = fp2_dbl(fp2_sub(S2, S1));
  if (fp2_is_zero(H)) {
    if (fp2_is_zero(rr))
      g8_dbl(p);
    else
      p = jac_infinity<fp2>();
    return;
  }
  // 5: J = H I (3), V = U1 I (3), r^2 (2)
  m = g8_mul(g8_pick(q, H.c0, H.c1, fp_add(H.c0, H.c1), U1.c0, U1.c1, fp_add(U1.c0, U1.c1), fp_add(rr.c0, rr.c1),
                     rr.c0),
             g8_pick(q, I.c0, I.c1, fp_add(I.c0, I.c1), I.c0, I.c1, fp_add(I.c0, I.c1), fp_sub(rr.c0, rr.c1), rr.c1));
  const fp2 J = g8_mul_out(g8_get(m, bs), g8_get(m, bs + 1), g8_get(m, bs + 2));
  const fp2 V = g8_mul_out(g8_get(m, bs + 3), g8_get(m, bs + 4), g8_get(m, bs + 5));
  const fp2 R2 = g8_sqr_out(g8_get(m, bs + 6), g8_get(m, bs + 7));
  const fp2 X3 = fp2_sub(fp2_sub(R2, J), fp2_dbl(V));
  // 6: r (V - X3) (3), S1 J (3)
  const fp2 W = fp2_sub(V, X3);
  m = g8_mul(g8_pick(q, rr.c0, rr.c1, fp_add(rr.c0, rr.c1), S1.c0, S1.c1, fp_add(S1.c0, S1.c1), S1.c0, S1.c0),
             g8_pick(q, W.c0, W.c1, fp_add(W.c0, W.c1), J.c0, J.c1, fp_add(J.c0, J.c1), J.c0, J.c0));
  const fp2 RW = g8_mul_out(g8_get(m, bs), g8_get(m, bs + 1), g8_get(m, bs + 2));
  const fp2 SJ = g8_mul_out(g8_get(m, bs + 3), g8_get(m, bs + 4), g8_get(m, bs + 5));
  p.x = X3;
  p.y = fp2_sub(RW, fp2_dbl(SJ));
  p.z = Z3;
}

// psi(p) (6 products, one level) and psi^2(p) (4 products, one level), as g2_psi / g2_psi2
__device__ __forceinline__ g2j g8_psi(const g2j& p) {
  const int q = g8_q(), bs = g8_base();
  const fp2 cx = fp2_load(LB_PSI_CX), cy = fp2_load(LB_PSI_CY);
  const fp2 ax = fp2_conj(p.x), ay = fp2_conj(p.y);
  const fp m = g8_mul(g8_pick(q, ax.c0, ax.c1, fp_add(ax.c0, ax.c1), ay.c0, ay.c1, fp_add(ay.c0, ay.c1), ax.c0, ax.c0),
                      g8_pick(q, cx.c0, cx.c1, fp_add(cx.c0, cx.c1), cy.c0, cy.c1, fp_add(cy.c0, cy.c1), cx.c0, cx.c0));
  g2j r;
  r.x = g8_mul_out(g8_get(m, bs), g8_get(m, bs + 1), g8_get(m, bs + 2));
  r.y = g8_mul_out(g8_get(m, bs + 3), g8_get(m, bs + 4), g8_get(m, bs + 5));
  r.z = fp2_conj(p.z);
  return r;
}
__device__ __forceinline__ g2j g8_psi2(const g2j& p) {
  const int q = g8_q(), bs = g8_base();
  const fp cx = fp_load(LB_PSI2_CX), cy = fp_load(LB_PSI2_CY);
  const fp m = g8_mul(g8_pick(q, p.x.c0, p.x.c1, p.y.c0, p.y.c1, p.x.c0, p.x.c0, p.x.c0, p.x.c0),
                      g8_pick(q, cx, cx, cy, cy, cx, cx, cx, cx));
  g2j r;
  r.x = fp2{g8_get(m, bs), g8_get(m, bs + 1)};
  r.y = fp2{g8_get(m, bs + 2), g8_get(m, bs + 3)};
  r.z = p.z;
  return r;
}

// [|x|] p (as jac_mul_xabs_i): 63 doublings, 5 additions
__device__ __forceinline__ g2j g8_mul_xabs(const g2j& p) {
  g2j acc = p;
#pragma clang loop unroll(disable)
  for (int i = 62; i >= 0; i--) {
    g8_dbl(acc);
    if ((LB_X_ABS >> i) & 1ull) g8_add(acc, p);
  }
  return acc;
}

// h_eff p via psi (as g2_clear_cofactor)
__device__ __forceinline__ g2j g8_clear_cofactor(const g2j& p) {
  const g2j t1 = jac_neg(g8_mul_xabs(p));  // [x] p
  g2j t2 = g8_psi(p);
  g2j t3 = p;
  g8_dbl(t3);
  t3 = g8_psi2(t3);
  g8_add(t3, jac_neg(t2));
  g8_add(t2, t1);
  t2 = jac_neg(g8_mul_xabs(t2));  // [x](t1 + t2)
  g8_add(t3, t2);
  g8_add(t3, jac_neg(t1));
  g8_add(t3, jac_neg(p));
  return t3;
}

// [r] P for a blinding word w = hi:lo standing for r = lo + hi lambda (as jac_mul_glv_i):
// t1 = P, t2 = [lambda] P, t3 = t1 + t2; 32 doublings and up to 32 additions, each addition of
// the term the two bits select (one conditional g8_add per step, the term picked before it).
// [k0] t1 + [k1] t2 by one joint double-and-add over `bits` bits (t3 = t1 + t2)
__device__ __forceinline__ g2j g8_mul_2d(const g2j& t1, const g2j& t2, const g2j& t3, uint64_t k0, uint64_t k1,
                                         int bits) {
  g2j acc = jac_infinity<fp2>();
#pragma clang loop unroll(disable)
  for (int i = bits - 1; i >= 0; i--) {
    g8_dbl(acc);
    const uint32_t d = (uint32_t)((k0 >> i) & 1u) | ((uint32_t)((k1 >> i) & 1u) << 1);
    if (d) g8_add(acc, d == 1u ? t1 : (d == 2u ? t2 : t3));
  }
  return acc;
}
__device__ __forceinline__ g2j g8_mul_glv(const g2j& t1, const g2j& t2, const g2j& t3, uint64_t w) {
  return g8_mul_2d(t1, t2, t3, w & 0xffffffffu, w >> 32, 32);
}

// The same with the long-lived points in LDS instead of registers: the replicated form holds p,
// [x]p, psi(p) + [x]p and the partial sum (4 x 72 words per lane) across both ladders, which the
// register file cannot hold beside a G2 addition's temporaries.  G: this group's 4 x 72 words of
// LDS (every lane of the group writes and reads the same replicated values).
__device__ __forceinline__ void g8_stash(lds_u32* G, int slot, const g2j& p) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&p);
  LB_UNROLL for (int k = 0; k < 72; k++) G[72 * slot + k] = w[k];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ g2j g8_unstash(const lds_u32* G, int slot) {
  g2j p;
  uint32_t* w = reinterpret_cast<uint32_t*>(&p);
  LB_UNROLL for (int k = 0; k < 72; k++) w[k] = G[72 * slot + k];
  return p;
}
// [|x|] (point in slot s), the base re-read at the five additions
__device__ __forceinline__ g2j g8_mul_xabs_st(const lds_u32* G, int s) {
  g2j acc = g8_unstash(G, s);
#pragma clang loop unroll(disable)
  for (int i = 62; i >= 0; i--) {
    g8_dbl(acc);
    if ((LB_X_ABS >> i) & 1ull) g8_add(acc, g8_unstash(G, s));
  }
  return acc;
}
// h_eff p via psi (as g8_clear_cofactor); slots: 0 p, 1 t1 = [x]p, 2 t3, 3 t2 = psi(p) + t1
__device__ __forceinline__ g2j g8_clear_cofactor_st(const g2j& p_in, lds_u32* G) {
  g8_stash(G, 0, p_in);
  g8_stash(G, 1, jac_neg(g8_mul_xabs_st(G, 0)));  // t1 = [x] p
  {
    g2j t3 = g8_unstash(G, 0);
    g8_dbl(t3);
    t3 = g8_psi2(t3);
    g8_add(t3, jac_neg(g8_psi(g8_unstash(G, 0))));  // psi^2(2p) - psi(p)
    g8_stash(G, 2, t3);
  }
  {
    g2j t2 = g8_psi(g8_unstash(G, 0));
    g8_add(t2, g8_unstash(G, 1));  // psi(p) + t1
    g8_stash(G, 3, t2);
  }
  const g2j t2x = jac_neg(g8_mul_xabs_st(G, 3));  // [x](t1 + t2)
  g2j t3 = g8_unstash(G, 2);
  g8_add(t3, t2x);
  g8_add(t3, jac_neg(g8_unstash(G, 1)));
  g8_add(t3, jac_neg(g8_unstash(G, 0)));
  return t3;
}
