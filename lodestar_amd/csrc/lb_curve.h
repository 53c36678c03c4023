// Short-Weierstrass (a = 0) group law in Jacobian coordinates, generic over the base
// field (fp for G1: y^2 = x^3 + 4, fp2 for G2: y^2 = x^3 + 4(1+u)).
// Replaces blst's POINTonE1/POINTonE2 arithmetic used by bls.PublicKey.aggregate
// (packages/beacon-node/src/chain/bls/utils.ts:11) and by Pairing.mul_n_aggregate
// (maybeBatch.ts:18-25).  Additions are complete with respect to the cases aggregation
// meets (duplicate keys P == Q, and P == -Q), as SURVEY.md §8 a3 requires.
#pragma once
#include "lb_field.h"

template <class F>
struct jac {
  F x, y, z;  // z == 0 <=> infinity
};
template <class F>
struct aff {
  F x, y;
};

typedef jac<fp> g1j;
typedef jac<fp2> g2j;
typedef aff<fp> g1a;
typedef aff<fp2> g2a;

// the same point over another field type of the same representation (fp <-> fpi)
template <class T, class S>
LB_HD aff<T> aff_as(const aff<S>& a) {
  return aff<T>{T{a.x}, T{a.y}};
}
template <class T, class S>
LB_HD jac<T> jac_as(const jac<S>& a) {
  return jac<T>{T{a.x}, T{a.y}, T{a.z}};
}

template <class F>
LB_HD jac<F> jac_infinity() {
  jac<F> r;
  f_set_one(r.x);
  f_set_one(r.y);
  f_set_zero(r.z);
  return r;
}
template <class F>
LB_HD bool jac_is_inf(const jac<F>& p) {
  return f_is_zero(p.z);
}
template <class F>
LB_HD jac<F> jac_from_aff(const aff<F>& a) {
  jac<F> r;
  r.x = a.x;
  r.y = a.y;
  f_set_one(r.z);
  return r;
}
template <class F>
LB_HD jac<F> jac_neg(const jac<F>& p) {
  return jac<F>{p.x, f_neg(p.y), p.z};
}

// Group operations come in two forms: jac_*_i is force-inlined (the loop bodies of the scalar
// multiplications use it, so the point stays in registers; a by-value jac<> argument of an
// out-of-line call travels through scratch memory), jac_* is the out-of-line wrapper for
// one-off uses.
// dbl-2009-l
template <class F>
LB_HD jac<F> jac_dbl_i(const jac<F>& p) {
  F A = f_sqr(p.x);
  F B = f_sqr(p.y);
  F C = f_sqr(B);
  F D = f_dbl(f_sub(f_sub(f_sqr(f_add(p.x, B)), A), C));
  F E = f_mul3(A);
  F Fv = f_sqr(E);
  jac<F> r;
  r.x = f_sub(Fv, f_dbl(D));
  r.y = f_sub(f_mul(E, f_sub(D, r.x)), f_mul8(C));
  r.z = f_dbl(f_mul(p.y, p.z));
  return r;
}

template <class F>
LB_NI jac<F> jac_dbl(jac<F> p) {
  return jac_dbl_i(p);
}

// add-2007-bl with the exceptional cases handled
// kInl = true keeps the exceptional doubling inline too (a kernel with no out-of-line calls).
template <class F, bool kInl = false>
LB_HD jac<F> jac_add_i(const jac<F>& p, const jac<F>& q) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  F Z1Z1 = f_sqr(p.z);
  F Z2Z2 = f_sqr(q.z);
  F U1 = f_mul(p.x, Z2Z2);
  F U2 = f_mul(q.x, Z1Z1);
  F S1 = f_mul(f_mul(p.y, q.z), Z2Z2);
  F S2 = f_mul(f_mul(q.y, p.z), Z1Z1);
  F H = f_sub(U2, U1);
  F rr = f_dbl(f_sub(S2, S1));
  if (f_is_zero(H)) {
    if (f_is_zero(rr)) {
      if constexpr (kInl) return jac_dbl_i(p);
      else return jac_dbl(p);
    }
    return jac_infinity<F>();
  }
  F I = f_sqr(f_dbl(H));
  F J = f_mul(H, I);
  F V = f_mul(U1, I);
  jac<F> r;
  r.x = f_sub(f_sub(f_sqr(rr), J), f_dbl(V));
  r.y = f_sub(f_mul(rr, f_sub(V, r.x)), f_dbl(f_mul(S1, J)));
  r.z = f_mul(f_sub(f_sub(f_sqr(f_add(p.z, q.z)), Z1Z1), Z2Z2), H);
  return r;
}

template <class F>
LB_NI jac<F> jac_add(jac<F> p, jac<F> q) {
  return jac_add_i(p, q);
}

// madd-2007-bl: p Jacobian + q affine (q not infinity)
template <class F, bool kInl = false>
LB_HD jac<F> jac_add_aff_i(const jac<F>& p, const aff<F>& q) {
  if (jac_is_inf(p)) return jac_from_aff(q);
  F Z1Z1 = f_sqr(p.z);
  F U2 = f_mul(q.x, Z1Z1);
  F S2 = f_mul(f_mul(q.y, p.z), Z1Z1);
  F H = f_sub(U2, p.x);
  F rr = f_dbl(f_sub(S2, p.y));
  if (f_is_zero(H)) {
    if (f_is_zero(rr)) {
      if constexpr (kInl) return jac_dbl_i(p);
      else return jac_dbl(p);
    }
    return jac_infinity<F>();
  }
  F HH = f_sqr(H);
  F I = f_dbl(f_dbl(HH));
  F J = f_mul(H, I);
  F V = f_mul(p.x, I);
  jac<F> r;
  r.x = f_sub(f_sub(f_sqr(rr), J), f_dbl(V));
  r.y = f_sub(f_mul(rr, f_sub(V, r.x)), f_dbl(f_mul(p.y, J)));
  r.z = f_sub(f_sub(f_sqr(f_add(p.z, H)), Z1Z1), HH);
  return r;
}

template <class F>
LB_NI jac<F> jac_add_aff(jac<F> p, aff<F> q) {
  return jac_add_aff_i(p, q);
}

template <class F>
LB_NI bool jac_eq(jac<F> p, jac<F> q) {
  bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  if (pi || qi) return pi && qi;
  F Z1Z1 = f_sqr(p.z), Z2Z2 = f_sqr(q.z);
  if (!f_eq(f_mul(p.x, Z2Z2), f_mul(q.x, Z1Z1))) return false;
  return f_eq(f_mul(f_mul(p.y, q.z), Z2Z2), f_mul(f_mul(q.y, p.z), Z1Z1));
}

// to affine; returns false for infinity
template <class F>
LB_NI bool jac_to_aff(aff<F>& out, jac<F> p) {
  F zi = f_inv(p.z);
  F zi2 = f_sqr(zi);
  out.x = f_mul(p.x, zi2);
  out.y = f_mul(f_mul(p.y, zi2), zi);
  return !jac_is_inf(p);
}

// Register-only affine conversions for lone-lane stages of the wave kernels (jac_to_aff takes its
// point by value through the stack: a private segment of ~0.7 KB per lane in kernels that run one
// such conversion on one lane).  The only call is the product; the inversion is the inline EEA.
LB_HD void g1_to_aff_inl(g1a& out, const g1j& p) {
  const fp zi = fp_inv_i(p.z), zi2 = fp_sqr(zi);
  out.x = fp_mul(p.x, zi2);
  out.y = fp_mul(fp_mul(p.y, zi2), zi);
}
LB_HD void g2_to_aff_inl(g2a& out, const g2j& p) {
  const fp ni = fp_inv_i(fp_add(fp_sqr(p.z.c0), fp_sqr(p.z.c1)));  // 1/z = conj(z) / N(z)
  const fp2 zi{fp_mul(p.z.c0, ni), fp_neg(fp_mul(p.z.c1, ni))};
  const fp2 zi2 = fp2_sqr(zi);
  out.x = fp2_mul(p.x, zi2);
  out.y = fp2_mul(fp2_mul(p.y, zi2), zi);
}

// [k]P for a 64-bit scalar, P affine (left-to-right double-and-add)
template <class F>
LB_NI jac<F> jac_mul_u64(aff<F> p, uint64_t k) {
  jac<F> acc = jac_infinity<F>();
  for (int i = 63; i >= 0; i--) {
    acc = jac_dbl_i(acc);
    if ((k >> i) & 1ull) acc = jac_add_aff_i(acc, p);
  }
  return acc;
}

// [r]P for a structured blinding scalar.  The 64-bit word w = hi:lo stands for
//   r = lo + hi * lambda  (mod q),  lambda = -x^2 mod q,
// and t1, t2, t3 = P, [lambda]P, P + [lambda]P (affine; free through the endomorphisms, see
// k_pk_blind / k_sig_blind).  Joint double-and-add over the 32 bit pairs: 32 doublings + 32
// mixed additions, against 64 + 64 for a plain 64-bit scalar on a wave (the random bits make
// every wave execute the addition of every step).  The table entry is selected by data, so all
// lanes follow one path.  Distinct words give distinct r (the lattice {(a, b): a + b lambda = 0
// mod q} has no non-zero vector with |a|, |b| < 2^32), so a uniform non-zero word is a uniform
// draw from 2^64 - 1 distinct blinding values, the set size behind blst's 64-bit randomness.
// (jac_mul_glv_i is the inline body: k_pk_blind keeps the table in registers.)
template <class F, bool kInl = false>
LB_HD jac<F> jac_mul_2d_i(const aff<F>& t1, const aff<F>& t2, const aff<F>& t3, uint64_t k0, uint64_t k1, int bits) {
  jac<F> acc = jac_infinity<F>();
  for (int i = bits - 1; i >= 0; i--) {
    acc = jac_dbl_i(acc);
    const uint32_t d = (uint32_t)((k0 >> i) & 1u) | ((uint32_t)((k1 >> i) & 1u) << 1);
    aff<F> t;
    t.x = d == 1u ? t1.x : (d == 2u ? t2.x : t3.x);
    t.y = d == 1u ? t1.y : (d == 2u ? t2.y : t3.y);
    jac<F> s = jac_add_aff_i<F, kInl>(acc, t);
    if (d != 0u) acc = s;
  }
  return acc;
}
template <class F, bool kInl = false>
LB_HD jac<F> jac_mul_glv_i(const aff<F>& t1, const aff<F>& t2, const aff<F>& t3, uint64_t w) {
  return jac_mul_2d_i<F, kInl>(t1, t2, t3, w & 0xffffffffu, w >> 32, 32);
}
template <class F>
LB_NI jac<F> jac_mul_glv(aff<F> t1, aff<F> t2, aff<F> t3, uint64_t w) {
  return jac_mul_glv_i(t1, t2, t3, w);
}

// [k]P for a 64-bit scalar, P Jacobian (used after aggregation, before the one inversion)
template <class F>
LB_NI jac<F> jac_mul_u64_jac(jac<F> p, uint64_t k) {
  jac<F> acc = jac_infinity<F>();
  for (int i = 63; i >= 0; i--) {
    acc = jac_dbl_i(acc);
    if ((k >> i) & 1ull) acc = jac_add_i(acc, p);
  }
  return acc;
}

// [k]P for a 256-bit scalar (8 little-endian u32 words), P affine.  Synthetic-data helper
// (SecretKey.toPublicKey / SecretKey.sign), not on the verification path.
template <class F>
LB_NI jac<F> jac_mul_u256(aff<F> p, const uint32_t* k) {
  jac<F> acc = jac_infinity<F>();
  for (int i = 255; i >= 0; i--) {
    acc = jac_dbl_i(acc);
    if ((k[i >> 5] >> (i & 31)) & 1u) acc = jac_add_aff_i(acc, p);
  }
  return acc;
}

// [|x|]P for the curve parameter |x| = 0xd201000000010000 (wave-uniform bits)
template <class F, bool kInl = false>
LB_HD jac<F> jac_mul_xabs_i(const jac<F>& p) {
  jac<F> acc = p;  // top bit
  for (int i = 62; i >= 0; i--) {
    acc = jac_dbl_i(acc);
    if ((LB_X_ABS >> i) & 1ull) acc = jac_add_i<F, kInl>(acc, p);
  }
  return acc;
}
template <class F>
LB_NI jac<F> jac_mul_xabs(jac<F> p) {
  return jac_mul_xabs_i(p);
}

// ------------------------------------------------------------------ G2 endomorphism psi
LB_HD g2j g2_psi(const g2j& p) {
  g2j r;
  r.x = fp2_mul(fp2_conj(p.x), fp2_load(LB_PSI_CX));
  r.y = fp2_mul(fp2_conj(p.y), fp2_load(LB_PSI_CY));
  r.z = fp2_conj(p.z);
  return r;
}
LB_HD g2j g2_psi2(const g2j& p) {
  g2j r;
  r.x = fp2_mul_fp(p.x, fp_load(LB_PSI2_CX));
  r.y = fp2_mul_fp(p.y, fp_load(LB_PSI2_CY));
  r.z = p.z;
  return r;
}

// Scott's G2 membership test (the one blst uses): P in G2 <=> psi(P) == [x]P, x < 0.
LB_HD bool g2_in_subgroup(const g2j& p) {
  if (jac_is_inf(p)) return true;
  g2j xp = jac_neg(jac_mul_xabs(p));
  return jac_eq(g2_psi(p), xp);
}

// The same test for an affine point that is not infinity (a decoded signature, z = 1):
// [|x|]P by mixed additions with the loop state in registers, and psi(P) kept affine, so the
// comparison with [x]P = -acc is psi.x Z^2 == X and psi.y Z^3 == -Y.
// Register-lean forms for the two-waves-per-SIMD signature kernels (256 VGPRs).  kInl = true
// inlines the Fp products (fp_mul28 / fp_sqr28): with out-of-line products every value live
// across a call must sit in the ~100 callee-saved VGPRs of the AMDGPU calling convention, which
// the G2 ladder's state overflows.  The statement order is the live-range order: each temporary
// dies as early as the formula allows (dbl-2009-l and madd-2007-bl, reordered; same results as
// jac_dbl_i / jac_add_aff_i).
// (inline products are fenced with scheduling barriers: interleaving the three independent
// products of an Fp2 multiplication would hold three 28-column accumulators at once)
template <bool kInl>
LB_HD fp lean_mul(const fp& a, const fp& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (kInl) {
    __builtin_amdgcn_sched_barrier(0);
    fp r = fp_mul28(a, b);
    __builtin_amdgcn_sched_barrier(0);
    return r;
  }
#endif
  return fp_mul(a, b);
}
template <bool kInl>
LB_HD fp lean_sqr(const fp& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (kInl) {
    __builtin_amdgcn_sched_barrier(0);
    fp r = fp_sqr28(a);
    __builtin_amdgcn_sched_barrier(0);
    return r;
  }
#endif
  return fp_sqr(a);
}
template <bool kInl>
LB_HD fp2 lean2_mul(const fp2& a, const fp2& b) {
  fp t0 = lean_mul<kInl>(a.c0, b.c0);
  fp t1 = lean_mul<kInl>(a.c1, b.c1);
  fp t2 = lean_mul<kInl>(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
  return fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}
template <bool kInl>
LB_HD fp2 lean2_sqr(const fp2& a) {
  fp t0 = lean_mul<kInl>(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1));
  fp t1 = lean_mul<kInl>(a.c0, a.c1);
  return fp2{t0, fp_dbl(t1)};
}
template <bool kInl>
LB_HD void g2_dbl_lean(g2j& p) {
  p.z = fp2_dbl(lean2_mul<kInl>(p.y, p.z));        // Z3 = 2 Y Z (Z dead)
  fp2 B = lean2_sqr<kInl>(p.y);                    // Y dead from here on
  fp2 C = lean2_sqr<kInl>(B);
  fp2 A = lean2_sqr<kInl>(p.x);
  fp2 D = lean2_sqr<kInl>(fp2_add(p.x, B));        // X, B dead
  D = fp2_dbl(fp2_sub(fp2_sub(D, A), C));
  fp2 E = fp2_mul3(A);                             // A dead
  p.x = fp2_sub(lean2_sqr<kInl>(E), fp2_dbl(D));   // X3
  p.y = fp2_sub(lean2_mul<kInl>(E, fp2_sub(D, p.x)), fp2_mul8(C));
}
// p + q for q affine, p finite (the exceptional cases P == +-Q are handled)
template <bool kInl>
LB_HD void g2_add_aff_lean(g2j& p, const g2a& q) {
  fp2 Z1Z1 = lean2_sqr<kInl>(p.z);
  fp2 H = fp2_sub(lean2_mul<kInl>(q.x, Z1Z1), p.x);    // U2 - X1
  fp2 rr = lean2_mul<kInl>(lean2_mul<kInl>(q.y, p.z), Z1Z1);   // S2
  rr = fp2_dbl(fp2_sub(rr, p.y));
  if (fp2_is_zero(H)) {
    if (fp2_is_zero(rr)) {
      g2_dbl_lean<kInl>(p);
    } else {
      p = jac_infinity<fp2>();
    }
    return;
  }
  fp2 HH = lean2_sqr<kInl>(H);
  p.z = fp2_sub(fp2_sub(lean2_sqr<kInl>(fp2_add(p.z, H)), Z1Z1), HH);  // Z, Z1Z1 dead
  fp2 I = fp2_mul4(HH);                                                  // HH dead
  fp2 J = lean2_mul<kInl>(H, I);                                         // H dead
  fp2 V = lean2_mul<kInl>(p.x, I);                                       // X, I dead
  fp2 YJ = fp2_dbl(lean2_mul<kInl>(p.y, J));                             // Y dead
  p.x = fp2_sub(fp2_sub(lean2_sqr<kInl>(rr), J), fp2_dbl(V));           // J dead
  p.y = fp2_sub(lean2_mul<kInl>(rr, fp2_sub(V, p.x)), YJ);
}

// p + q for Jacobian p, q (add-2007-bl with the exceptional cases, as jac_add_i), register-lean
// statement order for the lone-lane per-root kernels
template <bool kInl>
LB_HD void g2_add_lean(g2j& p, const g2j& q) {
  if (jac_is_inf(q)) return;
  if (jac_is_inf(p)) {
    p = q;
    return;
  }
  const fp2 Z1Z1 = lean2_sqr<kInl>(p.z), Z2Z2 = lean2_sqr<kInl>(q.z);
  const fp2 ZZ = fp2_sub(fp2_sub(lean2_sqr<kInl>(fp2_add(p.z, q.z)), Z1Z1), Z2Z2);  // 2 Z1 Z2
  const fp2 U1 = lean2_mul<kInl>(p.x, Z2Z2);
  const fp2 S1 = lean2_mul<kInl>(lean2_mul<kInl>(p.y, q.z), Z2Z2);
  const fp2 H = fp2_sub(lean2_mul<kInl>(q.x, Z1Z1), U1);
  const fp2 rr = fp2_dbl(fp2_sub(lean2_mul<kInl>(lean2_mul<kInl>(q.y, p.z), Z1Z1), S1));
  if (fp2_is_zero(H)) {
    if (fp2_is_zero(rr)) {
      p = q;
      g2_dbl_lean<kInl>(p);
    } else {
      p = jac_infinity<fp2>();
    }
    return;
  }
  p.z = lean2_mul<kInl>(ZZ, H);
  const fp2 I = lean2_sqr<kInl>(fp2_dbl(H));
  const fp2 J = lean2_mul<kInl>(H, I);
  const fp2 V = lean2_mul<kInl>(U1, I);
  p.x = fp2_sub(fp2_sub(lean2_sqr<kInl>(rr), J), fp2_dbl(V));
  p.y = fp2_sub(lean2_mul<kInl>(rr, fp2_sub(V, p.x)), fp2_dbl(lean2_mul<kInl>(S1, J)));
}

// The loop is kept rolled, and the base point is re-read from memory (`src`, the caller's
// copy) at the five additions instead of being held across the 63 doublings.
LB_HD bool g2_aff_in_subgroup_i(const g2a& a) {
  g2j acc = jac_from_aff(a);
#pragma clang loop unroll(disable)
  for (int i = 62; i >= 0; i--) {
    acc = jac_dbl_i(acc);
    if ((LB_X_ABS >> i) & 1ull) acc = jac_add_aff_i<fp2, true>(acc, a);
  }
  if (jac_is_inf(acc)) return false;  // psi(P) is finite
  fp2 z2 = fp2_sqr(acc.z);
  fp2 px = fp2_mul(fp2_conj(a.x), fp2_load(LB_PSI_CX));
  if (!fp2_eq(fp2_mul(px, z2), acc.x)) return false;
  fp2 py = fp2_mul(fp2_conj(a.y), fp2_load(LB_PSI_CY));
  return fp2_eq(fp2_mul(fp2_mul(py, z2), acc.z), fp2_neg(acc.y));
}

// h_eff * P via psi (RFC 9380 App. G.3 / Budroni-Pintore)
LB_NI g2j g2_clear_cofactor(g2j p) {
  g2j t1 = jac_neg(jac_mul_xabs(p));  // [x]P
  g2j t2 = g2_psi(p);
  g2j t3 = g2_psi2(jac_dbl(p));
  t3 = jac_add(t3, jac_neg(t2));
  t2 = jac_add(t1, t2);
  t2 = jac_neg(jac_mul_xabs(t2));  // [x](t1 + t2)
  t3 = jac_add(t3, t2);
  t3 = jac_add(t3, jac_neg(t1));
  return jac_add(t3, jac_neg(p));
}

// G1 curve check (affine, y^2 == x^3 + 4)
LB_HD bool g1_aff_on_curve(const g1a& a) {
  return fp_eq(fp_sqr(a.y), fp_add(fp_mul(fp_sqr(a.x), a.x), fp_load(LB_B1)));
}
LB_HD bool g2_aff_on_curve(const g2a& a) {
  return fp2_eq(fp2_sqr(a.y), fp2_add(fp2_mul(fp2_sqr(a.x), a.x), fp2_load(LB_B2)));
}
