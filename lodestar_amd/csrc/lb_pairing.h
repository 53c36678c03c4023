// Optimal-ate Miller loop and final exponentiation for BLS12-381 (M-type sextic twist,
// y^2 = x^3 + 4(1+u)).  Replaces blst's miller_loop_n / final_exp behind
// Pairing.commit + Pairing.finalverify (maybeBatch.ts:18-25).
//
// Lines are evaluated at the G1 point P = (xP, yP) and kept in the sparse form
//   l = l0 + l2 w^2 + l3 w^3      (Fp12 = Fp6[w]/(w^2 - v))
// which differs from the textbook line value only by factors in Fp4, killed by the
// final exponentiation.  The hard part computes f^(3(p^4-p^2+1)/r); cubing is a
// bijection on the order-r group, so "== 1" decides exactly as blst's finalverify.
#pragma once
#include "lb_curve.h"

// doubling step on T = (X, Y, Z) (homogeneous projective on the twist), line at P.
// 25 Fp multiplications: 3b' = 12(1 + u) is applied with additions, and the output is scaled
// by 4 (a homogeneous (X:Y:Z) ~ (4X:4Y:4Z)) so the textbook halvings of X3, Y3 disappear.
template <bool kInl = false>
LB_HD void miller_dbl(g2j& T, fp2& l0, fp2& l2, fp2& l3, const fp& xP, const fp& yP) {
  fp2 X = T.x, Y = T.y, Z = T.z;
  fp2 A = lean2_mul<kInl>(X, Y);             // XY
  fp2 B = lean2_sqr<kInl>(Y);
  fp2 C = lean2_sqr<kInl>(Z);
  fp2 E = fp2_mul3(fp2_dbl(fp2_dbl(fp2_mul_xi(C))));  // 3b' Z^2 = 12 (1 + u) Z^2
  fp2 F = fp2_mul3(E);               // 9b' Z^2
  fp2 H = fp2_sub(lean2_sqr<kInl>(fp2_add(Y, Z)), fp2_add(B, C));  // 2YZ
  fp2 XX3 = fp2_mul3(lean2_sqr<kInl>(X));
  // line: (B - E) + (-3X^2 xP) w^2 + (H yP) w^3
  l0 = fp2_sub(B, E);
  l2 = fp2_neg(fp2{lean_mul<kInl>(XX3.c0, xP), lean_mul<kInl>(XX3.c1, xP)});
  l3 = fp2{lean_mul<kInl>(H.c0, yP), lean_mul<kInl>(H.c1, yP)};
  // 4 x (X3, Y3, Z3) with X3 = XY/2 (B - F), Y3 = ((B+F)/2)^2 - 3E^2, Z3 = B H:
  //   X3' = 2 A (B - F),  Y3' = (B + F)^2 - 12 E^2,  Z3' = 4 B H
  T.x = fp2_dbl(lean2_mul<kInl>(A, fp2_sub(B, F)));
  T.y = fp2_sub(lean2_sqr<kInl>(fp2_add(B, F)), fp2_mul3(fp2_dbl(fp2_dbl(lean2_sqr<kInl>(E)))));
  T.z = fp2_dbl(fp2_dbl(lean2_mul<kInl>(B, H)));
}

// addition step T <- T + Q (Q affine), line through T and Q at P
template <bool kInl = false>
LB_HD void miller_add(g2j& T, const g2a& Q, fp2& l0, fp2& l2, fp2& l3, const fp& xP, const fp& yP) {
  fp2 theta = fp2_sub(T.y, lean2_mul<kInl>(Q.y, T.z));
  fp2 lam = fp2_sub(T.x, lean2_mul<kInl>(Q.x, T.z));
  // line: (theta xQ - lam yQ) + (-theta xP) w^2 + (lam yP) w^3
  l0 = fp2_sub(lean2_mul<kInl>(theta, Q.x), lean2_mul<kInl>(lam, Q.y));
  l2 = fp2_neg(fp2{lean_mul<kInl>(theta.c0, xP), lean_mul<kInl>(theta.c1, xP)});
  l3 = fp2{lean_mul<kInl>(lam.c0, yP), lean_mul<kInl>(lam.c1, yP)};
  fp2 C = lean2_sqr<kInl>(theta);
  fp2 D = lean2_sqr<kInl>(lam);
  fp2 E = lean2_mul<kInl>(lam, D);
  fp2 F = lean2_mul<kInl>(T.z, C);
  fp2 G = lean2_mul<kInl>(T.x, D);
  fp2 H = fp2_sub(fp2_add(E, F), fp2_dbl(G));
  T.x = lean2_mul<kInl>(lam, H);
  T.y = fp2_sub(lean2_mul<kInl>(theta, fp2_sub(G, H)), lean2_mul<kInl>(E, T.y));
  T.z = lean2_mul<kInl>(T.z, E);
}

// f_{|x|,Q}(P), conjugated (x < 0).  P, Q affine and not infinity.
LB_NI fp12 miller_loop(g1a P, g2a Q) {
  g2j T;
  T.x = Q.x;
  T.y = Q.y;
  T.z = fp2_one();
  fp2 l0, l2, l3;
  fp12 f = fp12_one();
  bool first = true;
  for (int i = 62; i >= 0; i--) {
    if (!first) f = fp12_sqr(f);
    miller_dbl(T, l0, l2, l3, P.x, P.y);
    if (first) {
      f = fp12_one();
      first = false;
    }
    f = fp12_mul_line(f, l0, l2, l3);
    if ((LB_X_ABS >> i) & 1ull) {
      miller_add(T, Q, l0, l2, l3, P.x, P.y);
      f = fp12_mul_line(f, l0, l2, l3);
    }
  }
  return fp12_conj(f);
}

// Same loop with the Fp12 squaring / line multiplication / point steps inlined, so f, T and
// the line values stay in registers (only fp_mul is a call).  The pointer-argument versions
// cost ~8 GB of scratch traffic per 19k-pair launch (profiles/r1_pmc_*).
LB_HD fp12 miller_loop_inl(const g1a& P, const g2a& Q) {
  g2j T;
  T.x = Q.x;
  T.y = Q.y;
  T.z = fp2_one();
  fp2 l0, l2, l3;
  fp12 f = fp12_one();
  bool first = true;
  for (int i = 62; i >= 0; i--) {
    if (!first) f = fp12_sqr_inl(f);
    miller_dbl(T, l0, l2, l3, P.x, P.y);
    if (first) {
      f = fp12_one();
      first = false;
    }
    f = fp12_mul_line_inl(f, l0, l2, l3);
    if ((LB_X_ABS >> i) & 1ull) {
      miller_add(T, Q, l0, l2, l3, P.x, P.y);
      f = fp12_mul_line_inl(f, l0, l2, l3);
    }
  }
  return fp12_conj(f);
}

// a^|x| for a in the cyclotomic subgroup
LB_NI fp12 fp12_pow_xabs(fp12 a) {
  fp12 r = a;
  for (int i = 62; i >= 0; i--) {
    r = fp12_sqr(r);
    if ((LB_X_ABS >> i) & 1ull) r = fp12_mul(r, a);
  }
  return r;
}

// f^(3 (p^12 - 1)/r)
LB_NI fp12 final_exponentiation(fp12 f) {
  // easy part: f^((p^6 - 1)(p^2 + 1))
  fp12 t = fp12_mul(fp12_conj(f), fp12_inv(f));
  t = fp12_mul(fp12_frob2(t), t);
  // hard part: t^((x-1)^2 (x+p) (x^2+p^2-1) + 3)
  fp12 a = fp12_conj(fp12_mul(fp12_pow_xabs(t), t));  // t^(x-1)
  a = fp12_conj(fp12_mul(fp12_pow_xabs(a), a));        // t^((x-1)^2)
  fp12 b = fp12_mul(fp12_conj(fp12_pow_xabs(a)), fp12_frob(a));  // a^(x+p)
  fp12 c = fp12_pow_xabs(fp12_pow_xabs(b));                        // b^(x^2)
  c = fp12_mul(fp12_mul(c, fp12_frob2(b)), fp12_conj(b));          // b^(x^2+p^2-1)
  fp12 t3 = fp12_mul(fp12_sqr(t), t);
  return fp12_mul(c, t3);
}
