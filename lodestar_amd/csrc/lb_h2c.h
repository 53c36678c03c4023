// hash_to_G2 for BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_ (RFC 9380), one message per
// thread.  Replaces the hashing blst performs inside Pairing.mul_n_aggregate /
// Pairing.aggregate(hash_or_encode = true) for every set (maybeBatch.ts:18-25, 36-37).
// Messages are Lodestar signing roots: exactly 32 bytes (ISignatureSet.signingRoot,
// packages/state-transition/src/util/signatureSets.ts:14).
#pragma once
#include "lb_curve.h"

// ------------------------------------------------------------------ SHA-256
LB_CONST uint32_t LB_SHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

LB_HD uint32_t lb_rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// one compression of a 16-word big-endian block into state h
LB_NI void sha256_compress(uint32_t h[8], const uint32_t blk[16]) {
  uint32_t w[16];
  LB_UNROLL for (int i = 0; i < 16; i++) w[i] = blk[i];
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  LB_UNROLL for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = lb_rotr(w15, 7) ^ lb_rotr(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = lb_rotr(w2, 17) ^ lb_rotr(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = lb_rotr(e, 6) ^ lb_rotr(e, 11) ^ lb_rotr(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = hh + S1 + ch + LB_SHA_K[i] + wi;
    uint32_t S0 = lb_rotr(a, 2) ^ lb_rotr(a, 13) ^ lb_rotr(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
  h[5] += f;
  h[6] += g;
  h[7] += hh;
}

LB_HD void sha256_init(uint32_t h[8]) {
  h[0] = 0x6a09e667; h[1] = 0xbb67ae85; h[2] = 0x3c6ef372; h[3] = 0xa54ff53a;
  h[4] = 0x510e527f; h[5] = 0x9b05688c; h[6] = 0x1f83d9ab; h[7] = 0x5be0cd19;
}

// Byte-addressed message builder over a 16-word block, big-endian within words.
LB_HD void blk_put(uint32_t blk[16], int pos, uint32_t byte) {
  int w = pos >> 2, sh = (3 - (pos & 3)) * 8;
  blk[w] |= (byte & 0xffu) << sh;
}

// DST' = DST || len(DST)
#define LB_DST_LEN 43
LB_CONST uint8_t LB_DST[LB_DST_LEN + 1] = {
    'B', 'L', 'S', '_', 'S', 'I', 'G', '_', 'B', 'L', 'S', '1', '2', '3', '8', '1', 'G', '2', '_', 'X', 'M', 'D',
    ':', 'S', 'H', 'A', '-', '2', '5', '6', '_', 'S', 'S', 'W', 'U', '_', 'R', 'O', '_', 'P', 'O', 'P', '_', 43};

// SHA-256 over (prefix[npre] || msg_tail) where the whole message is < 120 bytes after the
// optional 64-byte zero block; generic small-message helper used by expand_message_xmd.
// `m` holds the bytes (after any leading constant block), `len` bytes; `total` is the full
// message length for padding (includes a leading zero block when `zero_block` is set).
LB_HD void sha256_small(uint32_t out[8], const uint8_t* m, int len, bool zero_block) {
  uint32_t h[8];
  sha256_init(h);
  uint32_t blk[16];
  if (zero_block) {
    LB_UNROLL for (int i = 0; i < 16; i++) blk[i] = 0;
    sha256_compress(h, blk);
  }
  uint64_t total_bits = (uint64_t)(len + (zero_block ? 64 : 0)) * 8;
  // message + 0x80 + length (8 bytes) fits in at most 3 blocks here (len <= 150)
  int nblk = (len + 9 + 63) / 64;
  for (int b = 0; b < nblk; b++) {
    LB_UNROLL for (int i = 0; i < 16; i++) blk[i] = 0;
    for (int i = 0; i < 64; i++) {
      int pos = b * 64 + i;
      uint32_t byte = 0;
      if (pos < len)
        byte = m[pos];
      else if (pos == len)
        byte = 0x80;
      else if (pos >= nblk * 64 - 8)
        byte = (uint32_t)(total_bits >> (8 * (nblk * 64 - 1 - pos))) & 0xff;
      blk_put(blk, i, byte);
    }
    sha256_compress(h, blk);
  }
  LB_UNROLL for (int i = 0; i < 8; i++) out[i] = h[i];
}

// expand_message_xmd(msg32, DST, 256) -> 8 x 32-byte blocks (as big-endian words)
LB_NI void expand_message_xmd_256(uint32_t out[64], const uint8_t msg[32]) {
  uint8_t buf[32 + 2 + 1 + LB_DST_LEN + 1];
  // b0 = H(Z_pad || msg || I2OSP(256, 2) || I2OSP(0, 1) || DST')
  for (int i = 0; i < 32; i++) buf[i] = msg[i];
  buf[32] = 1;
  buf[33] = 0;
  buf[34] = 0;
  for (int i = 0; i < LB_DST_LEN + 1; i++) buf[35 + i] = LB_DST[i];
  uint32_t b0[8];
  sha256_small(b0, buf, 35 + LB_DST_LEN + 1, true);
  // b_i = H((b0 xor b_{i-1}) || I2OSP(i, 1) || DST')
  uint32_t prev[8];
  LB_UNROLL for (int k = 0; k < 8; k++) prev[k] = 0;
  for (int i = 1; i <= 8; i++) {
    for (int k = 0; k < 8; k++) {
      uint32_t wv = b0[k] ^ prev[k];
      buf[4 * k] = (uint8_t)(wv >> 24);
      buf[4 * k + 1] = (uint8_t)(wv >> 16);
      buf[4 * k + 2] = (uint8_t)(wv >> 8);
      buf[4 * k + 3] = (uint8_t)wv;
    }
    buf[32] = (uint8_t)i;
    for (int j = 0; j < LB_DST_LEN + 1; j++) buf[33 + j] = LB_DST[j];
    uint32_t bi[8];
    sha256_small(bi, buf, 33 + LB_DST_LEN + 1, false);
    for (int k = 0; k < 8; k++) {
      out[(i - 1) * 8 + k] = bi[k];
      prev[k] = bi[k];
    }
  }
}

// 64 big-endian bytes (as 16 BE words) -> element of Fp in Montgomery form (value mod p)
LB_HD fp fp_from_be64_words(const uint32_t* wds) {
  fp hi, lo;
  LB_UNROLL for (int i = 0; i < 12; i++) {
    hi.v[i] = 0;
    lo.v[i] = 0;
  }
  LB_UNROLL for (int i = 0; i < 8; i++) {
    hi.v[i] = wds[7 - i];
    lo.v[i] = wds[15 - i];
  }
  // both halves < 2^256 < p, so to_mont is exact
  fp him = fp_to_mont(hi), lom = fp_to_mont(lo);
  return fp_add(fp_mul(him, fp_load(LB_2P256)), lom);
}

// ------------------------------------------------------------------ SSWU + 3-isogeny
LB_NI g2j map_to_curve_g2(fp2 u) {
  const fp2 A = fp2_load(LB_SSWU_A), B = fp2_load(LB_SSWU_B), Z = fp2_load(LB_SSWU_Z);
  fp2 u2 = fp2_sqr(u);
  fp2 zu2 = fp2_mul(Z, u2);
  fp2 tv1 = fp2_add(fp2_sqr(zu2), zu2);
  bool exc = fp2_is_zero(tv1);
  fp2 x1 = fp2_mul(fp2_load(LB_SSWU_MBDIVA), fp2_add(fp2_one(), fp2_inv(tv1)));
  x1 = fp2_select(exc, fp2_load(LB_SSWU_BDIVZA), x1);
  fp2 gx1 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1), A), x1), B);
  fp2 x2 = fp2_mul(zu2, x1);
  fp2 gx2 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x2), A), x2), B);
  bool sq1 = fp2_is_square(gx1);
  fp2 x = fp2_select(sq1, x1, x2);
  fp2 gx = fp2_select(sq1, gx1, gx2);
  fp2 y;
  fp2_sqrt(y, gx);
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  // 3-isogeny E2' -> E2, output in Jacobian coordinates with Z = xden * yden
  fp2 xx = fp2_sqr(x), xxx = fp2_mul(xx, x);
  fp2 xn = fp2_add(fp2_add(fp2_add(fp2_mul(fp2_load(LB_ISO_XNUM3), xxx), fp2_mul(fp2_load(LB_ISO_XNUM2), xx)),
                           fp2_mul(fp2_load(LB_ISO_XNUM1), x)),
                   fp2_load(LB_ISO_XNUM0));
  fp2 xd = fp2_add(fp2_add(xx, fp2_mul(fp2_load(LB_ISO_XDEN1), x)), fp2_load(LB_ISO_XDEN0));
  fp2 yn = fp2_add(fp2_add(fp2_add(fp2_mul(fp2_load(LB_ISO_YNUM3), xxx), fp2_mul(fp2_load(LB_ISO_YNUM2), xx)),
                           fp2_mul(fp2_load(LB_ISO_YNUM1), x)),
                   fp2_load(LB_ISO_YNUM0));
  fp2 yd = fp2_add(fp2_add(fp2_add(xxx, fp2_mul(fp2_load(LB_ISO_YDEN2), xx)), fp2_mul(fp2_load(LB_ISO_YDEN1), x)),
                   fp2_load(LB_ISO_YDEN0));
  g2j r;
  fp2 yd2 = fp2_sqr(yd);
  fp2 xd2 = fp2_sqr(xd);
  r.z = fp2_mul(xd, yd);
  r.x = fp2_mul(fp2_mul(xn, xd), yd2);
  r.y = fp2_mul(fp2_mul(fp2_mul(y, yn), fp2_mul(xd2, xd)), yd2);
  return r;
}

// The same map with the SSWU denominator's inversion and gx1's Legendre symbol folded into the
// square root's first exponentiation, so the chain is two exponentiations by (p - 3) / 4 and a
// few dozen products (map_to_curve_g2 above: an Fp2 inversion, a Jacobi symbol, then the two
// exponentiations).  `pow(a, LB_EXP_ISQRT, 378)` returns a^((p-3)/4); the output is the same
// Jacobian point as map_to_curve_g2 (same affine x, y; Z = xden yden).
//   x1 = N / D (projective SSWU), gx1 = U / V with U = N^3 + A N D^2 + B D^3, V = D^3;
//   t = nu nv^3 (nu = norm U, nv = norm V), w = t^((p-3)/4), chi = w^2 t = t^((p-1)/2):
//     chi = legendre(norm gx1) (gx1 is a square in Fp2 iff its norm is one in Fp, or gx1 = 0),
//     1/nv = chi nu nv^2 w^2 (t != 0), so 1/V = conj(V) / nv and gx1, x1 are affine,
//     y1 = nu nv w: y1^2 = chi norm(gx1), i.e. sqrt(norm gx1) when chi = 1;
//   chi = -1: x2 = Z u^2 x1, gx2 = (Z u^2)^3 gx1, norm gx2 = 125 N(u)^6 norm gx1 (norm Z = 5), so
//     sqrt(norm gx2) = sqrt(-125) N(u)^3 y1;
//   then the complex method from alpha = sqrt(norm gx) (one more exponentiation), as fp2_sqrt_p.
// Generic over the field types (F2, F): fp2 / fp (lane arithmetic, the CPU harness) or rfp2 / rfp
// (lb_row.h: every product a row product, k_hash_map_row), through f_* and the fl_* policy below;
// pow: F -> F.  Decisions and the output go through canonical values (fl_out).
LB_HD fp fl_in(const fp& a, const fp*) { return a; }
LB_HD fp2 fl_in(const fp2& a, const fp2*) { return a; }
LB_HD fp fl_out(const fp& a) { return a; }
LB_HD fp2 fl_out(const fp2& a) { return a; }
LB_HD fp fl_norm(const fp2& a) { return fp_add(fp_sqr(a.c0), fp_sqr(a.c1)); }
LB_HD fp2 fl_mulb(const fp2& a, const fp& s) { return fp2_mul_fp(a, s); }
LB_HD fp2 fl_conj(const fp2& a) { return fp2_conj(a); }
LB_HD fp2 fl_make(const fp& a, const fp& b) { return fp2{a, b}; }
LB_HD fp fl_c0(const fp2& a) { return a.c0; }
LB_HD fp fl_c1(const fp2& a) { return a.c1; }
template <class F2, class F, class Pow>
LB_HD g2j map_to_curve_g2_fold_t(const fp2& u_in, Pow pow) {
  const F2* t2 = nullptr;
  const F* t1 = nullptr;
  auto C2 = [&](const uint32_t* c) { return fl_in(fp2_load(c), t2); };
  const F2 u = fl_in(u_in, t2);
  const F2 A = C2(LB_SSWU_A), B = C2(LB_SSWU_B), Z = C2(LB_SSWU_Z);
  const F2 zu2 = f_mul(Z, f_sqr(u));
  const F2 tv1 = f_add(f_sqr(zu2), zu2);
  const bool exc = fp2_is_zero(fl_out(tv1));
  F2 one;
  f_set_one(one);
  // x1 = -B (1 + 1/tv1) / A = -B (tv1 + 1) / (A tv1); tv1 = 0: B / (Z A)
  const F2 N = f_select(exc, B, f_neg(f_mul(B, f_add(tv1, one))));
  const F2 D = f_select(exc, f_mul(Z, A), f_mul(A, tv1));
  const F2 D2 = f_sqr(D), V = f_mul(D2, D);
  const F2 U = f_add(f_mul(f_add(f_sqr(N), f_mul(A, D2)), N), f_mul(B, V));
  const F nu = fl_norm(U), nv = fl_norm(V);
  const F nv2 = f_sqr(nv);
  const F t = f_mul(nu, f_mul(nv2, nv));
  const F w = pow(t, LB_EXP_ISQRT, 378);
  const F w2 = f_sqr(w);
  const fp chi = fl_out(f_mul(w2, t));
  const bool qr = !fp_eq(chi, fp_neg(fp_one()));  // chi = 1, or 0 (gx1 = 0 is a square)
  F inv_nv = f_mul(f_mul(nu, nv2), w2);
  if (!qr) inv_nv = f_neg(inv_nv);
  if (fp_is_zero(chi)) inv_nv = fl_in(fp_inv_i(fl_out(nv)), t1);  // gx1 = 0 (V != 0: D != 0 always)
  const F2 inv_v = fl_mulb(fl_conj(V), inv_nv);
  F2 x = f_mul(f_mul(N, D2), inv_v);  // N / D
  F2 gx = f_mul(U, inv_v);
  F alpha = f_mul(f_mul(nu, nv), w);
  if (!qr) {
    const F nuu = fl_norm(u);
    alpha = f_mul(alpha, f_mul(fl_in(fp_load(LB_SQRT_M125), t1), f_mul(f_sqr(nuu), nuu)));
    x = f_mul(zu2, x);
    gx = f_mul(gx, f_mul(f_sqr(zu2), zu2));
  }
  // complex method (fp2_sqrt_i) from alpha
  const F inv2 = fl_in(fp_load(LB_INV2), t1);
  const F g0 = fl_c0(gx);
  const F d1 = f_mul(f_add(g0, alpha), inv2);
  const F d2 = f_mul(f_sub(g0, alpha), inv2);
  const F delta = f_select(fp_is_zero(fl_out(d1)), d2, d1);
  const F z = pow(delta, LB_EXP_ISQRT, 378);
  const F s = f_mul(delta, z);
  const bool delta_qr = f_eq(f_sqr(s), delta);
  F tt = f_mul(z, inv2);
  if (!delta_qr) tt = f_neg(tt);
  const F q = f_mul(fl_c1(gx), tt);
  F2 y = fl_make(f_select(delta_qr, s, q), f_select(delta_qr, q, s));
  if (fp2_sgn0(u_in) != fp2_sgn0(fl_out(y))) y = f_neg(y);
  // 3-isogeny E2' -> E2 (as map_to_curve_g2)
  const F2 xx = f_sqr(x), xxx = f_mul(xx, x);
  const F2 xn = f_add(f_add(f_add(f_mul(C2(LB_ISO_XNUM3), xxx), f_mul(C2(LB_ISO_XNUM2), xx)), f_mul(C2(LB_ISO_XNUM1), x)),
                      C2(LB_ISO_XNUM0));
  const F2 xd = f_add(f_add(xx, f_mul(C2(LB_ISO_XDEN1), x)), C2(LB_ISO_XDEN0));
  const F2 yn = f_add(f_add(f_add(f_mul(C2(LB_ISO_YNUM3), xxx), f_mul(C2(LB_ISO_YNUM2), xx)), f_mul(C2(LB_ISO_YNUM1), x)),
                      C2(LB_ISO_YNUM0));
  const F2 yd = f_add(f_add(f_add(xxx, f_mul(C2(LB_ISO_YDEN2), xx)), f_mul(C2(LB_ISO_YDEN1), x)), C2(LB_ISO_YDEN0));
  const F2 yd2 = f_sqr(yd);
  g2j r;
  r.z = fl_out(f_mul(xd, yd));
  r.x = fl_out(f_mul(f_mul(xn, xd), yd2));
  r.y = fl_out(f_mul(f_mul(f_mul(y, yn), f_mul(f_sqr(xd), xd)), yd2));
  return r;
}
template <class Pow>
LB_HD g2j map_to_curve_g2_fold(const fp2& u, Pow pow) {
  return map_to_curve_g2_fold_t<fp2, fp>(u, pow);
}

// hash_to_G2(msg32) in Jacobian coordinates (RFC 9380 §3 hash_to_curve)
LB_HD g2j hash_to_g2(const uint8_t msg[32]) {
  uint32_t ub[64];
  expand_message_xmd_256(ub, msg);
  fp2 u0{fp_from_be64_words(ub + 0), fp_from_be64_words(ub + 16)};
  fp2 u1{fp_from_be64_words(ub + 32), fp_from_be64_words(ub + 48)};
  g2j q0 = map_to_curve_g2(u0);
  g2j q1 = map_to_curve_g2(u1);
  return g2_clear_cofactor(jac_add(q0, q1));
}
