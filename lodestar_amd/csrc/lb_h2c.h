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
