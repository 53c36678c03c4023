// ZCash BLS12-381 point encodings (flags 0x80 compressed, 0x40 infinity, 0x20 sign).
// Replaces blst's P1/P2 (de)serialisation reached from
//   * bls.Signature.fromBytes(sig, CoordType.affine, validate=true)   maybeBatch.ts:23,36
//   * bls.PublicKey.fromBytes(pk, CoordType.affine)                   multithread/worker.ts:112
//   * PublicKey.toBytes(PointFormat.uncompressed)                     multithread/index.ts:160
// Error codes follow blst's BLST_ERROR (lb_common.h).
#pragma once
#include "lb_curve.h"

// 96-byte compressed G2, as 24 little-endian-loaded words (w[k] = bytes 4k..4k+3) -> affine point
// (no subgroup check).  inf = point at infinity.
LB_HD int g2_decompress96_w(const uint32_t* w, g2a& out, bool& inf) {
  inf = false;
  const uint32_t f = w[0] & 0xffu;
  if (!(f & 0x80)) return LB_BAD_ENCODING;
  if (f & 0x40) {
    uint32_t acc = w[0] & 0xffffff3fu;
    for (int i = 1; i < 24; i++) acc |= w[i];
    if (acc) return LB_BAD_ENCODING;
    inf = true;
    out.x = fp2_zero();
    out.y = fp2_zero();
    return LB_OK;
  }
  fp x1, x0;
  bool ok1 = fp_plain_from_be48_w(x1, w, 0x1f);
  bool ok0 = fp_plain_from_be48_w(x0, w + 12, 0xff);
  if (!ok0 || !ok1) return LB_BAD_ENCODING;
  fp2 x{fp_to_mont(x0), fp_to_mont(x1)};
  fp2 rhs = fp2_add(fp2_mul(fp2_sqr(x), x), fp2_load(LB_B2));
  fp2 y;
  if (!fp2_sqrt_i<true>(y, rhs)) return LB_POINT_NOT_ON_CURVE;
  bool want_large = (f & 0x20) != 0;
  if (fp2_lex_larger(y) != want_large) y = fp2_neg(y);
  out.x = x;
  out.y = y;
  return LB_OK;
}
// the same with the square root's exponentiations by pow (k_decompress_sigs_row: on a row)
template <class Pow>
LB_HD int g2_decompress96_wp(const uint32_t* w, g2a& out, bool& inf, Pow pow) {
  inf = false;
  const uint32_t f = w[0] & 0xffu;
  if (!(f & 0x80)) return LB_BAD_ENCODING;
  if (f & 0x40) {
    uint32_t acc = w[0] & 0xffffff3fu;
    for (int i = 1; i < 24; i++) acc |= w[i];
    if (acc) return LB_BAD_ENCODING;
    inf = true;
    out.x = fp2_zero();
    out.y = fp2_zero();
    return LB_OK;
  }
  fp x1, x0;
  const bool ok1 = fp_plain_from_be48_w(x1, w, 0x1f);
  const bool ok0 = fp_plain_from_be48_w(x0, w + 12, 0xff);
  if (!ok0 || !ok1) return LB_BAD_ENCODING;
  const fp2 x{fp_to_mont(x0), fp_to_mont(x1)};
  const fp2 rhs = fp2_add(fp2_mul(fp2_sqr(x), x), fp2_load(LB_B2));
  fp2 y;
  if (!fp2_sqrt_p(y, rhs, pow)) return LB_POINT_NOT_ON_CURVE;
  const bool want_large = (f & 0x20) != 0;
  if (fp2_lex_larger(y) != want_large) y = fp2_neg(y);
  out.x = x;
  out.y = y;
  return LB_OK;
}
LB_HD int g2_decompress96(const uint8_t* b, g2a& out, bool& inf) {
  uint32_t w[24];
  LB_UNROLL for (int k = 0; k < 24; k++)
    w[k] = (uint32_t)b[4 * k] | ((uint32_t)b[4 * k + 1] << 8) | ((uint32_t)b[4 * k + 2] << 16) | ((uint32_t)b[4 * k + 3] << 24);
  return g2_decompress96_w(w, out, inf);
}

// 192-byte uncompressed G2 (x.c1 || x.c0 || y.c1 || y.c0) -> affine point, curve-checked
LB_HD int g2_deserialize192(const uint8_t* b, g2a& out, bool& inf) {
  inf = false;
  uint8_t f = b[0];
  if (f & 0x80) return LB_BAD_ENCODING;
  if (f & 0x40) {
    uint32_t acc = f & 0x3f;
    for (int i = 1; i < 192; i++) acc |= b[i];
    if (acc) return LB_BAD_ENCODING;
    inf = true;
    out.x = fp2_zero();
    out.y = fp2_zero();
    return LB_OK;
  }
  if (f & 0x20) return LB_BAD_ENCODING;
  fp x1, x0, y1, y0;
  bool ok = fp_plain_from_be48(x1, b, 0x1f);
  ok &= fp_plain_from_be48(x0, b + 48, 0xff);
  ok &= fp_plain_from_be48(y1, b + 96, 0xff);
  ok &= fp_plain_from_be48(y0, b + 144, 0xff);
  if (!ok) return LB_BAD_ENCODING;
  out.x = fp2{fp_to_mont(x0), fp_to_mont(x1)};
  out.y = fp2{fp_to_mont(y0), fp_to_mont(y1)};
  if (!g2_aff_on_curve(out)) return LB_POINT_NOT_ON_CURVE;
  return LB_OK;
}

// 96-byte uncompressed G1 (x || y) -> affine, curve-checked (no subgroup check)
LB_HD int g1_deserialize96(const uint8_t* b, g1a& out, bool& inf) {
  inf = false;
  uint8_t f = b[0];
  if (f & 0x80) return LB_BAD_ENCODING;
  if (f & 0x40) {
    uint32_t acc = f & 0x3f;
    for (int i = 1; i < 96; i++) acc |= b[i];
    if (acc) return LB_BAD_ENCODING;
    inf = true;
    out.x = fp_zero();
    out.y = fp_zero();
    return LB_OK;
  }
  if (f & 0x20) return LB_BAD_ENCODING;
  fp x, y;
  bool ok = fp_plain_from_be48(x, b, 0x1f);
  ok &= fp_plain_from_be48(y, b + 48, 0xff);
  if (!ok) return LB_BAD_ENCODING;
  out.x = fp_to_mont(x);
  out.y = fp_to_mont(y);
  if (!g1_aff_on_curve(out)) return LB_POINT_NOT_ON_CURVE;
  return LB_OK;
}

// 48-byte compressed G1 -> affine (no subgroup check)
LB_HD int g1_decompress48(const uint8_t* b, g1a& out, bool& inf) {
  inf = false;
  uint8_t f = b[0];
  if (!(f & 0x80)) return LB_BAD_ENCODING;
  if (f & 0x40) {
    uint32_t acc = f & 0x3f;
    for (int i = 1; i < 48; i++) acc |= b[i];
    if (acc) return LB_BAD_ENCODING;
    inf = true;
    out.x = fp_zero();
    out.y = fp_zero();
    return LB_OK;
  }
  fp x;
  if (!fp_plain_from_be48(x, b, 0x1f)) return LB_BAD_ENCODING;
  fp xm = fp_to_mont(x);
  fp rhs = fp_add(fp_mul(fp_sqr(xm), xm), fp_load(LB_B1));
  fp y = fp_sqrt_cand(rhs);
  if (!fp_eq(fp_sqr(y), rhs)) return LB_POINT_NOT_ON_CURVE;
  if (fp_plain_gt_half(fp_from_mont(y)) != ((f & 0x20) != 0)) y = fp_neg(y);
  out.x = xm;
  out.y = y;
  return LB_OK;
}

LB_HD void g1_serialize96(uint8_t* b, const g1a& a, bool inf) {
  if (inf) {
    b[0] = 0x40;
    for (int i = 1; i < 96; i++) b[i] = 0;
    return;
  }
  fp_plain_to_be48(b, fp_from_mont(a.x));
  fp_plain_to_be48(b + 48, fp_from_mont(a.y));
}

LB_HD void g1_compress48(uint8_t* b, const g1a& a, bool inf) {
  if (inf) {
    b[0] = 0xc0;
    for (int i = 1; i < 48; i++) b[i] = 0;
    return;
  }
  fp_plain_to_be48(b, fp_from_mont(a.x));
  b[0] |= 0x80;
  if (fp_plain_gt_half(fp_from_mont(a.y))) b[0] |= 0x20;
}

LB_HD void g2_compress96(uint8_t* b, const g2a& a, bool inf) {
  if (inf) {
    b[0] = 0xc0;
    for (int i = 1; i < 96; i++) b[i] = 0;
    return;
  }
  fp_plain_to_be48(b, fp_from_mont(a.x.c1));
  fp_plain_to_be48(b + 48, fp_from_mont(a.x.c0));
  b[0] |= 0x80;
  if (fp2_lex_larger(a.y)) b[0] |= 0x20;
}

// Fp12 -> 576 bytes, big-endian coefficients in tower order (c0.c0.c0, c0.c0.c1, c0.c1.c0, ...)
LB_HD void fp12_to_be576(uint8_t* b, const fp12& a) {
  const fp2* parts[6] = {&a.c0.c0, &a.c0.c1, &a.c0.c2, &a.c1.c0, &a.c1.c1, &a.c1.c2};
  for (int i = 0; i < 6; i++) {
    fp_plain_to_be48(b + 96 * i, fp_from_mont(parts[i]->c0));
    fp_plain_to_be48(b + 96 * i + 48, fp_from_mont(parts[i]->c1));
  }
}

// 576 bytes (layout of fp12_to_be576) -> Fp12; false if a coefficient is >= p
LB_HD bool fp12_from_be576(fp12& a, const uint8_t* b) {
  fp2* parts[6] = {&a.c0.c0, &a.c0.c1, &a.c0.c2, &a.c1.c0, &a.c1.c1, &a.c1.c2};
  bool ok = true;
  for (int i = 0; i < 6; i++) {
    fp x0, x1;
    ok &= fp_plain_from_be48(x0, b + 96 * i, 0xff);
    ok &= fp_plain_from_be48(x1, b + 96 * i + 48, 0xff);
    parts[i]->c0 = fp_to_mont(x0);
    parts[i]->c1 = fp_to_mont(x1);
  }
  return ok;
}
