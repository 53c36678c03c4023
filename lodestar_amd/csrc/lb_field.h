// BLS12-381 field tower for gfx950: Fp (12 x u32 Montgomery limbs), Fp2 = Fp[u]/(u^2+1),
// Fp6 = Fp2[v]/(v^3 - (1+u)), Fp12 = Fp6[w]/(w^2 - v).
//
// Replaces the blst field layer that @chainsafe/blst@0.2.7 runs under
// packages/beacon-node/src/chain/bls/maybeBatch.ts:18-37.
// Every element is kept fully reduced in [0, p) in Montgomery form (R = 2^384), so
// equality is limb equality and serialisation is one Montgomery multiply away.
// The 32x32->64 multiply-accumulate chains lower to v_mad_u64_u32 on gfx950.
#pragma once
#include "lb_common.h"
#include "lb_consts.h"
#include "lb_fpmul_gfx950.h"

struct fp {
  uint32_t v[12];
};
struct fp2 {
  fp c0, c1;
};
struct fp6 {
  fp2 c0, c1, c2;
};
struct fp12 {
  fp6 c0, c1;
};

// ------------------------------------------------------------------ Fp basics
LB_HD fp fp_load(const uint32_t* c) {
  fp r;
  LB_UNROLL for (int i = 0; i < 12; i++) r.v[i] = c[i];
  return r;
}
LB_HD fp2 fp2_load(const uint32_t* c) {
  fp2 r;
  r.c0 = fp_load(c);
  r.c1 = fp_load(c + 12);
  return r;
}
LB_HD fp fp_zero() {
  fp r;
  LB_UNROLL for (int i = 0; i < 12; i++) r.v[i] = 0;
  return r;
}
LB_HD fp fp_one() { return fp_load(LB_ONE); }

LB_HD bool fp_is_zero(const fp& a) {
  uint32_t t = 0;
  LB_UNROLL for (int i = 0; i < 12; i++) t |= a.v[i];
  return t == 0;
}
LB_HD bool fp_eq(const fp& a, const fp& b) {
  uint32_t t = 0;
  LB_UNROLL for (int i = 0; i < 12; i++) t |= a.v[i] ^ b.v[i];
  return t == 0;
}
LB_HD fp fp_select(bool c, const fp& a, const fp& b) {
  fp r;
  LB_UNROLL for (int i = 0; i < 12; i++) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

// r = a - p if a >= p (a given as 12 limbs + carry word)
LB_HD fp fp_reduce_once(const uint32_t* t, uint32_t top) {
  const uint32_t Pl[12] = {LB_P0, LB_P1, LB_P2, LB_P3, LB_P4, LB_P5, LB_P6, LB_P7, LB_P8, LB_P9, LB_P10, LB_P11};
  uint32_t s[12];
  uint32_t br = 0;
  LB_UNROLL for (int j = 0; j < 12; j++) s[j] = LB_SUBC(t[j], Pl[j], br, &br);
  bool ge = (top != 0) || (br == 0);
  fp r;
  LB_UNROLL for (int j = 0; j < 12; j++) r.v[j] = ge ? s[j] : t[j];
  return r;
}

LB_HD fp fp_add(const fp& a, const fp& b) {
  uint32_t t[12];
  uint32_t c = 0;
  LB_UNROLL for (int j = 0; j < 12; j++) t[j] = LB_ADDC(a.v[j], b.v[j], c, &c);
  return fp_reduce_once(t, c);
}

LB_HD fp fp_sub(const fp& a, const fp& b) {
  const uint32_t Pl[12] = {LB_P0, LB_P1, LB_P2, LB_P3, LB_P4, LB_P5, LB_P6, LB_P7, LB_P8, LB_P9, LB_P10, LB_P11};
  uint32_t t[12];
  uint32_t br = 0;
  LB_UNROLL for (int j = 0; j < 12; j++) t[j] = LB_SUBC(a.v[j], b.v[j], br, &br);
  // if borrow, add p back
  uint32_t m = 0u - br;
  fp r;
  uint32_t c = 0;
  LB_UNROLL for (int j = 0; j < 12; j++) r.v[j] = LB_ADDC(t[j], Pl[j] & m, c, &c);
  return r;
}

LB_HD fp fp_neg(const fp& a) { return fp_sub(fp_zero(), a); }
LB_HD fp fp_dbl(const fp& a) { return fp_add(a, a); }

// Montgomery multiplication a*b/R mod p, 12 x 32-bit limbs, operand scanning in carry-save
// form.  Textbook CIOS threads one carry through all 288 multiply-adds, so a lone wave waits
// on a 288-deep v_mad_u64_u32 dependency chain.  Here every row keeps the carry out of limb j
// *pending* for limb j+1 of the next row: u = a_i*b_j + t_j + cc_j <= (2^32-1)^2 + 2(2^32-1)
// < 2^64, so each row's 12 products are independent and the chain is ~7 deep per row.
// After the multiply row nothing is pending into limb 0, so m = t_0 * (-p^-1) mod 2^32 is
// exact; the reduction row zeroes limb 0 and the state shifts down one limb.
LB_HD fp fp_mul_body(const fp& a, const fp& b) {
  const uint32_t Pl[12] = {LB_P0, LB_P1, LB_P2, LB_P3, LB_P4, LB_P5, LB_P6, LB_P7, LB_P8, LB_P9, LB_P10, LB_P11};
  uint32_t t[13], cc[14];
  LB_UNROLL for (int j = 0; j < 13; j++) t[j] = 0;
  LB_UNROLL for (int j = 0; j < 14; j++) cc[j] = 0;
  LB_UNROLL for (int i = 0; i < 12; i++) {
    uint32_t n[14];
    n[0] = 0;
    LB_UNROLL for (int j = 0; j < 12; j++) {
      uint64_t u = (uint64_t)a.v[i] * b.v[j] + t[j] + cc[j];
      t[j] = (uint32_t)u;
      n[j + 1] = (uint32_t)(u >> 32);
    }
    {
      uint64_t u = (uint64_t)t[12] + cc[12];
      t[12] = (uint32_t)u;
      n[13] = (uint32_t)(u >> 32) + cc[13];
    }
    // reduction row: limb 0 has no pending carry now
    uint32_t m = t[0] * LB_PINV;
    uint32_t r[14];
    r[0] = 0;
    LB_UNROLL for (int j = 0; j < 12; j++) {
      uint64_t u = (uint64_t)m * Pl[j] + t[j] + n[j];
      t[j] = (uint32_t)u;
      r[j + 1] = (uint32_t)(u >> 32);
    }
    {
      uint64_t u = (uint64_t)t[12] + n[12];
      t[12] = (uint32_t)u;
      r[13] = (uint32_t)(u >> 32) + n[13];
    }
    // divide by 2^32: limb 0 is zero; pending carries shift with the limbs
    LB_UNROLL for (int j = 0; j < 12; j++) t[j] = t[j + 1];
    t[12] = 0;
    LB_UNROLL for (int j = 0; j < 13; j++) cc[j] = r[j + 1];
    cc[13] = 0;
  }
  // resolve the pending carries (value < 2p < 2^382, so nothing escapes limb 12)
  uint32_t o[12];
  uint32_t c = 0;
  LB_UNROLL for (int j = 0; j < 12; j++) o[j] = LB_ADDC(t[j], cc[j], c, &c);
  uint32_t top = t[12] + cc[12] + c;
  return fp_reduce_once(o, top);
}

// Montgomery multiplication on 14 x 28-bit unsaturated limbs (same R = 2^384 contract as
// fp_mul_body).  With 28-bit limbs every partial product is < 2^56 and a column collects at most
// 28 of them plus a 2^36 carry, so a 64-bit column accumulator never overflows: each of the 392
// products is ONE carry-free v_mad_u64_u32 (acc = a*b + acc), against 288 MADs + 288 carry adds
// for 32-bit limbs, and the rows carry nothing but one shift per row.
// R stays 2^384 although 14 rows divide by 2^392: the second operand is unpacked as b * 2^8
// (b * 2^8 < 2^392 fits), so the result is a b 2^8 / 2^392 = a b / R.  For a b < R p the output is
// below 2p (as for fp_mul_body), and one conditional subtraction finishes it.
LB_HD uint32_t lb_bits28(const uint32_t* w, int off) {  // bits [off, off + 28) of a 12-word value
  const int q = off >> 5, r = off & 31;
  const uint32_t lo = q < 12 ? w[q] : 0u;
  const uint32_t hi = q + 1 < 12 ? w[q + 1] : 0u;
  return (r ? ((lo >> r) | (hi << (32 - r))) : lo) & 0x0fffffffu;
}
LB_HD fp fp_mul28(const fp& a, const fp& b) {
  const uint32_t P28[14] = {LB_P28_0, LB_P28_1, LB_P28_2, LB_P28_3, LB_P28_4,  LB_P28_5,  LB_P28_6,
                            LB_P28_7, LB_P28_8, LB_P28_9, LB_P28_10, LB_P28_11, LB_P28_12, LB_P28_13};
  uint32_t A[14], B[14];
  LB_UNROLL for (int k = 0; k < 14; k++) A[k] = lb_bits28(a.v, 28 * k);
  B[0] = (b.v[0] << 8) & 0x0fffffffu;
  LB_UNROLL for (int k = 1; k < 14; k++) B[k] = lb_bits28(b.v, 28 * k - 8);
  uint64_t acc[28];
  LB_UNROLL for (int k = 0; k < 28; k++) acc[k] = 0;
  LB_UNROLL for (int i = 0; i < 14; i++) {
    LB_UNROLL for (int j = 0; j < 14; j++) acc[i + j] += (uint64_t)A[i] * B[j];
    const uint32_t m = ((uint32_t)acc[i] * LB_PINV28) & 0x0fffffffu;
    LB_UNROLL for (int j = 0; j < 14; j++) acc[i + j] += (uint64_t)m * P28[j];
    acc[i + 1] += acc[i] >> 28;  // column i is now a multiple of 2^28
  }
  uint32_t r[14];
  LB_UNROLL for (int k = 0; k < 13; k++) {
    r[k] = (uint32_t)acc[14 + k] & 0x0fffffffu;
    acc[15 + k] += acc[14 + k] >> 28;
  }
  r[13] = (uint32_t)acc[27];  // < 2^18: the value is below 2p < 2^382
  uint32_t o[12];
  LB_UNROLL for (int w = 0; w < 12; w++) {
    const int l = (32 * w) / 28, s = 32 * w - 28 * l;  // s <= 24: two limbs cover a word
    o[w] = (r[l] >> s) | (r[l + 1] << (28 - s));
  }
  return fp_reduce_once(o, 0u);
}

// Montgomery squaring on the same 14 x 28-bit limbs: 105 products instead of 196 for a * a.
// The operand is unpacked once as a' = a * 2^4, so a'^2 = a^2 2^8 and the 2^392 reduction again
// yields a^2 / R.  Off-diagonal products use 2 a'_i (29 bits): a column holds at most 7 of them
// (< 2^57 each), one square, 14 reduction products (< 2^56) and a 2^36 carry: < 2^61.
LB_HD fp fp_sqr28(const fp& a) {
  const uint32_t P28[14] = {LB_P28_0, LB_P28_1, LB_P28_2, LB_P28_3, LB_P28_4,  LB_P28_5,  LB_P28_6,
                            LB_P28_7, LB_P28_8, LB_P28_9, LB_P28_10, LB_P28_11, LB_P28_12, LB_P28_13};
  uint32_t A[14], D[14];
  A[0] = (a.v[0] << 4) & 0x0fffffffu;
  LB_UNROLL for (int k = 1; k < 14; k++) A[k] = lb_bits28(a.v, 28 * k - 4);
  LB_UNROLL for (int k = 0; k < 14; k++) D[k] = A[k] << 1;
  uint64_t acc[28];
  LB_UNROLL for (int k = 0; k < 28; k++) acc[k] = 0;
  LB_UNROLL for (int i = 0; i < 14; i++) {
    acc[2 * i] += (uint64_t)A[i] * A[i];
    LB_UNROLL for (int j = i + 1; j < 14; j++) acc[i + j] += (uint64_t)D[i] * A[j];
  }
  LB_UNROLL for (int i = 0; i < 14; i++) {
    const uint32_t m = ((uint32_t)acc[i] * LB_PINV28) & 0x0fffffffu;
    LB_UNROLL for (int j = 0; j < 14; j++) acc[i + j] += (uint64_t)m * P28[j];
    acc[i + 1] += acc[i] >> 28;
  }
  uint32_t r[14];
  LB_UNROLL for (int k = 0; k < 13; k++) {
    r[k] = (uint32_t)acc[14 + k] & 0x0fffffffu;
    acc[15 + k] += acc[14 + k] >> 28;
  }
  r[13] = (uint32_t)acc[27];
  uint32_t o[12];
  LB_UNROLL for (int w = 0; w < 12; w++) {
    const int l = (32 * w) / 28, s = 32 * w - 28 * l;
    o[w] = (r[l] >> s) | (r[l + 1] << (28 - s));
  }
  return fp_reduce_once(o, 0u);
}

#if defined(__HIPCC__)
// Out of line on the GPU: one body shared by every call site keeps the pipeline kernels inside
// the instruction cache and compile time bounded.  Operands and result travel as 16-wide
// vectors, which the AMDGPU calling convention keeps in VGPRs (a 48-byte struct would be
// passed through scratch memory).
typedef uint32_t lb_v16u __attribute__((ext_vector_type(16)));
__device__ __forceinline__ lb_v16u fp_pack(const fp& a) {
  lb_v16u r;
  LB_UNROLL for (int i = 0; i < 12; i++) r[i] = a.v[i];
  r[12] = r[13] = r[14] = r[15] = 0;
  return r;
}
__device__ __forceinline__ fp fp_unpack(lb_v16u a) {
  fp r;
  LB_UNROLL for (int i = 0; i < 12; i++) r.v[i] = a[i];
  return r;
}
static __device__ __attribute__((noinline)) lb_v16u fp_mul_v(lb_v16u a, lb_v16u b) {
#if defined(__HIP_DEVICE_COMPILE__)
#if defined(LB_FPMUL_ASM32)
  // 32-bit limbs, hand-scheduled MAD + carry chains (lb_fpmul_gfx950.h)
  fp x = fp_unpack(a), y = fp_unpack(b);
  uint32_t o[12], top;
  lbm_mont_mul(o, &top, x.v, y.v);
  return fp_pack(fp_reduce_once(o, top));
#else
  return fp_pack(fp_mul28(fp_unpack(a), fp_unpack(b)));
#endif
#else
  return fp_pack(fp_mul_body(fp_unpack(a), fp_unpack(b)));
#endif
}
__host__ __device__ __forceinline__ fp fp_mul(const fp& a, const fp& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return fp_unpack(fp_mul_v(fp_pack(a), fp_pack(b)));
#else
  return fp_mul_body(a, b);
#endif
}
static __device__ __attribute__((noinline)) lb_v16u fp_sqr_v(lb_v16u a) {
#if defined(__HIP_DEVICE_COMPILE__)
  return fp_pack(fp_sqr28(fp_unpack(a)));
#else
  return fp_pack(fp_mul_body(fp_unpack(a), fp_unpack(a)));
#endif
}
__host__ __device__ __forceinline__ fp fp_sqr(const fp& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  return fp_unpack(fp_sqr_v(fp_pack(a)));
#else
  return fp_mul_body(a, a);
#endif
}
#else
static inline fp fp_mul(const fp& a, const fp& b) {
  LB_COUNT_MUL();
  return fp_mul28(a, b);
}
// counted as one Fp multiplication (the roofline's unit stays the 300-MAC product)
static inline fp fp_sqr(const fp& a) {
  LB_COUNT_MUL();
  return fp_sqr28(a);
}
#endif

// small-constant multiples via additions
LB_HD fp fp_mul3(const fp& a) { return fp_add(fp_dbl(a), a); }
LB_HD fp fp_mul4(const fp& a) { return fp_dbl(fp_dbl(a)); }
LB_HD fp fp_mul8(const fp& a) { return fp_dbl(fp_mul4(a)); }

LB_HD fp fp_to_mont(const fp& a) { return fp_mul(a, fp_load(LB_R2)); }
LB_HD fp fp_from_mont(const fp& a) {
  fp one = fp_zero();
  one.v[0] = 1;
  return fp_mul(a, one);
}

// a^e for a constant exponent held in (constant) memory, bit top_bit set, by a sliding window
// of 4 bits over the odd powers a, a^3, ..., a^15: for the 379-bit sqrt exponents 378
// squarings + 86 multiplications instead of 378 + 228.  Exponent bits, window values and table
// indices are wave-uniform (scalar control flow on the GPU); the table is read through a switch
// so it stays in registers.
LB_HD fp lb_tab8(const fp* t, uint32_t k) {
  switch (k) {
    case 0: return t[0];
    case 1: return t[1];
    case 2: return t[2];
    case 3: return t[3];
    case 4: return t[4];
    case 5: return t[5];
    case 6: return t[6];
    default: return t[7];
  }
}
// Inline products for the exponentiation chains (fenced so the compiler keeps one product's
// columns live at a time): a lone lane's out-of-line product costs ~1.42 us of latency against
// ~1.05 us inline, and ~7 % more issue (tools/ubench/fpmul_ps.hip, profiles/r3_variants_ab.txt).
LB_HD fp fp_mul_inl(const fp& a, const fp& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_sched_barrier(0);
  const fp r = fp_mul28(a, b);
  __builtin_amdgcn_sched_barrier(0);
  return r;
#else
  return fp_mul(a, b);
#endif
}
LB_HD fp fp_sqr_inl(const fp& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_sched_barrier(0);
  const fp r = fp_sqr28(a);
  __builtin_amdgcn_sched_barrier(0);
  return r;
#else
  return fp_sqr(a);
#endif
}
// Limb-resident exponentiation chains.  fp_mul28 / fp_sqr28 spend ~110 of their 632 / 506 VALU
// instructions unpacking 12 x 32-bit operands into 28-bit limbs, repacking the result and
// reducing it below p.  A chain of products can stay in limbs: with Montgomery radix R' = 2^392
// (the 14 rows' own radix) the limbs of a * 2^8 ARE the R'-form of a's value (x R 2^8 = x R'),
// and a product's 14 output limbs feed the next product directly.  Values are not reduced between
// products: for inputs below 2^390 the output (ab + mp) / R' is below 2^388 + p, so every limb stays
// below 2^28 and the column bounds of fp_mul28 / fp_sqr28 hold.  The end converts back with one
// product by R mod p (r R / R' = r / 2^8 = x^e R), repacks and reduces once.
#ifndef LB_POW28
#define LB_POW28 1  // 0: the chains through fp_mul28 / fp_sqr28 (A/B builds)
#endif
struct fp28 {
  uint32_t l[14];
};
LB_HD fp28 fp28_mul_raw(const fp28& a, const fp28& b) {
  const uint32_t P28[14] = {LB_P28_0, LB_P28_1, LB_P28_2, LB_P28_3, LB_P28_4,  LB_P28_5,  LB_P28_6,
                            LB_P28_7, LB_P28_8, LB_P28_9, LB_P28_10, LB_P28_11, LB_P28_12, LB_P28_13};
  uint64_t acc[28];
  LB_UNROLL for (int k = 0; k < 28; k++) acc[k] = 0;
  LB_UNROLL for (int i = 0; i < 14; i++) {
    LB_UNROLL for (int j = 0; j < 14; j++) acc[i + j] += (uint64_t)a.l[i] * b.l[j];
    const uint32_t m = ((uint32_t)acc[i] * LB_PINV28) & 0x0fffffffu;
    LB_UNROLL for (int j = 0; j < 14; j++) acc[i + j] += (uint64_t)m * P28[j];
    acc[i + 1] += acc[i] >> 28;
  }
  fp28 r;
  LB_UNROLL for (int k = 0; k < 13; k++) {
    r.l[k] = (uint32_t)acc[14 + k] & 0x0fffffffu;
    acc[15 + k] += acc[14 + k] >> 28;
  }
  r.l[13] = (uint32_t)acc[27];
  return r;
}
LB_HD fp28 fp28_sqr_raw(const fp28& a) {
  const uint32_t P28[14] = {LB_P28_0, LB_P28_1, LB_P28_2, LB_P28_3, LB_P28_4,  LB_P28_5,  LB_P28_6,
                            LB_P28_7, LB_P28_8, LB_P28_9, LB_P28_10, LB_P28_11, LB_P28_12, LB_P28_13};
  uint32_t D[14];
  LB_UNROLL for (int k = 0; k < 14; k++) D[k] = a.l[k] << 1;
  uint64_t acc[28];
  LB_UNROLL for (int k = 0; k < 28; k++) acc[k] = 0;
  LB_UNROLL for (int i = 0; i < 14; i++) {
    acc[2 * i] += (uint64_t)a.l[i] * a.l[i];
    LB_UNROLL for (int j = i + 1; j < 14; j++) acc[i + j] += (uint64_t)D[i] * a.l[j];
  }
  LB_UNROLL for (int i = 0; i < 14; i++) {
    const uint32_t m = ((uint32_t)acc[i] * LB_PINV28) & 0x0fffffffu;
    LB_UNROLL for (int j = 0; j < 14; j++) acc[i + j] += (uint64_t)m * P28[j];
    acc[i + 1] += acc[i] >> 28;
  }
  fp28 r;
  LB_UNROLL for (int k = 0; k < 13; k++) {
    r.l[k] = (uint32_t)acc[14 + k] & 0x0fffffffu;
    acc[15 + k] += acc[14 + k] >> 28;
  }
  r.l[13] = (uint32_t)acc[27];
  return r;
}
LB_HD fp28 fp28_mul(const fp28& a, const fp28& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_sched_barrier(0);
  const fp28 r = fp28_mul_raw(a, b);
  __builtin_amdgcn_sched_barrier(0);
  return r;
#else
  return fp28_mul_raw(a, b);
#endif
}
LB_HD fp28 fp28_sqr(const fp28& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_sched_barrier(0);
  const fp28 r = fp28_sqr_raw(a);
  __builtin_amdgcn_sched_barrier(0);
  return r;
#else
  return fp28_sqr_raw(a);
#endif
}
LB_HD fp28 lb_tab8_28(const fp28* t, uint32_t k) {
  switch (k) {
    case 0: return t[0];
    case 1: return t[1];
    case 2: return t[2];
    case 3: return t[3];
    case 4: return t[4];
    case 5: return t[5];
    case 6: return t[6];
    default: return t[7];
  }
}
#ifndef LB_POW28_WIN
#define LB_POW28_WIN 4  // sliding-window width of the 28-bit-limb chains.  4: the 8 odd powers on the
                        // stack (448 B per lane, ~170 VGPRs: three waves per SIMD in the signature
                        // decode); 3: the 4 powers in registers, no stack, 222 VGPRs (two waves) and
                        // ~10 % more decode instructions: 1.5 % lower throughput at 7 in flight
                        // (profiles/r4_regress_ab.txt), for 268 -> 53 MB of decode traffic per batch
#endif
template <int NT>
LB_HD fp28 lb_tab_sel28(const fp28* t, uint32_t k) {  // t[k] by selects (k is wave-uniform)
  fp28 r = t[0];
  LB_UNROLL for (int c = 1; c < NT; c++) {
    const bool s = k == (uint32_t)c;
    LB_UNROLL for (int w = 0; w < 14; w++) r.l[w] = s ? t[c].l[w] : r.l[w];
  }
  return r;
}
LB_HD fp fp_pow_const_28(const fp& a, const uint32_t* e, int top_bit) {
  constexpr int WIN = LB_POW28_WIN, NT = 1 << (WIN - 1);
  fp28 tab[NT];
  tab[0].l[0] = (a.v[0] << 8) & 0x0fffffffu;  // the limbs of a * 2^8: a's value in R'-form
  LB_UNROLL for (int k = 1; k < 14; k++) tab[0].l[k] = lb_bits28(a.v, 28 * k - 8);
  const fp28 a2 = fp28_sqr(tab[0]);
  // odd powers one statement each: a loop here stays rolled (its body is too large for the
  // unroller's budget) and then indexes the table dynamically, i.e. on the stack
  if constexpr (NT == 8) {
    // through a loop the unroller leaves rolled: the table indexed dynamically, on the stack
    // (448 B per lane, cache-resident), at ~170 VGPRs
    for (int k = 1; k < 8; k++) tab[k] = fp28_mul(tab[k - 1], a2);
  } else {
    tab[1] = fp28_mul(tab[0], a2);
    if constexpr (NT >= 4) {
      tab[2] = fp28_mul(tab[1], a2);
      tab[3] = fp28_mul(tab[2], a2);
    }
  }
  static_assert(NT == 2 || NT == 4 || NT == 8, "window of 2, 3 or 4 bits");
  auto bit = [&](int i) -> uint32_t { return (e[i >> 5] >> (i & 31)) & 1u; };
  fp28 r = tab[0];
  bool first = true;
  int i = top_bit;
  while (i >= 0) {
    if (!bit(i)) {
      if (!first) r = fp28_sqr(r);
      i--;
      continue;
    }
    int j = i - (WIN - 1) > 0 ? i - (WIN - 1) : 0;
    while (!bit(j)) j++;
    uint32_t val = 0;
    for (int k = i; k >= j; k--) val = (val << 1) | bit(k);
    if (first) {
      r = NT == 8 ? lb_tab8_28(tab, val >> 1) : lb_tab_sel28<NT>(tab, val >> 1);
      first = false;
    } else {
      for (int k = i; k >= j; k--) r = fp28_sqr(r);
      r = fp28_mul(r, NT == 8 ? lb_tab8_28(tab, val >> 1) : lb_tab_sel28<NT>(tab, val >> 1));
    }
    i = j - 1;
  }
  // back to R-form: r * (R mod p) / R' = r / 2^8, below 2p; repack and reduce once
  const fp one = fp_one();
  fp28 c;
  LB_UNROLL for (int k = 0; k < 14; k++) c.l[k] = lb_bits28(one.v, 28 * k);
  const fp28 t = fp28_mul(r, c);
  uint32_t o[12];
  LB_UNROLL for (int w = 0; w < 12; w++) {
    const int l = (32 * w) / 28, s = 32 * w - 28 * l;
    o[w] = (t.l[l] >> s) | (t.l[l + 1] << (28 - s));
  }
  return fp_reduce_once(o, 0u);
}

template <bool kInlMul = false>
LB_HD fp fp_pow_const_i(fp a, const uint32_t* e, int top_bit) {
  if constexpr (kInlMul && LB_POW28) return fp_pow_const_28(a, e, top_bit);
  auto mul = [](const fp& x, const fp& y) { return kInlMul ? fp_mul_inl(x, y) : fp_mul(x, y); };
  auto sqr = [](const fp& x) { return kInlMul ? fp_sqr_inl(x) : fp_sqr(x); };
  fp tab[8];
  tab[0] = a;
  const fp a2 = sqr(a);
  LB_UNROLL for (int k = 1; k < 8; k++) tab[k] = mul(tab[k - 1], a2);
  auto bit = [&](int i) -> uint32_t { return (e[i >> 5] >> (i & 31)) & 1u; };
  fp r = fp_zero();
  bool first = true;
  int i = top_bit;
  while (i >= 0) {
    if (!bit(i)) {
      r = sqr(r);
      i--;
      continue;
    }
    int j = i - 3 > 0 ? i - 3 : 0;
    while (!bit(j)) j++;
    uint32_t val = 0;
    for (int k = i; k >= j; k--) val = (val << 1) | bit(k);
    if (first) {
      r = lb_tab8(tab, val >> 1);
      first = false;
    } else {
      for (int k = i; k >= j; k--) r = sqr(r);
      r = mul(r, lb_tab8(tab, val >> 1));
    }
    i = j - 1;
  }
  return r;
}

// ---- variable-time inversion (binary extended Euclid).  Every value this engine inverts is
// derived from public data (signatures, pubkeys, messages), so timing does not leak secrets;
// this replaces a 570-multiplication Fermat chain by ~400 cheap shift/subtract steps.
LB_HD bool lb_is_one_plain(const uint32_t* x) {
  uint32_t t = x[0] ^ 1u;
  LB_UNROLL for (int i = 1; i < 12; i++) t |= x[i];
  return t == 0;
}
LB_HD int lb_ctz32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_ctz(x);
#else
  return __builtin_ctz(x);
#endif
}
// x <- x / 2^k mod p for 1 <= k <= 31 (Montgomery-style: add m*p so the low k bits vanish)
LB_HD void lb_div2k_mod(uint32_t* x, int k) {
  const uint32_t Pl[12] = {LB_P0, LB_P1, LB_P2, LB_P3, LB_P4, LB_P5, LB_P6, LB_P7, LB_P8, LB_P9, LB_P10, LB_P11};
  uint32_t m = (x[0] * LB_PINV) & ((1u << k) - 1u);
  uint32_t t[13];
  uint64_t c = 0;
  LB_UNROLL for (int j = 0; j < 12; j++) {
    c = (uint64_t)m * Pl[j] + x[j] + (c >> 32);
    t[j] = (uint32_t)c;
  }
  t[12] = (uint32_t)(c >> 32);
  // (x + m p) < 2^k p, divisible by 2^k, result < p
  LB_UNROLL for (int j = 0; j < 12; j++) x[j] = (t[j] >> k) | (t[j + 1] << (32 - k));
}
// u <- u / 2^k (plain shift), 1 <= k <= 31
LB_HD void lb_shr(uint32_t* u, int k) {
  LB_UNROLL for (int j = 0; j < 11; j++) u[j] = (u[j] >> k) | (u[j + 1] << (32 - k));
  u[11] >>= k;
}
LB_HD bool lb_geq(const uint32_t* a, const uint32_t* b) {
  uint32_t br = 0;
  LB_UNROLL for (int j = 0; j < 12; j++) (void)LB_SUBC(a[j], b[j], br, &br);
  return br == 0;
}
LB_HD void lb_sub_in(uint32_t* a, const uint32_t* b) {
  uint32_t br = 0;
  LB_UNROLL for (int j = 0; j < 12; j++) a[j] = LB_SUBC(a[j], b[j], br, &br);
}
// plain a in [0, p) -> a^-1 mod p (plain), 0 -> 0.  fp_inv_plain_vt_i is the inline body (a
// kernel whose call graph is all inline keeps its own register budget), fp_inv_plain_vt the
// out-of-line entry.
LB_HD fp fp_inv_plain_vt_i(fp a) {
  if (fp_is_zero(a)) return a;
  uint32_t u[12], v[12];
  fp x1 = fp_zero(), x2 = fp_zero();
  x1.v[0] = 1;
  const uint32_t Pl[12] = {LB_P0, LB_P1, LB_P2, LB_P3, LB_P4, LB_P5, LB_P6, LB_P7, LB_P8, LB_P9, LB_P10, LB_P11};
  LB_UNROLL for (int j = 0; j < 12; j++) {
    u[j] = a.v[j];
    v[j] = Pl[j];
  }
  // invariant: x1 * a == u, x2 * a == v (mod p); u, v > 0, v odd at loop head
  while (true) {
    while (u[0] == 0) {  // rare: shift whole words
      LB_UNROLL for (int j = 0; j < 11; j++) u[j] = u[j + 1];
      u[11] = 0;
      lb_div2k_mod(x1.v, 16);
      lb_div2k_mod(x1.v, 16);
    }
    int k = lb_ctz32(u[0]);
    if (k) {
      lb_shr(u, k);
      lb_div2k_mod(x1.v, k);
    }
    if (lb_is_one_plain(u)) return x1;
    if (lb_geq(u, v)) {
      lb_sub_in(u, v);
      x1 = fp_sub(x1, x2);
    } else {
      lb_sub_in(v, u);
      x2 = fp_sub(x2, x1);
      // v - u is even (both odd): normalise v here
      while (v[0] == 0) {
        LB_UNROLL for (int j = 0; j < 11; j++) v[j] = v[j + 1];
        v[11] = 0;
        lb_div2k_mod(x2.v, 16);
        lb_div2k_mod(x2.v, 16);
      }
      int kv = lb_ctz32(v[0]);
      if (kv) {
        lb_shr(v, kv);
        lb_div2k_mod(x2.v, kv);
      }
      if (lb_is_one_plain(v)) return x2;
    }
  }
}
// ---- Bernstein-Yang "safegcd" inversion, variable time (jumps of 62 divsteps on the low 64 bits,
// then 2x2 transition matrices applied to the full-width values; the divstep loop and the
// update steps follow the structure of libsecp256k1's modinv64_var, written here for a 381-bit
// modulus in 7 signed 62-bit limbs).  ~12 jumps for a random input against the binary extended
// Euclid's ~760 word-array iterations: an inversion on a lone lane 184 us -> ~25 us
// (tools/ubench/row_bench.hip), on the critical path of every small batch (the final
// exponentiation's norm, each block's batched inversion in k_hash_finish / k_gsum_final /
// k_pk_blind, ML(-G1, S)'s affine S).  Public inputs only, so variable time is fine.
struct lb_s62 {
  int64_t v[7];
};
#define LB_S62_M 0x3fffffffffffffffLL
LB_HD lb_s62 lb_s62_p() {
  return lb_s62{{0x39feffffffffaaabLL, 0x3aaffffac54ffffeLL, 0x330d2a0f6b0f6241LL, 0x1dd2e13ce144afd9LL,
                 0x1ba7b6434bacd764LL, 0x0447a8e5ff9a692cLL, 0x1a0LL}};
}
#define LB_S62_PINV 0x360c000300030003ULL  // p^-1 mod 2^62
LB_HD int lb_ctz64(uint64_t x) { return __builtin_ctzll(x); }
// 62 divsteps on the low bits of f, g (f odd); returns the new eta, the matrix in t[4] = u, v, q, r
LB_HD int64_t lb_divsteps62(int64_t eta, uint64_t f0, uint64_t g0, int64_t t[4]) {
  uint64_t u = 1, v = 0, q = 0, r = 1, f = f0, g = g0, m, w;
  int i = 62;
  for (;;) {
    const int zeros = lb_ctz64(g | (~0ULL << i));  // sentinel at bit i
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    int limit;
    if (eta < 0) {  // swap with negation: (f, g) <- (g, -f)
      uint64_t tmp;
      eta = -eta;
      tmp = f; f = g; g = (uint64_t)0 - tmp;
      tmp = u; u = q; q = (uint64_t)0 - tmp;
      tmp = v; v = r; r = (uint64_t)0 - tmp;
      limit = (int)eta + 1 > i ? i : (int)eta + 1;
      m = (~0ULL >> (64 - limit)) & 63u;
      w = (f * g * (f * f - 2)) & m;  // cancels up to 6 low bits of g
    } else {
      limit = (int)eta + 1 > i ? i : (int)eta + 1;
      m = (~0ULL >> (64 - limit)) & 15u;
      w = f + (((f + 1) & 4) << 1);
      w = ((uint64_t)0 - w * g) & m;  // up to 4 bits
    }
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t[0] = (int64_t)u;
  t[1] = (int64_t)v;
  t[2] = (int64_t)q;
  t[3] = (int64_t)r;
  return eta;
}
// (f, g) <- (u f + v g, q f + r g) / 2^62 (exact)
LB_HD void lb_s62_update_fg(lb_s62& f, lb_s62& g, const int64_t t[4]) {
  const int64_t u = t[0], v = t[1], q = t[2], r = t[3];
  __int128 cf = (__int128)u * f.v[0] + (__int128)v * g.v[0];
  __int128 cg = (__int128)q * f.v[0] + (__int128)r * g.v[0];
  cf >>= 62;
  cg >>= 62;
  LB_UNROLL for (int i = 1; i < 7; i++) {
    cf += (__int128)u * f.v[i] + (__int128)v * g.v[i];
    cg += (__int128)q * f.v[i] + (__int128)r * g.v[i];
    f.v[i - 1] = (int64_t)cf & LB_S62_M;
    cf >>= 62;
    g.v[i - 1] = (int64_t)cg & LB_S62_M;
    cg >>= 62;
  }
  f.v[6] = (int64_t)cf;
  g.v[6] = (int64_t)cg;
}
// (d, e) <- (u d + v e, q d + r e) / 2^62 mod p, kept in (-2p, p)
LB_HD void lb_s62_update_de(lb_s62& d, lb_s62& e, const int64_t t[4]) {
  const lb_s62 M = lb_s62_p();
  const int64_t u = t[0], v = t[1], q = t[2], r = t[3];
  const int64_t sd = d.v[6] >> 63, se = e.v[6] >> 63;
  int64_t md = (u & sd) + (v & se), me = (q & sd) + (r & se);
  __int128 cd = (__int128)u * d.v[0] + (__int128)v * e.v[0];
  __int128 ce = (__int128)q * d.v[0] + (__int128)r * e.v[0];
  md -= (int64_t)((LB_S62_PINV * (uint64_t)cd + (uint64_t)md) & (uint64_t)LB_S62_M);
  me -= (int64_t)((LB_S62_PINV * (uint64_t)ce + (uint64_t)me) & (uint64_t)LB_S62_M);
  cd += (__int128)M.v[0] * md;
  ce += (__int128)M.v[0] * me;
  cd >>= 62;
  ce >>= 62;
  LB_UNROLL for (int i = 1; i < 7; i++) {
    cd += (__int128)u * d.v[i] + (__int128)v * e.v[i] + (__int128)M.v[i] * md;
    ce += (__int128)q * d.v[i] + (__int128)r * e.v[i] + (__int128)M.v[i] * me;
    d.v[i - 1] = (int64_t)cd & LB_S62_M;
    cd >>= 62;
    e.v[i - 1] = (int64_t)ce & LB_S62_M;
    ce >>= 62;
  }
  d.v[6] = (int64_t)cd;
  e.v[6] = (int64_t)ce;
}
// r in (-2p, p) -> r * sign (sign = +-1 as the sign of the top limb of f) in [0, p)
LB_HD void lb_s62_normalize(lb_s62& r, int64_t sign) {
  const lb_s62 M = lb_s62_p();
  int64_t cond = r.v[6] >> 63;
  LB_UNROLL for (int i = 0; i < 7; i++) r.v[i] += M.v[i] & cond;
  const int64_t neg = sign >> 63;
  LB_UNROLL for (int i = 0; i < 7; i++) r.v[i] = (r.v[i] ^ neg) - neg;
  LB_UNROLL for (int i = 0; i < 6; i++) {
    r.v[i + 1] += r.v[i] >> 62;
    r.v[i] &= LB_S62_M;
  }
  cond = r.v[6] >> 63;
  LB_UNROLL for (int i = 0; i < 7; i++) r.v[i] += M.v[i] & cond;
  LB_UNROLL for (int i = 0; i < 6; i++) {
    r.v[i + 1] += r.v[i] >> 62;
    r.v[i] &= LB_S62_M;
  }
}
LB_HD uint64_t lb_bits64(const uint32_t* w, int off, int nbits) {  // bits [off, off + nbits) of 12 words
  const int q = off >> 5, s = off & 31;
  uint64_t x = 0;
  LB_UNROLL for (int k = 0; k < 3; k++) {
    const int j = q + k;
    const uint64_t wj = j < 12 ? w[j] : 0u;
    if (k == 0) x = wj >> s;
    else x |= (32 * k - s) < 64 ? wj << (32 * k - s) : 0;
  }
  return nbits >= 64 ? x : (x & ((1ULL << nbits) - 1));
}
// The Jacobi symbol by "posdivsteps" (the Jacobi variant of the divsteps above, as in
// libsecp256k1's modinv64 jacobi): f, g stay non-negative (a swap does not negate), and the
// symbol's sign bit in jac flips when g loses an odd power of 2 while f = 3, 5 mod 8, and when a
// swap meets f = g = 3 mod 4.  ~20 jumps of 62 steps against the binary algorithm's ~760
// word-array iterations (hash_to_G2's is_square: ~184 us -> tens of us on a lone lane).
LB_HD int64_t lb_posdivsteps62(int64_t eta, uint64_t f0, uint64_t g0, int64_t t[4], int& jac) {
  uint64_t u = 1, v = 0, q = 0, r = 1, f = f0, g = g0, m, w;
  int i = 62;
  for (;;) {
    const int zeros = lb_ctz64(g | (~0ULL << i));
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    jac ^= (int)(zeros & ((f >> 1) ^ (f >> 2)));
    if (i == 0) break;
    int limit;
    if (eta < 0) {  // swap (no negation)
      uint64_t tmp;
      eta = -eta;
      tmp = f; f = g; g = tmp;
      tmp = u; u = q; q = tmp;
      tmp = v; v = r; r = tmp;
      jac ^= (int)((f & g) >> 1);
      limit = (int)eta + 1 > i ? i : (int)eta + 1;
      m = (~0ULL >> (64 - limit)) & 63u;
      w = (f * g * (f * f - 2)) & m;
    } else {
      limit = (int)eta + 1 > i ? i : (int)eta + 1;
      m = (~0ULL >> (64 - limit)) & 15u;
      w = f + (((f + 1) & 4) << 1);
      w = ((uint64_t)0 - w * g) & m;
    }
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t[0] = (int64_t)u;
  t[1] = (int64_t)v;
  t[2] = (int64_t)q;
  t[3] = (int64_t)r;
  return eta;
}
// (x | p) for x in [0, p) given as 12 words (0 counts as a square): 1 square, 0 non-square,
// -1 not settled within the jump budget (the caller falls back to the binary algorithm)
LB_HD int fp_is_square_sg(const fp& x) {
  if (fp_is_zero(x)) return 1;
  lb_s62 f = lb_s62_p(), g;
  LB_UNROLL for (int i = 0; i < 7; i++) g.v[i] = (int64_t)lb_bits64(x.v, 62 * i, 62);
  int64_t eta = -1, t[4];
  int jac = 0;
  for (int it = 0; it < 60; it++) {
    // 64 low bits (the symbol's updates read f mod 8 up to the 62nd step)
    eta = lb_posdivsteps62(eta, (uint64_t)f.v[0] | ((uint64_t)f.v[1] << 62), (uint64_t)g.v[0] | ((uint64_t)g.v[1] << 62),
                           t, jac);
    lb_s62_update_fg(f, g, t);
    if (f.v[0] == 1) {
      int64_t any = 0;
      LB_UNROLL for (int i = 1; i < 7; i++) any |= f.v[i];
      if (any == 0) return (jac & 1) ? 0 : 1;
    }
  }
  return -1;
}
// plain a in [0, p) -> a^-1 mod p (plain), 0 -> 0
LB_HD fp fp_inv_plain_by_i(const fp& a) {
  if (fp_is_zero(a)) return a;
  lb_s62 f = lb_s62_p(), g, d, e;
  LB_UNROLL for (int i = 0; i < 7; i++) {
    g.v[i] = (int64_t)lb_bits64(a.v, 62 * i, 62);
    d.v[i] = 0;
    e.v[i] = i == 0;
  }
  int64_t eta = -1, t[4];
  for (int it = 0; it < 40; it++) {  // (a 381-bit modulus needs <= 18 jumps)
    eta = lb_divsteps62(eta, (uint64_t)f.v[0], (uint64_t)g.v[0], t);
    lb_s62_update_de(d, e, t);
    lb_s62_update_fg(f, g, t);
    if (g.v[0] == 0) {
      int64_t any = 0;
      LB_UNROLL for (int i = 1; i < 7; i++) any |= g.v[i];
      if (any == 0) break;
    }
  }
  lb_s62_normalize(d, f.v[6]);  // f = +-1: the sign of its top limb
  fp r;
  LB_UNROLL for (int w = 0; w < 12; w++) {
    const int b = 32 * w, i = b / 62, sft = b - 62 * i;
    uint64_t x = (uint64_t)d.v[i] >> sft;
    if (i + 1 < 7 && sft > 30) x |= (uint64_t)d.v[i + 1] << (62 - sft);
    r.v[w] = (uint32_t)x;
  }
  return r;
}
#ifndef LB_INV_EEA
#define LB_INV_EEA 0  // 1: the binary extended Euclid above (A/B)
#endif
LB_NI fp fp_inv_plain_vt(fp a) { return LB_INV_EEA ? fp_inv_plain_vt_i(a) : fp_inv_plain_by_i(a); }
// Montgomery a R -> a^-1 R:  plain inverse of (a R) is a^-1 R^-1; times R^3 / R gives a^-1 R
LB_HD fp fp_inv(const fp& a) { return fp_mul(fp_inv_plain_vt(a), fp_load(LB_R3)); }  // inv(0)=0
LB_HD fp fp_inv_i(const fp& a) {
  return fp_mul(LB_INV_EEA ? fp_inv_plain_vt_i(a) : fp_inv_plain_by_i(a), fp_load(LB_R3));
}
#ifndef LB_POW_INL
#define LB_POW_INL true  // exponentiations with inline products (A/B: false = out-of-line fp_mul_v)
#endif
LB_NI fp fp_pow_const(fp a, const uint32_t* e, int top_bit) { return fp_pow_const_i<LB_POW_INL>(a, e, top_bit); }
LB_HD fp fp_sqrt_cand(const fp& a) { return fp_pow_const(a, LB_EXP_SQRT, 378); }   // a^((p+1)/4)
LB_HD fp fp_isqrt_cand(const fp& a) { return fp_pow_const(a, LB_EXP_ISQRT, 378); }  // a^((p-3)/4)
// Quadratic character by the binary Jacobi-symbol algorithm (variable time; every input is
// public: SSWU on hashed messages).  Works on the Montgomery representation directly:
// (aR / p) = (a / p) (R / p) and R = 2^384 is a square.  ~400 shift/subtract steps instead of
// the 570-multiplication Legendre exponentiation a^((p-1)/2).
LB_NI bool fp_is_square(fp a) {
  if (fp_is_zero(a)) return true;
  uint32_t u[12], v[12];
  const uint32_t Pl[12] = {LB_P0, LB_P1, LB_P2, LB_P3, LB_P4, LB_P5, LB_P6, LB_P7, LB_P8, LB_P9, LB_P10, LB_P11};
  LB_UNROLL for (int j = 0; j < 12; j++) {
    u[j] = a.v[j];
    v[j] = Pl[j];
  }
  int t = 1;  // (u / v) * t is the answer; v stays odd
  while (true) {
    // remove factors of two from u: (2 / v) = -1 iff v = 3, 5 (mod 8)
    while (u[0] == 0) {
      LB_UNROLL for (int j = 0; j < 11; j++) u[j] = u[j + 1];
      u[11] = 0;  // 2^32 is a square: no sign change
    }
    int k = lb_ctz32(u[0]);
    if (k) {
      lb_shr(u, k);
      uint32_t v8 = v[0] & 7u;
      if ((k & 1) && (v8 == 3u || v8 == 5u)) t = -t;
    }
    if (lb_is_one_plain(u)) return t == 1;
    // both odd: make u >= v by swapping (quadratic reciprocity), then u -= v
    if (!lb_geq(u, v)) {
      if ((u[0] & 3u) == 3u && (v[0] & 3u) == 3u) t = -t;
      LB_UNROLL for (int j = 0; j < 12; j++) {
        uint32_t x = u[j];
        u[j] = v[j];
        v[j] = x;
      }
      if (lb_is_one_plain(u)) return t == 1;
    }
    lb_sub_in(u, v);
    bool zero = true;
    LB_UNROLL for (int j = 0; j < 12; j++) zero &= u[j] == 0;
    if (zero) return false;  // gcd > 1 cannot happen for prime p and a != 0
  }
}

// canonical (non-Montgomery) value compared with (p-1)/2: returns a > (p-1)/2
LB_HD bool fp_plain_gt_half(const fp& plain) {
  uint32_t br = 0;
  LB_UNROLL for (int j = 0; j < 12; j++) {
    uint64_t d = (uint64_t)LB_HALF_P[j] - plain.v[j] - br;
    br = (uint32_t)(d >> 63);
  }
  return br != 0;  // half - a < 0
}

// 48-byte big-endian -> plain limbs; returns false if value >= p (blst BAD_ENCODING)
LB_HD bool fp_plain_from_be48(fp& out, const uint8_t* b, uint8_t first_byte_mask) {
  LB_UNROLL for (int i = 0; i < 12; i++) {
    int o = 44 - 4 * i;
    uint32_t b0 = b[o];
    if (i == 11) b0 &= first_byte_mask;
    out.v[i] = (b0 << 24) | ((uint32_t)b[o + 1] << 16) | ((uint32_t)b[o + 2] << 8) | b[o + 3];
  }
  const uint32_t Pl[12] = {LB_P0, LB_P1, LB_P2, LB_P3, LB_P4, LB_P5, LB_P6, LB_P7, LB_P8, LB_P9, LB_P10, LB_P11};
  uint32_t br = 0;
  LB_UNROLL for (int j = 0; j < 12; j++) {
    uint64_t d = (uint64_t)out.v[j] - Pl[j] - br;
    br = (uint32_t)(d >> 63);
  }
  return br != 0;  // out < p
}

// the same from 12 little-endian-loaded words of the 48 bytes (w[k] = bytes 4k..4k+3): no byte
// buffer, so a kernel keeps the encoding in registers
LB_HD uint32_t lb_bswap32(uint32_t x) { return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24); }
LB_HD bool fp_plain_from_be48_w(fp& out, const uint32_t* w, uint8_t first_byte_mask) {
  LB_UNROLL for (int i = 0; i < 12; i++) out.v[i] = lb_bswap32(w[11 - i]);
  out.v[11] &= ((uint32_t)first_byte_mask << 24) | 0x00ffffffu;
  const uint32_t Pl[12] = {LB_P0, LB_P1, LB_P2, LB_P3, LB_P4, LB_P5, LB_P6, LB_P7, LB_P8, LB_P9, LB_P10, LB_P11};
  uint32_t br = 0;
  LB_UNROLL for (int j = 0; j < 12; j++) {
    uint64_t d = (uint64_t)out.v[j] - Pl[j] - br;
    br = (uint32_t)(d >> 63);
  }
  return br != 0;  // out < p
}

LB_HD void fp_plain_to_be48(uint8_t* b, const fp& plain) {
  LB_UNROLL for (int i = 0; i < 12; i++) {
    int o = 44 - 4 * i;
    uint32_t w = plain.v[i];
    b[o] = (uint8_t)(w >> 24);
    b[o + 1] = (uint8_t)(w >> 16);
    b[o + 2] = (uint8_t)(w >> 8);
    b[o + 3] = (uint8_t)w;
  }
}

// ------------------------------------------------------------------ Fp2
LB_HD fp2 fp2_zero() { return fp2{fp_zero(), fp_zero()}; }
LB_HD fp2 fp2_one() { return fp2{fp_one(), fp_zero()}; }
LB_HD bool fp2_is_zero(const fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
LB_HD bool fp2_eq(const fp2& a, const fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
LB_HD fp2 fp2_select(bool c, const fp2& a, const fp2& b) { return fp2{fp_select(c, a.c0, b.c0), fp_select(c, a.c1, b.c1)}; }
LB_HD fp2 fp2_add(const fp2& a, const fp2& b) { return fp2{fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
LB_HD fp2 fp2_sub(const fp2& a, const fp2& b) { return fp2{fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
LB_HD fp2 fp2_dbl(const fp2& a) { return fp2{fp_dbl(a.c0), fp_dbl(a.c1)}; }
LB_HD fp2 fp2_neg(const fp2& a) { return fp2{fp_neg(a.c0), fp_neg(a.c1)}; }
LB_HD fp2 fp2_conj(const fp2& a) { return fp2{a.c0, fp_neg(a.c1)}; }
LB_HD fp2 fp2_mul_fp(const fp2& a, const fp& s) { return fp2{fp_mul(a.c0, s), fp_mul(a.c1, s)}; }
LB_HD fp2 fp2_mul3(const fp2& a) { return fp2{fp_mul3(a.c0), fp_mul3(a.c1)}; }
LB_HD fp2 fp2_mul4(const fp2& a) { return fp2{fp_mul4(a.c0), fp_mul4(a.c1)}; }
LB_HD fp2 fp2_mul8(const fp2& a) { return fp2{fp_mul8(a.c0), fp_mul8(a.c1)}; }

// Fp2 arithmetic is inline (its three products are calls to fp_mul); the Fp6 / Fp12 layers
// and the group law are out of line with pointer / by-value arguments.
LB_HD fp2 fp2_mul(const fp2& a, const fp2& b) {
  fp t0 = fp_mul(a.c0, b.c0);
  fp t1 = fp_mul(a.c1, b.c1);
  fp t2 = fp_mul(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
  return fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}
LB_HD fp2 fp2_sqr(const fp2& a) {
  fp t0 = fp_mul(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1));
  fp t1 = fp_mul(a.c0, a.c1);
  return fp2{t0, fp_dbl(t1)};
}
// multiply by the non-residue xi = 1 + u
LB_HD fp2 fp2_mul_xi(const fp2& a) { return fp2{fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; }

LB_NI fp2 fp2_inv(fp2 a) {
  fp n = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  fp ni = fp_inv(n);
  return fp2{fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni))};
}

LB_HD bool fp2_is_square(const fp2& a) { return fp_is_square(fp_add(fp_sqr(a.c0), fp_sqr(a.c1))); }

// Square root in Fp2 by the complex method (p = 3 mod 4): three Fp exponentiations,
// no data-dependent branches.  Returns true iff a is a square; `out` is some root.
// fp2_sqrt_i is the inline body (signature decoding keeps its point in registers), fp2_sqrt
// the out-of-line entry.
template <bool kInl = false>
LB_HD bool fp2_sqrt_i(fp2& out, const fp2& a) {
  fp norm = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  fp alpha;
  if constexpr (kInl) alpha = fp_pow_const_i<LB_POW_INL>(norm, LB_EXP_SQRT, 378);
  else alpha = fp_sqrt_cand(norm);  // sqrt(norm) if it exists
  fp inv2 = fp_load(LB_INV2);
  fp d1 = fp_mul(fp_add(a.c0, alpha), inv2);
  fp d2 = fp_mul(fp_sub(a.c0, alpha), inv2);
  // (a0 + alpha)/2 is zero only when a1 == 0 and alpha == -a0; use the other candidate
  fp delta = fp_select(fp_is_zero(d1), d2, d1);
  // z = delta^((p-3)/4), s = delta z = delta^((p+1)/4), and s z = delta^((p-1)/2) = +-1, so
  // 1/s = +-z: the square root and the inverse it needs come from one exponentiation
  fp z;
  if constexpr (kInl) z = fp_pow_const_i<LB_POW_INL>(delta, LB_EXP_ISQRT, 378);
  else z = fp_isqrt_cand(delta);
  fp s = fp_mul(delta, z);
  bool delta_qr = fp_eq(fp_sqr(s), delta);
  // if delta is a residue: x0 = s, x1 = a1/(2s); else (s^2 = -delta) x0 = a1/(2s), x1 = s
  fp t = fp_mul(z, inv2);
  if (!delta_qr) t = fp_neg(t);
  fp q = fp_mul(a.c1, t);
  out.c0 = fp_select(delta_qr, s, q);
  out.c1 = fp_select(delta_qr, q, s);
  return fp2_eq(fp2_sqr(out), a);
}
LB_NI bool fp2_sqrt(fp2& out, fp2 a) { return fp2_sqrt_i(out, a); }
// the same with the two exponentiations by pow(x, exponent words, top bit) (k_hash_map_row: on a row)
template <class Pow>
LB_HD bool fp2_sqrt_p(fp2& out, const fp2& a, Pow pow) {
  const fp norm = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  const fp alpha = pow(norm, LB_EXP_SQRT, 378);
  const fp inv2 = fp_load(LB_INV2);
  const fp d1 = fp_mul(fp_add(a.c0, alpha), inv2);
  const fp d2 = fp_mul(fp_sub(a.c0, alpha), inv2);
  const fp delta = fp_select(fp_is_zero(d1), d2, d1);
  const fp z = pow(delta, LB_EXP_ISQRT, 378);
  const fp s = fp_mul(delta, z);
  const bool delta_qr = fp_eq(fp_sqr(s), delta);
  fp t = fp_mul(z, inv2);
  if (!delta_qr) t = fp_neg(t);
  const fp q = fp_mul(a.c1, t);
  out.c0 = fp_select(delta_qr, s, q);
  out.c1 = fp_select(delta_qr, q, s);
  return fp2_eq(fp2_sqr(out), a);
}

// RFC 9380 sgn0 for Fp2 (on canonical values)
LB_HD uint32_t fp2_sgn0(const fp2& a) {
  fp p0 = fp_from_mont(a.c0), p1 = fp_from_mont(a.c1);
  uint32_t sign0 = p0.v[0] & 1u;
  uint32_t zero0 = fp_is_zero(p0) ? 1u : 0u;
  uint32_t sign1 = p1.v[0] & 1u;
  return sign0 | (zero0 & sign1);
}

// ZCash "lexicographically largest" for Fp2: decided by c1 unless c1 == 0
LB_HD bool fp2_lex_larger(const fp2& a) {
  fp p0 = fp_from_mont(a.c0), p1 = fp_from_mont(a.c1);
  return fp_is_zero(p1) ? fp_plain_gt_half(p0) : fp_plain_gt_half(p1);
}

// ------------------------------------------------------------------ Fp6
LB_HD fp6 fp6_zero() { return fp6{fp2_zero(), fp2_zero(), fp2_zero()}; }
LB_HD fp6 fp6_one() { return fp6{fp2_one(), fp2_zero(), fp2_zero()}; }
LB_HD fp6 fp6_add(const fp6& a, const fp6& b) { return fp6{fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)}; }
LB_HD fp6 fp6_sub(const fp6& a, const fp6& b) { return fp6{fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)}; }
LB_HD fp6 fp6_neg(const fp6& a) { return fp6{fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)}; }
LB_HD fp6 fp6_mul_v(const fp6& a) { return fp6{fp2_mul_xi(a.c2), a.c0, a.c1}; }

// Inline body (the Miller loop kernel keeps its Fp12 state in registers); fp6_mul_p is the
// out-of-line entry everything else calls.
LB_HD fp6 fp6_mul_inl(const fp6& a, const fp6& b) {
  fp2 t0 = fp2_mul(a.c0, b.c0);
  fp2 t1 = fp2_mul(a.c1, b.c1);
  fp2 t2 = fp2_mul(a.c2, b.c2);
  fp2 c0 = fp2_add(fp2_mul_xi(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c1, a.c2), fp2_add(b.c1, b.c2)), t1), t2)), t0);
  fp2 c1 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b.c0, b.c1)), t0), t1), fp2_mul_xi(t2));
  fp2 c2 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c2), fp2_add(b.c0, b.c2)), t0), t2), t1);
  return fp6{c0, c1, c2};
}
LB_NI void fp6_mul_p(fp6* r, const fp6* pa, const fp6* pb) { *r = fp6_mul_inl(*pa, *pb); }
LB_HD fp6 fp6_mul(const fp6& a, const fp6& b) {
  fp6 r;
  fp6_mul_p(&r, &a, &b);
  return r;
}

// a * (b0 + b1 v)  (sparse: c2 coefficient zero)
LB_HD fp6 fp6_mul_01(const fp6& a, const fp2& b0, const fp2& b1) {
  fp2 t0 = fp2_mul(a.c0, b0);
  fp2 t1 = fp2_mul(a.c1, b1);
  fp2 c0 = fp2_add(fp2_mul_xi(fp2_mul(a.c2, b1)), t0);
  fp2 c1 = fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b0, b1)), t0), t1);
  fp2 c2 = fp2_add(fp2_mul(a.c2, b0), t1);
  return fp6{c0, c1, c2};
}

// a * (b1 v)
LB_HD fp6 fp6_mul_1(const fp6& a, const fp2& b1) {
  return fp6{fp2_mul_xi(fp2_mul(a.c2, b1)), fp2_mul(a.c0, b1), fp2_mul(a.c1, b1)};
}

LB_NI fp6 fp6_inv(fp6 a) {
  fp2 t0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  fp2 t1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  fp2 t2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  fp2 d = fp2_add(fp2_mul(a.c0, t0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, t1), fp2_mul(a.c1, t2))));
  fp2 di = fp2_inv(d);
  return fp6{fp2_mul(t0, di), fp2_mul(t1, di), fp2_mul(t2, di)};
}

// ------------------------------------------------------------------ Fp12
LB_HD fp12 fp12_one() { return fp12{fp6_one(), fp6_zero()}; }
LB_HD bool fp12_is_one(const fp12& a) {
  return fp2_eq(a.c0.c0, fp2_one()) && fp2_is_zero(a.c0.c1) && fp2_is_zero(a.c0.c2) && fp2_is_zero(a.c1.c0) &&
         fp2_is_zero(a.c1.c1) && fp2_is_zero(a.c1.c2);
}
LB_HD fp12 fp12_conj(const fp12& a) { return fp12{a.c0, fp6_neg(a.c1)}; }

LB_NI void fp12_mul_p(fp12* r, const fp12* pa, const fp12* pb) {
  const fp12& a = *pa;
  const fp12& b = *pb;
  fp6 t0 = fp6_mul(a.c0, b.c0);
  fp6 t1 = fp6_mul(a.c1, b.c1);
  fp6 c1 = fp6_sub(fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), t0), t1);
  fp6 c0 = fp6_add(t0, fp6_mul_v(t1));
  *r = fp12{c0, c1};
}
LB_HD fp12 fp12_mul(const fp12& a, const fp12& b) {
  fp12 r;
  fp12_mul_p(&r, &a, &b);
  return r;
}

LB_HD fp12 fp12_sqr_inl(const fp12& a) {
  // complex squaring: (a0 + a1 w)^2 = a0^2 + v a1^2 + 2 a0 a1 w
  fp6 t = fp6_mul_inl(a.c0, a.c1);
  fp6 c0 = fp6_mul_inl(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1)));
  c0 = fp6_sub(fp6_sub(c0, t), fp6_mul_v(t));
  return fp12{c0, fp6_add(t, t)};
}
LB_NI void fp12_sqr_p(fp12* r, const fp12* pa) { *r = fp12_sqr_inl(*pa); }
LB_HD fp12 fp12_sqr(const fp12& a) {
  fp12 r;
  fp12_sqr_p(&r, &a);
  return r;
}

// multiply by a Miller-loop line  l = (l0 + l2 v) + (l3 v) w   (w-basis: l0 w^0 + l2 w^2 + l3 w^3)
LB_HD fp12 fp12_mul_line_inl(const fp12& a, const fp2& l0, const fp2& l2, const fp2& l3) {
  fp6 t0 = fp6_mul_01(a.c0, l0, l2);
  fp6 t1 = fp6_mul_1(a.c1, l3);
  fp6 c1 = fp6_sub(fp6_sub(fp6_mul_01(fp6_add(a.c0, a.c1), l0, fp2_add(l2, l3)), t0), t1);
  fp6 c0 = fp6_add(t0, fp6_mul_v(t1));
  return fp12{c0, c1};
}
LB_NI void fp12_mul_line_p(fp12* r, const fp12* pa, const fp2* pl0, const fp2* pl2, const fp2* pl3) {
  *r = fp12_mul_line_inl(*pa, *pl0, *pl2, *pl3);
}
LB_HD fp12 fp12_mul_line(const fp12& a, const fp2& l0, const fp2& l2, const fp2& l3) {
  fp12 r;
  fp12_mul_line_p(&r, &a, &l0, &l2, &l3);
  return r;
}

LB_NI fp12 fp12_inv(fp12 a) {
  fp6 t = fp6_sub(fp6_mul(a.c0, a.c0), fp6_mul_v(fp6_mul(a.c1, a.c1)));
  fp6 ti = fp6_inv(t);
  return fp12{fp6_mul(a.c0, ti), fp6_neg(fp6_mul(a.c1, ti))};
}

// Frobenius a -> a^p.  In the w-basis a = sum a_k w^k (a_0=c0.c0, a_1=c1.c0, a_2=c0.c1,
// a_3=c1.c1, a_4=c0.c2, a_5=c1.c2), a^p = sum conj(a_k) xi^(k(p-1)/6) w^k.
LB_NI fp12 fp12_frob(fp12 a) {
  fp12 r;
  r.c0.c0 = fp2_conj(a.c0.c0);
  r.c1.c0 = fp2_mul(fp2_conj(a.c1.c0), fp2_load(LB_FROB1_1));
  r.c0.c1 = fp2_mul(fp2_conj(a.c0.c1), fp2_load(LB_FROB1_2));
  r.c1.c1 = fp2_mul(fp2_conj(a.c1.c1), fp2_load(LB_FROB1_3));
  r.c0.c2 = fp2_mul(fp2_conj(a.c0.c2), fp2_load(LB_FROB1_4));
  r.c1.c2 = fp2_mul(fp2_conj(a.c1.c2), fp2_load(LB_FROB1_5));
  return r;
}
LB_NI fp12 fp12_frob2(fp12 a) {
  fp12 r;
  r.c0.c0 = a.c0.c0;
  r.c1.c0 = fp2_mul_fp(a.c1.c0, fp_load(LB_FROB2_1));
  r.c0.c1 = fp2_mul_fp(a.c0.c1, fp_load(LB_FROB2_2));
  r.c1.c1 = fp2_mul_fp(a.c1.c1, fp_load(LB_FROB2_3));
  r.c0.c2 = fp2_mul_fp(a.c0.c2, fp_load(LB_FROB2_4));
  r.c1.c2 = fp2_mul_fp(a.c1.c2, fp_load(LB_FROB2_5));
  return r;
}

// ------------------------------------------------------------------ overloads for generic curve code
LB_HD fp f_add(const fp& a, const fp& b) { return fp_add(a, b); }
LB_HD fp f_sub(const fp& a, const fp& b) { return fp_sub(a, b); }
LB_HD fp f_mul(const fp& a, const fp& b) { return fp_mul(a, b); }
LB_HD fp f_sqr(const fp& a) { return fp_sqr(a); }
LB_HD fp f_dbl(const fp& a) { return fp_dbl(a); }
LB_HD fp f_neg(const fp& a) { return fp_neg(a); }
LB_HD fp f_mul3(const fp& a) { return fp_mul3(a); }
LB_HD fp f_mul8(const fp& a) { return fp_mul8(a); }
LB_HD fp f_inv(const fp& a) { return fp_inv(a); }
LB_HD bool f_is_zero(const fp& a) { return fp_is_zero(a); }
LB_HD bool f_eq(const fp& a, const fp& b) { return fp_eq(a, b); }
LB_HD fp f_select(bool c, const fp& a, const fp& b) { return fp_select(c, a, b); }
LB_HD void f_set_zero(fp& a) { a = fp_zero(); }
LB_HD void f_set_one(fp& a) { a = fp_one(); }

// fp with inline (fenced) products: a kernel that instantiates the generic curve code on jac<fpi>
// runs its G1 formulas without out-of-line product calls (k_pk_blind's GLV ladder)
struct fpi : fp {};
LB_HD fpi fpi_of(const fp& a) { return fpi{a}; }
LB_HD fpi f_add(const fpi& a, const fpi& b) { return fpi{fp_add(a, b)}; }
LB_HD fpi f_sub(const fpi& a, const fpi& b) { return fpi{fp_sub(a, b)}; }
LB_HD fpi f_mul(const fpi& a, const fpi& b) { return fpi{fp_mul_inl(a, b)}; }
LB_HD fpi f_sqr(const fpi& a) { return fpi{fp_sqr_inl(a)}; }
LB_HD fpi f_dbl(const fpi& a) { return fpi{fp_dbl(a)}; }
LB_HD fpi f_neg(const fpi& a) { return fpi{fp_neg(a)}; }
LB_HD fpi f_mul3(const fpi& a) { return fpi{fp_mul3(a)}; }
LB_HD fpi f_mul8(const fpi& a) { return fpi{fp_mul8(a)}; }
LB_HD bool f_is_zero(const fpi& a) { return fp_is_zero(a); }
LB_HD bool f_eq(const fpi& a, const fpi& b) { return fp_eq(a, b); }
LB_HD fpi f_select(bool c, const fpi& a, const fpi& b) { return fpi{fp_select(c, a, b)}; }
LB_HD void f_set_zero(fpi& a) { a = fpi{fp_zero()}; }
LB_HD void f_set_one(fpi& a) { a = fpi{fp_one()}; }

LB_HD fp2 f_add(const fp2& a, const fp2& b) { return fp2_add(a, b); }
// ... and fp2 with inline products (the G2 bucket sums and reductions of the MSM)
struct fp2i : fp2 {};
LB_HD fp2i f_add(const fp2i& a, const fp2i& b) { return fp2i{fp2_add(a, b)}; }
LB_HD fp2i f_sub(const fp2i& a, const fp2i& b) { return fp2i{fp2_sub(a, b)}; }
LB_HD fp2i f_mul(const fp2i& a, const fp2i& b) {
  const fp t0 = fp_mul_inl(a.c0, b.c0);
  const fp t1 = fp_mul_inl(a.c1, b.c1);
  const fp t2 = fp_mul_inl(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
  return fp2i{fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)}};
}
LB_HD fp2i f_sqr(const fp2i& a) {
  const fp t0 = fp_mul_inl(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1));
  const fp t1 = fp_mul_inl(a.c0, a.c1);
  return fp2i{fp2{t0, fp_dbl(t1)}};
}
LB_HD fp2i f_dbl(const fp2i& a) { return fp2i{fp2_dbl(a)}; }
LB_HD fp2i f_neg(const fp2i& a) { return fp2i{fp2_neg(a)}; }
LB_HD fp2i f_mul3(const fp2i& a) { return fp2i{fp2_mul3(a)}; }
LB_HD fp2i f_mul8(const fp2i& a) { return fp2i{fp2_mul8(a)}; }
LB_HD bool f_is_zero(const fp2i& a) { return fp2_is_zero(a); }
LB_HD bool f_eq(const fp2i& a, const fp2i& b) { return fp2_eq(a, b); }
LB_HD fp2i f_select(bool c, const fp2i& a, const fp2i& b) { return fp2i{fp2_select(c, a, b)}; }
LB_HD void f_set_zero(fp2i& a) { a = fp2i{fp2_zero()}; }
LB_HD void f_set_one(fp2i& a) { a = fp2i{fp2_one()}; }
LB_HD fp2 f_sub(const fp2& a, const fp2& b) { return fp2_sub(a, b); }
LB_HD fp2 f_mul(const fp2& a, const fp2& b) { return fp2_mul(a, b); }
LB_HD fp2 f_sqr(const fp2& a) { return fp2_sqr(a); }
LB_HD fp2 f_dbl(const fp2& a) { return fp2_dbl(a); }
LB_HD fp2 f_neg(const fp2& a) { return fp2_neg(a); }
LB_HD fp2 f_mul3(const fp2& a) { return fp2_mul3(a); }
LB_HD fp2 f_mul8(const fp2& a) { return fp2_mul8(a); }
LB_HD fp2 f_inv(const fp2& a) { return fp2_inv(a); }
LB_HD bool f_is_zero(const fp2& a) { return fp2_is_zero(a); }
LB_HD bool f_eq(const fp2& a, const fp2& b) { return fp2_eq(a, b); }
LB_HD fp2 f_select(bool c, const fp2& a, const fp2& b) { return fp2_select(c, a, b); }
LB_HD void f_set_zero(fp2& a) { a = fp2_zero(); }
LB_HD void f_set_one(fp2& a) { a = fp2_one(); }
