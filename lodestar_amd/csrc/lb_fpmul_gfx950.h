// gfx950 Montgomery multiplication with hand-scheduled multiply-accumulate chains.
//
// Operand scanning into per-column accumulators: column k holds a 64-bit accumulator acc[k]
// plus an overflow word ovf[k] (value = acc + ovf * 2^64).  Each product a_i * b_j is one
//   v_mad_u64_u32 acc[i+j], cc, a_i, b_j, acc[i+j]    (cc = carry out of bit 64, an SGPR pair)
// followed later by
//   v_addc_co_u32 ovf[i+j], cc, 0, ovf[i+j], cc
// A row's products hit different columns, so they are independent: four MADs are issued before
// the first ADDC reads its carry (>= 2 wait states, the gfx950 VALU-SGPR-write -> VALU-carry-
// read hazard), so no s_nop is needed.  After row i (a_i * b, then m_i * p), column i is
// divisible by 2^32 and its high part folds into column i+1.
// Replaces the 1336-instruction compiler output of the carry-save C form (664 of them v_mov
// for zero-extension); fp_mul_body (lb_field.h) stays the reference and the CPU path, and
// tests/test_gpu_parity.py::test_fp_mul_kernel checks both agree on the GPU.
#pragma once
#include "lb_common.h"

#if defined(__HIP_DEVICE_COMPILE__)

// acc[k..k+3] += x * y[0..3]  (y in VGPRs)
__device__ __forceinline__ void lbm_mac4v(uint64_t* acc, uint32_t* ovf, uint32_t x, uint32_t y0, uint32_t y1,
                                          uint32_t y2, uint32_t y3) {
  uint64_t c0, c1, c2, c3;
  asm volatile(
      "v_mad_u64_u32 %0, %8, %12, %13, %0\n\t"
      "v_mad_u64_u32 %1, %9, %12, %14, %1\n\t"
      "v_mad_u64_u32 %2, %10, %12, %15, %2\n\t"
      "v_mad_u64_u32 %3, %11, %12, %16, %3\n\t"
      "v_addc_co_u32_e64 %4, %8, 0, %4, %8\n\t"
      "v_addc_co_u32_e64 %5, %9, 0, %5, %9\n\t"
      "v_addc_co_u32_e64 %6, %10, 0, %6, %10\n\t"
      "v_addc_co_u32_e64 %7, %11, 0, %7, %11"
      : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(ovf[0]), "+v"(ovf[1]), "+v"(ovf[2]),
        "+v"(ovf[3]), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3)
      : "v"(x), "v"(y0), "v"(y1), "v"(y2), "v"(y3));
}

// acc[k..k+3] += x * y[0..3]  (y constants in SGPRs)
__device__ __forceinline__ void lbm_mac4s(uint64_t* acc, uint32_t* ovf, uint32_t x, uint32_t y0, uint32_t y1,
                                          uint32_t y2, uint32_t y3) {
  uint64_t c0, c1, c2, c3;
  asm volatile(
      "v_mad_u64_u32 %0, %8, %12, %13, %0\n\t"
      "v_mad_u64_u32 %1, %9, %12, %14, %1\n\t"
      "v_mad_u64_u32 %2, %10, %12, %15, %2\n\t"
      "v_mad_u64_u32 %3, %11, %12, %16, %3\n\t"
      "v_addc_co_u32_e64 %4, %8, 0, %4, %8\n\t"
      "v_addc_co_u32_e64 %5, %9, 0, %5, %9\n\t"
      "v_addc_co_u32_e64 %6, %10, 0, %6, %10\n\t"
      "v_addc_co_u32_e64 %7, %11, 0, %7, %11"
      : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(ovf[0]), "+v"(ovf[1]), "+v"(ovf[2]),
        "+v"(ovf[3]), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3)
      : "v"(x), "s"(y0), "s"(y1), "s"(y2), "s"(y3));
}

// column k (low 32 bits zero) folds into column k+1
__device__ __forceinline__ void lbm_fold(uint64_t& acc_k, uint32_t ovf_k, uint64_t& acc_k1, uint32_t& ovf_k1) {
  uint32_t lo = (uint32_t)acc_k1, hi = (uint32_t)(acc_k1 >> 32), c0, c1;
  lo = __builtin_addc(lo, (uint32_t)(acc_k >> 32), 0u, &c0);
  hi = __builtin_addc(hi, ovf_k, c0, &c1);
  acc_k1 = ((uint64_t)hi << 32) | lo;
  ovf_k1 += c1;
}

__device__ __forceinline__ void lbm_mont_mul(uint32_t* out, uint32_t* top_out, const uint32_t* a, const uint32_t* b) {
  uint64_t acc[24];
  uint32_t ovf[24];
  LB_UNROLL for (int k = 0; k < 24; k++) {
    acc[k] = 0;
    ovf[k] = 0;
  }
  LB_UNROLL for (int i = 0; i < 12; i++) {
    lbm_mac4v(acc + i, ovf + i, a[i], b[0], b[1], b[2], b[3]);
    lbm_mac4v(acc + i + 4, ovf + i + 4, a[i], b[4], b[5], b[6], b[7]);
    lbm_mac4v(acc + i + 8, ovf + i + 8, a[i], b[8], b[9], b[10], b[11]);
    const uint32_t m = (uint32_t)acc[i] * LB_PINV;
    lbm_mac4s(acc + i, ovf + i, m, LB_P0, LB_P1, LB_P2, LB_P3);
    lbm_mac4s(acc + i + 4, ovf + i + 4, m, LB_P4, LB_P5, LB_P6, LB_P7);
    lbm_mac4s(acc + i + 8, ovf + i + 8, m, LB_P8, LB_P9, LB_P10, LB_P11);
    lbm_fold(acc[i], ovf[i], acc[i + 1], ovf[i + 1]);
  }
  // normalise columns 12..23 into 12 limbs (+ top word): value < 2p
  LB_UNROLL for (int k = 12; k < 23; k++) {
    out[k - 12] = (uint32_t)acc[k];
    lbm_fold(acc[k], ovf[k], acc[k + 1], ovf[k + 1]);
  }
  out[11] = (uint32_t)acc[23];
  *top_out = (uint32_t)(acc[23] >> 32);
}

#endif
