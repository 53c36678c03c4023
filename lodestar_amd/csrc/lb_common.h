// Common macros for the BLS12-381 engine.  Every arithmetic routine is written once as
// LB_HD (host+device, force-inlined) so the same source runs in the gfx950 kernels and
// in the CPU unit-test harness (tests/harness/), which is how the arithmetic is checked
// against oracle/ without a GPU.  The product path is only ever the HIP build.
#pragma once
#include <stdint.h>

// Split build (tools/gen_kdecls.py): a translation unit compiled with -DLB_KGROUP=g defines only
// the kernels of group g (`#if LB_KG(g)` around each definition); LB_KGROUP unset defines them all
#ifndef LB_KGROUP
#define LB_KGROUP -1
#endif
#define LB_KG(g) (LB_KGROUP < 0 || LB_KGROUP == (g))

// k_hash_map_row: map_to_curve_g2_fold on row pairs (1) or map_to_curve_g2_i on single rows (0, A/B);
// k_decompress_sigs_row: its square roots' exponentiations on row pairs (1) or single rows (0)
#ifndef LB_H2C_FOLD
#define LB_H2C_FOLD 1
#endif
// rfp2 products on the four rows of a wave (lb_row.h f_mul / f_sqr; k_hash_map_row one item per wave)
#ifndef LBR_FP2_W4
#define LBR_FP2_W4 1
#endif

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define LB_HD __host__ __device__ __forceinline__
#define LB_HDNI static __host__ __device__ __attribute__((noinline))
#define LB_NI static __host__ __device__ __attribute__((noinline))
#define LB_CONST static __constant__ const
#else
#define LB_HD static inline
#define LB_HDNI static
#define LB_NI static inline
#define LB_CONST static const
#endif

#define LB_UNROLL _Pragma("unroll")

// 32-bit add / subtract with carry.  On the GPU these lower to one v_add_co_u32 /
// v_addc_co_u32 (v_sub_co / v_subb_co) per limb; the uint64_t idiom costs ~6 instructions per
// limb (zero-extension moves + 64-bit adds).  g++ builds (CPU harness) use the portable form.
#if defined(__clang__)
#define LB_ADDC(a, b, cin, cout) __builtin_addc((a), (b), (cin), (cout))
#define LB_SUBC(a, b, bin, bout) __builtin_subc((a), (b), (bin), (bout))
#else
static inline uint32_t lb_addc_port(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
  uint64_t s = (uint64_t)a + b + cin;
  *cout = (uint32_t)(s >> 32);
  return (uint32_t)s;
}
static inline uint32_t lb_subc_port(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
  uint64_t d = (uint64_t)a - b - bin;
  *bout = (uint32_t)(d >> 63);
  return (uint32_t)d;
}
#define LB_ADDC(a, b, cin, cout) lb_addc_port((a), (b), (cin), (cout))
#define LB_SUBC(a, b, bin, bout) lb_subc_port((a), (b), (bin), (bout))
#endif

// Host-only operation counter (tools/count_ops.py builds the harness with -DLB_COUNT_OPS to
// derive the algorithmic Fp-multiplication count per pipeline stage for the roofline).
#if defined(LB_COUNT_OPS) && !defined(__HIPCC__)
extern unsigned long long lb_count_mul;
#define LB_COUNT_MUL() (lb_count_mul++)
#else
#define LB_COUNT_MUL() ((void)0)
#endif

// Status codes (blst BLST_ERROR values + Lodestar's own errors) are the public ones of
// the C ABI: include/lodestar_bls.h.  Per-set / per-job status uses them directly.
#include "lodestar_bls.h"
