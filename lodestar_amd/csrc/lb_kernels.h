// gfx950 kernels of the signature-set verification pipeline (one thread per work item).
//
// Pipeline for one batch of jobs (blst semantics of
// Pairing.mul_n_aggregate + commit + finalverify behind maybeBatch.ts:18-25):
//   k_decompress_sigs / k_sig_subgroup   per set : compressed G2 -> affine, psi subgroup check
//                                                   (Signature.fromBytes(.., true))
//   k_msg_*            per set   : group the sets by signing root (hash table, counting sort)
//   k_hash_map         per root x2: expand_message_xmd + SSWU + 3-isogeny     (hash_to_G2, first half)
//   k_hash_finish      per root  : Q0 + Q1, clear cofactor, to affine        (hash_to_G2, second half)
//   k_pk_chunks[_idx] / k_pk_blind per set: G1 aggregation (utils.ts:5-16), r*PK
//   k_gsum_*           per root  : P_u = sum r_i PK_i over the root's live sets
//   k_miller_lane / _g8 / _wave per root : ML(P_u, H(m_u))               (Pairing.mul_n_aggregate)
//   k_msm_*            per set   : S = sum r_i sig_i (bucket MSM)
//   k_tree_up_U / k_ml_S / k_root_check : product tree, ML(-G1, S), one final exponentiation
//   k_rmsm_*, k_range_pk, k_search_check : the invalid-set search after a failing root
// All intermediate arrays are structure-of-arrays, word-major: word w of element e lives at
// base[w * n + e], so a wave's 64 lanes touch 64 consecutive words per access.
#pragma once
#include "lb_serial.h"
#include "lb_h2c.h"
#include "lb_pairing.h"

#define LB_TPB 64  // one wave per workgroup: spreads few-thousand-item batches over all 256 CUs
#ifndef LB_MINW
#define LB_MINW 1  // min waves per SIMD (2 caps registers at 256 but spills: measured slower)
#endif
#ifndef LB_MINW_DEC
#define LB_MINW_DEC 2  // k_decode_sigs (all-inline call graph, so its own bound holds): spills,
                       // but half the register file lets another batch's kernels co-reside
#endif
#ifndef LB_MINW_SUB
#define LB_MINW_SUB LB_MINW_DEC  // k_sig_subgroup.  One wave per SIMD lets the compiler spill to
                       // AGPRs instead of scratch (8 B instead of 696 B per lane) but costs occupancy:
                       // 10.2 vs 10.6 M sets/s at 7 in flight, 4.9 vs 5.0 M at one (round-3 A/B,
                       // profiles/r3_variants_ab.txt); the ladder state in LDS instead (24 KB per
                       // wave) still spilled and ran 4.7 M at one in flight.
#endif
#ifndef LB_SUBGROUP_INL
#define LB_SUBGROUP_INL true  // k_sig_subgroup: Fp products inline (no call-boundary spills)
#endif
#ifndef LB_MINW_MSM
#define LB_MINW_MSM 1  // k_msm_chunks (2 spills; within noise under load)
#endif
#ifndef LB_MINW_GSUM
#define LB_MINW_GSUM 1  // k_gsum_chunks (all-inline)
#endif
#ifndef LB_G1_INL
#define LB_G1_INL 1  // k_pk_blind's GLV ladder with inline products (jac<fpi>); 0: out-of-line calls
#endif
#ifndef LB_G2_INL
#define LB_G2_INL 1  // the MSM's G2 additions (chunks, buckets, reduction) with inline products
#endif
#if LB_G1_INL
typedef fpi lb_g1f;  // the G1 chunk and per-root sums' additions with inline products
#else
typedef fp lb_g1f;
#endif
#ifndef LB_G2_INL_SB
#define LB_G2_INL_SB LB_G2_INL  // ... and k_sig_blind's per-set GLV ladder
#endif
#if LB_G2_INL
typedef fp2i lb_g2f;
#else
typedef fp2 lb_g2f;
#endif
typedef jac<lb_g2f> g2jm;
#ifndef LB_MINW_G1
#define LB_MINW_G1 2  // G1 kernels: one Fp multiply per step, so a second wave hides its latency
#endif

template <class T>
__device__ __forceinline__ T soa_ld(const uint32_t* __restrict__ base, uint32_t n, uint32_t e) {
  static_assert(sizeof(T) % 4 == 0, "word-sized types only");
  T r;
  uint32_t* w = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); i++) w[i] = base[(size_t)i * n + e];
  return r;
}
template <class T>
__device__ __forceinline__ void soa_st(uint32_t* __restrict__ base, uint32_t n, uint32_t e, const T& v) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); i++) base[(size_t)i * n + e] = w[i];
}

// Array-of-structures element e (16-byte vector accesses): for arrays read by gathers (a lane
// pulls its element's 144 or 192 contiguous bytes instead of one word from each of 36 or 48
// SoA rows, i.e. 36 or 48 separate cache lines).
template <class T>
__device__ __forceinline__ T aos_ld(const uint32_t* __restrict__ base, uint32_t e) {
  static_assert(sizeof(T) % 16 == 0, "16-byte multiples");
  T r;
  uint4* w = reinterpret_cast<uint4*>(&r);
  const uint4* s = reinterpret_cast<const uint4*>(base) + (size_t)e * (sizeof(T) / 16);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 16); i++) w[i] = s[i];
  return r;
}
template <class T>
__device__ __forceinline__ void aos_st(uint32_t* __restrict__ base, uint32_t e, const T& v) {
  static_assert(sizeof(T) % 16 == 0, "16-byte multiples");
  const uint4* w = reinterpret_cast<const uint4*>(&v);
  uint4* d = reinterpret_cast<uint4*>(base) + (size_t)e * (sizeof(T) / 16);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 16); i++) d[i] = w[i];
}

template <int N>
__device__ __forceinline__ void ld_bytes(uint8_t* dst, const uint8_t* __restrict__ src) {
  static_assert(N % 16 == 0, "16-byte multiples");
  const uint4* s = reinterpret_cast<const uint4*>(src);
#pragma unroll
  for (int i = 0; i < N / 16; i++) {
    uint4 v = s[i];
    uint32_t ws[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
      dst[16 * i + 4 * k + 0] = (uint8_t)ws[k];
      dst[16 * i + 4 * k + 1] = (uint8_t)(ws[k] >> 8);
      dst[16 * i + 4 * k + 2] = (uint8_t)(ws[k] >> 16);
      dst[16 * i + 4 * k + 3] = (uint8_t)(ws[k] >> 24);
    }
  }
}

__device__ __forceinline__ uint32_t lb_tid() { return blockIdx.x * blockDim.x + threadIdx.x; }

#include "lb_wave.h"
#include "lb_row.h"
// Row-engine forms (lb_row.h: one Fp product per 16-lane row, one 16-wave workgroup per item) of
// the final exponentiations, ML(-G1, S), the small-batch per-root Miller loops and the product
// tree: k_*_row next to the wave-engine kernels (one product per lane, one wave).  The engine runs
// the row forms only while the device has no other batch in flight (latency): a 16-wave
// workgroup needs a whole CU, which under load costs the batches in flight ~5 % of the headline
// (profiles/r5_row_ab.txt).
#include "lb_group_exec.h"
#include "lb_group.h"
#include "lb_ssz.h"

// ---------------------------------------------------------------- block-wide batch inversion
// Montgomery's trick across the LB_INV_TPB threads of a block: prefix and suffix products by
// cross-lane scans inside each wave, ONE field inversion per block (wave 0, on a value that is
// uniform across its lanes, so the variable-time binary EEA runs without divergence), then
// z_i^-1 = prefix_{i-1} * suffix_{i+1} * (wave total)^-1.  A per-lane inversion instead runs
// 64 divergent EEAs per wave: about half of k_pk_blind's instructions before this.
// Every thread of the block must call it; z must be non-zero (callers pass one for idle lanes).
#define LB_INV_TPB 64
__device__ __forceinline__ fp fp_shfl_up(const fp& a, unsigned d) {
  fp r;
  LB_UNROLL for (int j = 0; j < 12; j++) r.v[j] = __shfl_up(a.v[j], d, 64);
  return r;
}
__device__ __forceinline__ fp fp_shfl_down(const fp& a, unsigned d) {
  fp r;
  LB_UNROLL for (int j = 0; j < 12; j++) r.v[j] = __shfl_down(a.v[j], d, 64);
  return r;
}
template <bool kInl = false>
__device__ __forceinline__ fp fp_inv_block(const fp& z) {
  constexpr int NW = LB_INV_TPB / 64;
  __shared__ uint32_t s_tot[NW][12];
  __shared__ uint32_t s_inv[12];
  const unsigned lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  fp pre = z, suf = z;  // inclusive prefix / suffix products within the wave
  for (unsigned d = 1; d < 64; d <<= 1) {
    fp t = fp_shfl_up(pre, d);
    if (lane >= d) pre = fp_mul(pre, t);
  }
  for (unsigned d = 1; d < 64; d <<= 1) {
    fp t = fp_shfl_down(suf, d);
    if (lane + d < 64) suf = fp_mul(suf, t);
  }
  if (lane == 63) LB_UNROLL for (int j = 0; j < 12; j++) s_tot[wv][j] = pre.v[j];
  __syncthreads();
  if (wv == 0) {
    fp t = fp_load(s_tot[0]);
    for (int w = 1; w < NW; w++) t = fp_mul(t, fp_load(s_tot[w]));
    if constexpr (kInl) t = fp_inv_i(t);
    else t = fp_inv(t);
    if (lane == 0) LB_UNROLL for (int j = 0; j < 12; j++) s_inv[j] = t.v[j];
  }
  __syncthreads();
  fp winv = fp_load(s_inv);  // (product of all wave totals)^-1 -> this wave's total^-1
  for (int w = 0; w < NW; w++)
    if (w != (int)wv) winv = fp_mul(winv, fp_load(s_tot[w]));
  fp pe = fp_shfl_up(pre, 1), se = fp_shfl_down(suf, 1);
  if (lane == 0) pe = fp_one();
  if (lane == 63) se = fp_one();
  return fp_mul(fp_mul(pe, se), winv);
}

// ---------------------------------------------------------------- signatures
// Signature.fromBytes(sig, affine, validate=true) in two kernels, each small enough to run at two
// waves per SIMD without register spills (one kernel doing both spilled ~2.2 KB per lane, i.e.
// ~1.3 GB of scratch traffic per 116k-set launch, and its per-dispatch scratch grant exhausted
// the runtime's pool at 8 batches in flight):
//   k_decompress_sigs  ZCash decode + Fp2 square root  -> affine point (SoA + AoS), status
//   k_sig_subgroup     Scott's psi check on the decoded points whose status is still OK
// sig_status: LB_OK / decode error / LB_POINT_NOT_IN_GROUP / LB_INVALID_SIZE (host-flagged)
#if LB_KG(0)
__global__ void __launch_bounds__(LB_TPB, LB_MINW_DEC) k_decompress_sigs(uint32_t n, const uint8_t* __restrict__ sigs,
                                                            const uint32_t* __restrict__ sig_sizes,
                                                            uint32_t* __restrict__ sig_aff,
                                                            uint4* __restrict__ sig_aos,
                                                            uint32_t* __restrict__ sig_inf,
                                                            int32_t* __restrict__ sig_status) {
  uint32_t i = lb_tid();
  if (i >= n) return;
  int st = LB_OK;
  g2a a;
  bool inf = false;
  if (sig_sizes != nullptr && sig_sizes[i] != 96) {
    st = LB_INVALID_SIZE;
    a.x = fp2_zero();
    a.y = fp2_zero();
  } else {
    uint32_t w[24];
    const uint4* s = reinterpret_cast<const uint4*>(sigs + (size_t)96 * i);
    LB_UNROLL for (int k = 0; k < 6; k++) {
      const uint4 v = s[k];
      w[4 * k] = v.x, w[4 * k + 1] = v.y, w[4 * k + 2] = v.z, w[4 * k + 3] = v.w;
    }
    st = g2_decompress96_w(w, a, inf);
  }
  soa_st(sig_aff, n, i, a);
  // array-of-structures copy (192 B per set) for the MSM's gathers: one point = 12 x 16 B
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&a);
  LB_UNROLL for (int k = 0; k < 12; k++) sig_aos[(size_t)12 * i + k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
  sig_inf[i] = inf ? 1u : 0u;
  sig_status[i] = st;
}
#endif  // LB_KG

#if LB_KG(1)
__global__ void __launch_bounds__(LB_TPB, LB_MINW_SUB) k_sig_subgroup(uint32_t n, const uint32_t* __restrict__ sig_aff,
                                                         const uint32_t* __restrict__ sig_inf,
                                                         int32_t* __restrict__ sig_status) {
  uint32_t i = lb_tid();
  if (i >= n) return;
  if (sig_status[i] != LB_OK || sig_inf[i]) return;
  // Scott's test psi(P) == [x]P with [|x|]P by the register-lean ladder (lb_curve.h).  P is
  // re-read from memory coordinate by coordinate where the additions use it, through a base
  // pointer re-derived at each read: otherwise the compiler hoists the 48 row addresses (96
  // VGPRs) out of the ladder and spills them (696 B of private segment per lane before)
  auto load_f2 = [&](int o) {
    const uint32_t* base = sig_aff;
    asm volatile("" : "+s"(base));
    fp2 a;
    uint32_t* w = reinterpret_cast<uint32_t*>(&a);
    LB_UNROLL for (int k = 0; k < 24; k++) w[k] = __builtin_nontemporal_load(base + (size_t)(k + o) * n + i);
    return a;
  };
  g2j acc = jac_from_aff(g2a{load_f2(0), load_f2(24)});
  // the exceptional additions (acc == +-P: points of small order outside G2) reuse the loop's one
  // doubling: acc = P, and the next pass's doubling yields acc + P = 2P for the same bit (redo)
  bool redo = false;
#pragma clang loop unroll(disable)
  for (int b = 62; b >= 0;) {
    g2_dbl_lean<LB_SUBGROUP_INL>(acc);
    if (redo) {
      redo = false;
      b--;
      continue;
    }
    if ((LB_X_ABS >> b) & 1ull) {
      if (jac_is_inf(acc)) {
        acc = jac_from_aff(g2a{load_f2(0), load_f2(24)});
        b--;
        continue;
      }
      // acc + P (madd-2007-bl with Z3 = 2 Z1 H), ordered so Z1Z1 dies before the Karatsuba temporaries
      const fp2 Z1Z1 = lean2_sqr<LB_SUBGROUP_INL>(acc.z);
      const fp2 H = fp2_sub(lean2_mul<LB_SUBGROUP_INL>(load_f2(0), Z1Z1), acc.x);
      const fp2 t = lean2_mul<LB_SUBGROUP_INL>(acc.z, Z1Z1);
      const fp2 rr = fp2_dbl(fp2_sub(lean2_mul<LB_SUBGROUP_INL>(load_f2(24), t), acc.y));
      if (fp2_is_zero(H)) {
        if (fp2_is_zero(rr)) {  // acc == P
          acc = jac_from_aff(g2a{load_f2(0), load_f2(24)});
          redo = true;
        } else {  // acc == -P
          acc = jac_infinity<fp2>();
          b--;
        }
        continue;
      }
      acc.z = fp2_dbl(lean2_mul<LB_SUBGROUP_INL>(acc.z, H));
      const fp2 I = fp2_mul4(lean2_sqr<LB_SUBGROUP_INL>(H));
      const fp2 J = lean2_mul<LB_SUBGROUP_INL>(H, I);
      const fp2 V = lean2_mul<LB_SUBGROUP_INL>(acc.x, I);
      const fp2 YJ = fp2_dbl(lean2_mul<LB_SUBGROUP_INL>(acc.y, J));
      acc.x = fp2_sub(fp2_sub(lean2_sqr<LB_SUBGROUP_INL>(rr), J), fp2_dbl(V));
      acc.y = fp2_sub(lean2_mul<LB_SUBGROUP_INL>(rr, fp2_sub(V, acc.x)), YJ);
    }
    b--;
  }
  bool ok = !jac_is_inf(acc);  // psi(P) is finite
  if (ok) {
    const fp2 z2 = lean2_sqr<LB_SUBGROUP_INL>(acc.z);
    ok = fp2_eq(lean2_mul<LB_SUBGROUP_INL>(lean2_mul<LB_SUBGROUP_INL>(fp2_conj(load_f2(0)), fp2_load(LB_PSI_CX)), z2),
                acc.x);
    if (ok) {
      const fp2 py = lean2_mul<LB_SUBGROUP_INL>(fp2_conj(load_f2(24)), fp2_load(LB_PSI_CY));
      ok = fp2_eq(lean2_mul<LB_SUBGROUP_INL>(lean2_mul<LB_SUBGROUP_INL>(py, z2), acc.z), fp2_neg(acc.y));
    }
  }
  if (!ok) sig_status[i] = LB_POINT_NOT_IN_GROUP;
}
#endif  // LB_KG

// The same test with 8 lanes per signature (lb_group.h), for small batches (a 1-set call, a
// block): the |x| ladder's 63 doublings take 3 product levels each instead of 16 serial products.
#if LB_KG(1)
__global__ void __launch_bounds__(64) k_sig_subgroup_g8(uint32_t n, const uint32_t* __restrict__ sig_aff,
                                                        const uint32_t* __restrict__ sig_inf,
                                                        int32_t* __restrict__ sig_status) {
  __shared__ uint32_t g8s[8 * 72];  // the point, per group (re-read at the additions, not held)
  const uint32_t i = blockIdx.x * 8 + (threadIdx.x >> 3);
  if (i >= n) return;  // uniform within the group
  if (sig_status[i] != LB_OK || sig_inf[i]) return;
  lds_u32* G = (lds_u32*)g8s + (threadIdx.x >> 3) * 72;
  g8_stash(G, 0, jac_from_aff(soa_ld<g2a>(sig_aff, n, i)));
  const g2j acc = g8_mul_xabs_st(G, 0);
  bool ok = !jac_is_inf(acc);  // psi(P) is finite
  if (ok) ok = jac_eq(g8_psi(g8_unstash(G, 0)), jac_neg(acc));
  if (!ok && g8_q() == 0) sig_status[i] = LB_POINT_NOT_IN_GROUP;
}
#endif  // LB_KG

// The same check on the row engine for small batches while alone (one workgroup per signature):
// [|x|]P by the op list's fast ladder (a zero Z, the mark of any exceptional case, reruns it with
// the tested additions: inputs here are adversarial), psi(P) by one program, the comparison on
// thread 0 (jac_eq on the exported canonical words).
#if LB_KG(12)
__global__ void __launch_bounds__(LBR_NT) k_sig_subgroup_row(uint32_t n, const uint32_t* __restrict__ sig_aff,
                                                           const uint32_t* __restrict__ sig_inf,
                                                           int32_t* __restrict__ sig_status, uint32_t proj) {
  LBR_SHARED_N(S, LBR_PROGS_END - LBR_G2DBL);
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  if (sig_status[i] != LB_OK || sig_inf[i]) return;  // uniform
  r_init(S, LBR_PROGS_END - LBR_G2DBL, LBR_G2DBL);
  const int P = LBR_A(3), X = LBR_A(4), PSI = LBR_A(4) + 6;
  {
    const int t = r_tid();
    if (t < 6) {
      fp v;
      if (t < 4)
        LB_UNROLL for (int w = 0; w < 12; w++) v.v[w] = sig_aff[(size_t)(12 * t + w) * n + i];
      else
        v = t == 4 ? fp_one() : fp_zero();
      r_stage_fp(S, t, v);
    }
    r_sync();
    r_import_staged(S, P, 6);
  }
  if (proj) {
    // round 6: the [|x|] ladder in projective coordinates with the complete formulas (no
    // exceptional case, no rerun), then psi(P) = -acc <=> X1 Z2 = X2 Z1 and Y1 Z2 = -Y2 Z1 (PEQN;
    // an infinite acc leaves Y2 Z1 != 0)
    r_run(S, &LBR_OPS_XLADDER_P, LBR_OPS_XLADDER_P.n);
    r_g2_psi(S, PSI, P);
    r_gather(S, LBR_IN, 12, [&](int e) { return e < 6 ? PSI + e : X + e - 6; });
    r_exec(S, LBR_PEQN);
    const lds_i32* pq = r_progs(S) + LBR_PEQN;
    const uint32_t mz = r_zero_mask(S, 4, [&](int e) { return pq[2 + e]; });
    if (r_tid() == 0 && mz != 0xf) sig_status[i] = LB_POINT_NOT_IN_GROUP;
    return;
  }
  r_run(S, &LBR_OPS_XLADDER, LBR_OPS_XLADDER.n);
  if (r_zero_mask(S, 2, [&](int e) { return X + 4 + e; }) == 3) r_g2_mul_xabs<false>(S, X, P);
  r_g2_psi(S, PSI, P);
  // psi(P) == -acc on the row, from G2ADD's exceptional-case values (round 6: the lane-0 jac_eq
  // epilogue cost the kernel 1.5 KB of private segment per lane at the 1 024-thread workgroup's
  // 128 VGPRs): with both points finite, H = 0 <=> equal x, and then r = 0 <=> equal y, so
  // psi(P) = -acc <=> H = 0 and (r != 0 or y(acc) = 0).  Bits: 0-1 Z of psi(P), 2-3 Z of acc,
  // 4-5 H, 6-7 r, 8-9 y of acc (r_zero_mask tests canonical values: exact)
  r_gather(S, LBR_IN, 12, [&](int e) { return e < 6 ? PSI + e : X + e - 6; });
  r_exec(S, LBR_G2ADD);
  const lds_i32* prog = r_progs(S) + LBR_G2ADD;
  const uint32_t m = r_zero_mask(S, 10, [&](int e) {
    return e < 2 ? PSI + 4 + e : (e < 4 ? X + 2 + e : (e < 8 ? prog[4 + e] : X + 2 + (e - 8)));
  });
  const bool ok = (m & 0x3) != 0x3 && (m & 0xc) != 0xc && (m & 0x30) == 0x30 &&
                  ((m & 0xc0) != 0xc0 || (m & 0x300) == 0x300);
  if (r_tid() == 0 && !ok) sig_status[i] = LB_POINT_NOT_IN_GROUP;
}
#endif  // LB_KG

// ---------------------------------------------------------------- hash_to_G2
// ---- expand_message_xmd for a 32-byte message at word level (no byte buffers: the byte-wise
// SHA-256 message builder kept its buffers on the stack, ~1.5 KB of private segment per lane).
// With DST' = DST || 43 (44 bytes), every SHA-256 block but the message's own is constant:
//   b0 = H(Z_pad || msg || 01 00 || 00 || DST')  blocks: zeros | msg, 01 00 00, DST'[0..28] | DST'[29..43], pad
//   bi = H((b0 ^ b_{i-1}) || i || DST')         blocks: X, i, DST'[0..30] | DST'[31..43], pad
typedef uint32_t lb_v8u __attribute__((ext_vector_type(8)));
static __device__ __attribute__((noinline)) lb_v8u sha256_compress_v(lb_v8u hv, lb_v16u bv) {
  uint32_t h[8], blk[16];
  LB_UNROLL for (int i = 0; i < 8; i++) h[i] = hv[i];
  LB_UNROLL for (int i = 0; i < 16; i++) blk[i] = bv[i];
  sha256_compress(h, blk);
  lb_v8u r;
  LB_UNROLL for (int i = 0; i < 8; i++) r[i] = h[i];
  return r;
}
__device__ __forceinline__ uint32_t dst_byte(int k) { return k < LB_DST_LEN + 1 ? (uint32_t)LB_DST[k] : 0u; }
__device__ __forceinline__ uint32_t dst_word(int k) {  // big-endian word of DST' bytes [k, k + 4)
  return (dst_byte(k) << 24) | (dst_byte(k + 1) << 16) | (dst_byte(k + 2) << 8) | dst_byte(k + 3);
}
__device__ __forceinline__ lb_v8u sha256_iv_v() {
  lb_v8u h;
  h[0] = 0x6a09e667; h[1] = 0xbb67ae85; h[2] = 0x3c6ef372; h[3] = 0xa54ff53a;
  h[4] = 0x510e527f; h[5] = 0x9b05688c; h[6] = 0x1f83d9ab; h[7] = 0x5be0cd19;
  return h;
}
// field element u_which (which = 0: bytes [0, 128) of the 256-byte output, 1: [128, 256)) of
// hash_to_field(msg, 2) for the 32-byte message with big-endian words M
__device__ __forceinline__ fp2 hash_to_field_u(const uint32_t M[8], int which) {
  const lb_v8u iv = sha256_iv_v();
  lb_v16u blk;
  LB_UNROLL for (int i = 0; i < 16; i++) blk[i] = 0u;
  lb_v8u b0 = sha256_compress_v(iv, blk);  // the zero block Z_pad
  LB_UNROLL for (int i = 0; i < 8; i++) blk[i] = M[i];
  blk[8] = 0x01000000u | dst_byte(0);
  LB_UNROLL for (int i = 9; i < 16; i++) blk[i] = dst_word(4 * i - 35);
  b0 = sha256_compress_v(b0, blk);
  LB_UNROLL for (int i = 0; i < 4; i++) blk[i] = dst_word(29 + 4 * i);
  blk[3] = (dst_byte(41) << 24) | (dst_byte(42) << 16) | (dst_byte(43) << 8) | 0x80u;
  LB_UNROLL for (int i = 4; i < 15; i++) blk[i] = 0u;
  blk[15] = 143u * 8u;
  b0 = sha256_compress_v(b0, blk);
  uint32_t out[32];
  lb_v8u prev = b0 ^ b0;  // zero
  LB_UNROLL for (int i = 1; i <= 8; i++) {
    if ((i - 1) / 4 > which) break;  // later blocks belong to the other element
    lb_v16u bb;
    LB_UNROLL for (int k = 0; k < 8; k++) bb[k] = b0[k] ^ prev[k];
    bb[8] = ((uint32_t)i << 24) | (dst_byte(0) << 16) | (dst_byte(1) << 8) | dst_byte(2);
    LB_UNROLL for (int k = 9; k < 16; k++) bb[k] = dst_word(4 * k - 33);
    lb_v8u bi = sha256_compress_v(iv, bb);
    LB_UNROLL for (int k = 0; k < 3; k++) bb[k] = dst_word(31 + 4 * k);
    bb[3] = (dst_byte(43) << 24) | 0x00800000u;
    LB_UNROLL for (int k = 4; k < 15; k++) bb[k] = 0u;
    bb[15] = 77u * 8u;
    bi = sha256_compress_v(bi, bb);
    prev = bi;
    if ((i - 1) / 4 == which) LB_UNROLL for (int k = 0; k < 8; k++) out[8 * ((i - 1) & 3) + k] = bi[k];
  }
  return fp2{fp_from_be64_words(out), fp_from_be64_words(out + 16)};
}
// inline pieces of map_to_curve_g2 (register arguments only: by-value structs go through the stack)
__device__ __forceinline__ fp2 fp2_inv_i(const fp2& a) {
  const fp ni = fp_inv_i(fp_add(fp_sqr(a.c0), fp_sqr(a.c1)));
  return fp2{fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni))};
}
// binary Jacobi symbol (the fallback when posdivsteps has not settled)
__device__ __forceinline__ bool fp_is_square_bin_i(const fp& a) {
  if (fp_is_zero(a)) return true;
  uint32_t u[12], v[12];
  const uint32_t Pl[12] = {LB_P0, LB_P1, LB_P2, LB_P3, LB_P4, LB_P5, LB_P6, LB_P7, LB_P8, LB_P9, LB_P10, LB_P11};
  LB_UNROLL for (int j = 0; j < 12; j++) {
    u[j] = a.v[j];
    v[j] = Pl[j];
  }
  int t = 1;  // as fp_is_square (binary Jacobi symbol on the Montgomery form)
  while (true) {
    while (u[0] == 0) {
      LB_UNROLL for (int j = 0; j < 11; j++) u[j] = u[j + 1];
      u[11] = 0;
    }
    int k = lb_ctz32(u[0]);
    if (k) {
      lb_shr(u, k);
      uint32_t v8 = v[0] & 7u;
      if ((k & 1) && (v8 == 3u || v8 == 5u)) t = -t;
    }
    if (lb_is_one_plain(u)) return t == 1;
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
    if (zero) return false;
  }
}
#ifndef LB_JAC_SG
#define LB_JAC_SG 1  // 0: the binary Jacobi symbol only (A/B)
#endif
__device__ __forceinline__ bool fp_is_square_i(const fp& a) {
  if (LB_JAC_SG) {
    const int s = fp_is_square_sg(a);  // (aR | p) = (a | p): R = 2^384 is a square
    if (s >= 0) return s == 1;
  }
  return fp_is_square_bin_i(a);
}
// map_to_curve_g2 (SSWU + 3-isogeny, lb_h2c.h) with the inline pieces above; ROW: the square
// root's two exponentiations on the lane's 16-lane row (r1_pow_const; every lane of the row runs
// the same item)
template <bool ROW = false>
__device__ __forceinline__ g2j map_to_curve_g2_i(const fp2& u) {
  const fp2 A = fp2_load(LB_SSWU_A), B = fp2_load(LB_SSWU_B), Z = fp2_load(LB_SSWU_Z);
  const fp2 zu2 = fp2_mul(Z, fp2_sqr(u));
  const fp2 tv1 = fp2_add(fp2_sqr(zu2), zu2);
  const bool exc = fp2_is_zero(tv1);
  fp2 x1 = fp2_mul(fp2_load(LB_SSWU_MBDIVA), fp2_add(fp2_one(), fp2_inv_i(tv1)));
  x1 = fp2_select(exc, fp2_load(LB_SSWU_BDIVZA), x1);
  const fp2 gx1 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1), A), x1), B);
  const fp2 x2 = fp2_mul(zu2, x1);
  const fp2 gx2 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x2), A), x2), B);
  const bool sq1 = fp_is_square_i(fp_add(fp_sqr(gx1.c0), fp_sqr(gx1.c1)));
  const fp2 x = fp2_select(sq1, x1, x2);
  fp2 y;
  if constexpr (ROW)
    fp2_sqrt_p(y, fp2_select(sq1, gx1, gx2), [](const fp& a, const uint32_t* e, int top) { return r1_pow_const(a, e, top); });
  else
    fp2_sqrt_i<true>(y, fp2_select(sq1, gx1, gx2));
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  const fp2 xx = fp2_sqr(x), xxx = fp2_mul(xx, x);
  const fp2 xn = fp2_add(fp2_add(fp2_add(fp2_mul(fp2_load(LB_ISO_XNUM3), xxx), fp2_mul(fp2_load(LB_ISO_XNUM2), xx)),
                                 fp2_mul(fp2_load(LB_ISO_XNUM1), x)),
                         fp2_load(LB_ISO_XNUM0));
  const fp2 xd = fp2_add(fp2_add(xx, fp2_mul(fp2_load(LB_ISO_XDEN1), x)), fp2_load(LB_ISO_XDEN0));
  const fp2 yn = fp2_add(fp2_add(fp2_add(fp2_mul(fp2_load(LB_ISO_YNUM3), xxx), fp2_mul(fp2_load(LB_ISO_YNUM2), xx)),
                                 fp2_mul(fp2_load(LB_ISO_YNUM1), x)),
                         fp2_load(LB_ISO_YNUM0));
  const fp2 yd = fp2_add(fp2_add(fp2_add(xxx, fp2_mul(fp2_load(LB_ISO_YDEN2), xx)), fp2_mul(fp2_load(LB_ISO_YDEN1), x)),
                         fp2_load(LB_ISO_YDEN0));
  g2j r;
  const fp2 yd2 = fp2_sqr(yd);
  r.z = fp2_mul(xd, yd);
  r.x = fp2_mul(fp2_mul(xn, xd), yd2);
  r.y = fp2_mul(fp2_mul(fp2_mul(y, yn), fp2_mul(fp2_sqr(xd), xd)), yd2);
  return r;
}

// Hashing runs once per DISTINCT signing root (k_msg_insert below): launched over 2 nu threads
// (nu = distinct roots, read back by the host); thread t handles unique message t % nu, field
// element u_{t / nu}; output Jacobian points q (stride 2n: u_0 of root u at u, u_1 at n + u).
#if LB_KG(2)
__global__ void __launch_bounds__(LB_TPB, LB_MINW) k_hash_map(uint32_t n, uint32_t nu,
                                                     const uint32_t* __restrict__ uniq_set,
                                                     const uint8_t* __restrict__ msgs, uint32_t* __restrict__ q) {
  const uint32_t t = lb_tid();
  if (t >= 2 * nu) return;
  const uint32_t which = t < nu ? 0u : 1u;
  const uint32_t u = which ? t - nu : t;
  const uint4* m4 = reinterpret_cast<const uint4*>(msgs + (size_t)32 * uniq_set[u]);
  uint32_t M[8];
  LB_UNROLL for (int i = 0; i < 2; i++) {
    const uint4 v = m4[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    LB_UNROLL for (int k = 0; k < 4; k++) M[4 * i + k] = __builtin_bswap32(w[k]);  // big-endian words
  }
  soa_st(q, 2 * n, which * n + u, map_to_curve_g2_i(hash_to_field_u(M, (int)which)));
}
#endif  // LB_KG
// k_decompress_sigs with 16 lanes per signature (4 per wave): every lane of a row decodes the
// same signature and the square root's exponentiations run as row products (r1_pow_const), for
// small batches on a device running alone.
#if LB_KG(13)
__global__ void __launch_bounds__(64) k_decompress_sigs_row(uint32_t n, const uint8_t* __restrict__ sigs,
                                                            const uint32_t* __restrict__ sig_sizes,
                                                            uint32_t* __restrict__ sig_aff, uint4* __restrict__ sig_aos,
                                                            uint32_t* __restrict__ sig_inf,
                                                            int32_t* __restrict__ sig_status) {
  const uint32_t i = (blockIdx.x * 64 + threadIdx.x) >> (LB_H2C_FOLD ? 5 : 4);  // a row pair (r2_pow_const) / a row
  const uint32_t ic = i < n ? i : n - 1;  // rows past the end decode the last signature again
  int st = LB_OK;
  g2a a;
  bool inf = false;
  if (sig_sizes != nullptr && sig_sizes[ic] != 96) {
    st = LB_INVALID_SIZE;
    a.x = fp2_zero();
    a.y = fp2_zero();
  } else {
    uint32_t w[24];
    const uint4* s = reinterpret_cast<const uint4*>(sigs + (size_t)96 * ic);
    LB_UNROLL for (int k = 0; k < 6; k++) {
      const uint4 v = s[k];
      w[4 * k] = v.x, w[4 * k + 1] = v.y, w[4 * k + 2] = v.z, w[4 * k + 3] = v.w;
    }
#if LB_H2C_FOLD
    st = g2_decompress96_wp(w, a, inf, [](const fp& x, const uint32_t* e, int top) { return r2_pow_const(x, e, top); });
#else
    st = g2_decompress96_wp(w, a, inf, [](const fp& x, const uint32_t* e, int top) { return r1_pow_const(x, e, top); });
#endif
  }
  if (i >= n || (threadIdx.x & (LB_H2C_FOLD ? 31 : 15)) != 0) return;
  soa_st(sig_aff, n, i, a);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&a);
  LB_UNROLL for (int k = 0; k < 12; k++) sig_aos[(size_t)12 * i + k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
  sig_inf[i] = inf ? 1u : 0u;
  sig_status[i] = st;
}
#endif  // LB_KG
// The same with 16 lanes per field element (4 per wave): the lanes of a row run the same item and
// share its square roots' exponentiations as row products (lb_row.h r1_pow_const), for batches
// with few distinct roots on a device running alone (latency: 1.5 -> ~0.6 ms per call).
#if LB_KG(13)
__global__ void __launch_bounds__(64) k_hash_map_row(uint32_t n, uint32_t nu, const uint32_t* __restrict__ uniq_set,
                                                     const uint8_t* __restrict__ msgs, uint32_t* __restrict__ q) {
#if LB_H2C_FOLD
  // two items per wave, a row PAIR each: map_to_curve_g2_fold with row products (rfp2 / rfp) and
  // the exponentiations on the pair (r2_pow_rf)
#if LBR_FP2_W4
  const uint32_t t = blockIdx.x;  // one item per wave (rfp2 products on its four rows)
  if (t >= 2 * nu) return;        // (whole wave)
#else
  const uint32_t t = (blockIdx.x * 64 + threadIdx.x) >> 5;
  if (blockIdx.x * 2 >= 2 * nu) return;  // (whole wave)
#endif
  const uint32_t tc = t < 2 * nu ? t : 2 * nu - 1;
  const uint32_t which = tc < nu ? 0u : 1u;
  const uint32_t u = which ? tc - nu : tc;
  const uint4* m4 = reinterpret_cast<const uint4*>(msgs + (size_t)32 * uniq_set[u]);
  uint32_t M[8];
  LB_UNROLL for (int i = 0; i < 2; i++) {
    const uint4 v = m4[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    LB_UNROLL for (int k = 0; k < 4; k++) M[4 * i + k] = __builtin_bswap32(w[k]);
  }
  const g2j r = map_to_curve_g2_fold_t<rfp2, rfp>(hash_to_field_u(M, (int)which),
                                                [](const rfp& a, const uint32_t* e, int top) { return r2_pow_rf(a, e, top); });
  if (t < 2 * nu && (threadIdx.x & (LBR_FP2_W4 ? 63 : 31)) == 0) soa_st(q, 2 * n, which * n + u, r);
#else
  const uint32_t t = (blockIdx.x * 64 + threadIdx.x) >> 4;
  if (blockIdx.x * 4 >= 2 * nu) return;  // (whole wave)
  const uint32_t tc = t < 2 * nu ? t : 2 * nu - 1;  // rows past the end recompute the last item
  const uint32_t which = tc < nu ? 0u : 1u;
  const uint32_t u = which ? tc - nu : tc;
  const uint4* m4 = reinterpret_cast<const uint4*>(msgs + (size_t)32 * uniq_set[u]);
  uint32_t M[8];
  LB_UNROLL for (int i = 0; i < 2; i++) {
    const uint4 v = m4[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    LB_UNROLL for (int k = 0; k < 4; k++) M[4 * i + k] = __builtin_bswap32(w[k]);
  }
  const g2j r = map_to_curve_g2_i<true>(hash_to_field_u(M, (int)which));
  if (t < 2 * nu && (threadIdx.x & 15) == 0) soa_st(q, 2 * n, which * n + u, r);
#endif
}
#endif  // LB_KG

// Lone-lane state parked in an engine-owned global buffer (word w of slot k of root u at
// st[(k * 72 + w) * n + u]: a wave's lanes touch consecutive words), so long-lived points do not
// stay in registers across a 63-step ladder.  The memory clobber ends the register copy's life:
// later uses reload.  The runtime's private segment (scratch) is reserved per HIP queue for the
// device's whole wave capacity, so kilobytes of spill per lane in any kernel cap the engines per
// device; this buffer is sized by the launch.
__device__ __forceinline__ void lane_park(uint32_t* __restrict__ st, uint32_t n, uint32_t u, int k, const g2j& p) {
  soa_st(st + (size_t)k * 72 * n, n, u, p);
  __asm__ volatile("" ::: "memory");
}
__device__ __forceinline__ g2j lane_unpark(const uint32_t* __restrict__ st, uint32_t n, uint32_t u, int k) {
  __asm__ volatile("" ::: "memory");
  return soa_ld<g2j>(st + (size_t)k * 72 * n, n, u);
}
__device__ __forceinline__ void lane_park_aff(uint32_t* __restrict__ st, uint32_t n, uint32_t u, int k, const g2a& p) {
  soa_st(st + (size_t)k * 72 * n, n, u, p);
  __asm__ volatile("" ::: "memory");
}
__device__ __forceinline__ g2a lane_unpark_aff(const uint32_t* __restrict__ st, uint32_t n, uint32_t u, int k) {
  __asm__ volatile("" ::: "memory");
  return soa_ld<g2a>(st + (size_t)k * 72 * n, n, u);
}
// [|x|] (affine point in slot k; `inf`: the point at infinity, whose multiple is infinity): lean
// inline doublings and mixed additions, the base re-read at the five additions
__device__ __forceinline__ g2j g2_mul_xabs_parked(const uint32_t* st, uint32_t n, uint32_t u, int k, bool inf) {
  if (inf) return jac_infinity<fp2>();
  g2j acc = jac_from_aff(lane_unpark_aff(st, n, u, k));
#pragma clang loop unroll(disable)
  for (int i = 62; i >= 0; i--) {
    g2_dbl_lean<true>(acc);
    if ((LB_X_ABS >> i) & 1ull) {
      if (jac_is_inf(acc))
        acc = jac_from_aff(lane_unpark_aff(st, n, u, k));
      else
        g2_add_aff_lean<true>(acc, lane_unpark_aff(st, n, u, k));
    }
  }
  return acc;
}
__device__ __forceinline__ void g2_add_aff_or(g2j& p, const g2a& q) {
  if (jac_is_inf(p))
    p = jac_from_aff(q);
  else
    g2_add_aff_lean<true>(p, q);
}
__device__ __forceinline__ g2a g2_psi_aff(const g2a& a) {
  return g2a{fp2_mul(fp2_conj(a.x), fp2_load(LB_PSI_CX)), fp2_mul(fp2_conj(a.y), fp2_load(LB_PSI_CY))};
}
__device__ __forceinline__ g2a g2a_neg(const g2a& a) { return g2a{a.x, fp2_neg(a.y)}; }
// Jacobian -> affine for every lane of the block (fp_inv_block: one inversion per block); inf
// reports the point at infinity (its affine value is then meaningless)
__device__ __forceinline__ g2a g2_to_aff_block(const g2j& h, bool act, bool& inf) {
  const fp nz = fp_add(fp_sqr(h.z.c0), fp_sqr(h.z.c1));
  inf = !act || fp_is_zero(nz);
  const fp ni = fp_inv_block<true>(inf ? fp_one() : nz);  // inline EEA: no by-value call frames
  const fp2 zi{fp_mul(h.z.c0, ni), fp_neg(fp_mul(h.z.c1, ni))};
  const fp2 zi2 = fp2_sqr(zi);
  return g2a{fp2_mul(h.x, zi2), fp2_mul(fp2_mul(h.y, zi2), zi)};
}

// p + q for Jacobian p and a PARKED Jacobian q (slot k, negated if neg): q's coordinates are
// read when each is needed, so p, q and the formula's temporaries are never live together
// (add-2007-bl with Z1 Z2 by one product; the exceptional cases as g2_add_lean)
__device__ __forceinline__ void g2_add_parked(g2j& p, const uint32_t* st, uint32_t n, uint32_t u, int k, bool neg) {
  const uint32_t* b = st + (size_t)k * 72 * n;
  auto ld2 = [&](int c) {  // coordinate c of q
    __asm__ volatile("" ::: "memory");
    return soa_ld<fp2>(b + (size_t)24 * c * n, n, u);
  };
  const fp2 qz = ld2(2);
  if (fp2_is_zero(qz)) return;  // q = infinity
  if (jac_is_inf(p)) {
    p = lane_unpark(st, n, u, k);
    if (neg) p = jac_neg(p);
    return;
  }
  const fp2 Z2Z2 = lean2_sqr<true>(qz);
  const fp2 Z1Z2 = lean2_mul<true>(p.z, qz);
  const fp2 U1 = lean2_mul<true>(p.x, Z2Z2);
  const fp2 S1 = lean2_mul<true>(lean2_mul<true>(p.y, qz), Z2Z2);
  const fp2 Z1Z1 = lean2_sqr<true>(p.z);
  const fp2 H = fp2_sub(lean2_mul<true>(ld2(0), Z1Z1), U1);
  fp2 S2 = lean2_mul<true>(lean2_mul<true>(ld2(1), p.z), Z1Z1);
  if (neg) S2 = fp2_neg(S2);
  const fp2 rr = fp2_dbl(fp2_sub(S2, S1));
  if (fp2_is_zero(H)) {
    if (fp2_is_zero(rr)) {
      p = lane_unpark(st, n, u, k);
      if (neg) p = jac_neg(p);
      g2_dbl_lean<true>(p);
    } else {
      p = jac_infinity<fp2>();
    }
    return;
  }
  p.z = fp2_dbl(lean2_mul<true>(Z1Z2, H));
  const fp2 I = lean2_sqr<true>(fp2_dbl(H));
  const fp2 J = lean2_mul<true>(H, I);
  const fp2 V = lean2_mul<true>(U1, I);
  p.x = fp2_sub(fp2_sub(lean2_sqr<true>(rr), J), fp2_dbl(V));
  p.y = fp2_sub(lean2_mul<true>(rr, fp2_sub(V, p.x)), fp2_dbl(lean2_mul<true>(S1, J)));
}

// block of LB_INV_TPB threads (fp_inv_block).  h_eff Q via psi (as g2_clear_cofactor) with the
// two [x] ladders over AFFINE bases (the block's batch inversions make them affine: mixed
// additions, 5 x 14 fewer products per ladder and a smaller live set) and the long-lived points
// parked (slots: 0 Q, 1 t1 = [x]Q, 2 t3, 3 t1 + psi(Q); 4 x 72 words per lane, stride pn >= grid).
#if LB_KG(3)
__global__ void __launch_bounds__(LB_INV_TPB, 1) k_hash_finish(uint32_t n, const uint32_t* __restrict__ n_u,
                                                                  const uint32_t* __restrict__ q,
                                                                  uint32_t* __restrict__ h_aff,
                                                                  uint32_t* __restrict__ park, uint32_t pn) {
  const uint32_t i = blockIdx.x * LB_INV_TPB + threadIdx.x;
  const uint32_t nu = *n_u;
  if (blockIdx.x * LB_INV_TPB >= nu) return;  // whole block idle (uniform: fp_inv_block is safe)
  const bool act = i < nu;
  const uint32_t ic = act ? i : nu - 1;  // idle lanes compute a live root's values, store nothing
  // (each lane parks in its own column i < pn)
  bool inf0, inf1, inf2;
  {
    g2j h = soa_ld<g2j>(q, 2 * n, ic);
    g2_add_parked(h, q, 2 * n, n + ic, 0, false);  // Q = Q0 + Q1 (Q1: element n + ic of q, "slot 0")
    lane_park_aff(park, pn, i, 0, g2_to_aff_block(h, act, inf0));
  }
  lane_park(park, pn, i, 1, jac_neg(g2_mul_xabs_parked(park, pn, i, 0, inf0)));  // t1 = [x] Q
  g2j b = lane_unpark(park, pn, i, 1);
  if (!inf0) {
    const g2a qa = lane_unpark_aff(park, pn, i, 0);
    g2j t3 = jac_from_aff(qa);
    g2_dbl_lean<true>(t3);
    t3 = g2_psi2(t3);
    g2_add_aff_or(t3, g2a_neg(g2_psi_aff(qa)));  // psi^2(2Q) - psi(Q)
    lane_park(park, pn, i, 2, t3);
    g2_add_aff_or(b, g2_psi_aff(qa));  // t1 + psi(Q)
  } else {
    lane_park(park, pn, i, 2, jac_infinity<fp2>());
  }
  lane_park_aff(park, pn, i, 3, g2_to_aff_block(b, act, inf1));
  lane_park(park, pn, i, 3, jac_neg(g2_mul_xabs_parked(park, pn, i, 3, inf1)));  // t2x = [x](t1 + psi(Q))
  g2j h = lane_unpark(park, pn, i, 2);
  g2_add_parked(h, park, pn, i, 3, false);
  g2_add_parked(h, park, pn, i, 1, true);
  if (!inf0) g2_add_aff_or(h, g2a_neg(lane_unpark_aff(park, pn, i, 0)));
  // H(m) == infinity has negligible probability; its z = 0 gives x = y = 0 as jac_to_aff would
  const g2a a = g2_to_aff_block(h, act, inf2);
  if (!act) return;
  soa_st(h_aff, n, i, inf2 ? g2a{fp2_zero(), fp2_zero()} : a);
}
#endif  // LB_KG

// The same with 8 lanes per root (lb_group.h: each G2 doubling in 3 levels of Fp products, each
// addition in 6), for batches with few distinct roots, where k_hash_finish's lone-lane
// cofactor clearing (~2 700 serial Fp products) is the longest step of the per-root chain.
// Blocks of 64 threads = 8 roots; idle groups of the last block recompute the last root.
#if LB_KG(8)
__global__ void __launch_bounds__(64) k_hash_finish_g8(uint32_t n, const uint32_t* __restrict__ n_u,
                                                       const uint32_t* __restrict__ q, uint32_t* __restrict__ h_aff) {
  __shared__ uint32_t g8s[8 * 4 * 72];  // g8_clear_cofactor_st's points, per group
  const uint32_t nu = *n_u;
  if (blockIdx.x * 8 >= nu) return;  // whole block idle (uniform: fp_inv_block is safe)
  const uint32_t u = blockIdx.x * 8 + (threadIdx.x >> 3);
  const bool act = u < nu;
  const uint32_t uc = act ? u : nu - 1;
  g2j h = soa_ld<g2j>(q, 2 * n, uc);
  g8_add(h, soa_ld<g2j>(q, 2 * n, n + uc));
  h = g8_clear_cofactor_st(h, (lds_u32*)g8s + (threadIdx.x >> 3) * 4 * 72);
  const fp nz = fp_add(fp_sqr(h.z.c0), fp_sqr(h.z.c1));
  const bool zero = fp_is_zero(nz);
  const fp ni = fp_inv_block(zero ? fp_one() : nz);
  if (!act || g8_q() != 0) return;
  g2a a;
  if (zero) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  } else {
    const fp2 zi{fp_mul(h.z.c0, ni), fp_neg(fp_mul(h.z.c1, ni))};
    const fp2 zi2 = fp2_sqr(zi);
    a.x = fp2_mul(h.x, zi2);
    a.y = fp2_mul(fp2_mul(h.y, zi2), zi);
  }
  soa_st(h_aff, n, u, a);
}
#endif  // LB_KG

// The same with one workgroup (LBR_NT threads) per root on the row engine (lb_row.h
// r_g2_clear_cofactor: each Fp product of a doubling / addition on a 16-lane row), for a device
// running alone with few distinct roots: ~2.3x shorter than k_hash_finish_g8's chain.  Z^-1 on
// thread 0 (safegcd).
#if LB_KG(12)
__global__ void __launch_bounds__(LBR_NT) k_hash_finish_row(uint32_t n, const uint32_t* __restrict__ n_u,
                                                          const uint32_t* __restrict__ q, uint32_t* __restrict__ h_aff,
                                                          uint32_t careful) {
  LBR_SHARED_N(S, LBR_PROGS_END - LBR_G2DBL);
  const uint32_t u = blockIdx.x;
  if (u >= *n_u) return;
  r_init(S, LBR_PROGS_END - LBR_G2DBL, LBR_G2DBL);
  const int Q0 = LBR_A(3), Q1 = LBR_A(3) + 6, H = LBR_A(4);
  {
    const int t = r_tid();
    if (t < 12) {  // Q0 (element u of q) into Q0, Q1 (element n + u) into Q1
      const uint32_t e = t < 6 ? u : n + u, c = t < 6 ? t : t - 6;
      fp v;
      LB_UNROLL for (int w = 0; w < 12; w++) v.v[w] = q[(size_t)(12 * c + w) * (2 * n) + e];
      r_stage_fp(S, t, v);
    }
    r_sync();
    r_import_staged(S, Q0, 12);
  }
  // careful bit 0 (LB_HASH_ROW_CAREFUL, tests): the Jacobian chain with the exceptional-case
  // tests; bit 1 (LB_ROW_PROJ=0): the Jacobian fast chain (rerun with the tests on Z = 0).
  // Default (round 6): projective coordinates, complete additions, no rerun.
  const bool proj = careful == 0;
  if (proj) {
    r_g2_prog(S, LBR_JTOP, Q0, Q0);
    r_g2_prog(S, LBR_JTOP, Q1, Q1);
    r_run(S, &LBR_OPS_HASH_P, LBR_OPS_HASH_P.n);  // Q0 + Q1, cofactor clearing into H
  } else {
    r_copy(S, LBR_A(5), Q0, 12);  // Q0, Q1 kept for a recomputation
    r_run(S, &LBR_OPS_HASH, LBR_OPS_HASH.n);  // Q0 + Q1, cofactor clearing into H (fast path)
    // Z = 0 (or `careful` bit 0, LB_HASH_ROW_CAREFUL for the tests): again with the tests
    if (r_zero_mask(S, 2, [&](int e) { return H + 4 + e; }) == 3 || (careful & 1)) {
      r_copy(S, Q0, LBR_A(5), 12);
      r_g2_add(S, Q0, Q0, Q1);
      r_g2_clear_cofactor<false>(S, H, Q0);
    }
  }
  r_export(S, H, 6);
  if (r_tid() == 0) {
    g2j h;
    h.x = fp2{r_fp_of_staged(S, 0), r_fp_of_staged(S, 1)};
    h.y = fp2{r_fp_of_staged(S, 2), r_fp_of_staged(S, 3)};
    h.z = fp2{r_fp_of_staged(S, 4), r_fp_of_staged(S, 5)};
    const fp nz = fp_add(fp_sqr(h.z.c0), fp_sqr(h.z.c1));
    g2a a;
    if (fp_is_zero(nz)) {  // H(m) = O (negligible probability): x = y = 0 as the other forms
      a.x = fp2_zero();
      a.y = fp2_zero();
    } else {
      const fp ni = fp_inv_i(nz);
      const fp2 zi{fp_mul(h.z.c0, ni), fp_neg(fp_mul(h.z.c1, ni))};
      if (proj) {  // x = X / Z, y = Y / Z
        a.x = fp2_mul(h.x, zi);
        a.y = fp2_mul(h.y, zi);
      } else {  // x = X / Z^2, y = Y / Z^3
        const fp2 zi2 = fp2_sqr(zi);
        a.x = fp2_mul(h.x, zi2);
        a.y = fp2_mul(fp2_mul(h.y, zi2), zi);
      }
    }
    soa_st(h_aff, n, u, a);
  }
}
#endif  // LB_KG

// ---------------------------------------------------------------- pubkeys + blinding
// G1 aggregation (getAggregatedPubkey, utils.ts:5-16) is split into chunks of <= LB_PK_CHUNK
// keys so a 512-key sync aggregate costs one chunk's latency plus a short combine instead of
// 512 serial additions on one lane; chunk c covers pubkeys [chunk_lo[c], chunk_lo[c+1]) of one set.
#define LB_PK_CHUNK 16
#ifndef LB_PK_CHUNK_SMALL
#define LB_PK_CHUNK_SMALL 4  // ... for batches of up to row_max sets (lb_engine.hip batch_fill)
#endif
// chunk_lo[c] bit 31: chunk c is its set's first (lb_engine.hip batch_fill; the sentinel
// chunk_lo[nc] carries it too)
#define LB_CHUNK_FIRST 0x80000000u
#define LB_CHUNK_LO(v) ((v) & 0x7fffffffu)

// Round 6: the chunk sums of one set are combined by a segmented shuffle tree over the wave (64
// chunks per wave, one workgroup = one wave) instead of serially on one lane in k_pk_blind: lane
// t's segment is the run of lanes of its set inside the wave (heads from the LB_CHUNK_FIRST flags
// by ballot), and after log2(64) levels the segment's first lane holds the segment's sum.  A set's
// sum is then the sum of its segment heads: its first chunk and every later chunk at a wave
// boundary (c % 64 == 0), at most 1 + ceil(chunks / 64) of them (k_pk_blind).  The same for the
// per-root sums of a batch alone (k_gsum_wave).  (north_star: tree reduction for G1 aggregation.)
__device__ __forceinline__ g1j g1j_shfl_down(const g1j& a, unsigned d) {
  return g1j{fp_shfl_down(a.x, d), fp_shfl_down(a.y, d), fp_shfl_down(a.z, d)};
}
// v: this lane's partial; rel: lanes of its segment before it; left: lanes of its segment from it on
template <class F>
__device__ __forceinline__ jac<F> wave_seg_sum(jac<F> v, uint32_t rel, uint32_t left) {
  LB_UNROLL for (uint32_t s = 1; s < 64; s <<= 1) {
    const jac<F> o = jac_as<F>(g1j_shfl_down(jac_as<fp>(v), s));
    if ((rel & (2 * s - 1)) == 0 && s < left) v = jac_add_i<F, true>(v, o);
  }
  return v;
}
// segments of the wave from per-lane "starts a segment" flags (inactive lanes: pass true)
__device__ __forceinline__ void wave_segments(bool starts, uint32_t& rel, uint32_t& left) {
  const uint64_t heads = __ballot(starts) | 1ull;  // the wave's first lane always starts one
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
  const uint32_t hl = 63 - __clzll(heads & upto);
  const uint64_t after = heads & ~upto;
  const uint32_t el = after ? (uint32_t)__ffsll((long long)after) - 1 : 64;
  rel = lane - hl;
  left = el - lane;
}
#if LB_KG(4)
__global__ void __launch_bounds__(LB_TPB, LB_MINW) k_pk_chunks(uint32_t nc, const uint32_t* __restrict__ chunk_lo,
                                                      const uint8_t* __restrict__ pks, uint32_t* __restrict__ chunk_acc,
                                                      int32_t* __restrict__ chunk_status) {
  uint32_t c = lb_tid();
  if (blockIdx.x * LB_TPB >= nc) return;  // whole wave idle (uniform)
  const bool act = c < nc;
  const uint32_t cl = act ? chunk_lo[c] : LB_CHUNK_FIRST;
  int st = LB_OK;
  g1j acc = jac_infinity<fp>();
  if (act) {
    const uint32_t a = LB_CHUNK_LO(cl), e = LB_CHUNK_LO(chunk_lo[c + 1]);
    for (uint32_t k = a; k < e && st == LB_OK; k++) {
      uint8_t b[96];
      ld_bytes<96>(b, pks + (size_t)96 * k);
      g1a p;
      bool inf;
      st = g1_deserialize96(b, p, inf);
      if (st == LB_OK && !inf) acc = jac_add_aff(acc, p);
    }
  }
  uint32_t rel, left;
  wave_segments((cl & LB_CHUNK_FIRST) != 0, rel, left);
  acc = wave_seg_sum(acc, rel, left);
  if (!act) return;
  soa_st(chunk_acc, nc, c, acc);
  chunk_status[c] = st;
}
#endif  // LB_KG

// The resident pubkey table (the epoch cache's index2pubkey, pubkeyCache.ts:56-77): one 128-byte
// record per key, words 0-23 the affine Montgomery point (g1a), word 24 the flag (decode status
// << 1) | is_infinity.  A gather by validator index touches one L2 line (a word-major layout
// touched 24 lines + 1 for the flag: with a mainnet-sized table every one a miss).
#define LB_TABLE_REC 32
// an affine G1 point with beta x (the GLV endomorphism [lambda]P = (beta x, y)): 144 B, AoS
struct g1x3 {
  fp x, y, bx;
};
__device__ __forceinline__ g1a table_ld(const uint32_t* __restrict__ table, uint32_t t) {
  return aos_ld<g1a>(table + (size_t)LB_TABLE_REC * t, 0);
}
__device__ __forceinline__ uint32_t table_flag_ld(const uint32_t* __restrict__ table, uint32_t t) {
  return table[(size_t)LB_TABLE_REC * t + 24];
}

// Same as k_pk_chunks over the resident pubkey table.  idx = pk_indices.
#if LB_KG(4)
__global__ void __launch_bounds__(LB_TPB, LB_MINW_G1) k_pk_chunks_idx(uint32_t nc, const uint32_t* __restrict__ chunk_lo,
                                                          const uint32_t* __restrict__ idx,
                                                          const uint32_t* __restrict__ table, uint32_t table_n,
                                                          uint32_t* __restrict__ chunk_acc,
                                                          int32_t* __restrict__ chunk_status) {
  uint32_t c = lb_tid();
  if (blockIdx.x * LB_TPB >= nc) return;  // whole wave idle (uniform)
  const bool act = c < nc;
  const uint32_t cl = act ? chunk_lo[c] : LB_CHUNK_FIRST;
  int st = LB_OK;
  jac<lb_g1f> acc = jac_infinity<lb_g1f>();
  if (act) {
    const uint32_t a = LB_CHUNK_LO(cl), e = LB_CHUNK_LO(chunk_lo[c + 1]);
    for (uint32_t k = a; k < e; k++) {
      uint32_t t = idx[k];
      if (t >= table_n) {
        st = LB_ERR_ARGUMENT;
        break;
      }
      const uint32_t fl = table_flag_ld(table, t);
      if (fl >> 1) {
        st = (int)(fl >> 1);
        break;
      }
      if (fl & 1u) continue;  // infinity contributes nothing to the aggregate
      acc = jac_add_aff_i<lb_g1f, true>(acc, aff_as<lb_g1f>(table_ld(table, t)));
    }
  }
  uint32_t rel, left;
  wave_segments((cl & LB_CHUNK_FIRST) != 0, rel, left);
  acc = wave_seg_sum(acc, rel, left);
  if (!act) return;
  soa_st(chunk_acc, nc, c, jac_as<fp>(acc));
  chunk_status[c] = st;
}
#endif  // LB_KG

// decode keys into the resident table (48 B compressed or 96 B uncompressed)
#if LB_KG(0)
__global__ void __launch_bounds__(LB_TPB, LB_MINW) k_table_fill(uint32_t n, const uint8_t* __restrict__ keys,
                                                       uint32_t key_size, int32_t validate, uint32_t first,
                                                       uint32_t* __restrict__ table, int32_t* __restrict__ status) {
  uint32_t i = lb_tid();
  if (i >= n) return;
  g1a a;
  bool inf = false;
  int st;
  if (key_size == 48) {
    uint8_t b[48];
    for (int k = 0; k < 48; k++) b[k] = keys[(size_t)48 * i + k];
    st = g1_decompress48(b, a, inf);
  } else {
    uint8_t b[96];
    for (int k = 0; k < 96; k++) b[k] = keys[(size_t)96 * i + k];
    st = g1_deserialize96(b, a, inf);
  }
  if (st == LB_OK && validate) {
    if (inf) {
      st = LB_PK_IS_INFINITY;
    } else {
      const uint32_t rr[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                              0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
      if (!jac_is_inf(jac_mul_u256(a, rr))) st = LB_POINT_NOT_IN_GROUP;
    }
  }
  if (st != LB_OK) {
    a.x = fp_zero();
    a.y = fp_zero();
  }
  uint32_t* rec = table + (size_t)LB_TABLE_REC * (first + i);
  aos_st(rec, 0, a);
  uint4 tail = {((uint32_t)st << 1) | (inf ? 1u : 0u), 0u, 0u, 0u};
  reinterpret_cast<uint4*>(rec)[6] = tail;
  status[i] = st;
}
#endif  // LB_KG

// pk_status: LB_OK / pubkey decode error / LB_EMPTY_AGGREGATE_ARRAY / LB_PK_IS_INFINITY
// r * PK (Jacobian) for the per-root sums; the affine aggregate PK itself -> pk_aff.  block of LB_INV_TPB threads (fp_inv_block)
#if LB_KG(4)
__global__ void __launch_bounds__(LB_INV_TPB, LB_MINW_G1) k_pk_blind(uint32_t n, uint32_t nc, const uint32_t* __restrict__ set_chunk_off,
                                                         const uint32_t* __restrict__ chunk_acc,
                                                         const int32_t* __restrict__ chunk_status,
                                                         uint32_t* __restrict__ pk_aff,
                                                         const uint64_t* __restrict__ scalars,
                                                         uint32_t* __restrict__ rpk,
                                                         int32_t* __restrict__ pk_status, uint32_t mode,
                                                         uint32_t* __restrict__ pk3) {
  // mode 0: all; 1: the aggregate, its status and affine form only (pk_status, pk_aff: what the
  // job statuses need, ahead of the ladder); 2: the ladder only, from mode 1's pk_status / pk_aff.
  // pk3 (mode 1, optional): (x, y, beta x) per set, AoS, for the per-root Straus sums
  // (k_gsum_straus), which then replace the ladder
  const uint32_t i = blockIdx.x * LB_INV_TPB + threadIdx.x;
  const bool act = i < n;
  int st = LB_ERR_ARGUMENT;
  g1j rj = jac_infinity<fp>();
  if (mode == 2) {  // uniform
    if (!act) return;
    st = pk_status[i];
    if (st == LB_OK && scalars[i] == 1) {  // the unblinded 1-set call: r PK = PK, kept affine (Z = 1)
      const g1a pk = soa_ld<g1a>(pk_aff, n, i);
      rj = g1j{pk.x, pk.y, fp_one()};
    } else if (st == LB_OK) {
      const g1a pk = soa_ld<g1a>(pk_aff, n, i);
      const g1a t2{fp_mul(pk.x, fp_load(LB_GLV_BETA)), pk.y};
      const g1a t3{fp_mul(pk.x, fp_load(LB_GLV_BETA2)), fp_neg(pk.y)};
#if LB_G1_INL
      rj = jac_as<fp>(jac_mul_glv_i<fpi, true>(aff_as<fpi>(pk), aff_as<fpi>(t2), aff_as<fpi>(t3), scalars[i]));
#else
      rj = jac_mul_glv_i<fp, true>(pk, t2, t3, scalars[i]);
#endif
    }
    aos_st(rpk, i, rj);
    return;
  }
  if (act) {
    uint32_t c0 = set_chunk_off[i], c1 = set_chunk_off[i + 1];
    st = (c0 == c1) ? LB_EMPTY_AGGREGATE_ARRAY : LB_OK;
    g1j acc = jac_infinity<fp>();
    // every chunk's status, the segment heads' sums (k_pk_chunks[_idx]: the set's first chunk and
    // its chunks at wave boundaries)
    for (uint32_t c = c0; c < c1 && st == LB_OK; c++) {
      st = chunk_status[c];
      if (st == LB_OK && (c == c0 || (c & (LB_TPB - 1)) == 0))
        acc = (c == c0) ? soa_ld<g1j>(chunk_acc, nc, c) : jac_add_i<fp, true>(acc, soa_ld<g1j>(chunk_acc, nc, c));
    }
    if (st == LB_OK && jac_is_inf(acc)) st = LB_PK_IS_INFINITY;
    rj = acc;
  }
  // aggregate -> affine for the GLV table.  A single key comes out of its chunk with Z = 1, so a
  // block of single-key sets (every attestation) skips the batched inversion.
  const bool ok = act && st == LB_OK;
  const fp one = fp_one();
  const bool need = ok && !fp_eq(rj.z, one);
  g1a pk;
  if (__syncthreads_or(need)) {
    const fp ai = fp_inv_block<true>(need ? rj.z : one);
    const fp ai2 = fp_sqr(ai);
    pk.x = fp_mul(rj.x, ai2);
    pk.y = fp_mul(fp_mul(rj.y, ai2), ai);
  } else {
    pk.x = rj.x;
    pk.y = rj.y;
  }
  if (mode == 1) {  // uniform
    if (!act) return;
    if (ok) soa_st(pk_aff, n, i, pk);
    if (pk3 != nullptr) aos_st(pk3, i, g1x3{pk.x, pk.y, ok ? fp_mul(pk.x, fp_load(LB_GLV_BETA)) : fp_zero()});
    pk_status[i] = st;
    return;
  }
  if (ok) {
    // r * PK with r = lo + hi * lambda: t2 = [lambda]PK = (beta x, y), t3 = PK + t2 = (beta^2 x, -y)
    const g1a t2{fp_mul(pk.x, fp_load(LB_GLV_BETA)), pk.y};
    const g1a t3{fp_mul(pk.x, fp_load(LB_GLV_BETA2)), fp_neg(pk.y)};
#if LB_G1_INL
    rj = jac_as<fp>(jac_mul_glv_i<fpi, true>(aff_as<fpi>(pk), aff_as<fpi>(t2), aff_as<fpi>(t3), scalars[i]));
#else
    rj = jac_mul_glv_i<fp, true>(pk, t2, t3, scalars[i]);
#endif
  } else {
    rj = jac_infinity<fp>();
  }
  if (!act) return;
  aos_st(rpk, i, rj);  // AoS: the per-root sums and the search gather it by member
  if (ok) soa_st(pk_aff, n, i, pk);  // the unblinded aggregate, for single-set checks of the search
  pk_status[i] = st;
}
#endif  // LB_KG

// k_pk_blind's mode 2 (the r PK ladder, from mode 1's pk_status / pk_aff) for small batches on a
// device running alone: ONE WAVE per set, its four rows four product units (lb_row.h w4_mul: every
// row holds the whole state, each level's independent products one per row, the results handed to
// every row by permlane swaps).  A doubling (dbl-2009-l) is 3 product levels, a doubling plus a
// mixed addition (madd-2007-bl) 6 (the addition's first products ride along with the doubling's),
// against 7 and 18 serial products: a C2 block's ladders ~0.9 ms of lone-lane products (round 5),
// ~0.45 ms with one row per set, ~0.1 ms here.
#if LB_KG(13)
__global__ void __launch_bounds__(64) k_pk_blind_rowp(uint32_t n, const uint32_t* __restrict__ pk_aff,
                                                     const uint64_t* __restrict__ scalars, uint32_t* __restrict__ rpk,
                                                     const int32_t* __restrict__ pk_status) {
  const uint32_t i = blockIdx.x;
  if (i >= n) return;  // (n = 0: the scratch reservation's empty dispatch)
  const int st = pk_status[i];
  const uint64_t w = scalars[i];
  g1j rj = jac_infinity<fp>();
  if (st == LB_OK) {  // uniform (one set per wave)
    const g1a pk = soa_ld<g1a>(pk_aff, n, i);
    if (w == 1) {  // the unblinded 1-set call: r PK = PK, affine (Z = 1)
      rj = g1j{pk.x, pk.y, fp_one()};
    } else {
      // t2 = [lambda]PK = (beta x, y), t3 = PK + t2 = (beta^2 x, -y), as k_pk_blind
      const aff<rfp> t1 = rf_of(pk);
      const aff<rfp> t2{f_mul(t1.x, rf_of(fp_load(LB_GLV_BETA))), t1.y};
      const aff<rfp> t3{f_mul(t1.x, rf_of(fp_load(LB_GLV_BETA2))), f_neg(t1.y)};
      // the ladder from the top non-zero digit with untested additions: PK is in G1 (prime order
      // r) and not O, and the running scalar A + B lambda (0 <= A, B < 2^33, growing by doubling
      // from the top digit) never equals +-(d0 + d1 lambda) for a digit d != 0 -- the lattice
      // {(a, b): a + b lambda = 0 mod r} has no non-zero vector with |a|, |b| < 2^64 (reduced
      // basis (x^2, 1), (-1, x^2 - 1)) -- so acc != +-T_d and acc != O at every addition
      // (madd-2007-bl's exceptional cases)
      const uint32_t k0 = (uint32_t)w, k1 = (uint32_t)(w >> 32);
      auto digit = [&](int b) { return ((k0 >> b) & 1u) | (((k1 >> b) & 1u) << 1); };
      int b = 31;
      while (b > 0 && digit(b) == 0) b--;  // w != 0 (the engine's scalars are non-zero)
      auto tab = [&](uint32_t d) { return d == 1u ? t1 : (d == 2u ? t2 : t3); };
      const aff<rfp> top = tab(digit(b));
      rfp X = top.x, Y = top.y, Z;
      f_set_one(Z);
      // lazy sums inside a step (lb_row.h lz_*: |v| < 32 p as product operands), the carried point
      // reduced at its end
      for (b--; b >= 0; b--) {
        const uint32_t d = digit(b);  // uniform
        // doubling: A = X^2, B = Y^2, YZ; C = B^2, P = (X + B)^2, F = E^2 (E = 3A); E (D - X3)
        rfp o[4];
        w4_mul<3>({X, Y, Y}, {X, Y, Z}, o);
        const rfp A = o[0], B = o[1], E = lz_mul(A, 3), XB = lz_add(X, B);
        const rfp Z3 = rf_red(2 * (int64_t)o[2].v);
        if (d == 0u) {
          w4_mul<3>({B, XB, E}, {B, XB, E}, o);
          const rfp C = o[0], D = lz_mul(lz_sub(lz_sub(o[1], A), C), 2);
          X = rf_red((int64_t)o[2].v - 2 * (int64_t)D.v);
          w4_mul<1>({E}, {lz_sub(D, X)}, o);
          Y = rf_red((int64_t)o[0].v - 8 * (int64_t)C.v);
          Z = Z3;
          continue;
        }
        const aff<rfp> q = tab(d);
        // ... with the addition's Z1Z1 = Z3^2 alongside
        w4_mul<4>({B, XB, E, Z3}, {B, XB, E, Z3}, o);
        const rfp C = o[0], D = lz_mul(lz_sub(lz_sub(o[1], A), C), 2), Z1Z1 = o[3];
        const rfp X3 = rf_red((int64_t)o[2].v - 2 * (int64_t)D.v);
        // E (D - X3); U2 = x2 Z1Z1; y2 Z3
        w4_mul<3>({E, q.x, q.y}, {lz_sub(D, X3), Z1Z1, Z3}, o);
        const rfp Y3 = rf_red((int64_t)o[0].v - 8 * (int64_t)C.v), H = lz_sub(o[1], X3), Y2Z = o[2];
        // S2 = y2 Z3 Z1Z1; HH = H^2; (Z3 + H)^2
        const rfp ZH = lz_add(Z3, H);
        w4_mul<3>({Y2Z, H, ZH}, {Z1Z1, H, ZH}, o);
        const rfp rr = lz_mul(lz_sub(o[0], Y3), 2), HH = o[1], I = lz_mul(HH, 4);
        Z = rf_red((int64_t)o[2].v - Z1Z1.v - HH.v);
        // J = H I; V = X3 I; rr^2
        w4_mul<3>({H, X3, rr}, {I, I, rr}, o);
        const rfp J = o[0], V = o[1];
        X = rf_red((int64_t)o[2].v - J.v - 2 * (int64_t)V.v);
        // rr (V - X); Y3 J
        w4_mul<2>({rr, Y3}, {lz_sub(V, X), J}, o);
        Y = rf_red((int64_t)o[0].v - 2 * (int64_t)o[1].v);
      }
      rj = rf_fp(jac<rfp>{X, Y, Z});
    }
  }
  if (threadIdx.x == 0) aos_st(rpk, i, rj);
}
#endif  // LB_KG

// Small batches on a device running alone, one WAVE per signature (lb_row.h w4_g2_*: the four
// rows of the wave as four product units; a doubling in 4 product levels, a mixed addition in 8):
// the 16-wave row-engine kernels need a whole CU each, and a block's 131 subgroup checks, 131
// r_i sig_i ladders and ~70 cofactor clearings (k_hash_finish_row) asked for more CUs than the
// device has, so the per-root chain waited for CUs.
// The subgroup check: Scott's psi(P) == [x]P as k_sig_subgroup, [|x|]P without the exceptional
// additions; a zero final Z (an exceptional case on the way, the inputs being adversarial, or
// [|x|]P = O) reruns the lane ladder with the tested additions (g2_aff_in_subgroup_i).
#if LB_KG(13)
__global__ void __launch_bounds__(64) k_sig_subgroup_w4(uint32_t n, const uint32_t* __restrict__ sig_aff,
                                                       const uint32_t* __restrict__ sig_inf,
                                                       int32_t* __restrict__ sig_status) {
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  if (sig_status[i] != LB_OK || sig_inf[i]) return;  // uniform
  const g2a P = soa_ld<g2a>(sig_aff, n, i);
  const rfp2* t2 = nullptr;
  const rfp2 px = fl_in(P.x, t2), py = fl_in(P.y, t2);
  rfp2 X = px, Y = py, Z;
  f_set_one(Z);
#pragma clang loop unroll(disable)
  for (int b = 62; b >= 0; b--) {
    w4_g2_dbl(X, Y, Z);
    if ((LB_X_ABS >> b) & 1ull) w4_g2_madd(X, Y, Z, px, py);
  }
  bool ok;
  if (fp2_is_zero(fl_out(Z))) {
    ok = g2_aff_in_subgroup_i(P);
  } else {
    // psi(P) = (conj(x) cx, conj(y) cy) == -[|x|]P = (X / Z^2, -Y / Z^3)
    const rfp2 Z2 = f_sqr(Z);
    const rfp2 sx = f_mul(fl_conj(px), fl_in(fp2_load(LB_PSI_CX), t2));
    const rfp2 sy = f_mul(fl_conj(py), fl_in(fp2_load(LB_PSI_CY), t2));
    ok = fp2_eq(fl_out(f_mul(sx, Z2)), fl_out(X)) && fp2_eq(fl_out(f_mul(f_mul(sy, Z2), Z)), fl_out(f_neg(Y)));
  }
  if (!ok && threadIdx.x == 0) sig_status[i] = LB_POINT_NOT_IN_GROUP;
}
#endif  // LB_KG
// r_i sig_i of every decoded set (k_sig_blind_row's GLV double-and-add over sig, [lambda] sig =
// -psi^2(sig), [1 + lambda] sig = -psi^4(sig), all affine) without the exceptional additions: for
// sig in G2 the running scalar never meets +-T_d (the GLV lattice argument of k_pk_blind_rowp);
// a set whose signature is not in G2 is not live, and k_g2_sum_g8 masks its term.
#if LB_KG(13)
__global__ void __launch_bounds__(64) k_sig_blind_w4(uint32_t n, const uint32_t* __restrict__ sig_aff,
                                                    const uint64_t* __restrict__ scalars,
                                                    const uint32_t* __restrict__ sig_inf, uint32_t* __restrict__ terms) {
  const uint32_t i = blockIdx.x;
  if (i >= n) return;  // (n = 0: the scratch reservation's empty dispatch)
  const uint64_t w = scalars[i];
  g2j r = jac_infinity<fp2>();
  if (!sig_inf[i] && w != 0) {  // uniform
    const g2a S = soa_ld<g2a>(sig_aff, n, i);
    const rfp2* t2p = nullptr;
    const rfp* t1p = nullptr;
    const rfp2 x1 = fl_in(S.x, t2p), y1 = fl_in(S.y, t2p);
    const rfp c2x = fl_in(fp_load(LB_PSI2_CX), t1p), c2y = fl_in(fp_load(LB_PSI2_CY), t1p);
    const rfp c4x = fl_in(fp_load(LB_PSI4_CX), t1p), c4y = fl_in(fp_load(LB_PSI4_CY), t1p);
    const rfp2 x2 = fl_mulb(x1, c2x), y2 = f_neg(fl_mulb(y1, c2y));
    const rfp2 x3 = fl_mulb(x1, c4x), y3 = f_neg(fl_mulb(y1, c4y));
    const uint32_t k0 = (uint32_t)w, k1 = (uint32_t)(w >> 32);
    auto digit = [&](int b) { return ((k0 >> b) & 1u) | (((k1 >> b) & 1u) << 1); };
    int b = 31;
    while (b > 0 && digit(b) == 0) b--;
    const uint32_t d0 = digit(b);
    rfp2 X = d0 == 1u ? x1 : (d0 == 2u ? x2 : x3), Y = d0 == 1u ? y1 : (d0 == 2u ? y2 : y3), Z;
    f_set_one(Z);
#pragma clang loop unroll(disable)
    for (b--; b >= 0; b--) {
      w4_g2_dbl(X, Y, Z);
      const uint32_t d = digit(b);  // uniform
      if (d != 0u) w4_g2_madd(X, Y, Z, d == 1u ? x1 : (d == 2u ? x2 : x3), d == 1u ? y1 : (d == 2u ? y2 : y3));
    }
    r = g2j{fl_out(X), fl_out(Y), fl_out(Z)};
  }
  if (threadIdx.x == 0) soa_st(terms, n, i, r);
}
#endif  // LB_KG

// ---------------------------------------------------------------- Miller loops
// ML(P_u, H(m_u)) with P_u = sum of r_i PK_i over the live sets signing m_u (bilinearity:
// prod_i e(r_i PK_i, H(m)) = e(sum_i r_i PK_i, H(m))), written straight into leaf m + u of the
// message product tree (stride 2m).  Three forms, picked per launch (lb_engine.hip):
//   * k_miller_lane: one lane per root, 64 roots per wave.  The fewest instructions per root
//     (the tower formulas compiled straight, operand sums computed once), but ~12 ms of serial
//     products per lane and a large private segment; the form when the device is shared with
//     other batches in flight, whose waves fill the SIMDs while these wait.
//   * k_miller_g8 (lb_group_exec.h): 8 lanes per root, 32 roots per workgroup, the state in LDS:
//     ~3x shorter, ~2.5x more VALU work per root; the form for a large batch alone on the device.
//   * k_miller_wave below: one wave per root, for batches with few distinct roots.
// One lane per root with the Fp12 accumulator f in LDS (two 72-word slots per lane,
// lane-interleaved: 36 KB per wave, so LDS allows the same one wave per SIMD as the registers)
// and T and a tower temporary parked in global memory.  Held in registers across ~100
// out-of-line product calls per step, f, T, the lines and the temporaries spilled 6.7 KB per
// lane to the private segment, which the runtime reserves per HIP queue for the device's whole
// wave capacity (the per-device engine cap).
#ifndef LB_MILLER_LANE_REG
#define LB_MILLER_LANE_REG 0
#endif
typedef __attribute__((address_space(3))) uint32_t lds_w;
template <int NL>  // slots [0, NL) in LDS (2: f; 3: f and the temporary), the rest in global memory
struct lane_lds {
  lds_w* L;         // slots 0, 1: f.c0, f.c1
  uint32_t* g;      // slot 2 (a temporary) and slot 3 (T): word i of slot k at g[((k - 2) * 72 + i) * n + u]
  uint32_t n, u;
  int lane;
  __device__ __forceinline__ void put(int k, const fp6& v) const {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
    if (k < NL)
      LB_UNROLL for (int i = 0; i < 72; i++) L[(k * 72 + i) * 64 + lane] = w[i];
    else
      LB_UNROLL for (int i = 0; i < 72; i++) g[((size_t)(k - 2) * 72 + i) * n + u] = w[i];
    __asm__ volatile("" ::: "memory");
  }
  __device__ __forceinline__ fp6 get(int k) const {
    __asm__ volatile("" ::: "memory");
    fp6 v;
    uint32_t* w = reinterpret_cast<uint32_t*>(&v);
    if (k < NL)
      LB_UNROLL for (int i = 0; i < 72; i++) w[i] = L[(k * 72 + i) * 64 + lane];
    else
      LB_UNROLL for (int i = 0; i < 72; i++) w[i] = g[((size_t)(k - 2) * 72 + i) * n + u];
    return v;
  }
};
// f <- f^2 = (c0' - t - v t) + 2 t w, t = a0 a1, c0' = (a0 + a1)(a0 + v a1)  (slots 0, 1: f; 2: t)
template <class S_t>
__device__ __forceinline__ void lane_f_sqr(const S_t& S) {
  fp6 s1, s2;
  {
    const fp6 a0 = S.get(0), a1 = S.get(1);
    S.put(2, fp6_mul_inl(a0, a1));
    s1 = fp6_add(a0, a1);
    s2 = fp6_add(a0, fp6_mul_v(a1));
  }
  const fp6 c0 = fp6_mul_inl(s1, s2);
  const fp6 t = S.get(2);
  S.put(0, fp6_sub(fp6_sub(c0, t), fp6_mul_v(t)));
  S.put(1, fp6_add(t, t));
}
// f <- f (l0 + l2 v + l3 v w)  (as fp12_mul_line_inl; slot 2 holds t1 = a1 l3)
template <class S_t>
__device__ __forceinline__ void lane_f_line(const S_t& S, const fp2& l0, const fp2& l2, const fp2& l3) {
  fp6 s;
  {
    const fp6 a1 = S.get(1);
    S.put(2, fp6_mul_1(a1, l3));
    const fp6 a0 = S.get(0);
    s = fp6_add(a0, a1);
    S.put(0, fp6_mul_01(a0, l0, l2));  // t0 (f.c0 consumed)
  }
  const fp6 c1 = fp6_mul_01(s, l0, fp2_add(l2, l3));
  const fp6 t0 = S.get(0), t1 = S.get(2);
  S.put(1, fp6_sub(fp6_sub(c1, t0), t1));
  S.put(0, fp6_add(t0, fp6_mul_v(t1)));
}
// NL = 3 (f and the temporary in LDS, 54 KB per wave: two waves per CU) keeps the per-root chain
// fastest; NL = 2 (36 KB: one wave per SIMD, as the registers allow) for batches of so many
// distinct roots that the LDS bound would leave most of them waiting (lb_engine.hip).
#if LB_KG(4)
template <int NL>
__global__ void __launch_bounds__(LB_TPB, 1) k_miller_lane(uint32_t n, uint32_t m,
                                                           const uint32_t* __restrict__ n_u,
                                                           const uint32_t* __restrict__ gp_aff,
                                                           const uint32_t* __restrict__ gp_inf,
                                                           const uint32_t* __restrict__ h_aff,
                                                           uint32_t* __restrict__ treeP, uint32_t* __restrict__ tpark) {
#if LB_MILLER_LANE_REG  // A/B builds only: the round-3 register-resident kernel (6.7 KB private segment)
  const uint32_t u = lb_tid();
  if (u >= *n_u) return;
  fp12 f = fp12_one();
  if (!gp_inf[u]) f = miller_loop_inl(soa_ld<g1a>(gp_aff, n, u), soa_ld<g2a>(h_aff, n, u));
  soa_st(treeP, 2 * m, m + u, f);
  (void)tpark;
#else
  static_assert(LB_TPB == 64, "one wave per block: 64 lanes of LDS slots");
  __shared__ uint32_t lds[NL * 72 * 64];
  const uint32_t u = lb_tid();
  if (u >= *n_u) return;
  const lane_lds<NL> S{(lds_w*)lds, tpark, n, u, (int)threadIdx.x};
  S.put(0, fp6_one());
  S.put(1, fp6_zero());
  if (!gp_inf[u]) {
    auto park_t = [&](const g2j& T) { S.put(3, *reinterpret_cast<const fp6*>(&T)); };
    auto unpark_t = [&]() {
      const fp6 v = S.get(3);
      return *reinterpret_cast<const g2j*>(&v);
    };
    {
      const g2a Q = soa_ld<g2a>(h_aff, n, u);
      park_t(g2j{Q.x, Q.y, fp2_one()});
    }
    bool first = true;
#pragma clang loop unroll(disable)
    for (int i = 62; i >= 0; i--) {
      if (!first) lane_f_sqr(S);
      first = false;
      fp2 l0, l2, l3;
      {
        g2j T = unpark_t();
        const g1a P = soa_ld<g1a>(gp_aff, n, u);
        miller_dbl(T, l0, l2, l3, P.x, P.y);
        park_t(T);
      }
      lane_f_line(S, l0, l2, l3);
      if ((LB_X_ABS >> i) & 1ull) {
        {
          g2j T = unpark_t();
          const g1a P = soa_ld<g1a>(gp_aff, n, u);
          miller_add(T, soa_ld<g2a>(h_aff, n, u), l0, l2, l3, P.x, P.y);
          park_t(T);
        }
        lane_f_line(S, l0, l2, l3);
      }
    }
    S.put(1, fp6_neg(S.get(1)));  // conjugate (x < 0)
  }
  LB_UNROLL for (int h = 0; h < 2; h++) {
    const fp6 v = S.get(h);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
    LB_UNROLL for (int i = 0; i < 72; i++) treeP[(size_t)(72 * h + i) * (2 * m) + m + u] = w[i];
  }
#endif
}
#endif  // LB_KG

#if LB_KG(5)
__global__ void __launch_bounds__(64) k_miller_wave(uint32_t n, uint32_t m, const uint32_t* __restrict__ n_u,
                                                    const uint32_t* __restrict__ gp_aff,
                                                    const uint32_t* __restrict__ gp_inf,
                                                    const uint32_t* __restrict__ h_aff, uint32_t* __restrict__ treeP) {
  LBW_SHARED_MILLER(S);
  const uint32_t u = blockIdx.x;
  if (u >= *n_u) return;
  const int lane = threadIdx.x;
  w_init_consts(S, LBW_MILLER_COUNT, LBW_MILLER_FIRST);
  const bool inf = gp_inf[u] != 0;  // uniform
  if (inf) {
    w_set_one(S, LBW_A(0));
  } else {
    if (lane < 6) {
      const uint32_t* base = lane < 2 ? gp_aff + (size_t)12 * lane * n : h_aff + (size_t)12 * (lane - 2) * n;
      fp v;
      LB_UNROLL for (int w = 0; w < 12; w++) v.v[w] = base[(size_t)w * n + u];
      w_st(S, LBW_PT + lane, v);
    }
    w_sync();
    w_miller(S, LBW_A(0));
  }
  w_store_soa12(S, LBW_A(0), treeP, 2 * m, m + u);
}
#endif  // LB_KG

// ---------------------------------------------------------------- message grouping
// Sets that sign the same 32-byte root share one hash_to_G2 and one Miller loop (on mainnet a
// committee's unaggregated attestations all sign one AttestationData root, every aggregator of a
// slot signs the same selection-proof root, and all 512 sync-committee members sign one block
// root).  The batch equation is unchanged: prod_i e(r_i PK_i, H(m_i)) regrouped by message.
//
// k_msg_insert: open addressing over a table of set indices (capacity cap = pow2 >= 2n, every
// slot 0xffffffff), probed from a keyed hash of the root (key from the engine's CSPRNG, so crafted
// roots cannot be aimed at one probe chain); equality is decided on all 32 bytes.  A slot, once
// claimed by compare-and-swap, never changes, so a loser can compare against its owner at once.
// members summed per lane in k_gsum_chunks: 8 with the k_gsum_tree levels for a batch alone on
// the device (latency), 32 with the chunk sums added per root on one lane under load (the tree's
// wide launches cost the batches in flight throughput, profiles/r5_row_ab.txt); lb_engine.hip
#ifndef LB_GROUP_CHUNK_ALONE
#define LB_GROUP_CHUNK_ALONE 8
#endif
#define LB_GROUP_CHUNK 32
#ifndef LB_GROUP_CHUNK_WAVE
#define LB_GROUP_CHUNK_WAVE 4  // ... with k_gsum_wave's shuffle tree (64 chunks of a wave: 256 members)
#endif
#ifndef LB_GSUM_FAN
#define LB_GSUM_FAN 4     // partial sums combined per lane and level in k_gsum_tree
#endif
#ifndef LB_MSM_CHUNK
#define LB_MSM_CHUNK 16  // bucket members summed per lane in k_msm_chunks (the batch MSM's serial chain)
#endif
__device__ __forceinline__ bool msg_eq(const uint8_t* __restrict__ msgs, uint32_t a, uint32_t b) {
  const uint4* x = reinterpret_cast<const uint4*>(msgs + (size_t)32 * a);
  const uint4* y = reinterpret_cast<const uint4*>(msgs + (size_t)32 * b);
  const uint4 x0 = x[0], x1 = x[1], y0 = y[0], y1 = y[1];
  return ((x0.x ^ y0.x) | (x0.y ^ y0.y) | (x0.z ^ y0.z) | (x0.w ^ y0.w) | (x1.x ^ y1.x) | (x1.y ^ y1.y) |
          (x1.z ^ y1.z) | (x1.w ^ y1.w)) == 0u;
}
__device__ __forceinline__ uint32_t msg_hash(const uint8_t* __restrict__ msgs, uint32_t i, uint64_t key) {
  const uint4* x = reinterpret_cast<const uint4*>(msgs + (size_t)32 * i);
  const uint4 a = x[0], b = x[1];
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint64_t h = key;
  LB_UNROLL for (int k = 0; k < 8; k++) {
    h = (h ^ w[k]) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
  }
  return (uint32_t)(h >> 32);
}
#if LB_KG(0)
__global__ void __launch_bounds__(LB_TPB) k_msg_insert(uint32_t n, const uint8_t* __restrict__ msgs, uint64_t key,
                                                       uint32_t cap, uint32_t* __restrict__ tab,
                                                       uint32_t* __restrict__ rep_of) {
  const uint32_t i = lb_tid();
  if (i >= n) return;
  uint32_t h = msg_hash(msgs, i, key) & (cap - 1u), rep = i;
  for (uint32_t probe = 0; probe < cap; probe++) {  // cap > n: a free slot always exists
    const uint32_t old = atomicCAS(&tab[h], 0xffffffffu, i);
    if (old == 0xffffffffu) break;
    if (msg_eq(msgs, old, i)) {
      rep = old;
      break;
    }
    h = (h + 1u) & (cap - 1u);
  }
  rep_of[i] = rep;
}
#endif  // LB_KG
// The grouping of a ONE-set batch (what k_msg_insert .. k_msg_scatter produce for n = 1: one
// root of one member in one chunk) in one launch instead of three fills and six kernels
#if LB_KG(0)
__global__ void __launch_bounds__(64) k_dedup_one(uint32_t* __restrict__ rep_of, uint32_t* __restrict__ uid_of,
                                                  uint32_t* __restrict__ uniq_set, uint32_t* __restrict__ n_u,
                                                  uint32_t* __restrict__ set_uid, uint32_t* __restrict__ cnt,
                                                  uint32_t* __restrict__ pos, uint32_t* __restrict__ goff,
                                                  uint32_t* __restrict__ gch, uint32_t* __restrict__ chunk_beg,
                                                  uint32_t* __restrict__ chunk_end, uint32_t* __restrict__ chunk_root,
                                                  uint32_t* __restrict__ members) {
  if (threadIdx.x != 0) return;
  rep_of[0] = 0;
  uid_of[0] = 0;
  uniq_set[0] = 0;
  n_u[0] = 1;  // distinct roots
  n_u[1] = 1;  // chunks of the largest root
  set_uid[0] = 0;
  cnt[0] = 1;
  pos[0] = 0;
  goff[0] = 0;
  goff[1] = 1;
  gch[0] = 0;
  gch[1] = 1;
  chunk_beg[0] = 0;
  chunk_end[0] = 1;
  chunk_root[0] = 0;
  members[0] = 0;
}
#endif  // LB_KG
// Unique-message ids in input order (the first set of each root, LB_ROOT_SHUFFLE=0)
#if LB_KG(0)
__global__ void __launch_bounds__(LB_TPB) k_msg_uid_input(uint32_t n, const uint32_t* __restrict__ rep_of,
                                                          uint32_t* __restrict__ uid_of,
                                                          uint32_t* __restrict__ uniq_set, uint32_t* __restrict__ n_u) {
  const uint32_t i = lb_tid();
  if (i >= n || rep_of[i] != i) return;
  const uint32_t u = atomicAdd(n_u, 1u);
  uid_of[i] = u;
  uniq_set[u] = i;
}
#endif  // LB_KG
// Unique-message ids in TABLE-SLOT order (keyed hash: pseudo-random, not the input order): the
// roots' order is the root product tree's leaf order, and the invalid-set search's first-round
// subtrees are runs of it.  In input order a run of 64 roots held whole committees of one slot
// (16 k sets) and the failing subtrees' tests went through the 6-window bucket MSM; shuffled,
// a subtree holds ~3.5 committee roots on average.
#if LB_KG(0)
__global__ void __launch_bounds__(LB_TPB) k_msg_uid(uint32_t cap, const uint32_t* __restrict__ tab,
                                                    uint32_t* __restrict__ uid_of, uint32_t* __restrict__ uniq_set,
                                                    uint32_t* __restrict__ n_u) {
  const uint32_t h = lb_tid();
  if (h >= cap) return;
  const uint32_t i = tab[h];
  if (i == 0xffffffffu) return;  // each distinct root holds exactly one slot (its first claimer's)
  const uint32_t u = atomicAdd(n_u, 1u);
  uid_of[i] = u;
  uniq_set[u] = i;
}
#endif  // LB_KG

// set_uid[i] = unique-message id of set i; pos[i] = its rank inside the group (cnt zeroed)
#if LB_KG(0)
__global__ void __launch_bounds__(LB_TPB) k_msg_count(uint32_t n, const uint32_t* __restrict__ rep_of,
                                                      const uint32_t* __restrict__ uid_of,
                                                      uint32_t* __restrict__ set_uid, uint32_t* __restrict__ cnt,
                                                      uint32_t* __restrict__ pos) {
  const uint32_t i = lb_tid();
  if (i >= n) return;
  const uint32_t u = uid_of[rep_of[i]];
  set_uid[i] = u;
  pos[i] = atomicAdd(&cnt[u], 1u);
}
#endif  // LB_KG

// One block: exclusive scans of the group sizes (member offsets goff) and of their chunk
// counts (gch), and the member range of every chunk.  goff[n_u] / gch[n_u] = totals.
// (n_u == nullptr: nu_const groups; the MSM's buckets use it too)
#if LB_KG(0)
__global__ void __launch_bounds__(1024) k_msg_scan(const uint32_t* __restrict__ n_u, uint32_t nu_const, uint32_t chunk,
                                                   const uint32_t* __restrict__ cnt,
                                                   uint32_t* __restrict__ goff, uint32_t* __restrict__ gch,
                                                   uint32_t* __restrict__ chunk_beg, uint32_t* __restrict__ chunk_end,
                                                   uint32_t* __restrict__ chunk_root, uint32_t* __restrict__ max_chunks) {
  __shared__ uint32_t s_m[1024], s_c[1024], s_x;
  const uint32_t nu = n_u ? *n_u : nu_const, t = threadIdx.x, per = (nu + 1023u) / 1024u;
  const uint32_t a = min(t * per, nu), b = min(a + per, nu);
  uint32_t sm = 0, sc = 0, mx = 0;
  for (uint32_t u = a; u < b; u++) {
    sm += cnt[u];
    const uint32_t cu = (cnt[u] + chunk - 1) / chunk;
    sc += cu;
    mx = max(mx, cu);
  }
  if (t == 0) s_x = 0;
  s_m[t] = sm;
  s_c[t] = sc;
  __syncthreads();
  if (max_chunks) atomicMax(&s_x, mx);
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    const uint32_t vm = t >= d ? s_m[t - d] : 0u, vc = t >= d ? s_c[t - d] : 0u;
    __syncthreads();
    s_m[t] += vm;
    s_c[t] += vc;
    __syncthreads();
  }
  uint32_t om = s_m[t] - sm, oc = s_c[t] - sc;
  for (uint32_t u = a; u < b; u++) {
    const uint32_t c = cnt[u];
    goff[u] = om;
    gch[u] = oc;
    if (chunk_beg)  // (chunk_beg == nullptr: k_chunk_fill writes the chunk ranges, one lane per chunk)
      for (uint32_t k = 0; k < c; k += chunk) {
        chunk_beg[oc] = om + k;
        chunk_end[oc] = om + min(k + chunk, c);
        if (chunk_root) chunk_root[oc] = u;
        oc++;
      }
    else
      oc += (c + chunk - 1) / chunk;
    om += c;
  }
  if (t == 1023) {
    goff[nu] = s_m[1023];
    gch[nu] = s_c[1023];
  }
  if (max_chunks && t == 0) *max_chunks = s_x;  // (the atomics completed before the scan's barriers)
}
#endif  // LB_KG

// The member range and root of every chunk of the per-root grouping, one lane per chunk (root by
// binary search over the chunk offsets gch): the serial per-thread chunk loop of k_msg_scan took
// ~2 ms per 116 736-set batch with 4-member chunks (a thread owning the large roots wrote
// thousands of chunks), on the s1 path the host waits on.
#if LB_KG(0)
__global__ void __launch_bounds__(LB_TPB) k_chunk_fill(const uint32_t* __restrict__ n_u, uint32_t chunk,
                                                       const uint32_t* __restrict__ goff,
                                                       const uint32_t* __restrict__ gch,
                                                       uint32_t* __restrict__ chunk_beg, uint32_t* __restrict__ chunk_end,
                                                       uint32_t* __restrict__ chunk_root) {
  const uint32_t c = lb_tid(), nu = *n_u;
  if (c >= gch[nu]) return;
  uint32_t lo = 0, hi = nu;  // the last u with gch[u] <= c
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (gch[mid] <= c) lo = mid;
    else hi = mid;
  }
  const uint32_t b = goff[lo] + (c - gch[lo]) * chunk;
  chunk_beg[c] = b;
  chunk_end[c] = min(b + chunk, goff[lo + 1]);
  chunk_root[c] = lo;
}
#endif  // LB_KG

#if LB_KG(0)
__global__ void __launch_bounds__(LB_TPB) k_msg_scatter(uint32_t n, const uint32_t* __restrict__ set_uid,
                                                        const uint32_t* __restrict__ pos,
                                                        const uint32_t* __restrict__ goff,
                                                        uint32_t* __restrict__ members) {
  const uint32_t i = lb_tid();
  if (i >= n) return;
  members[goff[set_uid[i]] + pos[i]] = i;
}
#endif  // LB_KG

// ---------------------------------------------------------------- sum r_i sig_i by bucket MSM
// S = sum over live sets of r_i sig_i with r_i = lo_i + hi_i lambda (k_pk_blind): 2n points
// (sig_i with scalar lo_i, [lambda]sig_i = -psi^2(sig_i) with hi_i) and 32-bit scalars.
// Pippenger: LB_MSM_W windows of LB_MSM_C bits; every (point, window) with a non-zero digit d
// joins bucket (window, d); bucket sums come from chunked Jacobian sums of the members (the
// message-grouping machinery: count, k_msg_scan, scatter, chunks); one wave then forms
// sum_d d B_d per window and combines the windows.  About 8 mixed additions per set instead of
// the 32 doublings + 32 additions of a per-set r*sig.  The invalid-set search reuses the same
// machinery over ranges of sets (k_rmsm_*) after a failing root check.
#define LB_MSM_C 8
#define LB_MSM_W 4
#define LB_MSM_B (1 << LB_MSM_C)
#define LB_MSM_NB (LB_MSM_W * LB_MSM_B)  // bucket ids w * 256 + d (d = 0 unused)
// (set_live == nullptr: every decoded set; the caller masks the terms later, k_g2_sum_g8)
__device__ __forceinline__ bool msm_live(uint32_t i, const uint32_t* set_live, const uint32_t* sig_inf) {
  return (set_live == nullptr || set_live[i]) && !sig_inf[i];
}
#if LB_KG(6)
__global__ void __launch_bounds__(LB_TPB) k_msm_count(uint32_t n, const uint64_t* __restrict__ scalars,
                                                      const uint32_t* __restrict__ set_live,
                                                      const uint32_t* __restrict__ sig_inf, uint32_t* __restrict__ cnt) {
  const uint32_t i = lb_tid();
  if (i >= n || !msm_live(i, set_live, sig_inf)) return;
  const uint64_t wd = scalars[i];
  LB_UNROLL for (int h = 0; h < 2; h++) {
    const uint32_t k = (uint32_t)(wd >> (32 * h));
    LB_UNROLL for (int w = 0; w < LB_MSM_W; w++) {
      const uint32_t d = (k >> (LB_MSM_C * w)) & (LB_MSM_B - 1);
      if (d) atomicAdd(&cnt[w * LB_MSM_B + d], 1u);
    }
  }
}
#endif  // LB_KG
#if LB_KG(6)
__global__ void __launch_bounds__(LB_TPB) k_msm_scatter(uint32_t n, const uint64_t* __restrict__ scalars,
                                                        const uint32_t* __restrict__ set_live,
                                                        const uint32_t* __restrict__ sig_inf,
                                                        const uint32_t* __restrict__ boff, uint32_t* __restrict__ cursor,
                                                        uint32_t* __restrict__ members) {
  const uint32_t i = lb_tid();
  if (i >= n || !msm_live(i, set_live, sig_inf)) return;
  const uint64_t wd = scalars[i];
  LB_UNROLL for (int h = 0; h < 2; h++) {
    const uint32_t k = (uint32_t)(wd >> (32 * h));
    LB_UNROLL for (int w = 0; w < LB_MSM_W; w++) {
      const uint32_t d = (k >> (LB_MSM_C * w)) & (LB_MSM_B - 1);
      if (d) {
        const uint32_t b = w * LB_MSM_B + d;
        members[boff[b] + atomicAdd(&cursor[b], 1u)] = i | ((uint32_t)h << 31);
      }
    }
  }
}
#endif  // LB_KG
// chunk c of a bucket: Jacobian sum of its member points (AoS affine signatures; bit 31 of a
// member = the [lambda] image).  nb = bucket count (bch has nb + 1 entries).
#if LB_KG(6)
__global__ void __launch_bounds__(LB_TPB, LB_MINW_MSM) k_msm_chunks(const uint32_t* __restrict__ bch,
                                                       const uint32_t* __restrict__ chunk_beg,
                                                       const uint32_t* __restrict__ chunk_end,
                                                       const uint32_t* __restrict__ members,
                                                       const uint4* __restrict__ sig_aos, uint32_t cap,
                                                       uint32_t* __restrict__ bacc, uint32_t nb) {
  const uint32_t c = lb_tid();
  if (c >= bch[nb]) return;
  g2jm acc = jac_infinity<lb_g2f>();
  for (uint32_t k = chunk_beg[c]; k < chunk_end[c]; k++) {
    const uint32_t m = members[k], i = m & 0x7fffffffu;
    g2a p;
    uint32_t* w = reinterpret_cast<uint32_t*>(&p);
    LB_UNROLL for (int q = 0; q < 12; q++) {
      const uint4 v = sig_aos[(size_t)12 * i + q];
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
    if (m >> 31) {
      p.x = fp2_mul_fp(p.x, fp_load(LB_PSI2_CX));
      p.y = fp2_neg(fp2_mul_fp(p.y, fp_load(LB_PSI2_CY)));
    }
    acc = jac_add_aff_i<lb_g2f, true>(acc, aff_as<lb_g2f>(p));
  }
  soa_st(bacc, cap, c, jac_as<fp2>(acc));
}
#endif  // LB_KG
// bucket b = sum of its chunk sums (SoA, stride nb); empty buckets are infinity
#if LB_KG(6)
__global__ void __launch_bounds__(LB_TPB, LB_MINW) k_msm_buckets(const uint32_t* __restrict__ bch,
                                                        const uint32_t* __restrict__ bacc, uint32_t cap,
                                                        uint32_t* __restrict__ bsum, uint32_t nb) {
  const uint32_t b = lb_tid();
  if (b >= nb) return;
  g2jm acc = jac_infinity<lb_g2f>();
  for (uint32_t c = bch[b]; c < bch[b + 1]; c++)
    acc = jac_add_i<lb_g2f, true>(acc, jac_as<lb_g2f>(soa_ld<g2j>(bacc, cap, c)));
  soa_st(bsum, nb, b, jac_as<fp2>(acc));
}
#endif  // LB_KG
// One workgroup per MSM instance j of W windows (buckets [j W 256, (j+1) W 256) of bsum, stride
// nb), one wave per window: lane s owns digits [4 s, 4 s + 4).  A lane's running sums give
// Y_s = sum_j j B_{4s+j} and T_s = sum_j B_{4s+j} (5 additions); then
//   sum_d d B_d = sum_s (Y_s + 4 s T_s) = sum_s Y_s + 4 sum_{k >= 1} U_k,  U_k = sum_{s >= k} T_s,
// so a suffix scan of T across the wave (6 levels of shuffles + additions), V_s = Y_s + 4 U_s
// (s >= 1; two doublings) and a shuffle tree over V (6 levels) give the window sum W_w in lane 0.
// Lane 0 of wave 0 combines the windows Horner-style: S = sum_w 2^(8w) W_w -> element out0 + j of
// `out` (SoA, stride n_out).  The dependent chain is ~19 additions + 2 doublings + the Horner
// doublings, against 34 additions + 12 doublings + the Horner for 16 lanes of 16 digits.  W = 4
// (32-bit scalars) for the batch MSM, 6 for the search's weighted scalars (up to 43 bits).
__device__ __forceinline__ g2j g2j_shfl_down(const g2j& a, unsigned d) {
  return g2j{fp2{fp_shfl_down(a.x.c0, d), fp_shfl_down(a.x.c1, d)},
             fp2{fp_shfl_down(a.y.c0, d), fp_shfl_down(a.y.c1, d)},
             fp2{fp_shfl_down(a.z.c0, d), fp_shfl_down(a.z.c1, d)}};
}
#if LB_KG(6)
template <int W>
__global__ void __launch_bounds__(64 * W) k_msm_reduce(const uint32_t* __restrict__ bsum, uint32_t nb,
                                                       uint32_t* __restrict__ out, uint32_t n_out, uint32_t out0) {
  static_assert(LB_MSM_B == 256, "64 lanes of 4 digits per window");
  __shared__ g2j win[W];
  const uint32_t s = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint32_t* bw = bsum;  // bucket (instance, w, d) at element blockIdx.x * W * 256 + w * 256 + d
  const uint32_t e0 = blockIdx.x * (W * LB_MSM_B) + w * LB_MSM_B + 4 * s;
  // (out-of-line products here: inline ones grew this kernel's private segment 1.7 -> 4.3 KB)
  typedef fp2 rf;
  typedef jac<rf> g2jm;
  auto ld = [&](uint32_t e) { return soa_ld<g2j>(bw, nb, e); };
  auto add = [](const g2jm& a, const g2jm& b) { return jac_add_i(a, b); };
  auto shfl = [](const g2jm& a, unsigned d) { return g2j_shfl_down(a, d); };
  g2jm run = ld(e0 + 3);
  g2jm y = run;
  run = add(run, ld(e0 + 2));
  y = add(y, run);
  run = add(run, ld(e0 + 1));
  y = add(y, run);  // 3 B3 + 2 B2 + B1
  g2jm u = s ? add(run, ld(e0)) : run;  // digit 0 is unused
  // inclusive suffix scan: u_s = sum_{t >= s} T_t
  for (int l = 0; l < 6; l++) {  // rolled: the body is an inlined G2 addition
    const unsigned d = 1u << l;
    const g2jm o = shfl(u, d);
    if (s + d < 64) u = add(u, o);
  }
  g2jm v = y;
  if (s) v = add(v, jac_dbl_i(jac_dbl_i(u)));
  for (int l = 5; l >= 0; l--) {
    const unsigned d = 1u << l;
    const g2jm o = shfl(v, d);
    if (s < d) v = add(v, o);
  }
  if (s == 0) win[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    g2jm S = win[W - 1];
    for (int ww = W - 2; ww >= 0; ww--) {
      for (int b = 0; b < LB_MSM_C; b++) S = jac_dbl_i(S);
      S = add(S, win[ww]);
    }
    soa_st(out, n_out, out0 + blockIdx.x, S);
  }
}
#endif  // LB_KG

// ---- the same bucket reduction by 8-lane groups (lb_group.h), for the latency of the chain: a
// G2 addition is 6 product levels on a group instead of 43 serial products on a lone lane.
// Group point exchange through LDS (every lane of the group writes the same replicated words:
// a lane-dependent word index would put the point on the stack).
__device__ __forceinline__ void g8_put(lds_u32* X, int slot, const g2j& p) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&p);
  LB_UNROLL for (int k = 0; k < 72; k++) X[72 * slot + k] = w[k];
}
__device__ __forceinline__ g2j g8_take(const lds_u32* X, int slot) {
  g2j p;
  uint32_t* w = reinterpret_cast<uint32_t*>(&p);
  LB_UNROLL for (int k = 0; k < 72; k++) w[k] = X[72 * slot + k];
  return p;
}
__device__ __forceinline__ g2j g2j_shfl(const g2j& a, int src) {
  g2j r;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&a);
  uint32_t* o = reinterpret_cast<uint32_t*>(&r);
  LB_UNROLL for (int k = 0; k < 72; k++) o[k] = __shfl(w[k], src, 64);
  return r;
}
// bucket b = sum of its chunk sums: one wave per bucket, group g sums chunks g, g + 8, ..., then a
// 3-level shuffle tree over the groups (as k_msm_buckets, whose lone lane summed ~60 chunk sums
// serially)
#if LB_KG(9)
__global__ void __launch_bounds__(64) k_msm_buckets_g8(const uint32_t* __restrict__ bch,
                                                       const uint32_t* __restrict__ bacc, uint32_t cap,
                                                       uint32_t* __restrict__ bsum, uint32_t nb) {
  const uint32_t b = blockIdx.x;
  if (b >= nb) return;
  const int g = threadIdx.x >> 3;
  g2j acc = jac_infinity<fp2>();
#pragma clang loop unroll(disable)
  for (uint32_t c = bch[b] + g; c < bch[b + 1]; c += 8) g8_add(acc, soa_ld<g2j>(bacc, cap, c));
#pragma clang loop unroll(disable)
  for (int d = 4; d >= 1; d >>= 1) {
    const g2j o = g2j_shfl(acc, ((int)threadIdx.x + 8 * d) & 63);
    if (g < d) g8_add(acc, o);
  }
  if (threadIdx.x == 0) soa_st(bsum, nb, b, acc);
}
#endif  // LB_KG
// Window sums W_w = sum_d d B_d of k_msm_reduce, one workgroup of 4 waves per (instance, window)
// (one wave per SIMD: a group's G2 addition needs more than 256 registers): group s owns digits
// [8 s, 8 s + 8) (Y_s = sum_j j B_{8s+j}, T_s = sum_j B_{8s+j}: 13 additions), a 5-level suffix
// scan U_s = sum_{t >= s} T_t over the 32 groups, V_s = Y_s + 8 U_s (s >= 1), a 5-level tree:
// sum_d d B_d = sum_s (Y_s + 8 s T_s) = sum_s Y_s + 8 sum_{k >= 1} U_k.
// wsum: element blockIdx.x = instance * W + w.
#if LB_KG(9)
__global__ void __launch_bounds__(256) k_msm_window_g8(const uint32_t* __restrict__ bsum, uint32_t nb,
                                                       uint32_t* __restrict__ wsum, uint32_t n_w) {
  static_assert(LB_MSM_B == 256, "32 groups of 8 digits per window");
  __shared__ uint32_t xs[32 * 72], ys[32 * 72];
  lds_u32* X = (lds_u32*)xs;
  lds_u32* Y = (lds_u32*)ys;
  const int s = threadIdx.x >> 3;
  const uint32_t e0 = blockIdx.x * LB_MSM_B + 8 * s;  // bucket (instance, w, d) at instance*W*256 + w*256 + d
  g2j run = soa_ld<g2j>(bsum, nb, e0 + 7);
  g2j y = run;
#pragma clang loop unroll(disable)
  for (int j = 6; j >= 1; j--) {
    g8_add(run, soa_ld<g2j>(bsum, nb, e0 + j));
    g8_add(y, run);
  }
  if (s) g8_add(run, soa_ld<g2j>(bsum, nb, e0));  // digit 0 is unused
  g8_put(Y, s, y);
  // inclusive suffix scan: u_s = sum_{t >= s} T_t
#pragma clang loop unroll(disable)
  for (int d = 1; d < 32; d <<= 1) {
    g8_put(X, s, run);
    __syncthreads();
    g2j o = jac_infinity<fp2>();
    if (s + d < 32) o = g8_take(X, s + d);
    __syncthreads();
    if (s + d < 32) g8_add(run, o);
  }
  g2j v = g8_take(Y, s);
  if (s) {
    g8_dbl(run);
    g8_dbl(run);
    g8_dbl(run);
    g8_add(v, run);
  }
#pragma clang loop unroll(disable)
  for (int d = 16; d >= 1; d >>= 1) {
    g8_put(X, s, v);
    __syncthreads();
    g2j o = jac_infinity<fp2>();
    if (s < d) o = g8_take(X, s + d);
    __syncthreads();
    if (s < d) g8_add(v, o);
  }
  if (threadIdx.x == 0) soa_st(wsum, n_w, blockIdx.x, v);
}
#endif  // LB_KG
// S_j = sum_w 2^(8 w) W_w (Horner) for instance j = 8 blockIdx.x + group -> out0 + j of `out`
#if LB_KG(9)
template <int W>
__global__ void __launch_bounds__(64) k_msm_horner_g8(const uint32_t* __restrict__ wsum, uint32_t n_inst,
                                                      uint32_t* __restrict__ out, uint32_t n_out, uint32_t out0) {
  const uint32_t j = blockIdx.x * 8 + (threadIdx.x >> 3);
  if (j >= n_inst) return;  // uniform within the group
  const uint32_t n_w = n_inst * W;
  g2j S = soa_ld<g2j>(wsum, n_w, j * W + W - 1);
#pragma clang loop unroll(disable)
  for (int ww = W - 2; ww >= 0; ww--) {
#pragma clang loop unroll(disable)
    for (int b = 0; b < LB_MSM_C; b++) g8_dbl(S);
    g8_add(S, soa_ld<g2j>(wsum, n_w, j * W + ww));
  }
  if (g8_q() == 0) soa_st(out, n_out, out0 + j, S);
}
#endif  // LB_KG

// Small batches: S = sum r_i sig_i without the bucket MSM, whose chunk / bucket / reduction
// chain is a fixed ~5 ms of serial G2 additions however few the sets.  Each live set's r_i sig_i
// by 8 lanes (k_sig_blind_g8: GLV double-and-add, [lambda] sig = -psi^2(sig)), then 64:1 shuffle
// trees (k_g2_sum64) into treeS element 1, where k_msm_reduce would have put it.
#if LB_KG(9)
__global__ void __launch_bounds__(64) k_sig_blind_g8(uint32_t n, const uint32_t* __restrict__ sig_aff,
                                                     const uint64_t* __restrict__ scalars,
                                                     const uint32_t* __restrict__ set_live,
                                                     const uint32_t* __restrict__ sig_inf,
                                                     uint32_t* __restrict__ terms) {
  const uint32_t i = blockIdx.x * 8 + (threadIdx.x >> 3);
  if (i >= n) return;  // uniform within the group
  g2j r = jac_infinity<fp2>();
  if (msm_live(i, set_live, sig_inf)) {
    const g2a a = soa_ld<g2a>(sig_aff, n, i);
    const g2j t1 = jac_from_aff(a);
    g2j t2 = g8_psi2(t1);
    t2.y = fp2_neg(t2.y);  // [lambda] sig = -psi^2(sig)
    g2j t3 = t1;
    g8_add(t3, t2);
    r = g8_mul_glv(t1, t2, t3, scalars[i]);
  }
  if (g8_q() == 0) soa_st(terms, n, i, r);
}
#endif  // LB_KG
// A batch of ONE set verifies unblinded (Signature.verify: blst's single-set path, no random
// scalar needed): r = 1 and S = sig itself straight into treeS element 1 (no ladder, no tree).
#if LB_KG(9)
__global__ void __launch_bounds__(64) k_sig_unblinded(const uint32_t* __restrict__ sig_aff,
                                                      const uint32_t* __restrict__ set_live,
                                                      const uint32_t* __restrict__ sig_inf, uint32_t n_out,
                                                      uint32_t* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const g2j r = msm_live(0, set_live, sig_inf) ? jac_from_aff(soa_ld<g2a>(sig_aff, 1, 0)) : jac_infinity<fp2>();
  soa_st(out, n_out, 1, r);
}
#endif  // LB_KG
// The same terms one lane per set, for mid-size batches (a slot of gossip): 8-lane groups at
// ~20 k sets fill every SIMD's register file for ~5 ms and stall the per-root kernels of the
// other stream.  r sig = [lo] sig + [hi] [lambda] sig by jac_mul_glv_i over the affine table
// (sig, [lambda] sig, sig + [lambda] sig), the third made affine with one batched inversion per
// block (as k_pk_blind does for G1).
#if LB_KG(9)
__global__ void __launch_bounds__(LB_INV_TPB, LB_MINW) k_sig_blind(uint32_t n, const uint32_t* __restrict__ sig_aff,
                                                          const uint64_t* __restrict__ scalars,
                                                          const uint32_t* __restrict__ set_live,
                                                          const uint32_t* __restrict__ sig_inf,
                                                          uint32_t* __restrict__ terms) {
  const uint32_t i = blockIdx.x * LB_INV_TPB + threadIdx.x;
  const bool act = i < n && msm_live(i, set_live, sig_inf);
  g2a t1{fp2_one(), fp2_one()}, t2 = t1;
  g2j s = jac_infinity<fp2>();
  if (act) {
    t1 = soa_ld<g2a>(sig_aff, n, i);
    t2 = g2a{fp2_mul_fp(t1.x, fp_load(LB_PSI2_CX)), fp2_neg(fp2_mul_fp(t1.y, fp_load(LB_PSI2_CY)))};
    s = jac_add_aff_i<fp2, true>(jac_from_aff(t1), t2);  // finite: lambda + 1 != 0 mod r
  }
  const fp nz = fp_add(fp_sqr(s.z.c0), fp_sqr(s.z.c1));
  const bool ok = act && !fp_is_zero(nz);
  const fp ni = fp_inv_block(ok ? nz : fp_one());
  if (i >= n) return;
  g2j r = jac_infinity<fp2>();
  if (ok) {
    const fp2 zi{fp_mul(s.z.c0, ni), fp_neg(fp_mul(s.z.c1, ni))};
    const fp2 zi2 = fp2_sqr(zi);
    const g2a t3{fp2_mul(s.x, zi2), fp2_mul(fp2_mul(s.y, zi2), zi)};
#if LB_G2_INL_SB
    r = jac_as<fp2>(jac_mul_glv_i<fp2i, true>(aff_as<fp2i>(t1), aff_as<fp2i>(t2), aff_as<fp2i>(t3), scalars[i]));
#else
    r = jac_mul_glv_i<fp2, true>(t1, t2, t3, scalars[i]);
#endif
  }
  soa_st(terms, n, i, r);
}
#endif  // LB_KG

// element out0 + b of `out` (stride n_out) = sum of in[64 b .. 64 b + 63] (stride n_in)
#if LB_KG(9)
__global__ void __launch_bounds__(64) k_g2_sum64(uint32_t n_in, const uint32_t* __restrict__ in, uint32_t n_out,
                                                 uint32_t* __restrict__ out, uint32_t out0) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  g2j v = i < n_in ? soa_ld<g2j>(in, n_in, i) : jac_infinity<fp2>();
  for (int l = 5; l >= 0; l--) {
    const unsigned d = 1u << l;
    const g2j o = g2j_shfl_down(v, d);
    if (threadIdx.x < d) v = jac_add_i(v, o);
  }
  if (threadIdx.x == 0) soa_st(out, n_out, out0 + blockIdx.x, v);
}
#endif  // LB_KG

// The same sum for small n in ONE workgroup with 8-lane G2 additions (lb_group.h g8_add: 6
// product levels instead of 43 serial products per addition): 64 groups each add a strided share,
// then a 6-level tree over the groups through LDS.  For the small-S path up to small_s_g8_max
// terms (a block: ~0.6 ms of lone-lane 64:1 trees -> ~0.1 ms).
// r_i sig_i for small batches on the row engine (one workgroup per set; lb_row.h G2 programs):
// the GLV double-and-add of k_sig_blind_g8 over the table t1 = sig, t2 = [lambda] sig =
// -psi^2(sig), t3 = t1 + t2, starting from the top non-zero digit (no infinity in the ladder), the
// additions with the exceptional-case tests (r_g2_add).  Jacobian result, canonical words.
#if LB_KG(12)
__global__ void __launch_bounds__(LBR_NT) k_sig_blind_row(uint32_t n, const uint32_t* __restrict__ sig_aff,
                                                        const uint64_t* __restrict__ scalars,
                                                        const uint32_t* __restrict__ set_live,
                                                        const uint32_t* __restrict__ sig_inf,
                                                        uint32_t* __restrict__ terms, uint32_t proj) {
  LBR_SHARED_N(S, LBR_PROGS_END - LBR_G2DBL);
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  if (!msm_live(i, set_live, sig_inf)) {  // uniform
    if (threadIdx.x == 0) soa_st(terms, n, i, jac_infinity<fp2>());
    return;
  }
  r_init(S, LBR_PROGS_END - LBR_G2DBL, LBR_G2DBL);
  const int T1 = LBR_A(0), T2 = LBR_A(0) + 6, T3 = LBR_A(1), ACC = LBR_A(1) + 6;
  {
    const int t = r_tid();
    if (t < 6) {  // x.c0 x.c1 y.c0 y.c1 from the affine SoA, z = 1
      fp v;
      if (t < 4)
        LB_UNROLL for (int w = 0; w < 12; w++) v.v[w] = sig_aff[(size_t)(12 * t + w) * n + i];
      else
        v = t == 4 ? fp_one() : fp_zero();
      r_stage_fp(S, t, v);
    }
    r_sync();
    r_import_staged(S, T1, 6);
  }
  r_g2_psi2(S, T2, T1);
  r_g2_neg(S, T2);  // [lambda] sig = -psi^2(sig)
  // proj (round 6): the table and the ladder in projective coordinates with the complete
  // formulas (T1 = (x : y : 1) as it is; psi^2 and the negation act the same), the result back
  // to Jacobian (PTOJ) for the S sum
  if (proj) r_g2_prog(S, LBR_PADD, T3, T1, T2);
  else r_g2_add(S, T3, T1, T2);
  const uint64_t w = scalars[i];
  const uint32_t k0 = (uint32_t)w, k1 = (uint32_t)(w >> 32);
  auto digit = [&](int b) { return ((k0 >> b) & 1u) | (((k1 >> b) & 1u) << 1); };
  int b = 31;
  while (b >= 0 && digit(b) == 0) b--;
  if (b < 0) {  // r = 0 (never for the engine's scalars): the identity
    if (threadIdx.x == 0) soa_st(terms, n, i, jac_infinity<fp2>());
    return;
  }
  auto tab = [&](uint32_t d) { return d == 1 ? T1 : (d == 2 ? T2 : T3); };
  r_copy(S, ACC, tab(digit(b)), 6);
  for (b--; b >= 0; b--) {
    const uint32_t d = digit(b);
    if (proj) {
      r_g2_prog(S, LBR_PDBL1, ACC, ACC);
      if (d) r_g2_prog(S, LBR_PADD, ACC, ACC, tab(d));
    } else {
      r_g2_dbl(S, ACC, ACC);
      if (d) r_g2_add(S, ACC, ACC, tab(d));
    }
  }
  if (proj) r_g2_prog(S, LBR_PTOJ, ACC, ACC);
  r_export(S, ACC, 6);
  if (threadIdx.x < 6) {
    const fp v = r_fp_of_staged(S, threadIdx.x);
    LB_UNROLL for (int k = 0; k < 12; k++) terms[(size_t)(12 * threadIdx.x + k) * n + i] = v.v[k];
  }
}
#endif  // LB_KG
#define LB_SUM_G8_GROUPS 64
#if LB_KG(9)
__global__ void __launch_bounds__(8 * LB_SUM_G8_GROUPS) k_g2_sum_g8(uint32_t n, const uint32_t* __restrict__ in,
                                                                  uint32_t n_out, uint32_t* __restrict__ out,
                                                                  uint32_t out0, const uint32_t* __restrict__ live) {
  // live (optional): term i counts iff live[i] (terms computed before the job statuses were known)
  __shared__ uint32_t st[LB_SUM_G8_GROUPS * 72];
  const int g = threadIdx.x >> 3, q = g8_q();
  g2j acc = jac_infinity<fp2>();
  for (uint32_t i = g; i < n; i += LB_SUM_G8_GROUPS)
    if (live == nullptr || live[i]) g8_add(acc, soa_ld<g2j>(in, n, i));
  auto stash = [&](int slot, const g2j& v) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
    LB_UNROLL for (int k = 0; k < 9; k++) st[slot * 72 + 8 * k + q] = w[8 * k + q];
  };
  stash(g, acc);
  __syncthreads();
  for (int s = LB_SUM_G8_GROUPS / 2; s >= 1; s >>= 1) {
    if (g < s) {
      g2j o;
      uint32_t* w = reinterpret_cast<uint32_t*>(&o);
      LB_UNROLL for (int k = 0; k < 72; k++) w[k] = st[(g + s) * 72 + k];
      g8_add(acc, o);
    }
    __syncthreads();
    if (g < s) stash(g, acc);
    __syncthreads();
  }
  if (threadIdx.x == 0) soa_st(out, n_out, out0, acc);
}
#endif  // LB_KG

// ---------------------------------------------------------------- invalid-set search
// After a failing root check the engine searches for the failing sets over NODES: a node is a
// contiguous range [lo_j, lo_j + len_j) of the members array (sets sorted by signing root) and
// passes iff FE(P_j * ML(-G1, S_j)) == 1 with S_j = sum r_i sig_i over its live sets and
//   kind 0 (a subtree of the root product tree, whole roots): P_j = treeP[v_j];
//   kind 1 (part of one root u_j's members): P_j = ML(sum r_i PK_i, H(m_u));
//   kind 2 (one set i): Signature.verify itself, FE(ML(PK_i, H(m_i)) ML(-G1, sig_i)) == 1,
//          no blinding and no MSM (a set of a rejected job passes trivially).
// By bilinearity a node's verdict is the product of its children's, so a failing node has a
// failing child; the host descends until single sets (lb_engine.hip search_invalid).
// Search MSM: instance j covers member positions [lo_j, lo_j + len_j) (thread t of the
// T = sum len_j positions finds its instance by binary search of pre[]) with the scalar of set i
// multiplied by a small weight: mode 0 weight 1 (S of a node), mode 1 (a weighted test over
// subtrees of 2^b roots from root a) weight ((set_uid_i - a) >> b) + 1, mode 2 (a weighted test
// over parts of a members) weight (position offset / a) + 1.  Weights are <= LB_WT_MAX, so
// both 32-bit GLV halves of r_i w stay below 2^(32 + LB_WT_BITS) <= 2^48: LB_SMSM_W = 6 windows
// of 8 bits, instance j owning buckets [j LB_SMSM_NB, (j+1) LB_SMSM_NB).  A round of weight-1
// instances only (the first round's direct checks) takes LB_MSM_W = 4 windows (32-bit halves).
#define LB_WT_MAX 1024  // children of a weighted test over parts of one root (lb_engine.hip kWtParts)
#define LB_WT_BITS 11
#define LB_SMSM_W 6
#define LB_SMSM_NB (LB_SMSM_W * LB_MSM_B)
__device__ __forceinline__ uint32_t rmsm_node(const uint32_t* __restrict__ pre, uint32_t c, uint32_t t) {
  uint32_t lo = 0, hi = c;  // pre[lo] <= t < pre[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pre[mid] <= t) lo = mid;
    else hi = mid;
  }
  return lo;
}
struct smsm_args {
  const uint32_t *pre, *rlo, *mode, *wa, *wb;
};
__device__ __forceinline__ bool smsm_member(const smsm_args& a, uint32_t c, uint32_t t,
                                            const uint32_t* __restrict__ members,
                                            const uint32_t* __restrict__ set_uid, uint32_t& j, uint32_t& i,
                                            uint32_t& wt) {
  j = rmsm_node(a.pre, c, t);
  const uint32_t off = t - a.pre[j];
  i = members[a.rlo[j] + off];
  const uint32_t md = a.mode[j];
  wt = md == 0u ? 1u : (md == 1u ? ((set_uid[i] - a.wa[j]) >> a.wb[j]) + 1u : off / a.wa[j] + 1u);
  return true;
}
#if LB_KG(7)
template <int W>
__global__ void __launch_bounds__(LB_TPB) k_smsm_count(uint32_t T, uint32_t c, smsm_args a,
                                                       const uint32_t* __restrict__ members,
                                                       const uint32_t* __restrict__ set_uid,
                                                       const uint64_t* __restrict__ scalars,
                                                       const uint32_t* __restrict__ set_live,
                                                       const uint32_t* __restrict__ sig_inf,
                                                       uint32_t* __restrict__ cnt) {
  const uint32_t t = lb_tid();
  if (t >= T) return;
  uint32_t j, i, wt;
  smsm_member(a, c, t, members, set_uid, j, i, wt);
  if (!msm_live(i, set_live, sig_inf)) return;
  const uint64_t wd = scalars[i];
  LB_UNROLL for (int h = 0; h < 2; h++) {
    const uint64_t k = (uint64_t)(uint32_t)(wd >> (32 * h)) * wt;
    LB_UNROLL for (int w = 0; w < W; w++) {
      const uint32_t d = (uint32_t)(k >> (LB_MSM_C * w)) & (LB_MSM_B - 1);
      if (d) atomicAdd(&cnt[j * (W * LB_MSM_B) + w * LB_MSM_B + d], 1u);
    }
  }
}
#endif  // LB_KG
#if LB_KG(7)
template <int W>
__global__ void __launch_bounds__(LB_TPB) k_smsm_scatter(uint32_t T, uint32_t c, smsm_args a,
                                                         const uint32_t* __restrict__ members,
                                                         const uint32_t* __restrict__ set_uid,
                                                         const uint64_t* __restrict__ scalars,
                                                         const uint32_t* __restrict__ set_live,
                                                         const uint32_t* __restrict__ sig_inf,
                                                         const uint32_t* __restrict__ boff,
                                                         uint32_t* __restrict__ cursor, uint32_t* __restrict__ bmembers) {
  const uint32_t t = lb_tid();
  if (t >= T) return;
  uint32_t j, i, wt;
  smsm_member(a, c, t, members, set_uid, j, i, wt);
  if (!msm_live(i, set_live, sig_inf)) return;
  const uint64_t wd = scalars[i];
  LB_UNROLL for (int h = 0; h < 2; h++) {
    const uint64_t k = (uint64_t)(uint32_t)(wd >> (32 * h)) * wt;
    LB_UNROLL for (int w = 0; w < W; w++) {
      const uint32_t d = (uint32_t)(k >> (LB_MSM_C * w)) & (LB_MSM_B - 1);
      if (d) {
        const uint32_t b = j * (W * LB_MSM_B) + w * LB_MSM_B + d;
        bmembers[boff[b] + atomicAdd(&cursor[b], 1u)] = i | ((uint32_t)h << 31);
      }
    }
  }
}
#endif  // LB_KG
// Small search rounds (few thousand positions): the instances' weighted sums without the bucket
// MSM, whose chunk / bucket / reduction chain is a fixed ~5 ms per round.  Position t's term
// [w r_i] sig_i = [w lo] sig + [w hi] [lambda] sig (39-bit halves) by 8 lanes, then per-instance
// sums: blocks of <= 64 positions of one instance (k_seg_sum64), then each instance's block sums
// (k_seg_final, one wave).
#if LB_KG(7)
__global__ void __launch_bounds__(64) k_smsm_terms_g8(uint32_t T, uint32_t c, smsm_args a,
                                                      const uint32_t* __restrict__ members,
                                                      const uint32_t* __restrict__ set_uid,
                                                      const uint64_t* __restrict__ scalars,
                                                      const uint32_t* __restrict__ set_live,
                                                      const uint32_t* __restrict__ sig_inf,
                                                      const uint32_t* __restrict__ sig_aff, uint32_t n,
                                                      uint32_t* __restrict__ terms) {
  const uint32_t t = blockIdx.x * 8 + (threadIdx.x >> 3);
  if (t >= T) return;  // uniform within the group
  uint32_t j, i, wt;
  smsm_member(a, c, t, members, set_uid, j, i, wt);
  g2j r = jac_infinity<fp2>();
  if (msm_live(i, set_live, sig_inf)) {
    const g2j t1 = jac_from_aff(soa_ld<g2a>(sig_aff, n, i));
    g2j t2 = g8_psi2(t1);
    t2.y = fp2_neg(t2.y);  // [lambda] sig = -psi^2(sig)
    g2j t3 = t1;
    g8_add(t3, t2);
    const uint64_t wd = scalars[i];
    r = g8_mul_2d(t1, t2, t3, (wd & 0xffffffffu) * wt, (wd >> 32) * wt, 32 + LB_WT_BITS);
  }
  if (g8_q() == 0) soa_st(terms, T, t, r);
}
#endif  // LB_KG
// The same terms one lane per position (the form under load: the 8-lane groups issue several times
// the instructions of one lane's ladder, and a search round's terms were ~40 % of its work): the
// affine table (sig, [lambda] sig, sig + [lambda] sig) as in k_sig_blind, then the joint ladder
// over the two (32 + LB_WT_BITS)-bit weighted halves.
#if LB_KG(7)
__global__ void __launch_bounds__(LB_INV_TPB, LB_MINW) k_smsm_terms_lane(uint32_t T, uint32_t c, smsm_args a,
                                                                 const uint32_t* __restrict__ members,
                                                                 const uint32_t* __restrict__ set_uid,
                                                                 const uint64_t* __restrict__ scalars,
                                                                 const uint32_t* __restrict__ set_live,
                                                                 const uint32_t* __restrict__ sig_inf,
                                                                 const uint32_t* __restrict__ sig_aff, uint32_t n,
                                                                 uint32_t* __restrict__ terms) {
  const uint32_t t = blockIdx.x * LB_INV_TPB + threadIdx.x;
  uint32_t j = 0, i = 0, wt = 0;
  bool act = false;
  if (t < T) {
    smsm_member(a, c, t, members, set_uid, j, i, wt);
    act = msm_live(i, set_live, sig_inf);
  }
  g2a t1{fp2_one(), fp2_one()}, t2 = t1;
  g2j s = jac_infinity<fp2>();
  if (act) {
    t1 = soa_ld<g2a>(sig_aff, n, i);
    t2 = g2a{fp2_mul_fp(t1.x, fp_load(LB_PSI2_CX)), fp2_neg(fp2_mul_fp(t1.y, fp_load(LB_PSI2_CY)))};
    s = jac_add_aff_i<fp2, true>(jac_from_aff(t1), t2);  // finite: lambda + 1 != 0 mod r
  }
  const fp nz = fp_add(fp_sqr(s.z.c0), fp_sqr(s.z.c1));
  const bool ok = act && !fp_is_zero(nz);
  const fp ni = fp_inv_block(ok ? nz : fp_one());
  if (t >= T) return;
  g2j r = jac_infinity<fp2>();
  if (ok) {
    const fp2 zi{fp_mul(s.z.c0, ni), fp_neg(fp_mul(s.z.c1, ni))};
    const fp2 zi2 = fp2_sqr(zi);
    const g2a t3{fp2_mul(s.x, zi2), fp2_mul(fp2_mul(s.y, zi2), zi)};
    const uint64_t wd = scalars[i];
    r = jac_as<fp2>(jac_mul_2d_i<fp2i, true>(aff_as<fp2i>(t1), aff_as<fp2i>(t2), aff_as<fp2i>(t3),
                                            (wd & 0xffffffffu) * wt, (wd >> 32) * wt, 32 + LB_WT_BITS));
  }
  soa_st(terms, T, t, r);
}
#endif  // LB_KG
// block b sums positions [blo[b], bhi[b]) (<= 64, one instance) -> part[b] (stride nb); the
// term of position p is terms[perm ? perm[p] : p] (stride T)
#if LB_KG(7)
__global__ void __launch_bounds__(64) k_seg_sum64(const uint32_t* __restrict__ blo, const uint32_t* __restrict__ bhi,
                                                  uint32_t T, const uint32_t* __restrict__ terms, uint32_t nb,
                                                  uint32_t* __restrict__ part, const uint32_t* __restrict__ perm) {
  const uint32_t b = blockIdx.x, p = blo[b] + threadIdx.x;
  g2j v = p < bhi[b] ? soa_ld<g2j>(terms, T, perm ? perm[p] : p) : jac_infinity<fp2>();
  for (int l = 5; l >= 0; l--) {
    const unsigned d = 1u << l;
    const g2j o = g2j_shfl_down(v, d);
    if (threadIdx.x < d) v = jac_add_i(v, o);
  }
  if (threadIdx.x == 0) soa_st(part, nb, b, v);
}
#endif  // LB_KG
// instance j = sum of part[bo[j] .. bo[j+1]) -> out element j (stride n_out)
#if LB_KG(7)
__global__ void __launch_bounds__(64) k_seg_final(const uint32_t* __restrict__ bo, const uint32_t* __restrict__ part,
                                                  uint32_t nb, uint32_t* __restrict__ out, uint32_t n_out) {
  const uint32_t j = blockIdx.x;
  g2j v = jac_infinity<fp2>();
  for (uint32_t k = bo[j] + threadIdx.x; k < bo[j + 1]; k += 64) v = jac_add_i(v, soa_ld<g2j>(part, nb, k));
  for (int l = 5; l >= 0; l--) {
    const unsigned d = 1u << l;
    const g2j o = g2j_shfl_down(v, d);
    if (threadIdx.x < d) v = jac_add_i(v, o);
  }
  if (threadIdx.x == 0) soa_st(out, n_out, j, v);
}
#endif  // LB_KG

// Root-level search MSM (instances over whole roots: subtrees of the root product tree, modes 0
// and 1): position t of instance j is root u = rlo_j + (t - pre_j) with weight 1 (mode 0) or
// ((u - wa_j) >> wb_j) + 1 <= 64 (mode 1), term [w] S_u from the per-root sums S_u = sum r_i sig_i
// (search_root_sums), one lane per position: 7 doublings + <= 7 additions instead of a 39-bit
// weighted scalar per SET through the bucket MSM.
#if LB_KG(7)
__global__ void __launch_bounds__(LB_TPB) k_rsm_terms(uint32_t T, uint32_t c, smsm_args a,
                                                      const uint32_t* __restrict__ s_root, uint32_t nu,
                                                      uint32_t* __restrict__ terms) {
  const uint32_t t = lb_tid();
  if (t >= T) return;
  const uint32_t j = rmsm_node(a.pre, c, t);
  const uint32_t u = a.rlo[j] + (t - a.pre[j]);
  const uint32_t wt = a.mode[j] == 0u ? 1u : ((u - a.wa[j]) >> a.wb[j]) + 1u;
  const g2j su = soa_ld<g2j>(s_root, nu, u);
  g2j r = jac_infinity<fp2>();
  for (int b = 6; b >= 0; b--) {
    r = jac_dbl_i(r);
    if ((wt >> b) & 1u) r = jac_add_i<fp2, true>(r, su);
  }
  soa_st(terms, T, t, r);
}
#endif  // LB_KG

// The set-level instances of a round once the per-set terms T_i = r_i sig_i exist (search_root_sums
// keeps them): position t's term is [w] T_i, w <= LB_WT_MAX, by an LB_WT_BITS-bit ladder in one lane
// instead of the 43-bit weighted scalar by 8 lanes (k_smsm_terms_g8).
#if LB_KG(7)
__global__ void __launch_bounds__(LB_TPB) k_smsm_terms_pre(uint32_t T, uint32_t c, smsm_args a,
                                                           const uint32_t* __restrict__ members,
                                                           const uint32_t* __restrict__ set_uid,
                                                           const uint32_t* __restrict__ set_terms, uint32_t n,
                                                           uint32_t* __restrict__ terms) {
  const uint32_t t = lb_tid();
  if (t >= T) return;
  uint32_t j, i, wt;
  smsm_member(a, c, t, members, set_uid, j, i, wt);
  const g2j ti = soa_ld<g2j>(set_terms, n, i);  // infinity for a set outside the equation
  g2j r = jac_infinity<fp2>();
  for (int b = LB_WT_BITS - 1; b >= 0; b--) {
    r = jac_dbl_i(r);
    if ((wt >> b) & 1u) r = jac_add_i<fp2, true>(r, ti);
  }
  soa_st(terms, T, t, r);
}
#endif  // LB_KG

// direct kind-1 nodes: Jacobian sum of r_i PK_i over the part's live members -> pk_out (SoA,
// stride c)
#if LB_KG(7)
__global__ void __launch_bounds__(LB_TPB, LB_MINW_GSUM) k_range_pk(uint32_t c, const uint32_t* __restrict__ kind,
                                                       const uint32_t* __restrict__ rlo,
                                                       const uint32_t* __restrict__ rlen,
                                                       const uint32_t* __restrict__ members,
                                                       const uint32_t* __restrict__ set_live, uint32_t n,
                                                       const uint32_t* __restrict__ rpk, uint32_t* __restrict__ pk_out) {
  const uint32_t j = lb_tid();
  if (j >= c || kind[j] != 1u) return;
  g1j acc = jac_infinity<fp>();
  for (uint32_t k = rlo[j]; k < rlo[j] + rlen[j]; k++) {
    const uint32_t i = members[k];
    if (set_live[i]) acc = jac_add_i<fp, true>(acc, aos_ld<g1j>(rpk, i));
  }
  soa_st(pk_out, c, j, acc);
}
#endif  // LB_KG
// weighted tests over parts of one root (mode 2): sum_k (k + 1) sum_{i in part k} r_i PK_i,
// one workgroup per test, lane s owning parts k = s + 64 q (f <= LB_WT_MAX, q < 16): with A_q the
// part sums, sum_q (s + 1 + 64 q) A_q = (s + 1) sum_q A_q + 64 sum_q q A_q, the last by running
// sums (sum_q q A_q = sum_{j >= 1} sum_{q >= j} A_q): two additions per part and one 7-bit ladder
// per lane instead of a ladder per part.
#if LB_KG(7)
__global__ void __launch_bounds__(64) k_test_pk(uint32_t nt, const uint32_t* __restrict__ mode,
                                                const uint32_t* __restrict__ tlo, const uint32_t* __restrict__ tlen,
                                                const uint32_t* __restrict__ per, const uint32_t* __restrict__ members,
                                                const uint32_t* __restrict__ set_live, uint32_t n,
                                                const uint32_t* __restrict__ rpk, uint32_t* __restrict__ pk_out) {
  __shared__ g1j sh[64];
  const uint32_t t = blockIdx.x, lane = threadIdx.x;
  if (t >= nt || mode[t] != 2u) return;
  const uint32_t lo = tlo[t], len = tlen[t], pp = per[t];
  const uint32_t nparts = (len + pp - 1) / pp;
  g1j run = jac_infinity<fp>(), s1 = jac_infinity<fp>();
  if (lane < nparts) {
    const uint32_t qmax = (nparts - 1 - lane) / 64;
    for (int q = (int)qmax; q >= 0; q--) {
      const uint32_t k = lane + 64u * (uint32_t)q;
      const uint32_t a = lo + k * pp, e = lo + (k * pp + pp < len ? k * pp + pp : len);
      for (uint32_t x = a; x < e; x++) {
        const uint32_t i = members[x];
        if (set_live[i]) run = jac_add_i<fp, true>(run, aos_ld<g1j>(rpk, i));
      }
      if (q >= 1) s1 = jac_add_i<fp, true>(s1, run);
    }
  }
  g1j tot = jac_infinity<fp>();
  const uint32_t wt = lane + 1;  // <= 64: 7 bits
  for (int b = 6; b >= 0; b--) {
    tot = jac_dbl_i(tot);
    if ((wt >> b) & 1u) tot = jac_add_i<fp, true>(tot, run);
  }
  for (int b = 0; b < 6; b++) s1 = jac_dbl_i(s1);
  tot = jac_add_i<fp, true>(tot, s1);
  sh[lane] = tot;
  __syncthreads();
  for (uint32_t d = 32; d >= 1; d >>= 1) {
    if (lane < d) sh[lane] = jac_add_i<fp, true>(sh[lane], sh[lane + d]);
    __syncthreads();
  }
  if (lane == 0) soa_st(pk_out, nt, t, sh[0]);
}
#endif  // LB_KG

// ML(PK, H_u) of a G1 Jacobian point into area dst (1 for infinity); lane 0 stages the points
__device__ void w_miller_pk(fp* S, int dst, const g1j& pj_lane0, const uint32_t* __restrict__ h_aff, uint32_t n,
                            uint32_t u) {
  __shared__ int s_inf;
  if (w_lane() == 0) {
    s_inf = jac_is_inf(pj_lane0) ? 1 : 0;
    if (!s_inf) {
      g1a pa;
      g1_to_aff_inl(pa, pj_lane0);
      const g2a h = soa_ld<g2a>(h_aff, n, u);
      w_st(S, LBW_PT + 0, pa.x);
      w_st(S, LBW_PT + 1, pa.y);
      w_st(S, LBW_PT + 2, h.x.c0);
      w_st(S, LBW_PT + 3, h.x.c1);
      w_st(S, LBW_PT + 4, h.y.c0);
      w_st(S, LBW_PT + 5, h.y.c1);
    }
  }
  w_sync();
  const int inf = s_inf;
  w_sync();
  if (inf)
    w_set_one(S, dst);
  else
    w_miller(S, dst);
}
// ML(-G1, Q) of a G2 Jacobian point into area dst (1 for infinity)
__device__ void w_miller_negg1(fp* S, int dst, const g2j& q_lane0) {
  __shared__ int s_inf;
  if (w_lane() == 0) {
    s_inf = jac_is_inf(q_lane0) ? 1 : 0;
    if (!s_inf) {
      g2a a;
      g2_to_aff_inl(a, q_lane0);
      w_st(S, LBW_PT + 0, fp_load(LB_G1X));
      w_st(S, LBW_PT + 1, fp_load(LB_G1NEGY));
      w_st(S, LBW_PT + 2, a.x.c0);
      w_st(S, LBW_PT + 3, a.x.c1);
      w_st(S, LBW_PT + 4, a.y.c0);
      w_st(S, LBW_PT + 5, a.y.c1);
    }
  }
  w_sync();
  const int inf = s_inf;
  w_sync();
  if (inf)
    w_set_one(S, dst);
  else
    w_miller(S, dst);
}
__device__ bool w_eq(fp* S, int a, int b) {
  __shared__ int diff;
  if (w_lane() == 0) diff = 0;
  w_sync();
  if (w_lane() < 12 && !fp_eq(w_ld(S, a + w_lane()), w_ld(S, b + w_lane()))) atomicOr(&diff, 1);
  w_sync();
  const int r = diff;
  w_sync();
  return r == 0;
}

// One search round runs three launches over its items (direct checks first, then weighted
// tests), one wave each:
//   k_search_ml     two blocks per item: side 0 the P factor, side 1 ML(-G1, S);
//   k_search_fe     y_i = FE(P_i ML(-G1, S_i)), verdict of a direct check = (y_i == 1);
//   k_search_match  a test's z = y_{c+t} against the powers of its node's y.
// Direct check j (y_j = FE(X_j), Pairing.finalverify):
//   kind 0 (a subtree of the root product tree, whole roots): P_j = treeP[key_j];
//   kind 1 (part of one root u = key_j): P_j = ML(sum r_i PK_i, H(m_u)), S_j from the range MSM;
//   kind 2 (one set i = key_j): Signature.verify itself, FE(ML(PK_i, H(m_i)) ML(-G1, sig_i)),
//          no blinding and no MSM (a set of a rejected job passes trivially).
// Weighted test t over the f children of a failing node whose FE value y is known: with weights
// w_k = k + 1, z = FE(prod_k P_k^{w_k} ML(-G1, sum_k w_k S_k)) = prod_k y_k^{w_k}, so when
// exactly one child k* fails (y_k* = y), z = y^{k*+1} and the match returns k* + 1; it returns
// 0 when z is no power y^1..y^f (two or more failing children: the caller checks them directly).
// A wrong match needs prod over the other failing children of y_k^{w_k - w_k*} = 1, which the
// secret blinding scalars make as unlikely (2^-64) as a passing batch with an invalid set.
//   mode 1: the children are f consecutive nodes v0 + k of the root product tree: P side
//           prod_k treeP[v0 + k]^{k+1} by running products (2f Fp12 multiplications);
//   mode 2: the children are parts of root u: P side ML(sum_k (k+1) PKsum_k, H_u) (k_test_pk).
// A look-ahead test (t >= n_fresh) belongs to direct check tyidx[t] of the same round.  With
// skip_ahead it is launched after k_search_fe of the direct checks and skipped when that check
// passed (its y is 1): least work.  Without, everything is one launch pair: one FE latency less
// per round (LB_SEARCH_MERGE), k_search_match ignoring the tests of passing checks.
struct srch_items {
  uint32_t c, nt, n_fresh, skip_ahead;
  const uint32_t *kind, *key, *dmidx;                     // direct checks
  const uint32_t *tmode, *tf, *tv0, *tu, *tmidx, *tyidx;  // weighted tests
};
__device__ bool srch_skip(fp* S, const srch_items& I, uint32_t it, const uint32_t* __restrict__ ybuf) {
  if (!I.skip_ahead || it < I.c + I.n_fresh) return false;
  w_load_soa12(S, LBW_A(6), ybuf, I.c + I.nt, I.tyidx[it - I.c]);
  return w_is_one(S, LBW_A(6));
}
#if LB_KG(5)
__global__ void __launch_bounds__(64) k_search_ml(srch_items I, uint32_t it0, uint32_t cnt, uint32_t cm,
                                                  const uint32_t* __restrict__ treeP, uint32_t n2m,
                                                  const uint32_t* __restrict__ pk_d, const uint32_t* __restrict__ pk_t,
                                                  const uint32_t* __restrict__ h_aff, uint32_t n,
                                                  const uint32_t* __restrict__ s_out,
                                                  const uint32_t* __restrict__ pk_aff,
                                                  const uint32_t* __restrict__ sig_aff,
                                                  const uint32_t* __restrict__ sig_inf,
                                                  const uint32_t* __restrict__ set_live,
                                                  const uint32_t* __restrict__ set_uid,
                                                  const uint32_t* __restrict__ ybuf, uint32_t* __restrict__ ml) {
  LBW_SHARED_ML(S);
  if (blockIdx.x >= 2 * cnt) return;
  const uint32_t it = it0 + (blockIdx.x >> 1), side = blockIdx.x & 1u, N2 = 2 * (I.c + I.nt);
  const int lane = threadIdx.x;
  w_init_consts(S, LBW_PROGS_ALL);
  if (srch_skip(S, I, it, ybuf)) {
    w_set_one(S, LBW_A(0));
  } else if (it < I.c) {
    const uint32_t kd = I.kind[it], k = I.key[it];
    if (kd == 2u && !set_live[k]) {  // a set of a rejected job takes no part
      w_set_one(S, LBW_A(0));
    } else if (side == 0) {
      if (kd == 0u) {
        w_load_soa12(S, LBW_A(0), treeP, n2m, k);
      } else {
        g1j pj;
        uint32_t u = 0;
        if (lane == 0) {
          pj = kd == 1u ? soa_ld<g1j>(pk_d, I.c, it) : jac_from_aff(soa_ld<g1a>(pk_aff, n, k));
          u = kd == 1u ? k : set_uid[k];
        }
        w_miller_pk(S, LBW_A(0), pj, h_aff, n, u);
      }
    } else {
      g2j q;
      if (lane == 0) {
        if (kd == 2u) q = sig_inf[k] ? jac_infinity<fp2>() : jac_from_aff(soa_ld<g2a>(sig_aff, n, k));
        else q = soa_ld<g2j>(s_out, cm, I.dmidx[it]);
      }
      w_miller_negg1(S, LBW_A(0), q);
    }
  } else {
    const uint32_t t = it - I.c;
    if (side == 0) {
      if (I.tmode[t] == 1u) {
        const uint32_t v0 = I.tv0[t];
        w_set_one(S, LBW_A(0));
        w_set_one(S, LBW_A(1));
        for (int k = (int)I.tf[t] - 1; k >= 0; k--) {
          w_load_soa12(S, LBW_A(2), treeP, n2m, v0 + (uint32_t)k);
          w_mul(S, LBW_A(1), LBW_A(1), LBW_A(2));
          w_mul(S, LBW_A(0), LBW_A(0), LBW_A(1));
        }
      } else {
        g1j pj;
        if (lane == 0) pj = soa_ld<g1j>(pk_t, I.nt, t);
        w_miller_pk(S, LBW_A(0), pj, h_aff, n, I.tu[t]);
      }
    } else {
      g2j q;
      if (lane == 0) q = soa_ld<g2j>(s_out, cm, I.tmidx[t]);
      w_miller_negg1(S, LBW_A(0), q);
    }
  }
  w_store_soa12(S, LBW_A(0), ml, N2, 2 * it + side);
}
#endif  // LB_KG
#if LB_KG(5)
__global__ void __launch_bounds__(64) k_search_fe(srch_items I, uint32_t it0, uint32_t cnt,
                                                  const uint32_t* __restrict__ ml, uint32_t* __restrict__ ybuf,
                                                  int32_t* __restrict__ verdict) {
  LBW_SHARED(S);
  if (blockIdx.x >= cnt) return;
  const uint32_t it = it0 + blockIdx.x, N = I.c + I.nt;
  w_init_consts(S);
  if (srch_skip(S, I, it, ybuf)) {
    w_set_one(S, LBW_A(0));
  } else {
    w_load_soa12(S, LBW_A(0), ml, 2 * N, 2 * it);
    w_load_soa12(S, LBW_A(7), ml, 2 * N, 2 * it + 1);
    w_mul(S, LBW_A(0), LBW_A(0), LBW_A(7));
    w_final_exp(S, LBW_A(0), LBW_A(0));
  }
  const bool one = w_is_one(S, LBW_A(0));
  w_store_soa12(S, LBW_A(0), ybuf, N, it);
  if (threadIdx.x == 0 && it < I.c) verdict[it] = one ? 1 : 0;
}
#endif  // LB_KG
// z = y^k, 1 <= k <= f <= LB_WT_MAX, by baby steps / giant steps: baby[i] = y^(i+1) for i < m
// (m = min(f, 32), in LDS), then w = z y^(-m j) for j = 0, 1, ... (y^-1 = conj(y): FE values lie
// in the cyclotomic subgroup) compared by lanes i < m against baby[i] at once; k = m j + i + 1.
// At most 32 + 32 Fp12 multiplications, against f for the plain walk.
#define LB_BSGS_M 32
#if LB_KG(5)
__global__ void __launch_bounds__(64) k_search_match(srch_items I, const uint32_t* __restrict__ y_up,
                                                     const uint32_t* __restrict__ ybuf, int32_t* __restrict__ out_k) {
  LBW_SHARED(S);
  __shared__ uint32_t baby[LB_BSGS_M][144];
  __shared__ uint32_t s_hit;
  const uint32_t t = blockIdx.x;
  if (t >= I.nt) return;
  const uint32_t N = I.c + I.nt, f = I.tf[t];
  const int lane = w_lane();
  w_init_consts(S);
  if (t < I.n_fresh) w_load_soa12(S, LBW_A(7), y_up, I.n_fresh, t);
  else w_load_soa12(S, LBW_A(7), ybuf, N, I.tyidx[t]);
  if (w_is_one(S, LBW_A(7))) {
    if (threadIdx.x == 0) out_k[t] = 0;
    return;
  }
  w_load_soa12(S, LBW_A(0), ybuf, N, I.c + t);
  const uint32_t m = f < LB_BSGS_M ? f : LB_BSGS_M;
  w_conj(S, LBW_A(1), LBW_A(7));  // A1 runs over y^i (conj twice: a copy)
  w_conj(S, LBW_A(1), LBW_A(1));
  for (uint32_t i = 0; i < m; i++) {
    if (lane < 12) {
      const fp v = w_ld(S, LBW_A(1) + lane);
      LB_UNROLL for (int w = 0; w < 12; w++) baby[i][12 * lane + w] = v.v[w];
    }
    w_sync();
    if (i + 1 < m) w_mul(S, LBW_A(1), LBW_A(1), LBW_A(7));
  }
  w_conj(S, LBW_A(2), LBW_A(1));  // A1 = y^m after the loop: A2 = y^-m
  int hit = 0;
  for (uint32_t j = 0; m * j < f && !hit; j++) {
    if (lane == 0) s_hit = 0xffffffffu;
    w_sync();
    if ((uint32_t)lane < m) {
      uint32_t d = 0;
      for (int k = 0; k < 12; k++) {
        const fp v = w_ld(S, LBW_A(0) + k);
        LB_UNROLL for (int w = 0; w < 12; w++) d |= v.v[w] ^ baby[lane][12 * k + w];
      }
      const uint32_t kk = m * j + (uint32_t)lane + 1u;
      if (d == 0 && kk <= f) atomicMin(&s_hit, kk);
    }
    w_sync();
    const uint32_t h = s_hit;
    w_sync();
    if (h != 0xffffffffu) hit = (int)h;
    else if (m * (j + 1) < f) w_mul(S, LBW_A(0), LBW_A(0), LBW_A(2));
  }
  if (threadIdx.x == 0) out_k[t] = hit;
}
#endif  // LB_KG

// ---------------------------------------------------------------- per-job leaves
// Job status follows the reference's error precedence: aggregation / pubkey decoding happen
// first (main thread getAggregatedPubkey, worker deserializeSet), then every signature is
// decoded (maybeBatch.ts:18-25), then mul_n_aggregate rejects an infinite pubkey.
__device__ __forceinline__ int job_status_of(uint32_t a, uint32_t e, const int32_t* sig_status, const int32_t* pk_status) {
  int st = (a == e) ? LB_EMPTY_SIGNATURE_SET : LB_OK;
  for (uint32_t i = a; i < e && st == LB_OK; i++)
    if (pk_status[i] != LB_OK && pk_status[i] != LB_PK_IS_INFINITY) st = pk_status[i];
  for (uint32_t i = a; i < e && st == LB_OK; i++)
    if (sig_status[i] != LB_OK) st = sig_status[i];
  for (uint32_t i = a; i < e && st == LB_OK; i++)
    if (pk_status[i] != LB_OK) st = pk_status[i];
  return st;
}

// job_status[j] and, for each of its sets, whether the set takes part in the batch equation
#if LB_KG(0)
__global__ void __launch_bounds__(LB_TPB) k_job_status(uint32_t n_jobs, const uint32_t* __restrict__ job_off,
                                                       const int32_t* __restrict__ sig_status,
                                                       const int32_t* __restrict__ pk_status,
                                                       int32_t* __restrict__ job_status,
                                                       uint32_t* __restrict__ set_live) {
  const uint32_t j = lb_tid();
  if (j >= n_jobs) return;
  const uint32_t a = job_off[j], e = job_off[j + 1];
  const int st = job_status_of(a, e, sig_status, pk_status);
  job_status[j] = st;
  for (uint32_t i = a; i < e; i++) set_live[i] = st == LB_OK ? 1u : 0u;
}
#endif  // LB_KG

// Speculative liveness for the per-root sums: set_spec[i] = 1 iff set i's job would be live if
// every signature decodes (the pubkey statuses alone), so the per-root chain needs only the
// pubkey side, not the signature decode.  A decode failure can only clear a set's liveness:
// k_live_mismatch flags any set counted in the sums that the full statuses exclude.
#if LB_KG(0)
__global__ void __launch_bounds__(LB_TPB) k_spec_live(uint32_t n_jobs, const uint32_t* __restrict__ job_off,
                                                      const int32_t* __restrict__ pk_status,
                                                      uint32_t* __restrict__ set_spec) {
  const uint32_t j = lb_tid();
  if (j >= n_jobs) return;
  const uint32_t a = job_off[j], e = job_off[j + 1];
  bool live = a != e;
  for (uint32_t i = a; i < e; i++) live &= pk_status[i] == LB_OK;
  for (uint32_t i = a; i < e; i++) set_spec[i] = live ? 1u : 0u;
}
#endif  // LB_KG
#if LB_KG(0)
__global__ void __launch_bounds__(LB_TPB) k_live_mismatch(uint32_t n, const uint32_t* __restrict__ set_live,
                                                          const uint32_t* __restrict__ set_spec,
                                                          uint32_t* __restrict__ flag) {
  const uint32_t i = lb_tid();
  if (i < n && set_spec[i] && !set_live[i]) *flag = 1u;
}
#endif  // LB_KG

// chunk c of a group: Jacobian sum of r_i PK_i over its live members -> gacc (stride n)
#if LB_KG(4)
__global__ void __launch_bounds__(LB_TPB, LB_MINW_GSUM) k_gsum_chunks(uint32_t n, const uint32_t* __restrict__ n_u,
                                                        const uint32_t* __restrict__ gch,
                                                        const uint32_t* __restrict__ chunk_beg,
                                                        const uint32_t* __restrict__ chunk_end,
                                                        const uint32_t* __restrict__ members,
                                                        const uint32_t* __restrict__ set_live,
                                                        const uint32_t* __restrict__ rpk,
                                                        uint32_t* __restrict__ gacc) {
  const uint32_t c = lb_tid();
  if (c >= gch[*n_u]) return;
  jac<lb_g1f> acc = jac_infinity<lb_g1f>();
  for (uint32_t k = chunk_beg[c]; k < chunk_end[c]; k++) {
    const uint32_t i = members[k];
    if (!set_live[i]) continue;
    acc = jac_add_i<lb_g1f, true>(acc, jac_as<lb_g1f>(aos_ld<g1j>(rpk, i)));  // r*PK (infinity handled)
  }
  soa_st(gacc, n, c, jac_as<fp>(acc));
}
#endif  // LB_KG

// Chunk c of a group (<= LB_STRAUS_CHUNK members of one root): sum over its live members of
// r_i PK_i with the blinding folded in (round 6, the loaded-device form): r_i = lo_i + hi_i lambda,
// so the chunk sum is a joint (Straus) double-and-add over the 32 bit positions of all its
// members' lo / hi halves, ONE doubling chain per chunk instead of one per set:
//   acc = 2 acc;  acc += T_k[d_k]  for each member k with digit d_k = lo_k bit + 2 hi_k bit,
//   T_k = {PK, [lambda]PK = (beta x, y), PK + [lambda]PK = (beta^2 x, -y) = (-x - beta x, -y)}.
// Per set ~32 mixed additions + 32/8 doublings against k_pk_blind's per-set ladder (32 + 32) and
// the chunk sum's Jacobian addition.  Equal keys in a chunk (duplicate validators) meet P = +-Q:
// jac_add_aff_i handles them.  The per-set r_i PK_i (the search's) come from k_pk_blind mode 2
// when a search needs them.
#ifndef LB_STRAUS_CHUNK
#define LB_STRAUS_CHUNK 8
#endif
// The lanes take the chunks in order of decreasing member count (k_chunk_order: a counting sort
// by size), so a wave's chunks have equal counts but at its edges and the member loop runs to the
// wave's largest count: in root order the single-member roots' chunks (every aggregate-and-proof
// root) shared waves with 8-member chunks and idled 7 of 8 additions (measured: the Straus form
// 5 % below the per-set ladders before the ordering).
#if LB_KG(14)
__global__ void __launch_bounds__(LB_TPB) k_chunk_order(const uint32_t* __restrict__ n_u, const uint32_t* __restrict__ gch,
                                                        const uint32_t* __restrict__ chunk_beg,
                                                        const uint32_t* __restrict__ chunk_end,
                                                        uint32_t* __restrict__ cnt, uint32_t* __restrict__ order,
                                                        uint32_t pass) {
  // pass 0: cnt[m] = chunks of m members (m <= LB_STRAUS_CHUNK); pass 1: order (m descending),
  // cnt[LB_STRAUS_CHUNK + 1 + m] the per-size cursors (zeroed with the counts)
  const uint32_t c = lb_tid();
  if (c >= gch[*n_u]) return;
  const uint32_t m = chunk_end[c] - chunk_beg[c];
  if (pass == 0) {
    atomicAdd(&cnt[m], 1u);
    return;
  }
  uint32_t base = 0;
  for (uint32_t q = LB_STRAUS_CHUNK; q > m; q--) base += cnt[q];
  order[base + atomicAdd(&cnt[LB_STRAUS_CHUNK + 1 + m], 1u)] = c;
}
#endif  // LB_KG
#if LB_KG(14)
__global__ void __launch_bounds__(LB_TPB, LB_MINW_GSUM) k_gsum_straus(uint32_t n, const uint32_t* __restrict__ n_u,
                                                        const uint32_t* __restrict__ gch,
                                                        const uint32_t* __restrict__ chunk_beg,
                                                        const uint32_t* __restrict__ chunk_end,
                                                        const uint32_t* __restrict__ order,
                                                        const uint32_t* __restrict__ members,
                                                        const uint32_t* __restrict__ set_live,
                                                        const uint32_t* __restrict__ pk3,
                                                        const uint64_t* __restrict__ scalars,
                                                        uint32_t* __restrict__ gacc) {
  const uint32_t t = lb_tid(), nch = gch[*n_u];
  if (blockIdx.x * LB_TPB >= nch) return;  // whole wave idle (uniform)
  const bool act = t < nch;
  const uint32_t c = act ? order[t] : 0u;
  const uint32_t b = act ? chunk_beg[c] : 0u, m = act ? chunk_end[c] - b : 0u;
  // the wave's largest count: its first lane's (decreasing order)
  const uint32_t mw = (uint32_t)__builtin_amdgcn_readfirstlane((int)m);
  uint32_t idx[LB_STRAUS_CHUNK], lo[LB_STRAUS_CHUNK], hi[LB_STRAUS_CHUNK];
  LB_UNROLL for (int k = 0; k < LB_STRAUS_CHUNK; k++) {
    idx[k] = 0;
    lo[k] = hi[k] = 0;  // absent or dead members: digit 0 throughout
    if ((uint32_t)k < m) {
      const uint32_t i = members[b + k];
      idx[k] = i;
      if (set_live[i]) {
        const uint64_t w = scalars[i];
        lo[k] = (uint32_t)w;
        hi[k] = (uint32_t)(w >> 32);
      }
    }
  }
  jac<lb_g1f> acc = jac_infinity<lb_g1f>();
#pragma clang loop unroll(disable)
  for (int bit = 31; bit >= 0; bit--) {
    if (!jac_is_inf(acc)) acc = jac_dbl_i(acc);
    LB_UNROLL for (int k = 0; k < LB_STRAUS_CHUNK; k++) {
      if ((uint32_t)k >= mw) break;  // wave-uniform
      const uint32_t d = ((lo[k] >> bit) & 1u) | (((hi[k] >> bit) & 1u) << 1);
      if (d != 0u) {
        const g1x3 t = aos_ld<g1x3>(pk3, idx[k]);
        aff<lb_g1f> q;
        q.x = lb_g1f{d == 1u ? t.x : (d == 2u ? t.bx : fp_neg(fp_add(t.x, t.bx)))};
        q.y = lb_g1f{d == 3u ? fp_neg(t.y) : t.y};
        acc = jac_add_aff_i<lb_g1f, true>(acc, q);
      }
    }
  }
  if (act) soa_st(gacc, n, c, jac_as<fp>(acc));
}
#endif  // LB_KG

// Per-root sums of a batch alone (round 6; replaces k_gsum_chunks + the k_gsum_tree launches):
// the chunk sums of r_i PK_i (<= gchunk members per lane), then a segmented shuffle tree over the
// wave's 64 chunks by root (wave_seg_sum); the first lane of each (root, wave) segment writes the
// segment's sum to gacc, and k_gsum_final (mode 2) adds a root's segment heads.  One launch, the
// partials in registers, log2(64) levels.
#if LB_KG(14)
__global__ void __launch_bounds__(LB_TPB, LB_MINW_GSUM) k_gsum_wave(uint32_t n, const uint32_t* __restrict__ n_u,
                                                      const uint32_t* __restrict__ gch,
                                                      const uint32_t* __restrict__ chunk_beg,
                                                      const uint32_t* __restrict__ chunk_end,
                                                      const uint32_t* __restrict__ chunk_root,
                                                      const uint32_t* __restrict__ members,
                                                      const uint32_t* __restrict__ set_live,
                                                      const uint32_t* __restrict__ rpk,
                                                      uint32_t* __restrict__ gacc) {
  const uint32_t c = lb_tid(), nch = gch[*n_u];
  if (blockIdx.x * LB_TPB >= nch) return;  // whole wave idle (uniform)
  const bool act = c < nch;
  jac<lb_g1f> acc = jac_infinity<lb_g1f>();
  bool starts = true;
  if (act) {
    for (uint32_t k = chunk_beg[c]; k < chunk_end[c]; k++) {
      const uint32_t i = members[k];
      if (!set_live[i]) continue;
      acc = jac_add_i<lb_g1f, true>(acc, jac_as<lb_g1f>(aos_ld<g1j>(rpk, i)));
    }
    starts = c == gch[chunk_root[c]];
  }
  uint32_t rel, left;
  wave_segments(starts, rel, left);
  acc = wave_seg_sum(acc, rel, left);
  if (act && rel == 0) soa_st(gacc, n, c, jac_as<fp>(acc));
}
#endif  // LB_KG

// One level of the per-root sum tree over the chunk sums (in place, strided): at stride s, the
// lane of chunk c with (c - gch[u]) a multiple of LB_GSUM_FAN s adds the partials at c + k s,
// k = 1 .. LB_GSUM_FAN - 1, of its own root; after the levels with s < max chunks per root,
// gacc[gch[u]] holds P_u.  The reads of one lane, [c, c + FAN s), are nobody else's writes.
// (The serial chains this replaces, up to 32 members per lane and then up to 32 chunk sums per
// root on one lane, were the longest per-root latency of a batch alone: VERDICT r4.)
#if LB_KG(4)
__global__ void __launch_bounds__(LB_TPB, LB_MINW_GSUM) k_gsum_tree(uint32_t n, const uint32_t* __restrict__ n_u,
                                                      const uint32_t* __restrict__ gch,
                                                      const uint32_t* __restrict__ chunk_root, uint32_t s,
                                                      uint32_t* __restrict__ gacc) {
  const uint32_t c = lb_tid();
  if (c >= gch[*n_u]) return;
  const uint32_t u = chunk_root[c], base = gch[u], end = gch[u + 1];
  if ((c - base) % (LB_GSUM_FAN * s) != 0 || c + s >= end) return;
  jac<lb_g1f> acc = jac_as<lb_g1f>(soa_ld<g1j>(gacc, n, c));
  LB_UNROLL for (uint32_t k = 1; k < LB_GSUM_FAN; k++)
    if (c + k * s < end) acc = jac_add_i<lb_g1f, true>(acc, jac_as<lb_g1f>(soa_ld<g1j>(gacc, n, c + k * s)));
  soa_st(gacc, n, c, jac_as<fp>(acc));
}
#endif  // LB_KG

// P_u (the tree's root at gacc[gch[u]]) to affine (one batched inversion per block); gp_inf[u]
// flags P_u = infinity (no live member, or members cancelling), whose Miller value is 1.
#if LB_KG(4)
__global__ void __launch_bounds__(LB_INV_TPB, LB_MINW) k_gsum_final(uint32_t n, const uint32_t* __restrict__ n_u,
                                                           const uint32_t* __restrict__ gch,
                                                           const uint32_t* __restrict__ gacc,
                                                           uint32_t* __restrict__ gp_aff,
                                                           uint32_t* __restrict__ gp_inf, uint32_t serial) {
  const uint32_t u = blockIdx.x * LB_INV_TPB + threadIdx.x;
  const uint32_t nu = *n_u;
  if (blockIdx.x * LB_INV_TPB >= nu) return;  // whole block idle (uniform)
  const bool act = u < nu;
  g1j acc = jac_infinity<fp>();
  if (act) {
    if (serial == 1)  // (under load, and A/B: LB_GSUM_TREE=0) the root's chunk sums added on this lane
      for (uint32_t c = gch[u]; c < gch[u + 1]; c++) acc = jac_add(acc, soa_ld<g1j>(gacc, n, c));
    else if (serial == 2)  // k_gsum_wave: the root's segment heads (first chunk, then wave boundaries)
      for (uint32_t c = gch[u]; c < gch[u + 1]; c = (c / LB_TPB + 1) * LB_TPB) acc = jac_add(acc, soa_ld<g1j>(gacc, n, c));
    else  // k_gsum_tree: the tree's root
      acc = soa_ld<g1j>(gacc, n, gch[u]);
  }
  const bool zero = jac_is_inf(acc);
  // a block whose sums all have Z = 1 (the unblinded 1-set call's affine PK) skips the inversion
  const bool need = act && !zero && !fp_eq(acc.z, fp_one());
  const fp zi = __syncthreads_or(need) ? fp_inv_block(need ? acc.z : fp_one()) : fp_one();
  if (!act) return;
  g1a a;
  if (zero) {
    a.x = fp_zero();
    a.y = fp_zero();
  } else {
    const fp zi2 = fp_sqr(zi);
    a.x = fp_mul(acc.x, zi2);
    a.y = fp_mul(fp_mul(acc.y, zi2), zi);
  }
  soa_st(gp_aff, n, u, a);
  gp_inf[u] = zero ? 1u : 0u;
}
#endif  // LB_KG

// element e of an Fp12 SoA array (stride n) <- 1
#if LB_KG(0)
__global__ void __launch_bounds__(64) k_set_one(uint32_t* __restrict__ base, uint32_t n, uint32_t e) {
  if (threadIdx.x == 0) soa_st(base, n, e, fp12_one());
}
#endif  // LB_KG

// element e of a G2 Jacobian SoA array (stride n) <- infinity
#if LB_KG(0)
__global__ void __launch_bounds__(64) k_g2_set_inf(uint32_t* __restrict__ base, uint32_t n, uint32_t e) {
  if (threadIdx.x == 0) soa_st(base, n, e, jac_infinity<fp2>());
}
#endif  // LB_KG

// Message product tree, one level (one wave per node), over leaves [0, *n_u) only.  A node
// whose leaf range starts at or past *n_u is never read; one whose right half does is a copy.
#if LB_KG(5)
__global__ void __launch_bounds__(64) k_tree_up_U(uint32_t m, uint32_t lo, const uint32_t* __restrict__ n_u,
                                                  uint32_t* __restrict__ treeP) {
  LBW_SHARED(S);
  const uint32_t i = lo + blockIdx.x, span = m / lo, start = blockIdx.x * span, nu = *n_u;
  if (start >= nu) return;
  w_init_consts(S);  // the programs' padding reads the constant zero slot
  w_load_soa12(S, LBW_A(0), treeP, 2 * m, 2 * i);
  if (start + span / 2 < nu) {
    w_load_soa12(S, LBW_A(1), treeP, 2 * m, 2 * i + 1);
    w_mul(S, LBW_A(0), LBW_A(0), LBW_A(1));
  }
  w_store_soa12(S, LBW_A(0), treeP, 2 * m, i);
}
#endif  // LB_KG

// Row-engine forms of the per-root Miller loop and a product-tree level for batches with few
// distinct roots (latency: one 16-wave workgroup per root / node, lb_row.h); the engine picks
// them up to lb_engine::row_max items and the wave / lane forms above (less work per item) beyond.
#if LB_KG(10)
__global__ void __launch_bounds__(LBR_NT) k_miller_row(uint32_t n, uint32_t m, const uint32_t* __restrict__ n_u,
                                                        const uint32_t* __restrict__ gp_aff,
                                                        const uint32_t* __restrict__ gp_inf,
                                                        const uint32_t* __restrict__ h_aff, uint32_t* __restrict__ treeP) {
  LBR_SHARED_MILLER(S);
  const uint32_t u = blockIdx.x;
  if (u >= *n_u) return;
  const int t = threadIdx.x;
  r_init(S, LBR_MILLER_COUNT, LBR_MILLER_FIRST);
  if (gp_inf[u] != 0) {  // uniform
    r_set_one(S, LBR_A(0));
  } else {
    if (t < 6) {
      const uint32_t* base = t < 2 ? gp_aff + (size_t)12 * t * n : h_aff + (size_t)12 * (t - 2) * n;
      fp v;
      LB_UNROLL for (int w = 0; w < 12; w++) v.v[w] = base[(size_t)w * n + u];
      r_stage_fp(S, t, v);
    }
    r_sync();
    r_import_staged(S, LBR_PT, 6);
    r_miller(S, LBR_A(0));
  }
  r_store_soa12(S, LBR_A(0), treeP, 2 * m, m + u);
}
#endif  // LB_KG
#if LB_KG(10)
__global__ void __launch_bounds__(LBR_NT) k_tree_up_row(uint32_t m, uint32_t lo, const uint32_t* __restrict__ n_u,
                                                      uint32_t* __restrict__ treeP) {
  LBR_SHARED(S);
  const uint32_t i = lo + blockIdx.x, span = m / lo, start = blockIdx.x * span, nu = *n_u;
  if (start >= nu) return;
  r_init(S);
  r_load_soa12(S, LBR_A(0), treeP, 2 * m, 2 * i);
  if (start + span / 2 < nu) {
    r_load_soa12(S, LBR_A(1), treeP, 2 * m, 2 * i + 1);
    r_mul(S, LBR_A(0), LBR_A(0), LBR_A(1));
  }
  r_store_soa12(S, LBR_A(0), treeP, 2 * m, i);
}
#endif  // LB_KG

// fS = ML(-G1, S_root) (1 if S_root is infinity): the G2 half of the root partial product,
// computed while the per-set Miller loops still run.  Output: 12 Fp in Montgomery form.
#if LB_KG(5)
__global__ void __launch_bounds__(64) k_ml_S(uint32_t m, const uint32_t* __restrict__ treeS, uint32_t* __restrict__ fS) {
  LBW_SHARED_ML(S);
  __shared__ int s_inf;
  const int lane = threadIdx.x;
  w_init_consts(S, LBW_PROGS_ALL);
  if (lane == 0) {
    g2j Sj = soa_ld<g2j>(treeS, 2 * m, 1);
    s_inf = jac_is_inf(Sj) ? 1 : 0;
    if (!s_inf) {
      g2a a;
      g2_to_aff_inl(a, Sj);
      w_st(S, LBW_PT + 0, fp_load(LB_G1X));
      w_st(S, LBW_PT + 1, fp_load(LB_G1NEGY));
      w_st(S, LBW_PT + 2, a.x.c0);
      w_st(S, LBW_PT + 3, a.x.c1);
      w_st(S, LBW_PT + 4, a.y.c0);
      w_st(S, LBW_PT + 5, a.y.c1);
    }
  }
  w_sync();
  if (s_inf)
    w_set_one(S, LBW_A(7));
  else
    w_miller(S, LBW_A(7));
  w_store_soa12(S, LBW_A(7), fS, 1, 0);
}
#endif  // LB_KG
#if LB_KG(11)
__global__ void __launch_bounds__(LBR_NT) k_ml_S_row(uint32_t m, const uint32_t* __restrict__ treeS, uint32_t* __restrict__ fS) {
  LBR_SHARED_MILLER(S);
  __shared__ int s_inf;
  __shared__ fp pv[6];
  r_init(S, LBR_MILLER_COUNT, LBR_MILLER_FIRST);
  if (threadIdx.x == 0) {
    const g2j Sj = soa_ld<g2j>(treeS, 2 * m, 1);
    s_inf = jac_is_inf(Sj) ? 1 : 0;
    if (!s_inf) {
      g2a a;
      g2_to_aff_inl(a, Sj);
      pv[0] = fp_load(LB_G1X);
      pv[1] = fp_load(LB_G1NEGY);
      pv[2] = a.x.c0;
      pv[3] = a.x.c1;
      pv[4] = a.y.c0;
      pv[5] = a.y.c1;
    }
  }
  r_sync();
  if (s_inf) {
    r_set_one(S, LBR_A(7));
  } else {
    r_import_fps(S, LBR_PT, pv, 6);
    r_miller(S, LBR_A(7));
  }
  r_store_soa12(S, LBR_A(7), fS, 1, 0);
}
#endif  // LB_KG

// root verdict: FE(P_root * fS) == 1   (Pairing.finalverify over the whole batch)
// (the FE value y goes to y_out for the invalid-set search)
#if LB_KG(5)
__global__ void __launch_bounds__(64) k_root_check(uint32_t m, const uint32_t* __restrict__ treeP,
                                                   const uint32_t* __restrict__ fS, int32_t* __restrict__ verdict,
                                                   uint32_t* __restrict__ y_out) {
  LBW_SHARED(S);
  w_init_consts(S);
  w_load_soa12(S, LBW_A(0), treeP, 2 * m, 1);
  w_load_soa12(S, LBW_A(7), fS, 1, 0);
  w_mul(S, LBW_A(0), LBW_A(0), LBW_A(7));
  w_final_exp(S, LBW_A(0), LBW_A(0));
  bool one = w_is_one(S, LBW_A(0));
  w_store_soa12(S, LBW_A(0), y_out, 1, 0);
  if (threadIdx.x == 0) verdict[0] = one ? 1 : 0;
}
#endif  // LB_KG
#if LB_KG(11)
__global__ void __launch_bounds__(LBR_NT) k_root_check_row(uint32_t m, const uint32_t* __restrict__ treeP,
                                                       const uint32_t* __restrict__ fS, int32_t* __restrict__ verdict,
                                                       uint32_t* __restrict__ y_out) {
  LBR_SHARED(S);
  r_init(S);
  r_load_soa12(S, LBR_A(0), treeP, 2 * m, 1);
  r_load_soa12(S, LBR_A(7), fS, 1, 0);
  r_mul(S, LBR_A(0), LBR_A(0), LBR_A(7));
  r_final_exp(S, LBR_A(0), LBR_A(0));
  const bool one = r_is_one(S, LBR_A(0));
  r_store_soa12(S, LBR_A(0), y_out, 1, 0);
  if (threadIdx.x == 0) verdict[0] = one ? 1 : 0;
}
#endif  // LB_KG

// root partial product P_root * fS as 576 bytes (multi-GPU exchange format)
#if LB_KG(5)
__global__ void __launch_bounds__(64) k_root_partial(uint32_t m, const uint32_t* __restrict__ treeP,
                                                     const uint32_t* __restrict__ fS, uint8_t* __restrict__ out576) {
  LBW_SHARED(S);
  w_init_consts(S);
  w_load_soa12(S, LBW_A(0), treeP, 2 * m, 1);
  w_load_soa12(S, LBW_A(7), fS, 1, 0);
  w_mul(S, LBW_A(0), LBW_A(0), LBW_A(7));
  if (threadIdx.x < 12) fp_plain_to_be48(out576 + 48 * threadIdx.x, fp_from_mont(w_ld(S, LBW_A(0) + threadIdx.x)));
}
#endif  // LB_KG
#if LB_KG(11)
__global__ void __launch_bounds__(LBR_NT) k_root_partial_row(uint32_t m, const uint32_t* __restrict__ treeP,
                                                         const uint32_t* __restrict__ fS, uint8_t* __restrict__ out576) {
  LBR_SHARED(S);
  r_init(S);
  r_load_soa12(S, LBR_A(0), treeP, 2 * m, 1);
  r_load_soa12(S, LBR_A(7), fS, 1, 0);
  r_mul(S, LBR_A(0), LBR_A(0), LBR_A(7));
  r_export(S, LBR_A(0), 12);
  if (threadIdx.x < 12) fp_plain_to_be48(out576 + 48 * threadIdx.x, fp_from_mont(r_fp_of_staged(S, threadIdx.x)));
}
#endif  // LB_KG

#if LB_KG(5)
__global__ void __launch_bounds__(64) k_partials_check(uint32_t n, const uint8_t* __restrict__ parts,
                                                       int32_t* __restrict__ ok) {
  LBW_SHARED(S);
  __shared__ int bad;
  const int lane = threadIdx.x;
  if (lane == 0) bad = 0;
  w_init_consts(S);
  w_set_one(S, LBW_A(0));
  for (uint32_t i = 0; i < n; i++) {
    if (lane < 12) {
      fp x;
      if (!fp_plain_from_be48(x, parts + (size_t)576 * i + 48 * lane, 0xff)) atomicOr(&bad, 1);
      w_st(S, LBW_A(7) + lane, fp_to_mont(x));
    }
    w_sync();
    w_mul(S, LBW_A(0), LBW_A(0), LBW_A(7));
  }
  w_final_exp(S, LBW_A(0), LBW_A(0));
  bool one = w_is_one(S, LBW_A(0));
  if (lane == 0) *ok = (one && !bad) ? 1 : 0;
}
#endif  // LB_KG
#if LB_KG(11)
__global__ void __launch_bounds__(LBR_NT) k_partials_check_row(uint32_t n, const uint8_t* __restrict__ parts,
                                                           int32_t* __restrict__ ok) {
  LBR_SHARED(S);
  __shared__ int bad;
  const int t = threadIdx.x;
  if (t == 0) bad = 0;
  r_init(S);
  r_set_one(S, LBR_A(0));
  for (uint32_t i = 0; i < n; i++) {
    if (t < 12) {
      fp x;
      if (!fp_plain_from_be48(x, parts + (size_t)576 * i + 48 * t, 0xff)) atomicOr(&bad, 1);
      r_stage_fp(S, t, fp_to_mont(x));
    }
    r_sync();
    r_import_staged(S, LBR_A(7), 12);
    r_mul(S, LBR_A(0), LBR_A(0), LBR_A(7));
  }
  r_final_exp(S, LBR_A(0), LBR_A(0));
  const bool one = r_is_one(S, LBR_A(0));
  if (t == 0) *ok = (one && !bad) ? 1 : 0;
}
#endif  // LB_KG

// ---------------------------------------------------------------- pubkey aggregation only
// lb_aggregate_pubkeys (getAggregatedPubkey + toBytes(uncompressed), utils.ts:5-16,
// multithread/index.ts:126,160) since round 6: k_pk_chunks' chunk sums with the segmented wave
// tree, then per set the segment heads (first chunk, wave boundaries), affine, 96-byte encoding,
// with the statuses of the round-5 one-lane-per-set form (first failing key in order; no key:
// EMPTY_AGGREGATE_ARRAY) and its encoding of an infinite or failed aggregate (the infinity flag).
#if LB_KG(14)
__global__ void __launch_bounds__(LB_TPB, LB_MINW) k_pk_out96(uint32_t n, uint32_t nc, const uint32_t* __restrict__ set_chunk_off,
                                                     const uint32_t* __restrict__ chunk_acc,
                                                     const int32_t* __restrict__ chunk_status,
                                                     uint8_t* __restrict__ out96, int32_t* __restrict__ status) {
  const uint32_t i = lb_tid();
  if (i >= n) return;
  const uint32_t c0 = set_chunk_off[i], c1 = set_chunk_off[i + 1];
  int st = c0 == c1 ? LB_EMPTY_AGGREGATE_ARRAY : LB_OK;
  g1j acc = jac_infinity<fp>();
  for (uint32_t c = c0; c < c1 && st == LB_OK; c++) {
    st = chunk_status[c];
    if (st == LB_OK && (c == c0 || (c & (LB_TPB - 1)) == 0)) acc = jac_add(acc, soa_ld<g1j>(chunk_acc, nc, c));
  }
  uint8_t ob[96];
  g1a r;
  const bool fin = jac_to_aff(r, acc);
  g1_serialize96(ob, r, !fin || st != LB_OK);
  for (int k = 0; k < 96; k++) out96[(size_t)96 * i + k] = ob[k];
  status[i] = st;
}
#endif  // LB_KG

// ---------------------------------------------------------------- G2 signature aggregation
// bls.Signature.aggregate(signatures).toBytes() as the op pools use it for block production
// (beacon-node/src/chain/opPools/aggregatedAttestationPool.ts:321, attestationPool.ts:184,
// syncContributionAndProofPool.ts:185): signatures decoded by k_decompress_sigs (+ k_sig_subgroup
// when validating), summed in chunks of <= LB_PK_CHUNK per lane, then per group.
#if LB_KG(1)
__global__ void __launch_bounds__(LB_TPB, LB_MINW_MSM) k_sig_agg_chunks(uint32_t nc, const uint32_t* __restrict__ chunk_lo,
                                                           const uint32_t* __restrict__ sig_aff, uint32_t n,
                                                           const uint32_t* __restrict__ sig_inf,
                                                           const int32_t* __restrict__ sig_status,
                                                           uint32_t* __restrict__ chunk_acc,
                                                           int32_t* __restrict__ chunk_status) {
  const uint32_t c = lb_tid();
  if (c >= nc) return;
  int st = LB_OK;
  g2j acc = jac_infinity<fp2>();
  for (uint32_t i = chunk_lo[c]; i < chunk_lo[c + 1] && st == LB_OK; i++) {
    st = sig_status[i];
    if (st == LB_OK && !sig_inf[i]) acc = jac_add_aff_i<fp2, true>(acc, soa_ld<g2a>(sig_aff, n, i));
  }
  soa_st(chunk_acc, nc, c, acc);
  chunk_status[c] = st;
}
#endif  // LB_KG
#if LB_KG(1)
__global__ void __launch_bounds__(LB_TPB, LB_MINW) k_sig_agg_groups(uint32_t ng, const uint32_t* __restrict__ group_chunk_off,
                                                           const uint32_t* __restrict__ chunk_acc, uint32_t nc,
                                                           const int32_t* __restrict__ chunk_status,
                                                           uint8_t* __restrict__ out96, int32_t* __restrict__ status) {
  const uint32_t g = lb_tid();
  if (g >= ng) return;
  const uint32_t c0 = group_chunk_off[g], c1 = group_chunk_off[g + 1];
  int st = c0 == c1 ? LB_EMPTY_AGGREGATE_ARRAY : LB_OK;
  g2j acc = jac_infinity<fp2>();
  for (uint32_t c = c0; c < c1 && st == LB_OK; c++) {
    st = chunk_status[c];
    if (st == LB_OK) acc = jac_add(acc, soa_ld<g2j>(chunk_acc, nc, c));
  }
  g2a a;
  const bool fin = st == LB_OK && jac_to_aff(a, acc);
  uint8_t ob[96];
  g2_compress96(ob, a, !fin);
  for (int k = 0; k < 96; k++) out96[(size_t)96 * g + k] = ob[k];
  status[g] = st;
}
#endif  // LB_KG

// ---------------------------------------------------------------- G1 decompression
// 48-byte compressed pubkeys -> 96-byte uncompressed (the pubkey cache's one-time
// deserialisation, state-transition/src/cache/pubkeyCache.ts:56-77).  validate = subgroup
// + infinity check (PublicKey.keyValidate).
#if LB_KG(0)
__global__ void __launch_bounds__(LB_TPB, LB_MINW) k_g1_decompress(uint32_t n, const uint8_t* __restrict__ in48,
                                                          uint8_t* __restrict__ out96, int32_t* __restrict__ status,
                                                          int32_t validate) {
  uint32_t i = lb_tid();
  if (i >= n) return;
  uint8_t b[48];
  ld_bytes<48>(b, in48 + (size_t)48 * i);
  g1a a;
  bool inf;
  int st = g1_decompress48(b, a, inf);
  if (st == LB_OK && validate) {
    if (inf) {
      st = LB_PK_IS_INFINITY;
    } else {
      // r * P == O  (r = BLS12-381 subgroup order); plain check, one-time per key
      uint32_t rr[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                        0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
      if (!jac_is_inf(jac_mul_u256(a, rr))) st = LB_POINT_NOT_IN_GROUP;
    }
  }
  uint8_t ob[96];
  g1_serialize96(ob, a, inf || st != LB_OK);
  for (int k = 0; k < 96; k++) out96[(size_t)96 * i + k] = ob[k];
  status[i] = st;
}
#endif  // LB_KG

// ---------------------------------------------------------------- synthetic data (bench/tests)
// sk (32-byte big-endian, < r) -> 48-byte compressed and 96-byte uncompressed pubkey
#if LB_KG(2)
__global__ void __launch_bounds__(LB_TPB, LB_MINW) k_sk_to_pk(uint32_t n, const uint8_t* __restrict__ sks,
                                                     uint8_t* __restrict__ out48, uint8_t* __restrict__ out96) {
  uint32_t i = lb_tid();
  if (i >= n) return;
  uint32_t k[8];
  for (int w = 0; w < 8; w++) {
    const uint8_t* s = sks + (size_t)32 * i + 28 - 4 * w;
    k[w] = ((uint32_t)s[0] << 24) | ((uint32_t)s[1] << 16) | ((uint32_t)s[2] << 8) | s[3];
  }
  g1a g{fp_load(LB_G1X), fp_load(LB_G1Y)};
  g1a a;
  bool fin = jac_to_aff(a, jac_mul_u256(g, k));
  uint8_t c[48], u[96];
  g1_compress48(c, a, !fin);
  g1_serialize96(u, a, !fin);
  if (out48)
    for (int j = 0; j < 48; j++) out48[(size_t)48 * i + j] = c[j];
  if (out96)
    for (int j = 0; j < 96; j++) out96[(size_t)96 * i + j] = u[j];
}
#endif  // LB_KG

// sig = sk * H(m), 96-byte compressed
#if LB_KG(2)
__global__ void __launch_bounds__(LB_TPB, LB_MINW) k_sign(uint32_t n, const uint8_t* __restrict__ sks,
                                                 const uint8_t* __restrict__ msgs, uint8_t* __restrict__ out96) {
  uint32_t i = lb_tid();
  if (i >= n) return;
  uint32_t k[8];
  for (int w = 0; w < 8; w++) {
    const uint8_t* s = sks + (size_t)32 * i + 28 - 4 * w;
    k[w] = ((uint32_t)s[0] << 24) | ((uint32_t)s[1] << 16) | ((uint32_t)s[2] << 8) | s[3];
  }
  uint8_t m[32];
  for (int j = 0; j < 32; j++) m[j] = msgs[(size_t)32 * i + j];
  g2a h;
  jac_to_aff(h, hash_to_g2(m));
  g2a a;
  bool fin = jac_to_aff(a, jac_mul_u256(h, k));
  uint8_t c[96];
  g2_compress96(c, a, !fin);
  for (int j = 0; j < 96; j++) out96[(size_t)96 * i + j] = c[j];
}
#endif  // LB_KG
