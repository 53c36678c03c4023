// Grouped program engine: G = 8 lanes of a wave run one pairing instance, so a wave runs eight
// instances side by side and a workgroup of LBG_WAVES waves 8 * LBG_WAVES.  Programs come from
// tools/gen_group_programs.py (lb_group_progs.h): every Fp product is a task whose operands
// are small linear combinations of the instance's LDS slots, and the lanes of a group take a
// phase's tasks eight at a time.  Nothing of the pairing state lives in registers across tasks,
// so the kernels carry no spill scratch (the one-lane-per-root Miller loop spilled 6.7 KB per
// lane), and a phase costs one product per lane instead of the serial chain of a lone lane.
//
// LDS layout per workgroup: LBG_ROOTS instance blocks of 12 limb rows x LBG_NSP words (word k of
// slot s at k * LBG_NSP + s; the odd stride spreads a group's slots over the banks), one block
// holding the shared constants (slot s < 0 reads constant -1 - s), then the program image.
// A wave only ever touches its own instances, so phases are separated by wave-level fences, not
// workgroup barriers.
#pragma once
#include "lb_wave.h"
#include "lb_group_progs.h"

#ifndef LBG_WAVES
#define LBG_WAVES 4
#endif
#define LBG_G 8
#define LBG_ROOTS (LBG_WAVES * 64 / LBG_G)
#define LBG_NSP (LBG_NSLOT | 1)
#define LBG_BLOCK (12 * LBG_NSP)
#define LBG_LDS_WORDS ((LBG_ROOTS + 1) * LBG_BLOCK + (LBG_IMAGE + 1) / 2)
static_assert(LBG_LDS_WORDS * 4 <= 163840, "lb_group_exec.h: LDS budget (160 KB per CU)");
static_assert(LBW_N_CONST <= LBG_NSP, "lb_group_exec.h: constants block");

__device__ __forceinline__ void g_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ fp g_ld(const lds_u32* p) {
  fp r;
  LB_UNROLL for (int k = 0; k < 12; k++) r.v[k] = p[k * LBG_NSP];
  return r;
}
__device__ __forceinline__ void g_st(lds_u32* p, const fp& a) {
  LB_UNROLL for (int k = 0; k < 12; k++) p[k * LBG_NSP] = a.v[k];
}
__device__ __forceinline__ const lds_u32* g_slot(const lds_u32* R, const lds_u32* C, int s) {
  return s >= 0 ? R + s : C + (-1 - s);
}

// Accumulates sum_k c_k S[slot_k] over `cnt` (slot, coefficient) pairs into 64-bit limb sums.
// The pairs are read first, all at once; then the terms go in groups of four whose 48 limb loads
// issue together, padding terms getting coefficient 0 (cnt is phase-uniform, so the group loop
// branches on scalars).  One LDS round trip per group instead of two per term.
template <int MAXN>
__device__ __forceinline__ void g_acc(uint64_t* acc, const lds_u32* R, const lds_u32* C, const lds_u32* pr, int cnt) {
  uint32_t w[(MAXN + 3) & ~3];
  LB_UNROLL for (int k = 0; k < MAXN; k++) w[k] = k < cnt ? pr[k] : 0u;
  LB_UNROLL for (int k = MAXN; k < ((MAXN + 3) & ~3); k++) w[k] = 0u;
  LB_UNROLL for (int g = 0; g < MAXN; g += 4) {
    if (g < cnt) {
      fp v[4];
      LB_UNROLL for (int k = 0; k < 4; k++) v[k] = g_ld(g_slot(R, C, (int)(int16_t)(w[g + k] & 0xffffu)));
      LB_UNROLL for (int k = 0; k < 4; k++) {
        const uint32_t c = w[g + k] >> 16;
        LB_UNROLL for (int j = 0; j < 12; j++) acc[j] += (uint64_t)v[k].v[j] * c;
      }
    }
  }
}

// V = pos - neg (signed limb sums) reduced to [0, 3p) by the quotient estimate of lb_wave.h
// w_lin (below p if `full`)
__device__ __forceinline__ fp g_reduce(const uint64_t* pa, const uint64_t* na, bool full) {
  int64_t d[12];
  LB_UNROLL for (int j = 0; j < 12; j++) d[j] = (int64_t)(pa[j] - na[j]);
  const double wd = (double)d[11] * 4294967296.0 + (double)d[10];
  const int64_t q = (int64_t)floor(wd * LBW_INV_P320) - 1;
  const uint32_t P32[12] = {LB_P0, LB_P1, LB_P2, LB_P3, LB_P4, LB_P5, LB_P6, LB_P7, LB_P8, LB_P9, LB_P10, LB_P11};
  uint32_t r[13];
  int64_t carry = 0;
  LB_UNROLL for (int j = 0; j < 12; j++) {
    const int64_t t = d[j] - q * (int64_t)P32[j] + carry;
    r[j] = (uint32_t)t;
    carry = t >> 32;
  }
  r[12] = (uint32_t)carry;
  if (full) {
    w_csub13(r, LB_P_X2);
    w_csub13(r, LB_P_X1);
  }
  fp out;
  LB_UNROLL for (int j = 0; j < 12; j++) out.v[j] = r[j];
  return out;
}

// sum over np added and nn subtracted pairs at pr (np, nn <= MAXN, phase-uniform)
template <int MAXN>
__device__ __forceinline__ fp g_lin(const lds_u32* R, const lds_u32* C, const lds_u32* pr, int np, int nn, bool full) {
  uint64_t pa[12], na[12];
  LB_UNROLL for (int j = 0; j < 12; j++) pa[j] = na[j] = 0;
  g_acc<MAXN>(pa, R, C, pr, np);
  g_acc<MAXN>(na, R, C, pr + np, nn);
  return g_reduce(pa, na, full);
}

// Runs one program (image offset `off`) on this lane's instance R; q = lane within the group.
__device__ __forceinline__ void g_exec(lds_u32* R, const lds_u32* C, const lds_i16* img, int off, int q) {
  const lds_i16* prog = img + off;
  const int nph = __builtin_amdgcn_readfirstlane(prog[0]);
  int pos = 8;
#pragma clang loop unroll(disable)
  for (int ph = 0; ph < nph; ph++) {
    const int kind = __builtin_amdgcn_readfirstlane(prog[pos]), n = __builtin_amdgcn_readfirstlane(prog[pos + 1]);
    const int npa = __builtin_amdgcn_readfirstlane(prog[pos + 2]), nna = __builtin_amdgcn_readfirstlane(prog[pos + 3]);
    const int npb = __builtin_amdgcn_readfirstlane(prog[pos + 4]), nnb = __builtin_amdgcn_readfirstlane(prog[pos + 5]);
    const int rs = __builtin_amdgcn_readfirstlane(prog[pos + 6]);
    pos += 8;
    if (kind == 0) {
#pragma clang loop unroll(disable)
      for (int k = q; k - q < n; k += LBG_G) {
        if (k < n) {
          const lds_i16* rec = prog + pos + k * rs;
          const lds_u32* pr = (const lds_u32*)(rec + 2);
          uint64_t xa[12], xn[12], ya[12], yn[12];
          LB_UNROLL for (int j = 0; j < 12; j++) xa[j] = xn[j] = ya[j] = yn[j] = 0;
          g_acc<LBG_MAXP>(xa, R, C, pr, npa);
          g_acc<LBG_MAXP>(xn, R, C, pr + npa, nna);
          g_acc<LBG_MAXP>(ya, R, C, pr + npa + nna, npb);
          g_acc<LBG_MAXP>(yn, R, C, pr + npa + nna + npb, nnb);
          const int dst = rec[0];
          const fp x = g_reduce(xa, xn, false);
          const fp y = g_reduce(ya, yn, false);
          g_st(R + dst, fp_mul28(x, y));
        }
      }
    } else {
#pragma clang loop unroll(disable)
      for (int k = q; k - q < n; k += LBG_G) {
        if (k < n) {
          const lds_i16* rec = prog + pos + k * rs;
          const int dst = rec[0];
          g_st(R + (dst & ~LBW_OUT_FLAG), g_lin<LBG_MAXL>(R, C, (const lds_u32*)(rec + 2), npa, nna, (dst & LBW_OUT_FLAG) != 0));
        }
      }
    }
    pos += n * rs;
    g_sync();
  }
}

// Workgroup setup shared by the grouped kernels: the program image and the constants into LDS
// (every thread of the block takes part; one workgroup barrier).
__device__ __forceinline__ void g_setup(uint32_t* lds) {
  lds_u32* L = (lds_u32*)lds;
  lds_u32* C = L + LBG_ROOTS * LBG_BLOCK;
  lds_u32x4* img = (lds_u32x4*)(C + LBG_BLOCK);
  const int tid = threadIdx.x;
  const u32x4* src = reinterpret_cast<const u32x4*>(LBG_PROGS);
  for (int i = tid; i < LBG_IMAGE / 8; i += blockDim.x) img[i] = src[i];
  if (tid < LBW_N_CONST) {
    fp v;
    if (tid < 2)
      v = fp_load(LB_B2_3 + 12 * tid);
    else if (tid == 2)
      v = fp_load(LB_INV2);
    else if (tid < 13) {
      const int k = (tid - 3) / 2, c = (tid - 3) & 1;
      const uint32_t* tab[5] = {LB_FROB1_1, LB_FROB1_2, LB_FROB1_3, LB_FROB1_4, LB_FROB1_5};
      v = fp_load(tab[k] + 12 * c);
    } else if (tid < LBW_C_ZERO) {
      const uint32_t* tab[5] = {LB_FROB2_1, LB_FROB2_2, LB_FROB2_3, LB_FROB2_4, LB_FROB2_5};
      v = fp_load(tab[tid - 13]);
    } else {
      v = fp_zero();
    }
    g_st(C + tid, v);
  }
  __syncthreads();
}
static_assert(LBG_IMAGE % 8 == 0, "lb_group_exec.h: image is a 16-byte multiple");

// Miller loops f_{|x|, H(m_u)}(P_u), conjugated, for the distinct roots: 8 lanes per root, 8 roots
// per wave (as k_miller_wave, written into leaf m + u of the product tree).
// Roots u >= *n_u compute a clamped duplicate and store nothing; a root whose P_u is infinity
// stores the identity.
#if LB_KG(5)
__global__ void __launch_bounds__(64 * LBG_WAVES) k_miller_g8(uint32_t n, uint32_t m, const uint32_t* __restrict__ n_u,
                                                             const uint32_t* __restrict__ gp_aff,
                                                             const uint32_t* __restrict__ gp_inf,
                                                             const uint32_t* __restrict__ h_aff,
                                                             uint32_t* __restrict__ treeP) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[LBG_LDS_WORDS];
  const uint32_t nu = *n_u;
  if (blockIdx.x * LBG_ROOTS >= nu) return;  // whole block idle (uniform)
  g_setup(lds);
  const int q = threadIdx.x & (LBG_G - 1), rl = threadIdx.x / LBG_G;
  const uint32_t u = blockIdx.x * LBG_ROOTS + rl;
  const uint32_t uc = u < nu ? u : nu - 1;
  lds_u32* L = (lds_u32*)lds;
  lds_u32* R = L + rl * LBG_BLOCK;
  const lds_u32* C = L + LBG_ROOTS * LBG_BLOCK;
  const lds_i16* img = (const lds_i16*)(C + LBG_BLOCK);
  // state: f = 1, T = (xQ, yQ, 1), P, Q (slot 18 + k = P.x, P.y, Q.x.c0, Q.x.c1, Q.y.c0, Q.y.c1)
  for (int s = q; s < LBG_N_STATE; s += LBG_G) {
    fp v;
    if (s >= LBG_S_P) {
      const int k = s - LBG_S_P;
      const uint32_t* base = k < 2 ? gp_aff + (size_t)12 * k * n : h_aff + (size_t)12 * (k - 2) * n;
      LB_UNROLL for (int w = 0; w < 12; w++) v.v[w] = base[(size_t)w * n + uc];
    } else if (s >= LBG_S_T) {
      const int k = s - LBG_S_T;
      if (k < 4) {
        const uint32_t* base = h_aff + (size_t)12 * k * n;
        LB_UNROLL for (int w = 0; w < 12; w++) v.v[w] = base[(size_t)w * n + uc];
      } else {
        v = k == 4 ? fp_one() : fp_zero();
      }
    } else {
      v = s == 0 ? fp_one() : fp_zero();
    }
    g_st(R + s, v);
  }
  g_sync();
#pragma clang loop unroll(disable)
  for (int i = 62; i >= 0; i--) {
    g_exec(R, C, img, LBG_DBL, q);
    if ((LB_X_ABS >> i) & 1ull) g_exec(R, C, img, LBG_ADD, q);
  }
  if (u >= nu) return;
  const bool inf = gp_inf[u] != 0;
  for (int s = q; s < 12; s += LBG_G) {
    fp v = g_ld(R + s);
    if (s >= 6) v = fp_neg(v);  // conjugate (x < 0)
    if (inf) v = s == 0 ? fp_one() : fp_zero();
    LB_UNROLL for (int w = 0; w < 12; w++) treeP[(size_t)(12 * s + w) * (2 * m) + m + u] = v.v[w];
  }
}
#endif  // LB_KG
