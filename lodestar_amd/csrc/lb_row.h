// Row engine: the Fp12 programs of lb_wave.h (final exponentiation, Miller loops, product-tree
// nodes) with every Fp product split over one 16-lane ROW of a wave instead of one lane.
//
// Why: a lone lane runs one 381-bit Montgomery product in ~2 500 cycles (~630 dependent VALU
// instructions), so a final exponentiation or a Miller loop on the wave engine is a chain of
// ~1 us product phases plus the per-lane operand sums (12 LDS words per term).  Here lane k of a
// row holds limb k of an element (14 signed 28-bit limbs; lanes 14, 15 hold 0): an operand sum is
// one LDS word per term per lane, and a product is a systolic pass over the row (~200 VALU
// instructions, the shifts by DPP row_shr / row_shl), so a phase of <= 16 products takes ~1/3 of
// a lone-lane product on a 4-wave workgroup (16 rows, one wave per SIMD).
//
// Representation (tools/gen_row_programs.py mirrors it exactly): a slot holds an integer v in
// (-2p, 2p) congruent to x R' (mod p), R' = 2^392, as v = sum_k l_k 2^(28 k) with l_0..l_12 in
// [-1, 2^28 + 2) and l_13 a small signed top limb.  Slot s, limb k at LDS word 16 s + k.
//
// Product (rp_mul): x replicated in every lane of the row (14 registers), y distributed.
//   columns of x y: lane k accumulates column k (lo) and column k + 16 (hi), 64-bit, while y
//   shifts by row_shr:i / row_shl:(16 - i);
//   m = (x y mod 2^392)(-p^-1) mod 2^392 from the low columns normalised to ~28-bit limbs;
//   U = x y + m p; its low half is C 2^392 with C = ceil((U13 + U12 / 2^28 + U11 / 2^56) / 2^28)
//   (the lower columns move that by < 2^-17); the result is U's high columns + C, normalised.
//   |result| < |x y| / 2^392 + 1.0001 p.
// Operand / linear sums: signed limb sums (64-bit), then q = floor(v / p) estimated from the top
// two limbs in double precision (lane 13), broadcast over the row (ds_swizzle), v - q p: [0, p)
// up to an error far below p.
// Everything is collective over the workgroup (LBR_NT threads); one wave per SIMD.
#pragma once
#include "lb_pairing.h"
#include "lb_row_progs.h"
#include "lb_pdbl_tab.h"
#include "lb_mul12_tab.h"
#include "lb_row_compiled.h"

#ifndef LBR_WAVES
#define LBR_WAVES 16  // one workgroup of 16 waves (4 per SIMD): a phase of <= 64 products in one round
#endif
#define LBR_NT (64 * LBR_WAVES)
#define LBR_NROWS (4 * LBR_WAVES)
#define LBR_PERSIST (LBR_TEMP + LBR_MAX_TEMPS)
#define LBR_A(k) (LBR_PERSIST + 12 * (k))  // caller-owned Fp12 areas
#define LBR_N_AREAS 8
#define LBR_PT (LBR_PERSIST + 12 * LBR_N_AREAS)  // Miller loop: P (2), Q (4), T (6)
#define LBR_XS (LBR_PT + 16)                     // staging slots for import / export (16)
#define LBR_ROWX (LBR_XS + 16)                   // one operand slot per row
#define LBR_SLOTS (LBR_ROWX + LBR_NROWS)
#define LBR_SLOT_WORDS (16 * LBR_SLOTS)
#define LBR_MISC 8  // words after the slots: [0] first staged program word, [1] flag, [2] scratch
// The per-workgroup LDS block: the slots, misc words, the staged program image (a prefix / range
// of LBR_PROGS).  LBR_SHARED_N(name, words)
#define LBR_SHARED_N(name, nprog)                                                                 \
  __shared__ __attribute__((aligned(16))) int32_t name##_lds[LBR_SLOT_WORDS + LBR_MISC + (nprog)]; \
  int32_t* name = name##_lds
#define LBR_SHARED(name) LBR_SHARED_N(name, LBR_PROGS_FE)
#define LBR_SHARED_ML(name) LBR_SHARED_N(name, LBR_PROGS_ALL)
#define LBR_MILLER_FIRST LBR_DBL_STEP
#define LBR_MILLER_COUNT (LBR_PROGS_ALL - LBR_DBL_STEP)
#define LBR_SHARED_MILLER(name) LBR_SHARED_N(name, LBR_MILLER_COUNT)
static_assert(LBR_DBL_STEP >= LBR_PROGS_FE && LBR_ADD_STEP > LBR_DBL_STEP, "lb_row.h: program image order");

typedef __attribute__((address_space(3))) int32_t lds_i32;
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) i32x4 lds_i32x4;

__device__ __forceinline__ void r_sync() { __syncthreads(); }
__device__ __forceinline__ int r_tid() { return threadIdx.x; }
__device__ __forceinline__ int r_limb() { return threadIdx.x & 15; }
__device__ __forceinline__ int r_row() { return threadIdx.x >> 4; }
__device__ __forceinline__ lds_i32* r_lds(int32_t* S) { return (lds_i32*)S; }

// ---------------------------------------------------------------- DPP within a row
template <int CTRL>
__device__ __forceinline__ int r_dpp(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);  // bound_ctrl: out-of-row sources read 0
}
template <int CTRL>
__device__ __forceinline__ int64_t r_dpp64(int64_t v) {
  const int lo = r_dpp<CTRL>((int)(uint32_t)(uint64_t)v), hi = r_dpp<CTRL>((int)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
#define LBR_SHR(n) (0x110 + (n))  // lane k <- lane k - n of the row (0 below the row)
#define LBR_SHL(n) (0x100 + (n))  // lane k <- lane k + n of the row (0 above the row)
// broadcast lane 13 of each row (ds_swizzle bit mode: lane' = (lane & 0x10) | 13 within 32)
// lane I of the row to every lane of the row (DPP row_newbcast: a VALU move, no LDS round trip)
template <int I>
__device__ __forceinline__ int r_bcast(int v) {
  return __builtin_amdgcn_mov_dpp(v, 0x150 + I, 0xF, 0xF, false);
}
__device__ __forceinline__ int r_bcast13(int v) {
#ifdef LBR_SWIZZLE_BCAST
  return __builtin_amdgcn_ds_swizzle(v, 0x10 | (13 << 5));
#else
  return r_bcast<13>(v);
#endif
}
// a distributed element (lane k: limb k) replicated in every lane of the row
__device__ __forceinline__ void r_rep(int v, int (&x)[14]) {
  x[0] = r_bcast<0>(v); x[1] = r_bcast<1>(v); x[2] = r_bcast<2>(v); x[3] = r_bcast<3>(v);
  x[4] = r_bcast<4>(v); x[5] = r_bcast<5>(v); x[6] = r_bcast<6>(v); x[7] = r_bcast<7>(v);
  x[8] = r_bcast<8>(v); x[9] = r_bcast<9>(v); x[10] = r_bcast<10>(v); x[11] = r_bcast<11>(v);
  x[12] = r_bcast<12>(v); x[13] = r_bcast<13>(v);
}

#define LBR_M28 0x0fffffff
struct lbr_k {
  static constexpr int P[14] = {LBR_P_LIMBS};
  static constexpr int PINV[14] = {LBR_PINV_LIMBS};
  static constexpr int K_EXPORT[14] = {LBR_K_EXPORT};
  static constexpr int K_PLAIN[14] = {LBR_K_PLAIN};
  static constexpr int ONE[14] = {LBR_ONE};
};
// p's limb for this lane (0 in lanes 14, 15)
__device__ __forceinline__ int r_plimb(int k) {
  int v = 0;
  LB_UNROLL for (int i = 0; i < 14; i++) v = k == i ? lbr_k::P[i] : v;
  return v;
}

// Two carry rounds: 64-bit (the carry split in two 28-bit pieces), then 32-bit.  KEEP: limb 13
// keeps its whole value and takes limb 12's carry whole (a value, not a residue mod 2^392);
// otherwise carries out of limb 13 are dropped (mod 2^392).  Lanes 14, 15: 0 with KEEP.
template <bool KEEP>
__device__ __forceinline__ int r_norm(int64_t v, int k) {
  const int64_t q = v >> 28;
  int l = (int)(v & LBR_M28);
  int qlo = (int)(q & LBR_M28), qhi = (int)(q >> 28);
  if (KEEP) {
    if (k == 12) {
      qlo = (int)q;
      qhi = 0;
    }
    if (k >= 13) {
      l = k == 13 ? (int)v : 0;
      qlo = qhi = 0;
    }
  }
  l += r_dpp<LBR_SHR(1)>(qlo) + r_dpp<LBR_SHR(2)>(qhi);
  int c = l >> 28, l2 = l & LBR_M28;
  if (KEEP && k >= 13) {
    c = 0;
    l2 = k == 13 ? l : 0;
  }
  return l2 + r_dpp<LBR_SHR(1)>(c);
}

// lo += sum_i X[i] * y[k - i], hi += sum_{i>=1} X[i] * y[k + 16 - i]  (X replicated / constant);
// even and odd terms into separate accumulators (two independent MAD chains)
template <int I, bool HI, class XS>
__device__ __forceinline__ void r_sys(const XS& x, int y, int64_t (&lo)[2], int64_t (&hi)[2]) {
  if constexpr (I < 14) {
    if constexpr (I == 0) {
      lo[0] += (int64_t)x[0] * y;
    } else {
      lo[I & 1] += (int64_t)x[I] * r_dpp<LBR_SHR(I)>(y);
      if constexpr (HI) hi[I & 1] += (int64_t)x[I] * r_dpp<LBR_SHL(16 - I)>(y);
    }
    r_sys<I + 1, HI>(x, y, lo, hi);
  }
}
struct r_cx_p {
  __device__ __forceinline__ int operator[](int i) const { return lbr_k::P[i]; }
};
struct r_cx_pinv {
  __device__ __forceinline__ int operator[](int i) const { return lbr_k::PINV[i]; }
};

// The row Montgomery product of x (replicated: x[0..13] in every lane of the row) and y (lane k:
// limb k, lanes 14, 15: 0): this lane's limb of x y / 2^392 (mod p).
template <class XS>
__device__ __forceinline__ int rp_mul(const XS& x, int y, int k) {
  int64_t l2[2] = {0, 0}, h2[2] = {0, 0};
  r_sys<0, true>(x, y, l2, h2);
  int64_t lo = l2[0] + l2[1];
  // m = (x y mod 2^392) (-p^-1) mod 2^392
  int t = r_norm<false>(lo, k);
  t = k < 14 ? t : 0;
  int64_t m2[2] = {0, 0}, dummy[2] = {0, 0};
  r_sys<0, false>(r_cx_pinv{}, t, m2, dummy);
  int m = r_norm<false>(m2[0] + m2[1], k);
  m = k < 14 ? m : 0;
  // U = x y + m p
  l2[0] = lo;
  l2[1] = 0;
  r_sys<0, true>(r_cx_p{}, m, l2, h2);
  lo = l2[0] + l2[1];
  const int64_t hi = h2[0] + h2[1];
  // carry of the low half (a multiple of 2^392) into column 14
  const int64_t u13 = r_dpp64<LBR_SHR(1)>(lo), u12 = r_dpp64<LBR_SHR(2)>(lo), u11 = r_dpp64<LBR_SHR(3)>(lo);
  const int64_t E = u13 + (u12 >> 28) + (u11 >> 56);
  const int64_t C = (E + LBR_M28) >> 28;
  const int64_t w = k == 14 ? lo + C : (k == 15 ? lo : 0);
  const int64_t r = r_dpp64<LBR_SHL(14)>(w) + r_dpp64<LBR_SHR(2)>(hi);
  return r_norm<true>(r, k);
}
struct r_cx_arr {
  const int* a;
  __device__ __forceinline__ int operator[](int i) const { return a[i]; }
};
template <int N>
struct r_cx_const {
  const int (&a)[N];
  __device__ __forceinline__ int operator[](int i) const { return a[i]; }
};

// limb-sum reduction: v (64-bit limb sums) -> v - q p with q = floor(v / p) from the top limbs;
// pk = p's limb for this lane (r_plimb, hoisted by the callers)
__device__ __forceinline__ int r_reduce(int64_t acc, int k, int pk) {
  const int64_t a12 = r_dpp64<LBR_SHR(1)>(acc);  // lane 13 sees limb 12
  const double w = (double)acc * 268435456.0 + (double)a12;
  int q = (int)floor(w * LBR_INV_P336);
  q = r_bcast13(q);
  acc -= (int64_t)q * pk;
  return r_norm<true>(acc, k);
}
__device__ __forceinline__ int r_reduce(int64_t acc, int k) { return r_reduce(acc, k, r_plimb(k)); }

// operand / linear sum over `n` (<= 8 * NB) (slot, coef) pairs at LDS words rec[0..n): the pair
// words of a block of 8 and then their 8 limbs are loaded together (one LDS round trip each per
// block instead of two per term)
// Branch-free: every term of a block reads a valid record word (index clamped to n - 1; n >= 1)
// and its slot, the terms past n get coefficient 0, so the block's 8 record reads and then its 8
// limb reads issue together (guarded loads compiled to a branch per term).
template <int NB>
__device__ __forceinline__ int64_t r_acc(const lds_i32* S, const lds_i32* rec, int n, int k) {
  int64_t acc = 0;
  LB_UNROLL for (int b = 0; b < NB; b++) {
    if (8 * b < n) {
      int w[8], v[8];
      LB_UNROLL for (int j = 0; j < 8; j++) w[j] = rec[min(8 * b + j, n - 1)];
      LB_UNROLL for (int j = 0; j < 8; j++) v[j] = S[16 * (w[j] & 0xffff) + k];
      LB_UNROLL for (int j = 0; j < 8; j++) acc += (int64_t)(8 * b + j < n ? (w[j] >> 16) : 0) * v[j];
    }
  }
  return acc;
}
template <int NB>
__device__ __forceinline__ int r_sum(const lds_i32* S, const lds_i32* rec, int n, int k, int pk) {
  return r_reduce(r_acc<NB>(S, rec, n, k), k, pk);
}
// a product operand: with a coefficient sum <= 16 (phase flag clear) only the limb carries run
__device__ __forceinline__ int r_operand(const lds_i32* S, const lds_i32* rec, int n, int k, bool red, int pk) {
  const int64_t acc = r_acc<1>(S, rec, n, k);
  if (red) return r_reduce(acc, k, pk);
  return r_norm<true>(acc, k);
}

__device__ __forceinline__ void r_load_rep(const lds_i32* S, int slot, int (&x)[14]) {
  const lds_i32x4* q = (const lds_i32x4*)(S + 16 * slot);
  const i32x4 a = q[0], b = q[1], c = q[2], d = q[3];
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
  x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  x[8] = c.x; x[9] = c.y; x[10] = c.z; x[11] = c.w;
  x[12] = d.x; x[13] = d.y;
}

// base of the staged program image as seen from LDS (words below `first` are never used)
__device__ __forceinline__ const lds_i32* r_progs(int32_t* S) {
  const lds_i32* s = r_lds(S);
  return s + LBR_SLOT_WORDS + LBR_MISC - s[LBR_SLOT_WORDS + 0];
}

// ---------------------------------------------------------------- the interpreter
// Software-pipelined: the program words a row needs for phase ph + 1 (the header, and its task
// record: destination and up to 16 (slot, coef) pairs) are read while phase ph's product runs
// (program words are read-only, so only the slot reads wait for the barrier); one LDS round trip
// (the slot limbs) remains between a barrier and the product instead of four (header, record,
// slots; the operand's replicated copy).  Tasks past the first LBR_NROWS of a phase take the
// unpipelined path (r_exec_tail).
struct r_pref {
  int dst;
  int w[16];
};
__device__ __forceinline__ void r_prefetch(const lds_i32* prog, int pos, int h0, int h1, int row, r_pref& p) {
  const int kind = h0 & 0xff, n = h0 >> 16, nx = h1 & 0xffff, ny = h1 >> 16;
  int t, rs, nA, offB, nB;
  if (kind == 0) {
    t = row;
    rs = 1 + nx + ny;
    nA = nx;
    offB = 1 + nx;
    nB = ny;
  } else {
    t = (row - ny + 4 * LBR_NROWS) % LBR_NROWS;
    rs = 1 + nx;
    nA = min(nx, 8);
    offB = 9;
    nB = nx - 8;
  }
  if (t >= n) return;  // an idle row (its words are not used)
  const lds_i32* rec = prog + pos + t * rs;
  p.dst = rec[0];
  // in blocks of 4 terms: the second block only when the phase's operands have more than 4
  // (nA, nB are phase-uniform: scalar branches)
  LB_UNROLL for (int j = 0; j < 4; j++) p.w[j] = rec[1 + min(j, nA - 1)];
  if (nA > 4) LB_UNROLL for (int j = 4; j < 8; j++) p.w[j] = rec[1 + min(j, nA - 1)];
  LB_UNROLL for (int j = 0; j < 4; j++) p.w[8 + j] = rec[nB > 0 ? offB + min(j, nB - 1) : 1];
  if (nB > 4) LB_UNROLL for (int j = 4; j < 8; j++) p.w[8 + j] = rec[offB + min(j, nB - 1)];
}
// sum of the 4 prefetched terms w[O .. O + 4) (tools/gen_row_programs.py pads every non-plain
// operand and linear task to whole blocks of 4 with zero-coefficient pairs: no mask)
template <int O>
__device__ __forceinline__ int64_t r_acc4(const lds_i32* S, const r_pref& p, int, int k) {
  int v[4];
  LB_UNROLL for (int j = 0; j < 4; j++) v[j] = S[16 * (p.w[O + j] & 0xffff) + k];
  int64_t acc = 0;
  LB_UNROLL for (int j = 0; j < 4; j++) acc += (int64_t)(p.w[O + j] >> 16) * v[j];
  return acc;
}
// sum of up to 8 prefetched terms w[O .. O + 8) (n of them)
template <int O>
__device__ __forceinline__ int64_t r_acc_w(const lds_i32* S, const r_pref& p, int n, int k) {
  int64_t acc = r_acc4<O>(S, p, n, k);
  if (n > 4) acc += r_acc4<O + 4>(S, p, n - 4, k);
  return acc;
}
template <int O>
__device__ __forceinline__ int r_operand_w(const lds_i32* S, const r_pref& p, int n, bool plain, bool red, int k,
                                           int pk) {
  if (plain) return S[16 * (p.w[O] & 0xffff) + k];
  const int64_t acc = r_acc_w<O>(S, p, n, k);
  return red ? r_reduce(acc, k, pk) : r_norm<true>(acc, k);
}
// tasks LBR_NROWS.. of a phase (records at prog + pos)
__device__ void r_exec_tail(lds_i32* S, const lds_i32* prog, int pos, int h0, int h1) {
  const int k = r_limb(), row = r_row(), pk = r_plimb(k);
  const int kind = h0 & 0xff, flags = (h0 >> 8) & 0xff, n = h0 >> 16;
  const int nx = h1 & 0xffff, ny = h1 >> 16;
  if (kind == 0) {
    const int rs = 1 + nx + ny;
    for (int base = LBR_NROWS; base < n; base += LBR_NROWS) {
      const int t = base + row;
      if (t < n) {
        const lds_i32* rec = prog + pos + t * rs;
        const int y = (flags & 2) ? S[16 * (rec[1 + nx] & 0xffff) + k] : r_operand(S, rec + 1 + nx, ny, k, flags & 8, pk);
        int x[14];
        r_rep((flags & 1) ? S[16 * (rec[1] & 0xffff) + k] : r_operand(S, rec + 1, nx, k, flags & 4, pk), x);
        S[16 * rec[0] + k] = rp_mul(x, y, k);
      }
    }
  } else {
    const int rs = 1 + nx, rr = (row - ny + 4 * LBR_NROWS) % LBR_NROWS;
    for (int base = LBR_NROWS; base < n; base += LBR_NROWS) {
      const int t = base + rr;
      if (t < n) {
        const lds_i32* rec = prog + pos + t * rs;
        S[16 * rec[0] + k] = r_sum<3>(S, rec + 1, nx, k, pk);
      }
    }
  }
}

#ifndef LBR_EXEC_ATTR
#define LBR_EXEC_ATTR __attribute__((noinline))
#endif
#ifndef LBR_EXEC_V1
// Run one program (offset `off` in the image): inputs already in IN, outputs left in the temps
// the header lists.  r_exec_inl is inlined once into r_run's loop (lb_row.h, end): a call of the
// out-of-line r_exec costs ~0.9 us of callee-saved scratch round trips, on the order of a phase.
#ifndef LBR_TL
#define LBR_TL(i)
#endif
__device__ __forceinline__ void r_exec_inl(int32_t* S_generic, int off) {
  LBR_TL(0);
  lds_i32* S = r_lds(S_generic);
  const lds_i32* prog = r_progs(S_generic) + off;
  const int k = r_limb(), row = r_row(), pk = r_plimb(k);
  const int nph = __builtin_amdgcn_readfirstlane(prog[0]), nout = __builtin_amdgcn_readfirstlane(prog[1]);
  int pos = 2 + nout;
  int h0 = __builtin_amdgcn_readfirstlane(prog[pos]), h1 = __builtin_amdgcn_readfirstlane(prog[pos + 1]);
  pos += 2;
  r_pref p;
  r_prefetch(prog, pos, h0, h1, row, p);
  LBR_TL(1);
  for (int ph = 0; ph < nph; ph++) {
    const int kind = h0 & 0xff, flags = (h0 >> 8) & 0xff, n = h0 >> 16;
    const int nx = h1 & 0xffff, ny = h1 >> 16;
    const int npos = pos + n * (kind == 0 ? 1 + nx + ny : 1 + nx);
    const bool more = ph + 1 < nph;
    int nh0v = 0, nh1v = 0;
    if (more) {
      nh0v = prog[npos];
      nh1v = prog[npos + 1];
    }
    const int dst = p.dst;
    int yv = 0, xv = 0;
    bool act;
    if (kind == 0) {
      act = row < n;
      if (act) {
        yv = r_operand_w<8>(S, p, ny, flags & 2, flags & 8, k, pk);
        xv = r_operand_w<0>(S, p, nx, flags & 1, flags & 4, k, pk);
      }
    } else {
      act = (row - ny + 4 * LBR_NROWS) % LBR_NROWS < n;
      if (act) {
        int64_t acc = r_acc_w<0>(S, p, min(nx, 8), k);
        if (nx > 8) acc += r_acc_w<8>(S, p, nx - 8, k);
        if (nx > 16) {
          const int t = (row - ny + 4 * LBR_NROWS) % LBR_NROWS;
          acc += r_acc<1>(S, prog + pos + t * (1 + nx) + 17, nx - 16, k);
        }
        yv = r_reduce(acc, k, pk);
      }
    }
    LBR_TL(2);
    int nh0 = 0, nh1 = 0;
    if (more) {
      nh0 = __builtin_amdgcn_readfirstlane(nh0v);
      nh1 = __builtin_amdgcn_readfirstlane(nh1v);
      r_prefetch(prog, npos + 2, nh0, nh1, row, p);
    }
    LBR_TL(3);
    if (act) {
      if (kind == 0) {
        int x[14];
        r_rep(xv, x);
        yv = rp_mul(x, yv, k);
      }
      S[16 * dst + k] = yv;
    }
    LBR_TL(4);
    if (n > LBR_NROWS) r_exec_tail(S, prog, pos, h0, h1);
    if (kind != 0 || !(flags & 16)) r_sync();  // flag 16: the next (linear) phase reads nothing of this one
    LBR_TL(5);
#ifdef LBR_PHASE_HOOK
    LBR_PHASE_HOOK(ph, kind, n);
#endif
    pos = npos + 2;
    h0 = nh0;
    h1 = nh1;
  }
}
__device__ LBR_EXEC_ATTR void r_exec(int32_t* S_generic, int off) { r_exec_inl(S_generic, off); }
#else
__device__ __attribute__((noinline)) void r_exec(int32_t* S_generic, int off) {
  lds_i32* S = r_lds(S_generic);
  const lds_i32* prog = r_progs(S_generic) + off;
  const int k = r_limb(), row = r_row(), pk = r_plimb(k);
  const int nph = __builtin_amdgcn_readfirstlane(prog[0]), nout = __builtin_amdgcn_readfirstlane(prog[1]);
  int pos = 2 + nout;
  for (int ph = 0; ph < nph; ph++) {
    const int h0 = __builtin_amdgcn_readfirstlane(prog[pos]), h1 = __builtin_amdgcn_readfirstlane(prog[pos + 1]);
    pos += 2;
    const int kind = h0 & 0xff, flags = (h0 >> 8) & 0xff, n = h0 >> 16;
    const int nx = h1 & 0xffff, ny = h1 >> 16;
    if (kind == 0) {
      const int rs = 1 + nx + ny;
      for (int base = 0; base < n; base += LBR_NROWS) {
        const int t = base + row;
        if (t < n) {
          const lds_i32* rec = prog + pos + t * rs;
          const int dst = rec[0];
#ifdef LBR_SUB_HOOK
          LBR_SUB_HOOK(1, dst);
#endif
          const int y = (flags & 2) ? S[16 * (rec[1 + nx] & 0xffff) + k] : r_operand(S, rec + 1 + nx, ny, k, flags & 8, pk);
#ifdef LBR_SUB_HOOK
          LBR_SUB_HOOK(2, y);
#endif
          int x[14];
#ifdef LBR_LDS_REP
          int xs;
          if (flags & 1) {
            xs = rec[1] & 0xffff;
          } else {
            xs = LBR_ROWX + row;
            S[16 * xs + k] = r_operand(S, rec + 1, nx, k, flags & 4, pk);
          }
          r_load_rep(S, xs, x);
#else
          r_rep((flags & 1) ? S[16 * (rec[1] & 0xffff) + k] : r_operand(S, rec + 1, nx, k, flags & 4, pk), x);
#endif
#ifdef LBR_SUB_HOOK
          LBR_SUB_HOOK(3, x[13]);
#endif
          const int rv = rp_mul(x, y, k);
#ifdef LBR_SUB_HOOK
          LBR_SUB_HOOK(4, rv);
#endif
          S[16 * dst + k] = rv;
        }
      }
      pos += n * rs;
    } else {
      // ny: row offset (a linear phase merged into the product phase before it runs on the rows
      // after the products')
      const int rs = 1 + nx, rr = (row - ny + 4 * LBR_NROWS) % LBR_NROWS;
      for (int base = 0; base < n; base += LBR_NROWS) {
        const int t = base + rr;
        if (t < n) {
          const lds_i32* rec = prog + pos + t * rs;
          S[16 * rec[0] + k] = r_sum<3>(S, rec + 1, nx, k, pk);
        }
      }
      pos += n * rs;
    }
    if (kind != 0 || !(flags & 16)) r_sync();  // flag 16: the next (linear) phase reads nothing of this one
#ifdef LBR_PHASE_HOOK
    LBR_PHASE_HOOK(ph, kind, n);
#endif
  }
}
__device__ __forceinline__ void r_exec_inl(int32_t* S_generic, int off) { r_exec(S_generic, off); }
#endif  // LBR_EXEC_V1

// ---------------------------------------------------------------- element moves (limb-parallel)
// dst[e] = src(e) for e < n (src(e) a slot index; every source read before any write)
template <class F>
__device__ __forceinline__ void r_gather(int32_t* S_generic, int dst, int n, F src) {
  lds_i32* S = r_lds(S_generic);
  const int k = r_limb(), row = r_row();
  constexpr int J = (32 + LBR_NROWS - 1) / LBR_NROWS;  // n <= 32
  int v[J];
  LB_UNROLL for (int j = 0; j < J; j++) {
    const int e = row + LBR_NROWS * j;
    if (e < n) v[j] = S[16 * src(e) + k];
  }
  r_sync();
  LB_UNROLL for (int j = 0; j < J; j++) {
    const int e = row + LBR_NROWS * j;
    if (e < n) S[16 * (dst + e) + k] = v[j];
  }
  r_sync();
}
// the same when source and destination slots are disjoint (one barrier)
template <class F>
__device__ __forceinline__ void r_gather_dj(int32_t* S_generic, int dst, int n, F src) {
  lds_i32* S = r_lds(S_generic);
  const int k = r_limb(), row = r_row();
  for (int e = row; e < n; e += LBR_NROWS) S[16 * (dst + e) + k] = S[16 * src(e) + k];
  r_sync();
}
__device__ __forceinline__ void r_copy(int32_t* S, int dst, int src, int n) {
  r_gather(S, dst, n, [&](int e) { return src + e; });
}
__device__ __forceinline__ void r_out(int32_t* S, int off, int first, int n, int dst) {
  const lds_i32* prog = r_progs(S) + off;
  r_gather(S, dst, n, [&](int e) { return prog[2 + first + e]; });
}
__device__ __forceinline__ void r_set_one(int32_t* S_generic, int dst) {
  lds_i32* S = r_lds(S_generic);
  const int t = r_tid();
  if (t < 12 * 16) {
    const int e = t >> 4, k = t & 15;
    int v = 0;
    LB_UNROLL for (int i = 0; i < 14; i++) v = (e == 0 && k == i) ? lbr_k::ONE[i] : v;
    S[16 * (dst + e) + k] = v;
  }
  r_sync();
}
// dst = conj(a): coefficients of w negated (limb-wise: the value stays in (-2p, 2p))
__device__ __forceinline__ void r_conj(int32_t* S_generic, int dst, int a) {
  lds_i32* S = r_lds(S_generic);
  const int t = r_tid();
  int v = 0;
  if (t < 12 * 16) {
    v = S[16 * (a + (t >> 4)) + (t & 15)];
    if ((t >> 4) >= 6) v = -v;
  }
  r_sync();
  if (t < 12 * 16) S[16 * (dst + (t >> 4)) + (t & 15)] = v;
  r_sync();
}

// ---------------------------------------------------------------- import / export (one lane per element)
// The raw limbs of a 2^384-Montgomery element's value times 2^8 (= x 2^392, < 2^389) into staging
// slot LBR_XS + e; r_import_staged reduces them (quotient estimate) into dst + e.
__device__ __forceinline__ void r_stage_fp(int32_t* S_generic, int e, const fp& a) {
  lds_i32* S = r_lds(S_generic);
  S[16 * (LBR_XS + e) + 0] = (int)((a.v[0] << 8) & LBR_M28);
  LB_UNROLL for (int k = 1; k < 14; k++) S[16 * (LBR_XS + e) + k] = (int)lb_bits28(a.v, 28 * k - 8);
  S[16 * (LBR_XS + e) + 14] = 0;
  S[16 * (LBR_XS + e) + 15] = 0;
}
__device__ __forceinline__ void r_import_staged(int32_t* S_generic, int dst, int n) {
  lds_i32* S = r_lds(S_generic);
  const int k = r_limb();
  for (int e = r_row(); e < n; e += LBR_NROWS) S[16 * (dst + e) + k] = r_reduce((int64_t)S[16 * (LBR_XS + e) + k], k);
  r_sync();
}
// canonical 2^384-Montgomery words of the signed limb value sum_k l_k 2^(28 k), |v| < 4p
__device__ __forceinline__ fp r_canon(const int32_t* l) {
  int32_t n[14];
  int64_t c = 0;
  LB_UNROLL for (int k = 0; k < 13; k++) {
    const int64_t v = (int64_t)l[k] + c;
    n[k] = (int32_t)(v & LBR_M28);
    c = v >> 28;
  }
  n[13] = (int32_t)((int64_t)l[13] + c);
  for (int it = 0; it < 4 && n[13] < 0; it++) {  // add p
    int64_t cc = 0;
    LB_UNROLL for (int k = 0; k < 14; k++) {
      const int64_t v = (int64_t)n[k] + lbr_k::P[k] + cc;
      n[k] = k < 13 ? (int32_t)(v & LBR_M28) : (int32_t)v;
      cc = k < 13 ? (v >> 28) : 0;
    }
  }
  for (int it = 0; it < 4; it++) {  // subtract p while v >= p
    int32_t d[14];
    int64_t cc = 0;
    LB_UNROLL for (int k = 0; k < 14; k++) {
      const int64_t v = (int64_t)n[k] - lbr_k::P[k] + cc;
      d[k] = k < 13 ? (int32_t)(v & LBR_M28) : (int32_t)v;
      cc = k < 13 ? (v >> 28) : 0;
    }
    if (d[13] < 0) break;
    LB_UNROLL for (int k = 0; k < 14; k++) n[k] = d[k];
  }
  fp r;
  LB_UNROLL for (int w = 0; w < 12; w++) {
    const int b = 32 * w, q = b / 28, s = b - 28 * q;
    uint32_t v = (uint32_t)n[q] >> s;
    if (q + 1 < 14) v |= (uint32_t)n[q + 1] << (28 - s);
    if (s > 24 && q + 2 < 14) v |= (uint32_t)n[q + 2] << (56 - s);
    r.v[w] = v;
  }
  return r;
}
// slots src .. src + n - 1 -> 2^384-Montgomery words in staging (R' -> R: one row product by
// 2^384 mod p), canonical on lane e's read (r_fp_of)
__device__ __forceinline__ void r_export(int32_t* S_generic, int src, int n) {
  lds_i32* S = r_lds(S_generic);
  const int k = r_limb();
  for (int e = r_row(); e < n; e += LBR_NROWS) {
    const int y = S[16 * (src + e) + k];
    S[16 * (LBR_XS + e) + k] = rp_mul(r_cx_const<14>{lbr_k::K_EXPORT}, y, k);
  }
  r_sync();
}
__device__ __forceinline__ fp r_fp_of_staged(int32_t* S_generic, int e) {
  lds_i32* S = r_lds(S_generic);
  int32_t l[14];
  LB_UNROLL for (int k = 0; k < 14; k++) l[k] = S[16 * (LBR_XS + e) + k];
  return r_canon(l);
}

// Fp12 element e of a word-major SoA array (n elements) <-> an area
__device__ __forceinline__ void r_load_soa12(int32_t* S, int dst, const uint32_t* base, uint32_t n, uint32_t e) {
  const int t = r_tid();
  if (t < 12) {
    fp v;
    for (int w = 0; w < 12; w++) v.v[w] = base[(size_t)(12 * t + w) * n + e];
    r_stage_fp(S, t, v);
  }
  r_sync();
  r_import_staged(S, dst, 12);
}
__device__ __forceinline__ void r_store_soa12(int32_t* S, int src, uint32_t* base, uint32_t n, uint32_t e) {
  r_export(S, src, 12);
  const int t = r_tid();
  if (t < 12) {
    const fp v = r_fp_of_staged(S, t);
    for (int w = 0; w < 12; w++) base[(size_t)(12 * t + w) * n + e] = v.v[w];
  }
  r_sync();
}
// n (<= 16) elements given by lane 0 in `vals` (shared memory) -> slots dst ..
__device__ __forceinline__ void r_import_fps(int32_t* S, int dst, const fp* vals, int n) {
  const int t = r_tid();
  if (t < n) r_stage_fp(S, t, vals[t]);
  r_sync();
  r_import_staged(S, dst, n);
}

// ---------------------------------------------------------------- program loading
__device__ void r_init(int32_t* S_generic, int nprog = LBR_PROGS_FE, int first = 0) {
  lds_i32* S = r_lds(S_generic);
  const int t = r_tid();
  {
    lds_i32x4* dst = (lds_i32x4*)(S + LBR_SLOT_WORDS + LBR_MISC);
    const i32x4* src = reinterpret_cast<const i32x4*>(LBR_PROGS + first);
    for (int i = t; i < nprog / 4; i += LBR_NT) dst[i] = src[i];
    if (t == 0) S[LBR_SLOT_WORDS + 0] = first;
  }
  for (int i = t; i < LBR_N_CONST * 16; i += LBR_NT) S[16 * LBR_CONST + i] = LBR_CONST_LIMBS[i >> 4][i & 15];
  r_sync();
}

// ---------------------------------------------------------------- Fp12 ops on 12-slot areas
// The Fp12 product (MUL12) written out the same way: phase 1, rows 0..53: the 54 Karatsuba
// products, each operand a sum of <= 8 input slots (a: 0..11, b: 12..23); phase 2, rows 0..11: the
// outputs, <= 36 product terms each (tools/gen_mul12_fast.py -> lb_mul12_tab.h, checked against
// the oracle's tower product).  dst may equal a or b.
#ifndef LBR_MUL12_FAST
#define LBR_MUL12_FAST 1
#endif
__device__ __forceinline__ void r_mul12_fast(int32_t* S_generic, int dst, int a, int b) {
  lds_i32* S = r_lds(S_generic);
  const int k = r_limb(), row = r_row();
  const int T = LBR_TEMP;
  if (row < 54) {
    int64_t x = 0, y = 0;
    LB_UNROLL for (int j = 0; j < LBR_M12_NX; j++) {
      const int sx = LBR_M12P[row][2 * j], sy = LBR_M12P[row][2 * LBR_M12_NX + 2 * j];
      x += (int64_t)LBR_M12P[row][2 * j + 1] * S[16 * (sx < 12 ? a + sx : b + sx - 12) + k];
      y += (int64_t)LBR_M12P[row][2 * LBR_M12_NX + 2 * j + 1] * S[16 * (sy < 12 ? a + sy : b + sy - 12) + k];
    }
    int xr[14];
    r_rep(r_norm<true>(x, k), xr);
    S[16 * (T + row) + k] = rp_mul(xr, r_norm<true>(y, k), k);
  }
  r_sync();
  if (row < 12) {
    int64_t acc = 0;
    LB_UNROLL for (int j = 0; j < LBR_M12_NO; j++)
      acc += (int64_t)LBR_M12O[row][2 * j + 1] * S[16 * (T + LBR_M12O[row][2 * j]) + k];
    S[16 * (dst + row) + k] = r_reduce(acc, k);
  }
  r_sync();
}

__device__ void r_mul(int32_t* S, int dst, int a, int b) {
  if (LBR_MUL12_FAST) {
    r_mul12_fast(S, dst, a, b);
    return;
  }
  r_gather(S, LBR_IN, 24, [&](int e) { return e < 12 ? a + e : b + e - 12; });
  r_exec(S, LBR_MUL12);
  r_out(S, LBR_MUL12, 0, 12, dst);
}
__device__ void r_sqr(int32_t* S, int dst, int a) {
  r_copy(S, LBR_IN, a, 12);
  r_exec(S, LBR_SQR12);
  r_out(S, LBR_SQR12, 0, 12, dst);
}
// Granger-Scott cyclotomic squaring written out for the workgroup instead of interpreted
// (CSQR12): the interpreter's per-phase work -- program header and record reads, the next phase's
// prefetch, the operand records, the IN / output copies of r_run -- cost ~2.2 us of a 3.1 us
// squaring (profiles/r6_row_bench_tl.txt), the 18 products ~0.9 us.  Here each row's task follows
// from its row number:
//   products (rows 0..17): pair q = row / 6 of (x, y) in {(a00, a11), (a10, a02), (a01, a12)},
//     j = row % 6: x^2 = ((x0 + x1)(x0 - x1), 2 x0 x1), y^2 likewise, (x + y)^2 likewise;
//   outputs (rows 0..11), Fp4 squares r0 = xi y^2 + x^2, r1 = (x + y)^2 - x^2 - y^2:
//     c00 = 3 t0.r0 - 2 a00, c01 = 3 t1.r0 - 2 a01, c02 = 3 t2.r0 - 2 a02,
//     c10 = 3 xi t2.r1 + 2 a10, c11 = 3 t0.r1 + 2 a11, c12 = 3 t1.r1 + 2 a12
// (tools/gen_row_programs.py cyclotomic_sqr; slot k = c{k/6}.c{(k%6)/2}.c{k%2}).  Two barriers per
// squaring; dst may equal src (output k reads only input k).
#ifndef LBR_CSQR_FAST
#define LBR_CSQR_FAST 1
#endif
__device__ __forceinline__ void r_csqr_fast(int32_t* S_generic, int dst, int src) {
  lds_i32* S = r_lds(S_generic);
  const int k = r_limb(), row = r_row();
  const int T = LBR_TEMP;
  if (row < 18) {
    const int q = row / 6, j = row - 6 * q;
    const int xs = q == 0 ? 0 : (q == 1 ? 6 : 2), ys = q == 0 ? 8 : (q == 1 ? 4 : 10);
    const int x0 = S[16 * (src + xs) + k], x1 = S[16 * (src + xs + 1) + k];
    const int y0 = S[16 * (src + ys) + k], y1 = S[16 * (src + ys + 1) + k];
    // coefficients of (x0, x1, y0, y1) in the product's two operands, by j
    const int ax0 = (j == 0 || j == 1 || j >= 4) ? 1 : 0, ax1 = (j == 0 || j == 4) ? 1 : 0;
    const int ay0 = (j == 2 || j == 3 || j >= 4) ? 1 : 0, ay1 = (j == 2 || j == 4) ? 1 : 0;
    const int bx0 = (j == 0 || j == 4) ? 1 : 0, bx1 = (j == 0 || j == 4) ? -1 : (j == 1 || j == 5 ? 1 : 0);
    const int by0 = (j == 2 || j == 4) ? 1 : 0, by1 = (j == 2 || j == 4) ? -1 : (j == 3 || j == 5 ? 1 : 0);
    const int xv = r_norm<true>((int64_t)ax0 * x0 + (int64_t)ax1 * x1 + (int64_t)ay0 * y0 + (int64_t)ay1 * y1, k);
    const int yv = r_norm<true>((int64_t)bx0 * x0 + (int64_t)bx1 * x1 + (int64_t)by0 * y0 + (int64_t)by1 * y1, k);
    int xr[14];
    r_rep(xv, xr);
    S[16 * (T + row) + k] = rp_mul(xr, yv, k);
  }
  r_sync();
  if (row < 12) {
    // output row -> pair q and form: 0 r0.c0, 1 r0.c1, 2 r1.c0, 3 r1.c1, 4 (xi r1).c0, 5 (xi r1).c1
    const int q = (row < 2 || row == 8 || row == 9) ? 0 : ((row < 4 || row >= 10) ? 1 : 2);
    const int f = row < 6 ? (row & 1) : (row < 8 ? 4 + (row & 1) : 2 + (row & 1));
    // coefficients of the pair's products p0..p5 and of the input slot, per form
    const int c0 = f == 0 ? 3 : ((f == 1 || f == 3) ? 0 : -3);
    const int c1 = f == 1 ? 6 : (f == 3 ? -6 : (f == 4 ? 6 : (f == 5 ? -6 : 0)));
    const int c2 = f < 2 ? 3 : (f == 3 ? 0 : -3);
    const int c3 = f == 0 ? -6 : (f == 1 ? 6 : (f == 2 ? 0 : (f == 4 ? 6 : -6)));
    const int c4 = f >= 2 && f != 3 ? 3 : 0;
    const int c5 = f == 3 ? 6 : (f == 4 ? -6 : (f == 5 ? 6 : 0));
    const int ci = f < 2 ? -2 : 2;
    const int b = T + 6 * q;
    int64_t acc = (int64_t)ci * S[16 * (src + row) + k];
    acc += (int64_t)c0 * S[16 * (b + 0) + k] + (int64_t)c1 * S[16 * (b + 1) + k] + (int64_t)c2 * S[16 * (b + 2) + k];
    acc += (int64_t)c3 * S[16 * (b + 3) + k] + (int64_t)c4 * S[16 * (b + 4) + k] + (int64_t)c5 * S[16 * (b + 5) + k];
    S[16 * (dst + row) + k] = r_reduce(acc, k);
  }
  r_sync();
}

// The projective G2 doubling (RCB Algorithm 9, PDBL1) written out the same way: phase 1, rows
// 0..9: the level-1 products P (Y^2, YZ, Z^2, XY); phase 2, rows 0..11: the four Fp2 products of
// level 2 (Karatsuba) over combinations of P; phase 3, rows 0..5: the outputs.  Each row's integer
// coefficients come from tools/gen_pdbl_fast.py (lb_pdbl_tab.h), which checks the three phases
// against the oracle's doubling.  dst may equal src.
#ifndef LBR_PDBL_FAST
#define LBR_PDBL_FAST 1
#endif
__device__ __forceinline__ void r_pdbl_fast(int32_t* S_generic, int dst, int src) {
  lds_i32* S = r_lds(S_generic);
  const int k = r_limb(), row = r_row();
  const int T = LBR_TEMP;  // P at T .. T + 9, Q at T + 10 .. T + 21
  if (row < 10) {
    int64_t x = 0, y = 0;
    LB_UNROLL for (int e = 0; e < 6; e++) {
      const int v = S[16 * (src + e) + k];
      x += (int64_t)LBR_PD1[row][e] * v;
      y += (int64_t)LBR_PD1[row][6 + e] * v;
    }
    int xr[14];
    r_rep(r_norm<true>(x, k), xr);
    S[16 * (T + row) + k] = rp_mul(xr, r_norm<true>(y, k), k);
  }
  r_sync();
  if (row < 12) {
    int64_t x = 0, y = 0;
    LB_UNROLL for (int e = 0; e < 10; e++) {
      const int v = S[16 * (T + e) + k];
      x += (int64_t)LBR_PD2[row][e] * v;
      y += (int64_t)LBR_PD2[row][10 + e] * v;
    }
    int xr[14];
    r_rep(r_reduce(x, k), xr);
    S[16 * (T + 10 + row) + k] = rp_mul(xr, r_reduce(y, k), k);
  }
  r_sync();
  if (row < 6) {
    int64_t acc = 0;
    LB_UNROLL for (int e = 0; e < 12; e++) acc += (int64_t)LBR_PD3[row][e] * S[16 * (T + 10 + e) + k];
    S[16 * (dst + row) + k] = r_reduce(acc, k);
  }
  r_sync();
}

// a^2 for a in the cyclotomic subgroup (Granger-Scott: 18 products instead of 36)
__device__ void r_csqr(int32_t* S, int dst, int a) {
  if (LBR_CSQR_FAST) {
    r_csqr_fast(S, dst, a);
    return;
  }
  r_copy(S, LBR_IN, a, 12);
  r_exec(S, LBR_CSQR12);
  r_out(S, LBR_CSQR12, 0, 12, dst);
}
__device__ void r_frob(int32_t* S, int dst, int a) {
  r_copy(S, LBR_IN, a, 12);
  r_exec(S, LBR_FROB);
  r_out(S, LBR_FROB, 0, 12, dst);
}
__device__ void r_frob2(int32_t* S, int dst, int a) {
  r_copy(S, LBR_IN, a, 12);
  r_exec(S, LBR_FROB2);
  r_out(S, LBR_FROB2, 0, 12, dst);
}
// 1 if area a is 1 (exact: canonical words compared)
__device__ bool r_is_one(int32_t* S_generic, int a) {
  lds_i32* S = r_lds(S_generic);
  r_export(S_generic, a, 12);
  const int t = r_tid();
  if (t == 0) S[LBR_SLOT_WORDS + 1] = 0;
  r_sync();
  if (t < 12) {
    const fp v = r_fp_of_staged(S_generic, t);
    const fp want = t == 0 ? fp_one() : fp_zero();
    if (!fp_eq(v, want)) atomicOr((int*)&S_generic[LBR_SLOT_WORDS + 1], 1);
  }
  r_sync();
  const int r = S[LBR_SLOT_WORDS + 1];
  r_sync();
  return r == 0;
}
// areas a and b equal (canonical comparison)
__device__ bool r_eq(int32_t* S_generic, int a, int b) {
  lds_i32* S = r_lds(S_generic);
  __shared__ fp va[12];
  r_export(S_generic, a, 12);
  const int t = r_tid();
  if (t < 12) va[t] = r_fp_of_staged(S_generic, t);
  if (t == 0) S[LBR_SLOT_WORDS + 1] = 0;
  r_sync();
  r_export(S_generic, b, 12);
  if (t < 12 && !fp_eq(va[t], r_fp_of_staged(S_generic, t))) atomicOr((int*)&S_generic[LBR_SLOT_WORDS + 1], 1);
  r_sync();
  const int r = S[LBR_SLOT_WORDS + 1];
  r_sync();
  return r == 0;
}
// ---------------------------------------------------------------- one-row exponentiation
// An Fp exponentiation by a constant on one 16-lane row of a wave, every lane of the row holding
// the same fp (the four rows of a wave: four independent items): the chain's products are row
// products (rp_mul, ~0.45 us each, issue-bound on its 64-bit MADs) with the operand replicated
// by DPP row broadcasts -- no LDS, no barriers -- instead of lone-lane products (~1.1 us).  The
// square roots of hash_to_G2's SSWU map use it for small batches (k_hash_map_row).
__device__ __forceinline__ int r1_sqr(int v, int k) {
  int x[14];
  r_rep(v, x);
  return rp_mul(x, v, k);
}
__device__ __forceinline__ int r1_mul(int v, int w, int k) {
  int x[14];
  r_rep(v, x);
  return rp_mul(x, w, k);
}
// this lane's limb of a * 2^8 (= a's value in R'-form: a R 2^8 = a R')
__device__ __forceinline__ int r1_import(const fp& a, int k) {
  int v = 0;
  LB_UNROLL for (int i = 0; i < 14; i++) {
    const int li = i == 0 ? (int)((a.v[0] << 8) & LBR_M28) : (int)lb_bits28(a.v, 28 * i - 8);
    v = k == i ? li : v;
  }
  return v;
}
// a row value (R'-form) -> canonical fp (R-form) in every lane of the row
__device__ __forceinline__ fp r1_export(int v, int k) {
  const int y = rp_mul(r_cx_const<14>{lbr_k::K_EXPORT}, k < 14 ? v : 0, k);
  int l[14];
  r_rep(y, l);
  return r_canon(l);
}
template <int NT>
__device__ __forceinline__ int r1_sel(const int (&t)[NT], uint32_t i) {
  int r = t[0];
  LB_UNROLL for (int c = 1; c < NT; c++) r = i == (uint32_t)c ? t[c] : r;
  return r;
}
// a^e (e: top_bit + 1 bits, a constant), 4-bit windows over odd powers as fp_pow_const_28
__device__ fp r1_pow_const(const fp& a, const uint32_t* e, int top_bit) {
  const int k = r_limb();
  int tab[8];
  tab[0] = r1_import(a, k);
  const int a2 = r1_sqr(tab[0], k);
  LB_UNROLL for (int c = 1; c < 8; c++) tab[c] = r1_mul(tab[c - 1], a2, k);
  auto bit = [&](int i) -> uint32_t { return (e[i >> 5] >> (i & 31)) & 1u; };
  int r = tab[0];
  bool first = true;
  int i = top_bit;
  while (i >= 0) {
    if (!bit(i)) {
      if (!first) r = r1_sqr(r, k);
      i--;
      continue;
    }
    int j = i - 3 > 0 ? i - 3 : 0;
    while (!bit(j)) j++;
    uint32_t val = 0;
    for (int c = i; c >= j; c--) val = (val << 1) | bit(c);
    if (first) {
      r = r1_sel(tab, val >> 1);
      first = false;
    } else {
      for (int c = i; c >= j; c--) r = r1_sqr(r, k);
      r = r1_mul(r, r1_sel(tab, val >> 1), k);
    }
    i = j - 1;
  }
  return r1_export(r, k);
}

// ---------------------------------------------------------------- a row field element
// rfp: one Fp element on a 16-lane row (lane k: limb k, R'-form, as r1_* above), with the f_*
// overloads of the generic curve code (lb_curve.h), so jac_mul_glv_i<rfp> & co. run with every
// product a row product (~0.45 us) instead of a lone-lane one (~1.1 us).  Every lane of the row
// runs the same item's control flow; sums are reduced (r_reduce) so any chain of them stays a
// valid rp_mul operand; zero tests export the canonical value (one product).
struct rfp {
  int v;
};
__device__ __forceinline__ rfp rf_of(const fp& a) { return rfp{r1_import(a, r_limb())}; }
__device__ __forceinline__ fp rf_fp(const rfp& a) { return r1_export(a.v, r_limb()); }
__device__ __forceinline__ rfp rf_red(int64_t acc) { return rfp{r_reduce(acc, r_limb())}; }
__device__ __forceinline__ rfp f_add(const rfp& a, const rfp& b) { return rf_red((int64_t)a.v + b.v); }
__device__ __forceinline__ rfp f_sub(const rfp& a, const rfp& b) { return rf_red((int64_t)a.v - b.v); }
__device__ __forceinline__ rfp f_dbl(const rfp& a) { return rf_red(2 * (int64_t)a.v); }
__device__ __forceinline__ rfp f_neg(const rfp& a) { return rf_red(-(int64_t)a.v); }
__device__ __forceinline__ rfp f_mul3(const rfp& a) { return rf_red(3 * (int64_t)a.v); }
__device__ __forceinline__ rfp f_mul8(const rfp& a) { return rf_red(8 * (int64_t)a.v); }
__device__ __forceinline__ rfp f_mul(const rfp& a, const rfp& b) {
  int x[14];
  r_rep(a.v, x);
  return rfp{rp_mul(x, b.v, r_limb())};
}
__device__ __forceinline__ rfp f_sqr(const rfp& a) { return f_mul(a, a); }
__device__ __forceinline__ bool f_is_zero(const rfp& a) { return fp_is_zero(rf_fp(a)); }
__device__ __forceinline__ bool f_eq(const rfp& a, const rfp& b) { return f_is_zero(f_sub(a, b)); }
__device__ __forceinline__ rfp f_select(bool c, const rfp& a, const rfp& b) { return rfp{c ? a.v : b.v}; }
__device__ __forceinline__ void f_set_zero(rfp& a) { a.v = 0; }
__device__ __forceinline__ void f_set_one(rfp& a) { a = rf_of(fp_one()); }
__device__ __forceinline__ aff<rfp> rf_of(const g1a& a) { return aff<rfp>{rf_of(a.x), rf_of(a.y)}; }
__device__ __forceinline__ g1j rf_fp(const jac<rfp>& a) { return g1j{rf_fp(a.x), rf_fp(a.y), rf_fp(a.z)}; }

// ---- the four rows of a wave as four product units for ONE item (every row holds the whole
// state, the same values): w4_mul computes up to four independent products in one row product,
// row j the j-th, and hands every row all four results (three v_permlane*_swap, VALU ops).
// permlane16_swap(v, v) = {rows (v0 v0 v2 v2), rows (v1 v1 v3 v3)}; permlane32_swap(u, u) of those:
// {(u0 u0 u0 u0) -> v0 / v1, (u2 ...) -> v2 / v3}.
__device__ __forceinline__ void w4_gather(int v, int (&o)[4]) {
  const auto e = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  const auto a = __builtin_amdgcn_permlane32_swap(e[0], e[0], false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(e[1], e[1], false, false);
  o[0] = a[0];
  o[1] = b[0];
  o[2] = a[1];
  o[3] = b[1];
}
template <int N>
__device__ __forceinline__ void w4_mul(const rfp (&x)[N], const rfp (&y)[N], rfp* o) {
  static_assert(N >= 1 && N <= 4, "w4_mul: one product per row");
  const int r = (threadIdx.x >> 4) & 3;
  int xv = x[0].v, yv = y[0].v;
  LB_UNROLL for (int j = 1; j < N; j++) {
    xv = r == j ? x[j].v : xv;
    yv = r == j ? y[j].v : yv;
  }
  int xr[14];
  r_rep(xv, xr);
  int g[4];
  w4_gather(rp_mul(xr, yv, r_limb()), g);
  LB_UNROLL for (int j = 0; j < N; j++) o[j].v = g[j];
}

// rfp2: Fp2 over rfp (Karatsuba products: three row products), and the map_to_curve_g2_fold_t
// policy (lb_h2c.h: fl_*)
struct rfp2 {
  rfp c0, c1;
};
__device__ __forceinline__ rfp2 f_add(const rfp2& a, const rfp2& b) { return rfp2{f_add(a.c0, b.c0), f_add(a.c1, b.c1)}; }
__device__ __forceinline__ rfp2 f_sub(const rfp2& a, const rfp2& b) { return rfp2{f_sub(a.c0, b.c0), f_sub(a.c1, b.c1)}; }
__device__ __forceinline__ rfp2 f_neg(const rfp2& a) { return rfp2{f_neg(a.c0), f_neg(a.c1)}; }
__device__ __forceinline__ rfp2 f_dbl(const rfp2& a) { return rfp2{f_dbl(a.c0), f_dbl(a.c1)}; }
// LBR_FP2_W4 (default): every rfp2 user runs one item per WAVE (the four rows hold the same
// values), so the Karatsuba products take one row product on rows 0..2 (w4_mul) instead of three
// in sequence on each row
__device__ __forceinline__ rfp2 f_mul(const rfp2& a, const rfp2& b) {
#if LBR_FP2_W4
  {
    const int k = r_limb();
    const rfp x[3] = {a.c0, a.c1, rfp{r_norm<true>((int64_t)a.c0.v + a.c1.v, k)}};
    const rfp y[3] = {b.c0, b.c1, rfp{r_norm<true>((int64_t)b.c0.v + b.c1.v, k)}};
    rfp t[3];
    w4_mul<3>(x, y, t);
    return rfp2{rf_red((int64_t)t[0].v - t[1].v), rf_red((int64_t)t[2].v - t[0].v - t[1].v)};
  }
#endif
  const rfp t0 = f_mul(a.c0, b.c0), t1 = f_mul(a.c1, b.c1);
  const int k = r_limb();
  // (a0 + a1)(b0 + b1): operand sums by carry rounds only (|sum| < 4p, a valid rp_mul operand)
  int x[14];
  r_rep(r_norm<true>((int64_t)a.c0.v + a.c1.v, k), x);
  const int t2 = rp_mul(x, r_norm<true>((int64_t)b.c0.v + b.c1.v, k), k);
  return rfp2{rf_red((int64_t)t0.v - t1.v), rf_red((int64_t)t2 - t0.v - t1.v)};
}
__device__ __forceinline__ rfp2 f_sqr(const rfp2& a) {
  const int k = r_limb();
#if LBR_FP2_W4
  {
    const rfp x[2] = {rfp{r_norm<true>((int64_t)a.c0.v + a.c1.v, k)}, a.c0};
    const rfp y[2] = {rfp{r_norm<true>((int64_t)a.c0.v - a.c1.v, k)}, a.c1};
    rfp t[2];
    w4_mul<2>(x, y, t);
    return rfp2{t[0], f_dbl(t[1])};
  }
#endif
  int x[14];
  r_rep(r_norm<true>((int64_t)a.c0.v + a.c1.v, k), x);
  const int t0 = rp_mul(x, r_norm<true>((int64_t)a.c0.v - a.c1.v, k), k);
  const rfp t1 = f_mul(a.c0, a.c1);
  return rfp2{rfp{t0}, f_dbl(t1)};
}
__device__ __forceinline__ bool f_is_zero(const rfp2& a) { return f_is_zero(a.c0) && f_is_zero(a.c1); }
__device__ __forceinline__ rfp2 f_select(bool c, const rfp2& a, const rfp2& b) {
  return rfp2{f_select(c, a.c0, b.c0), f_select(c, a.c1, b.c1)};
}
__device__ __forceinline__ rfp fl_in(const fp& a, const rfp*) { return rf_of(a); }
__device__ __forceinline__ rfp2 fl_in(const fp2& a, const rfp2*) { return rfp2{rf_of(a.c0), rf_of(a.c1)}; }
__device__ __forceinline__ fp fl_out(const rfp& a) { return rf_fp(a); }
__device__ __forceinline__ fp2 fl_out(const rfp2& a) { return fp2{rf_fp(a.c0), rf_fp(a.c1)}; }
__device__ __forceinline__ rfp fl_norm(const rfp2& a) { return f_add(f_sqr(a.c0), f_sqr(a.c1)); }
__device__ __forceinline__ rfp2 fl_mulb(const rfp2& a, const rfp& s) { return rfp2{f_mul(a.c0, s), f_mul(a.c1, s)}; }
__device__ __forceinline__ rfp2 fl_conj(const rfp2& a) { return rfp2{a.c0, f_neg(a.c1)}; }
__device__ __forceinline__ rfp2 fl_make(const rfp& a, const rfp& b) { return rfp2{a, b}; }
__device__ __forceinline__ rfp2 f_mul3(const rfp2& a) { return rfp2{f_mul3(a.c0), f_mul3(a.c1)}; }
__device__ __forceinline__ rfp2 f_mul8(const rfp2& a) { return rfp2{f_mul8(a.c0), f_mul8(a.c1)}; }
__device__ __forceinline__ rfp fl_c0(const rfp2& a) { return a.c0; }
__device__ __forceinline__ rfp fl_c1(const rfp2& a) { return a.c1; }
__device__ __forceinline__ void f_set_zero(rfp2& a) { a.c0.v = a.c1.v = 0; }
__device__ __forceinline__ void f_set_one(rfp2& a) {
  f_set_one(a.c0);
  a.c1.v = 0;
}

// ---- G2 in Jacobian coordinates over rfp2 on the four rows of a wave (w4_mul levels of four Fp
// products; every row holds the point): one wave per point instead of a 16-wave row-engine
// workgroup, for the small-batch ladders (k_sig_subgroup_w4, k_sig_blind_w4).  No exceptional-case
// tests: any exceptional case of the formulas (an operand at infinity, P = +-Q, Y = 0) yields Z = 0,
// which every later doubling and mixed addition keeps (as the row engine's fast chains).
__device__ __forceinline__ rfp rf_lz(int64_t v) { return rfp{r_norm<true>(v, r_limb())}; }  // carries only
__device__ __forceinline__ rfp rf_sum(const rfp& a, const rfp& b) { return rf_lz((int64_t)a.v + b.v); }
__device__ __forceinline__ rfp rf_dif(const rfp& a, const rfp& b) { return rf_lz((int64_t)a.v - b.v); }
// lazy sums (carry rounds only, no quotient-estimate reduction): a value stays a valid product
// operand while its coefficients sum to <= 16 over reduced / product-output terms (|v| < 32 p);
// the ladders reduce only the point they carry from step to step (f_* below)
__device__ __forceinline__ rfp lz_add(const rfp& a, const rfp& b) { return rf_lz((int64_t)a.v + b.v); }
__device__ __forceinline__ rfp lz_sub(const rfp& a, const rfp& b) { return rf_lz((int64_t)a.v - b.v); }
__device__ __forceinline__ rfp lz_mul(const rfp& a, int c) { return rf_lz((int64_t)c * a.v); }
__device__ __forceinline__ rfp2 lz_add(const rfp2& a, const rfp2& b) { return rfp2{lz_add(a.c0, b.c0), lz_add(a.c1, b.c1)}; }
__device__ __forceinline__ rfp2 lz_sub(const rfp2& a, const rfp2& b) { return rfp2{lz_sub(a.c0, b.c0), lz_sub(a.c1, b.c1)}; }
__device__ __forceinline__ rfp2 lz_mul(const rfp2& a, int c) { return rfp2{lz_mul(a.c0, c), lz_mul(a.c1, c)}; }
// Karatsuba's third product t2 = (a0 + a1)(b0 + b1) -> (t0 - t1, t2 - t0 - t1), lazy (< 2p, 3p)
__device__ __forceinline__ rfp2 rf2_kara(const rfp& t0, const rfp& t1, const rfp& t2) {
  return rfp2{lz_sub(t0, t1), rf_lz((int64_t)t2.v - t0.v - t1.v)};
}
// the complex squaring's (o0, 2 o1)
__device__ __forceinline__ rfp2 rf2_sq(const rfp& o0, const rfp& o1) { return rfp2{o0, lz_mul(o1, 2)}; }
// reduce the limb-wise combination sum_j c_j a_j (64-bit limb sums) of each component
#define RF2_RED(E0, E1) (rfp2{rf_red((int64_t)(E0)), rf_red((int64_t)(E1))})
#define I64(x) ((int64_t)(x))
// dbl-2009-l: A = X^2, B = Y^2 | C = B^2, F = E^2 (E = 3A) | P = (X + B)^2, y0 z0, y1 z1 |
// (y0 + y1)(z0 + z1), E (D - X3): four levels of four products.  In: X, Y, Z reduced (< p); out
// reduced.  Bounds (in p): A, B, C, F, P < 2; E < 6; D < 12; X3 reduced; W < 13.
__device__ __forceinline__ void w4_g2_dbl(rfp2& X, rfp2& Y, rfp2& Z) {
  rfp o[4];
  w4_mul<4>({rf_sum(X.c0, X.c1), X.c0, rf_sum(Y.c0, Y.c1), Y.c0}, {rf_dif(X.c0, X.c1), X.c1, rf_dif(Y.c0, Y.c1), Y.c1}, o);
  const rfp2 A = rf2_sq(o[0], o[1]), B = rf2_sq(o[2], o[3]);
  const rfp2 E = lz_mul(A, 3);
  w4_mul<4>({rf_sum(B.c0, B.c1), B.c0, rf_sum(E.c0, E.c1), E.c0}, {rf_dif(B.c0, B.c1), B.c1, rf_dif(E.c0, E.c1), E.c1}, o);
  const rfp2 C = rf2_sq(o[0], o[1]), F = rf2_sq(o[2], o[3]);
  const rfp2 XB = lz_add(X, B);
  w4_mul<4>({rf_sum(XB.c0, XB.c1), XB.c0, Y.c0, Y.c1}, {rf_dif(XB.c0, XB.c1), XB.c1, Z.c0, Z.c1}, o);
  const rfp2 P = rf2_sq(o[0], o[1]);
  const rfp yz0 = o[2], yz1 = o[3];
  const rfp2 D = lz_mul(lz_sub(lz_sub(P, A), C), 2);
  const rfp2 X3 = RF2_RED(I64(F.c0.v) - 2 * I64(D.c0.v), I64(F.c1.v) - 2 * I64(D.c1.v));
  const rfp2 W = lz_sub(D, X3);
  w4_mul<4>({rf_sum(Y.c0, Y.c1), E.c0, E.c1, rf_sum(E.c0, E.c1)}, {rf_sum(Z.c0, Z.c1), W.c0, W.c1, rf_sum(W.c0, W.c1)}, o);
  const rfp2 YZ = rf2_kara(yz0, yz1, o[0]);
  const rfp2 EW = rf2_kara(o[1], o[2], o[3]);
  Y = RF2_RED(I64(EW.c0.v) - 8 * I64(C.c0.v), I64(EW.c1.v) - 8 * I64(C.c1.v));
  X = X3;
  Z = RF2_RED(2 * I64(YZ.c0.v), 2 * I64(YZ.c1.v));
}
// madd-2007-bl (Q affine, reduced): 29 products in eight levels.  In / out as w4_g2_dbl.
// Bounds (in p): Z1Z1, HH < 2; U2, S2, J, V < 3; H < 4; ZH < 5; R < 8; I < 8; W < 4.
__device__ __forceinline__ void w4_g2_madd(rfp2& X, rfp2& Y, rfp2& Z, const rfp2& qx, const rfp2& qy) {
  rfp o[4];
  // Z1Z1 = Z1^2; qy0 z0, qy1 z1
  w4_mul<4>({rf_sum(Z.c0, Z.c1), Z.c0, qy.c0, qy.c1}, {rf_dif(Z.c0, Z.c1), Z.c1, Z.c0, Z.c1}, o);
  const rfp2 ZZ = rf2_sq(o[0], o[1]);
  const rfp a0 = o[2], a1 = o[3];
  // (qy0 + qy1)(z0 + z1); U2 = qx Z1Z1
  w4_mul<4>({rf_sum(qy.c0, qy.c1), qx.c0, qx.c1, rf_sum(qx.c0, qx.c1)}, {rf_sum(Z.c0, Z.c1), ZZ.c0, ZZ.c1, rf_sum(ZZ.c0, ZZ.c1)}, o);
  const rfp2 QZ = rf2_kara(a0, a1, o[0]);
  const rfp2 U2 = rf2_kara(o[1], o[2], o[3]);
  const rfp2 H = lz_sub(U2, X);
  // S2 = qy Z1 Z1Z1; (h0 + h1)(h0 - h1)
  w4_mul<4>({QZ.c0, QZ.c1, rf_sum(QZ.c0, QZ.c1), rf_sum(H.c0, H.c1)}, {ZZ.c0, ZZ.c1, rf_sum(ZZ.c0, ZZ.c1), rf_dif(H.c0, H.c1)}, o);
  const rfp2 S2 = rf2_kara(o[0], o[1], o[2]);
  const rfp hh0 = o[3];
  const rfp2 R = lz_mul(lz_sub(S2, Y), 2);
  const rfp2 ZH = lz_add(Z, H);
  // h0 h1; (Z1 + H)^2; (r0 + r1)(r0 - r1)
  w4_mul<4>({H.c0, rf_sum(ZH.c0, ZH.c1), ZH.c0, rf_sum(R.c0, R.c1)}, {H.c1, rf_dif(ZH.c0, ZH.c1), ZH.c1, rf_dif(R.c0, R.c1)}, o);
  const rfp2 HH = rf2_sq(hh0, o[0]), ZH2 = rf2_sq(o[1], o[2]);
  const rfp r2a = o[3];
  const rfp2 I = lz_mul(HH, 4);
  // r0 r1; J = H I
  w4_mul<4>({R.c0, H.c0, H.c1, rf_sum(H.c0, H.c1)}, {R.c1, I.c0, I.c1, rf_sum(I.c0, I.c1)}, o);
  const rfp2 R2 = rf2_sq(r2a, o[0]);
  const rfp2 J = rf2_kara(o[1], o[2], o[3]);
  // V = X1 I; y0 j0
  w4_mul<4>({X.c0, X.c1, rf_sum(X.c0, X.c1), Y.c0}, {I.c0, I.c1, rf_sum(I.c0, I.c1), J.c0}, o);
  const rfp2 V = rf2_kara(o[0], o[1], o[2]);
  const rfp yj0 = o[3];
  const rfp2 X3 = RF2_RED(I64(R2.c0.v) - I64(J.c0.v) - 2 * I64(V.c0.v), I64(R2.c1.v) - I64(J.c1.v) - 2 * I64(V.c1.v));
  const rfp2 W = lz_sub(V, X3);
  // r W; y1 j1
  w4_mul<4>({R.c0, R.c1, rf_sum(R.c0, R.c1), Y.c1}, {W.c0, W.c1, rf_sum(W.c0, W.c1), J.c1}, o);
  const rfp2 RW = rf2_kara(o[0], o[1], o[2]);
  const rfp yj1 = o[3];
  // (y0 + y1)(j0 + j1)
  w4_mul<1>({rf_sum(Y.c0, Y.c1)}, {rf_sum(J.c0, J.c1)}, o);
  const rfp2 YJ = rf2_kara(yj0, yj1, o[0]);
  Y = RF2_RED(I64(RW.c0.v) - 2 * I64(YJ.c0.v), I64(RW.c1.v) - 2 * I64(YJ.c1.v));
  X = X3;
  Z = RF2_RED(I64(ZH2.c0.v) - I64(ZZ.c0.v) - I64(HH.c0.v), I64(ZH2.c1.v) - I64(ZZ.c1.v) - I64(HH.c1.v));
}

// An Fp exponentiation by a constant on a PAIR of rows (rows 2j, 2j + 1 of a wave; every lane of
// both rows holds the same fp): right to left, the even row squares (s = a^(2^i)) while the odd
// row multiplies its accumulator by the same s when bit i is set, in the same row product; then
// the even row's new s moves to the odd row (v_permlane16_swap, a VALU op).  The chain is one
// product per exponent bit (378 for (p-3)/4) against r1_pow_const's squarings plus one product
// per 4-bit window (~460).
// (rfp in and out: both rows of the pair hold the same value)
__device__ __forceinline__ rfp r2_pow_rf(const rfp& a, const uint32_t* e, int top_bit) {
  const int k = r_limb();
  const bool odd = (threadIdx.x >> 4) & 1;
  int s = a.v;
  int acc = r1_import(fp_one(), k);
  for (int i = 0; i <= top_bit; i++) {
    const bool b = (e[i >> 5] >> (i & 31)) & 1u;  // uniform
    int x[14];
    r_rep(s, x);
    const int r = rp_mul(x, odd ? acc : s, k);
    const int even_r = __builtin_amdgcn_permlane16_swap(r, r, false, false)[0];  // odd rows: the even row's r
    if (odd) {
      if (b) acc = r;
      s = even_r;
    } else {
      s = r;
    }
  }
  const int odd_acc = __builtin_amdgcn_permlane16_swap(acc, acc, false, false)[1];  // even rows: the odd row's acc
  return rfp{odd ? acc : odd_acc};
}
__device__ __forceinline__ fp r2_pow_const(const fp& a, const uint32_t* e, int top_bit) {
  return rf_fp(r2_pow_rf(rf_of(a), e, top_bit));
}

// ---------------------------------------------------------------- op lists (one r_exec site)
// A fixed sequence of Fp12 / G2 / Miller-step operations as a table of (kind, dst, a, b) words
// built at compile time (constexpr), run by r_run: one loop with the interpreter inlined once, so
// the final exponentiation's ~360 programs, a Miller loop's 68 steps and the cofactor clearing's
// ~140 point operations pay no call overhead per program.
enum {
  RK_MUL,    // dst = a b (Fp12)
  RK_SQR,    // dst = a^2
  RK_CSQR,   // dst = a^2, a cyclotomic
  RK_CSQR2,  // dst = a^4, a cyclotomic (CSQR12X2)
  RK_FROB,   // dst = a^p
  RK_FROB2,  // dst = a^(p^2)
  RK_G2DBL,  // dst = 2a (6-slot Jacobian G2)
  RK_G2DBL2, // dst = 4a
  RK_G2DBL4, // dst = 16a
  RK_G2ADD,  // dst = a + b (no exceptional cases)
  RK_PSI,    // dst = psi(a)
  RK_PSI2,   // dst = psi^2(a)
  RK_MLDBL,  // Miller doubling step: f = dst (12), T at LBR_PT + 6, P at LBR_PT
  RK_MLADD,  // Miller addition step: the same with Q at LBR_PT + 2
  RK_CONJ,   // dst = conj(a) (Fp12)
  RK_COPY,   // dst[0, b) = a[0, b)
  RK_G2NEG,  // a = -a (G2)
  // round 6: homogeneous projective G2 with the complete formulas (gen_row_programs.py g2_pdbl /
  // g2_padd: 2 product levels per doubling and per addition, no exceptional cases)
  RK_PDBL,   // dst = 2a
  RK_PDBL2,  // dst = 4a
  RK_PDBL4,  // dst = 16a
  RK_PADD,   // dst = a + b (complete)
};
#define LBR_MAX_OPS 400
struct r_opl {
  int n = 0;
  int w[2 * LBR_MAX_OPS] = {};
  constexpr void op(int kind, int dst, int a, int b = 0) {
    w[2 * n] = kind | (dst << 16);
    w[2 * n + 1] = a | (b << 16);
    n++;
  }
  // dst = a^|x| (a cyclotomic, dst != a)
  constexpr void csqrs(int dst, int run) {  // run chained squarings, two per program
    // (4 or 8 chained squarings in one program measured 8 / 21 phases in the generator: the
    // operand sums outgrow the flattening bound; two per program, 3 phases, stays the best)
    for (; run >= 2; run -= 2) op(RK_CSQR2, dst, dst);
    if (run) op(RK_CSQR, dst, dst);
  }
  constexpr void pow_xabs(int dst, int a) {
    op(RK_COPY, dst, a, 12);
    int run = 0;  // squarings pending
    for (int i = 62; i >= 0; i--) {
      run++;
      if ((LB_X_ABS >> i) & 1ull) {
        csqrs(dst, run);
        run = 0;
        op(RK_MUL, dst, dst, a);
      }
    }
    csqrs(dst, run);
  }
  // dst = [|x|] a (G2, dst != a)
  constexpr void g2_dbls(int dst, int run) {
    for (; run >= 4; run -= 4) op(RK_G2DBL4, dst, dst);
    for (; run >= 2; run -= 2) op(RK_G2DBL2, dst, dst);
    if (run) op(RK_G2DBL, dst, dst);
  }
  constexpr void g2_mul_xabs(int dst, int a) {
    op(RK_COPY, dst, a, 6);
    int run = 0;  // doublings pending (issued four / two at a time)
    for (int i = 62; i >= 0; i--) {
      run++;
      if ((LB_X_ABS >> i) & 1ull) {
        g2_dbls(dst, run);
        run = 0;
        op(RK_G2ADD, dst, dst, a);
      }
    }
    g2_dbls(dst, run);
  }
  // the same in projective coordinates (complete additions)
  constexpr void p_dbls(int dst, int run) {
    for (; run >= 4; run -= 4) op(RK_PDBL4, dst, dst);
    for (; run >= 2; run -= 2) op(RK_PDBL2, dst, dst);
    if (run) op(RK_PDBL, dst, dst);
  }
  constexpr void p_mul_xabs(int dst, int a) {
    op(RK_COPY, dst, a, 6);
    int run = 0;
    for (int i = 62; i >= 0; i--) {
      run++;
      if ((LB_X_ABS >> i) & 1ull) {
        p_dbls(dst, run);
        run = 0;
        op(RK_PADD, dst, dst, a);
      }
    }
    p_dbls(dst, run);
  }
};
// r_final_exp after the inversion (Y0 = f^-1): the chain of lb_pairing.h final_exponentiation
constexpr r_opl r_ops_fe_tail(int dst, int f) {
  r_opl o;
  const int T0 = LBR_A(1), A0 = LBR_A(2), B0 = LBR_A(3), C0 = LBR_A(4), X0 = LBR_A(5), Y0 = LBR_A(6);
  o.op(RK_CONJ, X0, f);
  o.op(RK_MUL, T0, X0, Y0);
  o.op(RK_FROB2, X0, T0);
  o.op(RK_MUL, T0, X0, T0);
  o.pow_xabs(X0, T0);
  o.op(RK_MUL, X0, X0, T0);
  o.op(RK_CONJ, A0, X0);
  o.pow_xabs(X0, A0);
  o.op(RK_MUL, X0, X0, A0);
  o.op(RK_CONJ, A0, X0);
  o.pow_xabs(X0, A0);
  o.op(RK_CONJ, X0, X0);
  o.op(RK_FROB, Y0, A0);
  o.op(RK_MUL, B0, X0, Y0);
  o.pow_xabs(X0, B0);
  o.pow_xabs(C0, X0);
  o.op(RK_FROB2, X0, B0);
  o.op(RK_MUL, C0, C0, X0);
  o.op(RK_CONJ, X0, B0);
  o.op(RK_MUL, C0, C0, X0);
  o.op(RK_CSQR, X0, T0);
  o.op(RK_MUL, X0, X0, T0);
  o.op(RK_MUL, dst, C0, X0);
  return o;
}
// the Miller loop's steps into area dst (after r_miller's setup, before its final conjugation)
constexpr r_opl r_ops_miller(int dst) {
  r_opl o;
  for (int i = 62; i >= 0; i--) {
    o.op(RK_MLDBL, dst, 0);
    if ((LB_X_ABS >> i) & 1ull) o.op(RK_MLADD, dst, 0);
  }
  return o;
}
// Q0 + Q1 (slots q .. q + 11), then h_eff (Q0 + Q1) via psi into dst (as r_g2_clear_cofactor<true>)
constexpr r_opl r_ops_hash_finish(int dst, int q) {
  r_opl o;
  const int T1 = LBR_A(0), T3 = LBR_A(0) + 6, T2 = LBR_A(1), X = LBR_A(1) + 6, W = LBR_A(2);
  const int p = q;
  o.op(RK_G2ADD, p, q, q + 6);
  o.g2_mul_xabs(T1, p);
  o.op(RK_G2NEG, T1, T1);
  o.op(RK_G2DBL, T3, p);
  o.op(RK_PSI2, T3, T3);
  o.op(RK_PSI, T2, p);
  o.op(RK_COPY, W, T2, 6);
  o.op(RK_G2NEG, W, W);
  o.op(RK_G2ADD, T3, T3, W);
  o.op(RK_G2ADD, T2, T2, T1);
  o.g2_mul_xabs(X, T2);
  o.op(RK_G2NEG, X, X);
  o.op(RK_G2ADD, T3, T3, X);
  o.op(RK_G2NEG, T1, T1);
  o.op(RK_G2ADD, T3, T3, T1);
  o.op(RK_COPY, W, p, 6);
  o.op(RK_G2NEG, W, W);
  o.op(RK_G2ADD, dst, T3, W);
  return o;
}
// the same chain in projective coordinates with the complete additions (k_hash_finish_row's
// default since round 6; q .. q + 11 projective): no exceptional case, so no rerun
constexpr r_opl r_ops_hash_finish_p(int dst, int q) {
  r_opl o;
  const int T1 = LBR_A(0), T3 = LBR_A(0) + 6, T2 = LBR_A(1), X = LBR_A(1) + 6, W = LBR_A(2);
  const int p = q;
  o.op(RK_PADD, p, q, q + 6);
  o.p_mul_xabs(T1, p);
  o.op(RK_G2NEG, T1, T1);
  o.op(RK_PDBL, T3, p);
  o.op(RK_PSI2, T3, T3);
  o.op(RK_PSI, T2, p);
  o.op(RK_COPY, W, T2, 6);
  o.op(RK_G2NEG, W, W);
  o.op(RK_PADD, T3, T3, W);
  o.op(RK_PADD, T2, T2, T1);
  o.p_mul_xabs(X, T2);
  o.op(RK_G2NEG, X, X);
  o.op(RK_PADD, T3, T3, X);
  o.op(RK_G2NEG, T1, T1);
  o.op(RK_PADD, T3, T3, T1);
  o.op(RK_COPY, W, p, 6);
  o.op(RK_G2NEG, W, W);
  o.op(RK_PADD, dst, T3, W);
  return o;
}
constexpr r_opl r_ops_xladder_p(int dst, int p) {
  r_opl o;
  o.p_mul_xabs(dst, p);
  return o;
}
static __device__ const r_opl LBR_OPS_HASH_P = r_ops_hash_finish_p(LBR_A(4), LBR_A(3));
static __device__ const r_opl LBR_OPS_XLADDER_P = r_ops_xladder_p(LBR_A(4), LBR_A(3));
static __device__ const r_opl LBR_OPS_FE_A0 = r_ops_fe_tail(LBR_A(0), LBR_A(0));
static __device__ const r_opl LBR_OPS_ML_A0 = r_ops_miller(LBR_A(0));
static __device__ const r_opl LBR_OPS_ML_A7 = r_ops_miller(LBR_A(7));
static __device__ const r_opl LBR_OPS_HASH = r_ops_hash_finish(LBR_A(4), LBR_A(3));
// [|x|] p for the signature subgroup check (k_sig_subgroup_row): A(4) = [|x|] A(3), fast additions
constexpr r_opl r_ops_xladder(int dst, int p) {
  r_opl o;
  o.g2_mul_xabs(dst, p);
  return o;
}
static __device__ const r_opl LBR_OPS_XLADDER = r_ops_xladder(LBR_A(4), LBR_A(3));
static_assert(r_ops_fe_tail(LBR_A(0), LBR_A(0)).n <= LBR_MAX_OPS && r_ops_hash_finish(LBR_A(4), LBR_A(3)).n <= LBR_MAX_OPS,
              "lb_row.h: op list size");

// ---------------------------------------------------------------- compiled programs
// The Miller loop's step programs (DBL_STEP, ADD_STEP) run by a fixed-phase executor instead of
// the interpreter: each phase's kind, flags and term counts are compile-time constants
// (tools/gen_row_compiled.py -> lb_row_compiled.h), so a phase is straight-line code; a row reads
// its own record (dst, operand pairs) from a per-row table; the program's input slots (IN) are
// mapped to the operation's sources instead of copied in (one copy phase and barrier fewer).
#ifndef LBR_ML_COMPILED
#define LBR_ML_COMPILED 1
#endif
struct rc_dbl_step {
  static constexpr int NPH = LBC_DBL_STEP_NPH, RS = LBC_DBL_STEP_RS, NOUT = LBC_DBL_STEP_NOUT;
  static constexpr int ph(int p, int f) { return LBC_DBL_STEP_PH[p][f]; }
  __device__ static const int32_t* rec(int p, int row) { return &LBC_DBL_STEP_REC[p][row][0]; }
  __device__ static int out(int e) { return LBC_DBL_STEP_OUT[e]; }
};
struct rc_add_step {
  static constexpr int NPH = LBC_ADD_STEP_NPH, RS = LBC_ADD_STEP_RS, NOUT = LBC_ADD_STEP_NOUT;
  static constexpr int ph(int p, int f) { return LBC_ADD_STEP_PH[p][f]; }
  __device__ static const int32_t* rec(int p, int row) { return &LBC_ADD_STEP_REC[p][row][0]; }
  __device__ static int out(int e) { return LBC_ADD_STEP_OUT[e]; }
};
template <int N, class M>
__device__ __forceinline__ int64_t rc_acc(const lds_i32* S, const int* w, int k, M map) {
  int64_t acc = 0;
  LB_UNROLL for (int j = 0; j < N; j++) acc += (int64_t)(w[j] >> 16) * S[16 * map(w[j] & 0xffff) + k];
  return acc;
}
template <class P, int I>
struct rc_w {
  static constexpr int n = 1 + P::ph(I, 3) + P::ph(I, 4);  // record words of phase I
};
template <class P, int I>
__device__ __forceinline__ void rc_load(int row, int (&w)[rc_w<P, I>::n]) {
  const int32_t* rec = P::rec(I, row);
  LB_UNROLL for (int j = 0; j < rc_w<P, I>::n; j++) w[j] = rec[j];
}
// phase I with its record already in registers; phase I + 1's record is loaded before this
// phase's operand reads (software pipelining: the table read overlaps the phase's work)
template <class P, int I, class M>
__device__ __forceinline__ void rc_phases(lds_i32* S, int k, int row, int pk, M map, const int (&w)[rc_w<P, I>::n]) {
  constexpr int kind = P::ph(I, 0), flags = P::ph(I, 1), nx = P::ph(I, 3), ny = P::ph(I, 4), bar = P::ph(I, 5);
  constexpr int IN = I + 1 < P::NPH ? I + 1 : I;
  int wn[rc_w<P, IN>::n];
  if constexpr (I + 1 < P::NPH) rc_load<P, IN>(row, wn);
  const int dst = w[0];
  if (dst >= 0) {  // uniform within the row
    if constexpr (kind == 0) {
      int xv, yv;
      if constexpr ((flags & 1) != 0) xv = S[16 * map(w[1] & 0xffff) + k];
      else {
        const int64_t a = rc_acc<nx>(S, w + 1, k, map);
        xv = (flags & 4) ? r_reduce(a, k, pk) : r_norm<true>(a, k);
      }
      if constexpr ((flags & 2) != 0) yv = S[16 * map(w[1 + nx] & 0xffff) + k];
      else {
        const int64_t a = rc_acc<ny>(S, w + 1 + nx, k, map);
        yv = (flags & 8) ? r_reduce(a, k, pk) : r_norm<true>(a, k);
      }
      int xr[14];
      r_rep(xv, xr);
      S[16 * dst + k] = rp_mul(xr, yv, k);
    } else {
      S[16 * dst + k] = r_reduce(rc_acc<nx>(S, w + 1, k, map), k, pk);
    }
  }
  if constexpr (bar != 0) r_sync();
  if constexpr (I + 1 < P::NPH) rc_phases<P, I + 1>(S, k, row, pk, map, wn);
}
// a Miller step on the areas of r_run: f at `f` (12 slots), T at tt (6), P at pp (2), Q at qq (4,
// ADD_STEP); outputs f <- f^2 l (or f l), T <- 2T (or T + Q)
template <class P>
__device__ __forceinline__ void rc_miller_step(int32_t* S_generic, int f, int tt, int pp, int qq, bool add) {
  lds_i32* S = r_lds(S_generic);
  const int k = r_limb(), row = r_row(), pk = r_plimb(k);
  auto map = [&](int s) -> int {
    if (s >= 24) return s;  // (LBR_IN = 0: the program's inputs are slots 0 .. 23)
    if (s < 12) return f + s;
    if (s < 18) return tt + s - 12;
    if (!add) return pp + s - 18;
    return s < 22 ? qq + s - 18 : pp + s - 22;
  };
  int w0[rc_w<P, 0>::n];
  rc_load<P, 0>(row, w0);
  rc_phases<P, 0>(S, k, row, pk, map, w0);
  for (int e = row; e < P::NOUT; e += LBR_NROWS) {
    const int d = e < 12 ? f + e : tt + e - 12;
    S[16 * d + k] = S[16 * P::out(e) + k];
  }
  r_sync();
}

// run ops[0, n): every program through one inlined interpreter
__device__ __attribute__((noinline)) void r_run(int32_t* S_generic, const r_opl* ops, int n) {
  lds_i32* S = r_lds(S_generic);
  const int k = r_limb(), row = r_row(), t = r_tid();
  const int PP = LBR_PT, QQ = LBR_PT + 2, TT = LBR_PT + 6;
  for (int i = 0; i < n; i++) {
    const int w0 = __builtin_amdgcn_readfirstlane(ops->w[2 * i]), w1 = __builtin_amdgcn_readfirstlane(ops->w[2 * i + 1]);
    const int kind = w0 & 0xffff, dst = w0 >> 16, a = w1 & 0xffff, b = w1 >> 16;
    if (kind == RK_CONJ) {
      r_conj(S_generic, dst, a);
      continue;
    }
    if (kind == RK_COPY) {
      r_copy(S_generic, dst, a, b);
      continue;
    }
    if (LBR_PDBL_FAST && (kind == RK_PDBL || kind == RK_PDBL2 || kind == RK_PDBL4)) {
      const int nd = kind == RK_PDBL ? 1 : (kind == RK_PDBL2 ? 2 : 4);
      r_pdbl_fast(S_generic, dst, a);
      for (int q = 1; q < nd; q++) r_pdbl_fast(S_generic, dst, dst);
      continue;
    }
    if (LBR_MUL12_FAST && kind == RK_MUL) {
      r_mul12_fast(S_generic, dst, a, b);
      continue;
    }
    if (LBR_CSQR_FAST && (kind == RK_CSQR || kind == RK_CSQR2)) {
      r_csqr_fast(S_generic, dst, a);
      if (kind == RK_CSQR2) r_csqr_fast(S_generic, dst, dst);
      continue;
    }
    if (kind == RK_G2NEG) {  // in place (dst == a)
      if (t < 32) S[16 * (a + 2) + t] = -S[16 * (a + 2) + t];
      r_sync();
      continue;
    }
    int prog, na, nb, nout;
    switch (kind) {
      case RK_MUL: prog = LBR_MUL12; na = 12; nb = 12; nout = 12; break;
      case RK_SQR: prog = LBR_SQR12; na = 12; nb = 0; nout = 12; break;
      case RK_CSQR: prog = LBR_CSQR12; na = 12; nb = 0; nout = 12; break;
      case RK_CSQR2: prog = LBR_CSQR12X2; na = 12; nb = 0; nout = 12; break;
      case RK_FROB: prog = LBR_FROB; na = 12; nb = 0; nout = 12; break;
      case RK_FROB2: prog = LBR_FROB2; na = 12; nb = 0; nout = 12; break;
      case RK_G2DBL: prog = LBR_G2DBL; na = 6; nb = 0; nout = 6; break;
      case RK_G2DBL2: prog = LBR_G2DBL2; na = 6; nb = 0; nout = 6; break;
      case RK_G2DBL4: prog = LBR_G2DBL4; na = 6; nb = 0; nout = 6; break;
      case RK_G2ADD: prog = LBR_G2ADD; na = 6; nb = 6; nout = 6; break;
      case RK_PSI: prog = LBR_PSI; na = 6; nb = 0; nout = 6; break;
      case RK_PSI2: prog = LBR_PSI2; na = 6; nb = 0; nout = 6; break;
      case RK_PDBL: prog = LBR_PDBL1; na = 6; nb = 0; nout = 6; break;
      case RK_PDBL2: prog = LBR_PDBL2; na = 6; nb = 0; nout = 6; break;
      case RK_PDBL4: prog = LBR_PDBL4; na = 6; nb = 0; nout = 6; break;
      case RK_PADD: prog = LBR_PADD; na = 6; nb = 6; nout = 6; break;
      case RK_MLDBL: prog = LBR_DBL_STEP; na = 12; nb = 0; nout = 18; break;
      default: prog = LBR_ADD_STEP; na = 12; nb = 0; nout = 18; break;  // RK_MLADD
    }
    const bool ml = kind == RK_MLDBL || kind == RK_MLADD;
    const int src_a = ml ? dst : a;
    // inputs into IN (sources never in IN: one barrier)
    const int nin = ml ? (kind == RK_MLDBL ? 20 : 24) : na + nb;
    for (int e = row; e < nin; e += LBR_NROWS) {
      int sl;
      if (e < na) sl = src_a + e;
      else if (!ml) sl = b + e - na;
      else if (e < 18) sl = TT + e - 12;
      else if (kind == RK_MLDBL) sl = PP + e - 18;
      else sl = e < 22 ? QQ + e - 18 : PP + e - 22;
      S[16 * (LBR_IN + e) + k] = S[16 * sl + k];
    }
    r_sync();
    r_exec_inl(S_generic, prog);
    // outputs (temps) to dst (and T for the Miller steps)
    const lds_i32* pr = r_progs(S_generic) + prog;
    for (int e = row; e < nout; e += LBR_NROWS) {
      const int d = e < 12 || !ml ? dst + e : TT + e - 12;
      S[16 * d + k] = S[16 * pr[2 + e] + k];
    }
    r_sync();
  }
}

// the Miller loop's op list (only RK_MLDBL / RK_MLADD) on the compiled steps; a separate function
// so the other op lists' interpreter (r_run) keeps its code size
__device__ __attribute__((noinline)) void r_run_ml(int32_t* S_generic, const r_opl* ops, int n) {
  const int PP = LBR_PT, QQ = LBR_PT + 2, TT = LBR_PT + 6;
  for (int i = 0; i < n; i++) {
    const int w0 = __builtin_amdgcn_readfirstlane(ops->w[2 * i]);
    const int kind = w0 & 0xffff, dst = w0 >> 16;
    if (kind == RK_MLDBL) rc_miller_step<rc_dbl_step>(S_generic, dst, TT, PP, QQ, false);
    else rc_miller_step<rc_add_step>(S_generic, dst, TT, PP, QQ, true);
  }
}

// dst = a^-1 by norms down to Fp2 (lb_wave.h w_inv): one Fp inversion on thread 0 (inline EEA)
__device__ void r_inv(int32_t* S, int dst, int a, int t1, int t2, int t3) {
  __shared__ fp nv[2];
  r_conj(S, t1, a);     // X
  r_mul(S, t2, a, t1);  // t
  r_frob2(S, t3, t2);   // t^(p^2)
  r_frob2(S, dst, t3);  // t^(p^4)
  r_mul(S, t3, t3, dst);  // u
  r_mul(S, t2, t2, t3);   // n = t u (slots 0, 1)
  r_export(S, t2, 2);
  if (r_tid() == 0) {
    const fp n0 = r_fp_of_staged(S, 0), n1 = r_fp_of_staged(S, 1);
    const fp ni = fp_inv_i(fp_add(fp_sqr(n0), fp_sqr(n1)));
    nv[0] = fp_mul(n0, ni);
    nv[1] = fp_neg(fp_mul(n1, ni));
  }
  r_sync();
  r_import_fps(S, t2, nv, 2);  // slots 2..11 of t2 are zero (n lies in Fp2)
  r_mul(S, t3, t3, t2);  // t^-1
  r_mul(S, dst, t1, t3);
}
// dst = a^|x| for a in the cyclotomic subgroup (a must not alias dst)
__device__ void r_pow_xabs(int32_t* S, int dst, int a) {
  r_copy(S, dst, a, 12);
  for (int i = 62; i >= 0; i--) {
    r_csqr(S, dst, dst);
    if ((LB_X_ABS >> i) & 1ull) r_mul(S, dst, dst, a);
  }
}
// f^(3 (p^12 - 1) / r), the chain of lb_pairing.h final_exponentiation (areas 1..6); after the
// easy part every value lies in the cyclotomic subgroup, so the squarings are r_csqr
__device__ void r_final_exp(int32_t* S, int dst, int f) {
  const int T0 = LBR_A(1), A0 = LBR_A(2), B0 = LBR_A(3), C0 = LBR_A(4), X0 = LBR_A(5), Y0 = LBR_A(6);
  r_inv(S, Y0, f, A0, B0, C0);
#ifndef LBR_NO_OPLIST
  if (dst == LBR_A(0) && f == LBR_A(0)) {
    r_run(S, &LBR_OPS_FE_A0, LBR_OPS_FE_A0.n);
    return;
  }
#endif
  r_conj(S, X0, f);
  r_mul(S, T0, X0, Y0);
  r_frob2(S, X0, T0);
  r_mul(S, T0, X0, T0);
  r_pow_xabs(S, X0, T0);
  r_mul(S, X0, X0, T0);
  r_conj(S, A0, X0);
  r_pow_xabs(S, X0, A0);
  r_mul(S, X0, X0, A0);
  r_conj(S, A0, X0);
  r_pow_xabs(S, X0, A0);
  r_conj(S, X0, X0);
  r_frob(S, Y0, A0);
  r_mul(S, B0, X0, Y0);
  r_pow_xabs(S, X0, B0);
  r_pow_xabs(S, C0, X0);
  r_frob2(S, X0, B0);
  r_mul(S, C0, C0, X0);
  r_conj(S, X0, B0);
  r_mul(S, C0, C0, X0);
  r_csqr(S, X0, T0);
  r_mul(S, X0, X0, T0);
  r_mul(S, dst, C0, X0);
}
// Miller loop f_{|x|,Q}(P), conjugated, into area dst; P at LBR_PT (xP, yP), Q at LBR_PT + 2
// (xq.c0, xq.c1, yq.c0, yq.c1); T at LBR_PT + 6..11.  Same steps as lb_wave.h w_miller.
__device__ void r_miller(int32_t* S_generic, int dst) {
  lds_i32* S = r_lds(S_generic);
  const int PP = LBR_PT, QQ = LBR_PT + 2, TT = LBR_PT + 6;
  r_set_one(S_generic, dst);
  {
    const int t = r_tid();
    if (t < 6 * 16) {
      const int e = t >> 4, k = t & 15;
      int v;
      if (e < 4) v = S[16 * (QQ + e) + k];
      else if (e == 4) {
        v = 0;
        LB_UNROLL for (int i = 0; i < 14; i++) v = k == i ? lbr_k::ONE[i] : v;
      } else v = 0;
      S[16 * (TT + e) + k] = v;
    }
    r_sync();
  }
#ifndef LBR_NO_OPLIST
  if (dst == LBR_A(0) || dst == LBR_A(7)) {
    if (LBR_ML_COMPILED) r_run_ml(S_generic, dst == LBR_A(0) ? &LBR_OPS_ML_A0 : &LBR_OPS_ML_A7, LBR_OPS_ML_A0.n);
    else r_run(S_generic, dst == LBR_A(0) ? &LBR_OPS_ML_A0 : &LBR_OPS_ML_A7, LBR_OPS_ML_A0.n);
    r_conj(S_generic, dst, dst);
    return;
  }
#endif
  for (int i = 62; i >= 0; i--) {
    r_gather(S_generic, LBR_IN, 20, [&](int e) { return e < 12 ? dst + e : (e < 18 ? TT + e - 12 : PP + e - 18); });
    r_exec(S_generic, LBR_DBL_STEP);
    r_out(S_generic, LBR_DBL_STEP, 0, 12, dst);
    r_out(S_generic, LBR_DBL_STEP, 12, 6, TT);
    if ((LB_X_ABS >> i) & 1ull) {
      r_gather(S_generic, LBR_IN, 24, [&](int e) {
        return e < 12 ? dst + e : (e < 18 ? TT + e - 12 : (e < 22 ? QQ + e - 18 : PP + e - 22));
      });
      r_exec(S_generic, LBR_ADD_STEP);
      r_out(S_generic, LBR_ADD_STEP, 0, 12, dst);
      r_out(S_generic, LBR_ADD_STEP, 12, 6, TT);
    }
  }
  r_conj(S_generic, dst, dst);
}

// ---------------------------------------------------------------- G2 points (6 slots: X, Y, Z in Fp2)
// hash_to_G2's cofactor clearing on rows (k_hash_finish_row): the chain of lb_group.h
// g8_clear_cofactor_st with every doubling / addition one row program (G2DBL: 16 products in 3
// levels, G2ADD: 43 products; tools/gen_row_programs.py g2_dbl / g2_add).  Infinity is a zero Z
// (a doubling keeps it); each addition tests its operands' Z and its H and r (canonical values,
// one lane per slot) for the exceptional cases, as jac_add_i / g8_add do.
// bit e of the result: slot src(e) is 0 mod p (e < n <= 16)
template <class F>
__device__ uint32_t r_zero_mask(int32_t* S_generic, int n, F src) {
  lds_i32* S = r_lds(S_generic);
  const int t = r_tid();
  if (t == 0) S[LBR_SLOT_WORDS + 2] = 0;
  r_sync();
  if (t < n) {
    int32_t l[14];
    const int s = src(t);
    LB_UNROLL for (int k = 0; k < 14; k++) l[k] = S[16 * s + k];
    if (fp_is_zero(r_canon(l))) atomicOr((int*)&S_generic[LBR_SLOT_WORDS + 2], 1 << t);
  }
  r_sync();
  const uint32_t m = (uint32_t)S[LBR_SLOT_WORDS + 2];
  r_sync();
  return m;
}
// program outputs (temps) to disjoint slots
__device__ __forceinline__ void r_out_dj(int32_t* S, int off, int first, int n, int dst) {
  const lds_i32* prog = r_progs(S) + off;
  r_gather_dj(S, dst, n, [&](int e) { return prog[2 + first + e]; });
}
__device__ void r_g2_dbl(int32_t* S, int dst, int a) {
  r_copy(S, LBR_IN, a, 6);
  r_exec(S, LBR_G2DBL);
  r_out(S, LBR_G2DBL, 0, 6, dst);
}
// a 6-slot G2 program: dst = prog(a) or prog(a, b) (b: a second 6-slot input, -1 for none)
__device__ void r_g2_prog(int32_t* S, int prog, int dst, int a, int b = -1) {
  r_gather(S, LBR_IN, b < 0 ? 6 : 12, [&](int e) { return e < 6 ? a + e : b + e - 6; });
  r_exec(S, prog);
  r_out(S, prog, 0, 6, dst);
}
__device__ void r_g2_psi(int32_t* S, int dst, int a) {
  r_copy(S, LBR_IN, a, 6);
  r_exec(S, LBR_PSI);
  r_out(S, LBR_PSI, 0, 6, dst);
}
__device__ void r_g2_psi2(int32_t* S, int dst, int a) {
  r_copy(S, LBR_IN, a, 6);
  r_exec(S, LBR_PSI2);
  r_out(S, LBR_PSI2, 0, 6, dst);
}
// a = -a (Y negated limb-wise, as r_conj)
__device__ void r_g2_neg(int32_t* S_generic, int a) {
  lds_i32* S = r_lds(S_generic);
  const int t = r_tid();
  if (t < 32) S[16 * (a + 2) + t] = -S[16 * (a + 2) + t];
  r_sync();
}
// dst = a + b (dst may alias a or b)
__device__ void r_g2_add(int32_t* S_generic, int dst, int a, int b) {
  r_gather(S_generic, LBR_IN, 12, [&](int e) { return e < 6 ? a + e : b + e - 6; });
  r_exec(S_generic, LBR_G2ADD);
  const lds_i32* prog = r_progs(S_generic) + LBR_G2ADD;
  // bits 0-1: a's Z, 2-3: b's Z, 4-5: H, 6-7: r (G2ADD's outputs 6..9)
  const uint32_t m = r_zero_mask(S_generic, 8, [&](int e) { return e < 2 ? a + 4 + e : (e < 4 ? b + 2 + e : prog[4 + e]); });
  if ((m & 0xc) == 0xc) {  // b = O
    if (dst != a) r_copy(S_generic, dst, a, 6);
  } else if ((m & 0x3) == 0x3) {  // a = O
    if (dst != b) r_copy(S_generic, dst, b, 6);
  } else if ((m & 0x30) == 0x30) {  // a = +-b
    if ((m & 0xc0) == 0xc0) r_g2_dbl(S_generic, dst, a);
    else r_gather(S_generic, dst, 6, [&](int) { return LBR_CONST + LBR_C_ZERO; });
  } else {
    r_out(S_generic, LBR_G2ADD, 0, 6, dst);
  }
}
// dst = [|x|] a (dst must not alias a).  FAST: the accumulator stays in IN (slots 0..5, the base
// in 6..11), each step one program and one move of its outputs back into IN; additions without
// the exceptional-case tests (see r_g2_clear_cofactor).
template <bool FAST>
__device__ void r_g2_mul_xabs(int32_t* S, int dst, int a) {
  if (FAST) {
    r_gather_dj(S, LBR_IN, 12, [&](int e) { return a + (e < 6 ? e : e - 6); });
    for (int i = 62; i >= 0; i--) {
      r_exec(S, LBR_G2DBL);
      r_out_dj(S, LBR_G2DBL, 0, 6, LBR_IN);
      if ((LB_X_ABS >> i) & 1ull) {
        r_exec(S, LBR_G2ADD);
        r_out_dj(S, LBR_G2ADD, 0, 6, LBR_IN);
      }
    }
    r_gather_dj(S, dst, 6, [&](int e) { return LBR_IN + e; });
    return;
  }
  r_copy(S, dst, a, 6);
  for (int i = 62; i >= 0; i--) {
    r_g2_dbl(S, dst, dst);
    if ((LB_X_ABS >> i) & 1ull) r_g2_add(S, dst, dst, a);
  }
}
// dst = a + b without the exceptional cases (dst may alias a or b)
__device__ void r_g2_add_fast(int32_t* S, int dst, int a, int b) {
  r_gather_dj(S, LBR_IN, 12, [&](int e) { return e < 6 ? a + e : b + e - 6; });
  r_exec(S, LBR_G2ADD);
  r_out_dj(S, LBR_G2ADD, 0, 6, dst);
}
// h_eff p via psi (as g8_clear_cofactor_st) for p in slots p .. p + 5; result in dst.  Uses
// areas 0..2 besides.  FAST: no exceptional-case tests.  Every exceptional case of the
// formulas (an operand at infinity, P = +-Q in an addition, a doubling of a point of order 2)
// yields Z = 0, and a zero Z stays zero through every later doubling, addition, psi and psi^2:
// a FAST result with Z != 0 is exact; Z = 0 (negligible probability for hash outputs) is
// recomputed with the tests (k_hash_finish_row).
template <bool FAST>
__device__ void r_g2_clear_cofactor(int32_t* S, int dst, int p) {
  const int T1 = LBR_A(0), T3 = LBR_A(0) + 6, T2 = LBR_A(1), X = LBR_A(1) + 6, W = LBR_A(2);
  auto add = [&](int d, int a, int b) {
    if (FAST) r_g2_add_fast(S, d, a, b);
    else r_g2_add(S, d, a, b);
  };
  r_g2_mul_xabs<FAST>(S, T1, p);
  r_g2_neg(S, T1);  // t1 = [x] p
  r_g2_dbl(S, T3, p);
  r_g2_psi2(S, T3, T3);
  r_g2_psi(S, T2, p);
  r_copy(S, W, T2, 6);
  r_g2_neg(S, W);
  add(T3, T3, W);  // psi^2(2p) - psi(p)
  add(T2, T2, T1);  // psi(p) + t1
  r_g2_mul_xabs<FAST>(S, X, T2);
  r_g2_neg(S, X);  // [x](t1 + t2)
  add(T3, T3, X);
  r_g2_neg(S, T1);
  add(T3, T3, T1);
  r_copy(S, W, p, 6);
  r_g2_neg(S, W);
  add(dst, T3, W);
}
