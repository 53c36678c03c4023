// Row engine vs wave engine latencies (tools/, not product code): cycles (s_memtime at 100 MHz
// -> converted by the host with the shader clock it measures with s_memrealtime? no: wall ns
// from clock64 deltas of the realtime counter) per operation of one workgroup.
//   tools/ubench/row_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#define LB_KGROUP 99
__device__ unsigned long long g_ph[64][3];
__device__ int g_ph_n;
#ifdef UB_HOOKS
#define LBR_PHASE_HOOK(ph, kind, n)                                  \
  if (threadIdx.x == 0 && g_ph_n < 64) {                             \
    g_ph[g_ph_n][0] = __builtin_readcyclecounter();                  \
    g_ph[g_ph_n][1] = kind;                                          \
    g_ph[g_ph_n][2] = n;                                             \
    g_ph_n++;                                                        \
  }
// sub-phase points of the first product of a phase (thread 0), after the value v is ready
#define LBR_SUB_HOOK(tag, v)                                                        \
  if (threadIdx.x == 0 && g_ph_n < 64) {                                             \
    asm volatile("" ::"v"(v));                                                       \
    __builtin_amdgcn_s_waitcnt(0);                                                   \
    g_ph[g_ph_n][0] = __builtin_readcyclecounter();                                  \
    g_ph[g_ph_n][1] = 10 + (tag);                                                    \
    g_ph[g_ph_n][2] = 0;                                                             \
    g_ph_n++;                                                                        \
  }
#endif
#ifdef UB_TL
// a timeline of r_exec_inl (lb_row.h LBR_TL points): thread 0 of each wave adds the s_memtime
// delta since the previous point to its wave's LDS slot (no global memory inside the loop)
static __shared__ unsigned long long g_tl[16][8];
static __shared__ unsigned long long g_tl_prev[16];
#define LBR_TL(i)                                                    \
  if ((threadIdx.x & 63) == 0) {                                    \
    const unsigned long long now = __builtin_amdgcn_s_memtime();    \
    g_tl[threadIdx.x >> 6][i] += now - g_tl_prev[threadIdx.x >> 6]; \
    g_tl_prev[threadIdx.x >> 6] = now;                              \
  }
__device__ unsigned long long g_tl_out[16][8];
#endif
#include "lb_kernels.h"

__device__ __forceinline__ uint64_t rt() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz

// one row: a chain of rp_mul
__global__ void __launch_bounds__(64) k_rp_chain(int iters, uint64_t* out, int* sink) {
  const int k = threadIdx.x & 15;
  int y = k < 13 ? (k * 12345 + 7) & LBR_M28 : (k == 13 ? 1000 : 0);
  int x[14];
  for (int i = 0; i < 14; i++) x[i] = (i * 777 + 3) & LBR_M28;
  const uint64_t t0 = rt();
  for (int it = 0; it < iters; it++) {
    y = rp_mul(x, y, k);
    x[it % 14] ^= y & 1;  // keep x live / varying
  }
  const uint64_t t1 = rt();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[threadIdx.x] = y;
}
template <int OP>
__global__ void __launch_bounds__(LBR_NT) k_row_ops(int iters, uint64_t* out) {
  LBR_SHARED(S);
  r_init(S);
  r_set_one(S, LBR_A(0));
  r_set_one(S, LBR_A(1));
  r_sync();
  const uint64_t t0 = rt();
  for (int it = 0; it < iters; it++) {
    if (OP == 0) r_sqr(S, LBR_A(0), LBR_A(0));
    if (OP == 1) r_mul(S, LBR_A(0), LBR_A(0), LBR_A(1));
    if (OP == 2) r_copy(S, LBR_IN, LBR_A(0), 12);
    if (OP == 3) r_exec(S, LBR_SQR12);
    if (OP == 4) r_csqr(S, LBR_A(0), LBR_A(0));
    if (OP == 5) r_final_exp(S, LBR_A(0), LBR_A(0));
    if (OP == 6) r_inv(S, LBR_A(2), LBR_A(0), LBR_A(3), LBR_A(4), LBR_A(5));
    if (OP == 7) r_pow_xabs(S, LBR_A(2), LBR_A(0));
  }
  r_sync();
  const uint64_t t1 = rt();
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
// G2 point ops on (1, 1, 1)-filled slots (any values: timing only)
__device__ void ub_fill_ones(int32_t* S, int dst, int n) {
  const int t = r_tid();
  if (t < 16 * n) {
    int v = 0;
    for (int i = 0; i < 14; i++) v = (t & 15) == i ? lbr_k::ONE[i] : v;
    S[16 * (dst + (t >> 4)) + (t & 15)] = v + ((t >> 4) == 3 ? 5 : 0);
  }
  r_sync();
}
template <int OP>
__global__ void __launch_bounds__(LBR_NT) k_g2_ops(int iters, uint64_t* out) {
  LBR_SHARED_N(S, LBR_PROGS_END);
  r_init(S, LBR_PROGS_END, 0);
  ub_fill_ones(S, LBR_A(0), 12);
  const uint64_t t0 = rt();
  for (int it = 0; it < iters; it++) {
    if (OP == 0) r_g2_dbl(S, LBR_A(0), LBR_A(0));
    if (OP == 1) r_g2_add(S, LBR_A(0), LBR_A(0), LBR_A(0) + 6);
    if (OP == 2) r_exec(S, LBR_G2DBL);
    if (OP == 3) r_g2_clear_cofactor<true>(S, LBR_A(4), LBR_A(3));
    if (OP == 4) r_zero_mask(S, 8, [&](int e) { return LBR_A(0) + e; });
    if (OP == 5) r_out(S, LBR_G2DBL, 0, 6, LBR_IN);
    if (OP == 6) r_run(S, &LBR_OPS_HASH, LBR_OPS_HASH.n);
  }
  r_sync();
  const uint64_t t1 = rt();
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
// dependent LDS load chain (latency of one ds_read round trip), NT threads each chasing
template <int NT>
__global__ void __launch_bounds__(NT) k_lds_chase(int iters, uint64_t* out, int* sink) {
  __shared__ int A[4096];
  for (int i = threadIdx.x; i < 4096; i += NT) A[i] = (i * 77 + 13) & 4095;
  __syncthreads();
  int p = threadIdx.x & 4095;
  const uint64_t t0 = rt();
  for (int it = 0; it < iters; it++) p = A[p];
  __syncthreads();
  const uint64_t t1 = rt();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[threadIdx.x] = p;
}
// pieces of k_hash_map_row's lone-lane part (one wave; every lane the same item)
template <int OP>
__global__ void __launch_bounds__(64) k_h2c_parts(int iters, uint64_t* out, uint32_t* sink) {
  uint32_t M[8];
  for (int i = 0; i < 8; i++) M[i] = 0x01020304u * (i + 1) + threadIdx.x / 16;
  fp2 u = hash_to_field_u(M, 0);
  uint32_t acc = 0;
  const uint64_t t0 = rt();
  for (int it = 0; it < iters; it++) {
    if (OP == 0) { u = hash_to_field_u(M, 0); M[0] ^= u.c0.v[0]; }
    if (OP == 1) { acc += fp_is_square_i(fp_add(u.c0, fp_one())) ? 1 : 0; u.c0 = fp_add(u.c0, fp_one()); }
    if (OP == 2) { u = fp2_inv_i(u); }
    if (OP == 3) { const g2j r = map_to_curve_g2_i<true>(u); u.c0 = fp_add(u.c0, r.x.c0); }
    if (OP == 4) { u.c0 = r1_pow_const(u.c0, LB_EXP_SQRT, 378); }
    if (OP == 5) { u = fp2_mul(u, u); }
  }
  const uint64_t t1 = rt();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[threadIdx.x] = u.c0.v[0] + u.c1.v[3] + acc;
}
// synthetic one-phase programs written over the image at offset 0: the cost of a phase's parts
template <int V>
__global__ void __launch_bounds__(LBR_NT) k_synth(int iters, uint64_t* out) {
  LBR_SHARED(S);
  r_init(S);
  ub_fill_ones(S, LBR_A(0), 12);
  if (threadIdx.x == 0) {
    lds_i32* P = r_lds(S) + LBR_SLOT_WORDS + LBR_MISC;
    int w = 0;
    const int A0 = LBR_A(0);
    auto pair = [&](int slot, int c) { return (slot & 0xffff) | (c << 16); };
    const int nprod = V == 6 ? 16 : (V == 8 ? 64 : 1);
    P[w++] = 1;  // phases
    P[w++] = 0;  // outputs
    if (V <= 2 || V == 6 || V == 8) {
      const int nt = V == 0 || V == 6 || V == 8 ? 1 : 8, flags = V == 0 || V == 6 || V == 8 ? 3 : (V == 2 ? 12 : 0);
      P[w++] = 0 | (flags << 8) | (nprod << 16);
      P[w++] = nt | (nt << 16);
      for (int t = 0; t < nprod; t++) {
        P[w++] = LBR_TEMP + t;
        for (int j = 0; j < 2 * nt; j++) P[w++] = pair(A0 + (j % 12), 1);
      }
    } else if (V == 3 || V == 4) {
      const int nt = V == 3 ? 1 : 8;
      P[w++] = 1 | (1 << 16);
      P[w++] = nt;
      P[w++] = LBR_TEMP;
      for (int j = 0; j < nt; j++) P[w++] = pair(A0 + j, 1);
    }
  }
  r_sync();
  const uint64_t t0 = rt();
  for (int it = 0; it < iters; it++) {
    if (V == 7) r_sync();
    else r_exec(S, 0);
  }
  r_sync();
  const uint64_t t1 = rt();
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
#ifdef UB_TL
// timeline of r_exec_inl over `iters` runs of program `prog` (image staged in full)
__global__ void __launch_bounds__(LBR_NT) k_tl(int iters, int prog, int g2) {
  LBR_SHARED_N(S, LBR_PROGS_END);
  r_init(S, LBR_PROGS_END, 0);
  ub_fill_ones(S, LBR_A(0), 12);
  r_copy(S, LBR_IN, LBR_A(0), 24);
  if ((threadIdx.x & 63) == 0) {
    for (int i = 0; i < 8; i++) g_tl[threadIdx.x >> 6][i] = 0;
    g_tl_prev[threadIdx.x >> 6] = __builtin_amdgcn_s_memtime();
  }
  r_sync();
  for (int it = 0; it < iters; it++) r_exec_inl(S, prog);
  r_sync();
  if ((threadIdx.x & 63) == 0)
    for (int i = 0; i < 8; i++) g_tl_out[threadIdx.x >> 6][i] = g_tl[threadIdx.x >> 6][i];
}
#endif
template <int OP>
__global__ void __launch_bounds__(LBR_NT) k_phases(unsigned long long* out) {
  LBR_SHARED_N(S, LBR_PROGS_END);
  r_init(S, LBR_PROGS_END, 0);
  r_set_one(S, LBR_A(0));
  if (threadIdx.x == 0) g_ph_n = 0;
  r_copy(S, LBR_IN, LBR_A(0), 24);
  r_sync();
  const unsigned long long t0 = __builtin_readcyclecounter();
  if (OP == 0) r_exec(S, LBR_CSQR12);
  if (OP == 1) r_exec(S, LBR_MUL12);
  if (OP == 2) r_exec(S, LBR_DBL_STEP);
  if (OP == 3) r_exec(S, LBR_G2DBL);
  if (OP == 4) r_exec(S, LBR_G2ADD);
  if (OP == 5) r_exec(S, LBR_ADD_STEP);
  const unsigned long long t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) { out[0] = t0; out[1] = t1; }
}
template <int OP>
__global__ void __launch_bounds__(64) k_wave_ops(int iters, uint64_t* out) {
  LBW_SHARED(S);
  w_init_consts(S);
  w_set_one(S, LBW_A(0));
  w_set_one(S, LBW_A(1));
  const uint64_t t0 = rt();
  for (int it = 0; it < iters; it++) {
    if (OP == 0) w_sqr(S, LBW_A(0), LBW_A(0));
    if (OP == 1) w_mul(S, LBW_A(0), LBW_A(0), LBW_A(1));
  }
  w_sync();
  const uint64_t t1 = rt();
  if (threadIdx.x == 0) out[0] = t1 - t0;
}


// ---- 32-lane group variant: column g at lane g (0..27), shifts by wave_shr:1
#define WSHR1 0x138
template <int TOP>  // TOP < 0: carries out of lane 13 dropped (mod 2^392); else lane TOP keeps whole
__device__ __forceinline__ int n32(int64_t v, int g) {
  const int64_t q = v >> 28;
  int l = (int)(v & LBR_M28);
  int qlo = (int)(q & LBR_M28), qhi = (int)(q >> 28);
  if (TOP >= 0) {
    if (g == TOP - 1) { qlo = (int)q; qhi = 0; }
    if (g >= TOP) { l = g == TOP ? (int)v : 0; qlo = qhi = 0; }
  }
  const int s1 = r_dpp<WSHR1>(qlo), s2 = r_dpp<WSHR1>(r_dpp<WSHR1>(qhi));
  l += s1 + s2;
  int c = l >> 28, l2 = l & LBR_M28;
  if (TOP >= 0 && g >= TOP) { c = 0; l2 = g == TOP ? l : 0; }
  return l2 + r_dpp<WSHR1>(c);
}
template <int I, class XS>
__device__ __forceinline__ void s32(const XS& x, int yi, int64_t (&a)[2]) {
  if constexpr (I < 14) {
    if constexpr (I > 0) yi = r_dpp<WSHR1>(yi);
    a[I & 1] += (int64_t)x[I] * yi;
    s32<I + 1>(x, yi, a);
  }
}
template <class XS>
__device__ __forceinline__ int rp_mul32(const XS& x, int y, int g) {
  int64_t a[2] = {0, 0};
  s32<0>(x, y, a);
  int64_t lo = a[0] + a[1];
  int t = n32<-1>(lo, g);
  t = g < 14 ? t : 0;
  int64_t b[2] = {0, 0};
  s32<0>(r_cx_pinv{}, t, b);
  int m = n32<-1>(b[0] + b[1], g);
  m = g < 14 ? m : 0;
  a[0] = lo; a[1] = 0;
  s32<0>(r_cx_p{}, m, a);
  lo = a[0] + a[1];
  const int64_t u13 = r_dpp64<LBR_SHR(1)>(lo), u12 = r_dpp64<LBR_SHR(2)>(lo), u11 = r_dpp64<LBR_SHR(3)>(lo);
  const int64_t E = u13 + (u12 >> 28) + (u11 >> 56);
  const int64_t C = (E + LBR_M28) >> 28;
  const int64_t r = g == 14 ? lo + C : ((g > 14 && g < 28) ? lo : 0);
  return n32<27>(r, g);  // limb g - 14 at lanes 14..27
}
__global__ void __launch_bounds__(64) k_rp32_chain(int iters, uint64_t* out, int* sink) {
  __shared__ int buf[2][32];
  const int g = threadIdx.x & 31, h = threadIdx.x >> 5;
  int y = g < 13 ? (g * 12345 + 7) & LBR_M28 : (g == 13 ? 1000 : 0);
  int x[14];
  for (int i = 0; i < 14; i++) x[i] = (i * 777 + 3) & LBR_M28;
  const uint64_t t0 = rt();
  for (int it = 0; it < iters; it++) {
    const int r = rp_mul32(x, y, g);
    // move limbs from lanes 14..27 to 0..13 through LDS (as the engine's slot store + reload)
    if (g >= 14 && g < 28) buf[h][g - 14] = r;
    if (g >= 28) buf[h][g - 14] = 0;
    y = g < 14 ? buf[h][g] : 0;
    x[it % 14] ^= y & 1;
  }
  const uint64_t t1 = rt();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[threadIdx.x] = y;
}
// correctness: one product each way, limbs out
__global__ void k_cmp(const int* xin, const int* yin, int* o16, int* o32) {
  const int k = threadIdx.x & 15, g = threadIdx.x & 31;
  int x[14];
  for (int i = 0; i < 14; i++) x[i] = xin[i];
  if (threadIdx.x < 16) o16[k] = rp_mul(x, k < 14 ? yin[k] : 0, k);
  if (threadIdx.x < 32) {
    const int r = rp_mul32(x, g < 14 ? yin[g] : 0, g);
    if (g >= 14 && g < 28) o32[g - 14] = r;
  }
}

template <int T>
__global__ void __launch_bounds__(T) k_inv_chain(int iters, uint64_t* out, uint32_t* sink) {
  fp a = fp_one();
  a.v[0] ^= threadIdx.x + 12345;
  a.v[5] ^= 0x9e3779b9u;
  const uint64_t t0 = rt();
  if (threadIdx.x == 0)
    for (int it = 0; it < iters; it++) a = fp_inv_i(fp_add(a, fp_one()));
  __syncthreads();
  const uint64_t t1 = rt();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[threadIdx.x] = a.v[0];
}
int main() {
  uint64_t* d;
  int* sink;
  hipMalloc(&d, 64);
  hipMalloc(&sink, 8192);
  uint64_t h;
  auto run = [&](const char* name, auto launch, int iters) {
    launch(iters);  // warm
    hipDeviceSynchronize();
    launch(iters);
    hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    printf("%-28s %8.3f us per op\n", name, (double)h * 10.0 / 1000.0 / iters);
  };
  run("rp_mul chain (1 row)", [&](int n) { hipLaunchKernelGGL(k_rp_chain, dim3(1), dim3(64), 0, 0, n, d, sink); }, 2000);
  run("rp_mul32 chain (1 group)", [&](int n) { hipLaunchKernelGGL(k_rp32_chain, dim3(1), dim3(64), 0, 0, n, d, sink); }, 2000);
  {
    int hx[14], hy[14];
    for (int i = 0; i < 14; i++) { hx[i] = (i * 7919 + 13) & 0x0fffffff; hy[i] = (i * 104729 + 5) & 0x0fffffff; }
    hx[13] = 1000; hy[13] = 77777;
    int *dx, *dy, *o16, *o32;
    hipMalloc(&dx, 64); hipMalloc(&dy, 64); hipMalloc(&o16, 64); hipMalloc(&o32, 64);
    hipMemcpy(dx, hx, 56, hipMemcpyHostToDevice); hipMemcpy(dy, hy, 56, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_cmp, dim3(1), dim3(64), 0, 0, dx, dy, o16, o32);
    int a[14], b[14];
    hipMemcpy(a, o16, 56, hipMemcpyDeviceToHost); hipMemcpy(b, o32, 56, hipMemcpyDeviceToHost);
    printf("x:"); for (int i = 0; i < 14; i++) printf(" %d", hx[i]); printf("\ny:"); for (int i = 0; i < 14; i++) printf(" %d", hy[i]);
    printf("\nr16:"); for (int i = 0; i < 14; i++) printf(" %d", a[i]); printf("\nr32:"); for (int i = 0; i < 14; i++) printf(" %d", b[i]); printf("\n");
  }
  run("row SQR12 (1024 thr)", [&](int n) { hipLaunchKernelGGL(k_row_ops<0>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 200);
  run("row MUL12", [&](int n) { hipLaunchKernelGGL(k_row_ops<1>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 200);
  run("row copy12", [&](int n) { hipLaunchKernelGGL(k_row_ops<2>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 200);
  run("row exec SQR12 only", [&](int n) { hipLaunchKernelGGL(k_row_ops<3>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 200);
  run("row CSQR12", [&](int n) { hipLaunchKernelGGL(k_row_ops<4>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 200);
  run("fp_inv_i lane0 (64 thr)", [&](int n) { hipLaunchKernelGGL(k_inv_chain<64>, dim3(1), dim3(64), 0, 0, n, d, (uint32_t*)sink); }, 50);
  run("fp_inv_i lane0 (1024 thr)", [&](int n) { hipLaunchKernelGGL(k_inv_chain<1024>, dim3(1), dim3(1024), 0, 0, n, d, (uint32_t*)sink); }, 50);
  run("row inv", [&](int n) { hipLaunchKernelGGL(k_row_ops<6>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 20);
  run("row pow_xabs", [&](int n) { hipLaunchKernelGGL(k_row_ops<7>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 5);
  run("row final exp", [&](int n) { hipLaunchKernelGGL(k_row_ops<5>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 3);
  {
    unsigned long long* dd;
    hipMalloc(&dd, 64);
    const char* nm[6] = {"CSQR12", "MUL12", "DBL_STEP", "G2DBL", "G2ADD", "ADD_STEP"};
    for (int op = 0; op < 6; op++) {
      if (op == 3) hipLaunchKernelGGL(k_phases<3>, dim3(1), dim3(LBR_NT), 0, 0, dd);
      if (op == 4) hipLaunchKernelGGL(k_phases<4>, dim3(1), dim3(LBR_NT), 0, 0, dd);
      if (op == 5) hipLaunchKernelGGL(k_phases<5>, dim3(1), dim3(LBR_NT), 0, 0, dd);
      if (op == 0) hipLaunchKernelGGL(k_phases<0>, dim3(1), dim3(LBR_NT), 0, 0, dd);
      if (op == 1) hipLaunchKernelGGL(k_phases<1>, dim3(1), dim3(LBR_NT), 0, 0, dd);
      if (op == 2) hipLaunchKernelGGL(k_phases<2>, dim3(1), dim3(LBR_NT), 0, 0, dd);
      hipDeviceSynchronize();
      unsigned long long tt[2], ph[64][3];
      int np;
      hipMemcpy(tt, dd, 16, hipMemcpyDeviceToHost);
      hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_ph), sizeof(ph));
      hipMemcpyFromSymbol(&np, HIP_SYMBOL(g_ph_n), 4);
      printf("%s: %llu cycles total;", nm[op], tt[1] - tt[0]);
      unsigned long long prev = tt[0];
      for (int i = 0; i < np; i++) {
        if (ph[i][1] >= 10) printf(" s%llu:%llu", ph[i][1] - 10, ph[i][0] - prev);
        else printf(" %s%llu:%llu |", ph[i][1] ? "L" : "P", ph[i][2], ph[i][0] - prev);
        prev = ph[i][0];
      }
      printf("\n");
    }
  }
  run("lds chase (64 thr)", [&](int n) { hipLaunchKernelGGL(k_lds_chase<64>, dim3(1), dim3(64), 0, 0, n, d, sink); }, 10000);
  run("lds chase (1024 thr)", [&](int n) { hipLaunchKernelGGL(k_lds_chase<1024>, dim3(1), dim3(1024), 0, 0, n, d, sink); }, 10000);
  run("h2c hash_to_field", [&](int n) { hipLaunchKernelGGL(k_h2c_parts<0>, dim3(1), dim3(64), 0, 0, n, d, (uint32_t*)sink); }, 20);
  run("h2c is_square (Jacobi)", [&](int n) { hipLaunchKernelGGL(k_h2c_parts<1>, dim3(1), dim3(64), 0, 0, n, d, (uint32_t*)sink); }, 20);
  run("h2c fp2 inverse", [&](int n) { hipLaunchKernelGGL(k_h2c_parts<2>, dim3(1), dim3(64), 0, 0, n, d, (uint32_t*)sink); }, 20);
  run("h2c map_to_curve (row pows)", [&](int n) { hipLaunchKernelGGL(k_h2c_parts<3>, dim3(1), dim3(64), 0, 0, n, d, (uint32_t*)sink); }, 5);
  run("h2c one row pow", [&](int n) { hipLaunchKernelGGL(k_h2c_parts<4>, dim3(1), dim3(64), 0, 0, n, d, (uint32_t*)sink); }, 10);
  run("h2c fp2 mul (lane)", [&](int n) { hipLaunchKernelGGL(k_h2c_parts<5>, dim3(1), dim3(64), 0, 0, n, d, (uint32_t*)sink); }, 200);
  run("synth P1 plain", [&](int n) { hipLaunchKernelGGL(k_synth<0>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 1000);
  run("synth P1 8+8 terms", [&](int n) { hipLaunchKernelGGL(k_synth<1>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 1000);
  run("synth P1 8+8 reduce", [&](int n) { hipLaunchKernelGGL(k_synth<2>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 1000);
  run("synth L1 1 term", [&](int n) { hipLaunchKernelGGL(k_synth<3>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 1000);
  run("synth L1 8 terms", [&](int n) { hipLaunchKernelGGL(k_synth<4>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 1000);
  run("synth P16 plain", [&](int n) { hipLaunchKernelGGL(k_synth<6>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 1000);
  run("synth P64 plain", [&](int n) { hipLaunchKernelGGL(k_synth<8>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 1000);
  run("synth barrier", [&](int n) { hipLaunchKernelGGL(k_synth<7>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 1000);
#ifdef UB_TL
  {
    const int progs[4] = {LBR_G2DBL, LBR_CSQR12, LBR_MUL12, LBR_G2ADD};
    const char* names[4] = {"G2DBL", "CSQR12", "MUL12", "G2ADD"};
    for (int q = 0; q < 4; q++) {
      hipLaunchKernelGGL(k_tl, dim3(1), dim3(LBR_NT), 0, 0, 100, progs[q], 0);
      hipDeviceSynchronize();
      unsigned long long tl[16][8];
      hipMemcpyFromSymbol(tl, HIP_SYMBOL(g_tl_out), sizeof(tl));
      printf("timeline %s (s_memtime ticks per exec, waves 0..3): entry->prologue, operands, next-prefetch, product+store, barrier, loop-back\n", names[q]);
      for (int w = 0; w < 4; w++) {
        printf("  wave %d:", w);
        for (int i = 0; i < 6; i++) printf(" %8.1f", tl[w][(i + 1) % 6] / 100.0);
        printf("\n");
      }
    }
  }
#endif
  run("row G2 dbl", [&](int n) { hipLaunchKernelGGL(k_g2_ops<0>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 200);
  run("row G2 add", [&](int n) { hipLaunchKernelGGL(k_g2_ops<1>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 200);
  run("row G2DBL exec only", [&](int n) { hipLaunchKernelGGL(k_g2_ops<2>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 200);
  run("row zero mask (8)", [&](int n) { hipLaunchKernelGGL(k_g2_ops<4>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 200);
  run("row out (6)", [&](int n) { hipLaunchKernelGGL(k_g2_ops<5>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 200);
  run("row clear cofactor", [&](int n) { hipLaunchKernelGGL(k_g2_ops<3>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 2);
  run("row hash finish op list", [&](int n) { hipLaunchKernelGGL(k_g2_ops<6>, dim3(1), dim3(LBR_NT), 0, 0, n, d); }, 2);
  run("wave SQR12 (64 thr)", [&](int n) { hipLaunchKernelGGL(k_wave_ops<0>, dim3(1), dim3(64), 0, 0, n, d); }, 200);
  run("wave MUL12", [&](int n) { hipLaunchKernelGGL(k_wave_ops<1>, dim3(1), dim3(64), 0, 0, n, d); }, 200);
  return 0;
}
