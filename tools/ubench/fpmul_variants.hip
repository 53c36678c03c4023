// Microbenchmark: per-thread Fp2-multiplication latency/throughput under three code structures,
// to choose how the pipeline kernels call the field layer (tools/, not product code).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "lb_field.h"

typedef uint32_t v16u __attribute__((ext_vector_type(16)));

__device__ __forceinline__ v16u pack(const fp& a) { v16u r; 
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = a.v[i];
  r[12] = r[13] = r[14] = r[15] = 0; return r; }
__device__ __forceinline__ fp unpack(v16u a) { fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = a[i]; return r; }

// inline CIOS body (copy of lb_field.h fp_mul as force-inline)
__device__ __forceinline__ fp mul_inl(const fp& a, const fp& b) {
  const uint32_t Pl[12] = {LB_P0, LB_P1, LB_P2, LB_P3, LB_P4, LB_P5, LB_P6, LB_P7, LB_P8, LB_P9, LB_P10, LB_P11};
  uint32_t t[14];
#pragma unroll
  for (int j = 0; j < 14; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) { c = (uint64_t)a.v[i] * b.v[j] + t[j] + (c >> 32); t[j] = (uint32_t)c; }
    c = (uint64_t)t[12] + (c >> 32); t[12] = (uint32_t)c; t[13] = (uint32_t)(c >> 32);
    uint32_t m = t[0] * LB_PINV;
    c = (uint64_t)m * Pl[0] + t[0];
#pragma unroll
    for (int j = 1; j < 12; j++) { c = (uint64_t)m * Pl[j] + t[j] + (c >> 32); t[j - 1] = (uint32_t)c; }
    c = (uint64_t)t[12] + (c >> 32); t[11] = (uint32_t)c; t[12] = t[13] + (uint32_t)(c >> 32);
  }
  return fp_reduce_once(t, t[12]);
}
__device__ __attribute__((noinline)) v16u mul_vec(v16u a, v16u b) { return pack(mul_inl(unpack(a), unpack(b))); }
__device__ __forceinline__ fp mul_v(const fp& a, const fp& b) { return unpack(mul_vec(pack(a), pack(b))); }

template <int V>
__device__ __forceinline__ fp2 f2mul(const fp2& a, const fp2& b) {
  if (V == 0) return fp2_mul(a, b);  // product: inline fp2 -> noinline carry-save fp_mul_v (VGPR args)
  if (V == 3) {  // carry-save body fully inline
    fp u0 = fp_mul_body(a.c0, b.c0), u1 = fp_mul_body(a.c1, b.c1), u2 = fp_mul_body(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
    return fp2{fp_sub(u0, u1), fp_sub(fp_sub(u2, u0), u1)};
  }
  fp t0, t1, t2;
  if (V == 1) { t0 = mul_v(a.c0, b.c0); t1 = mul_v(a.c1, b.c1); t2 = mul_v(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1)); }
  else { t0 = mul_inl(a.c0, b.c0); t1 = mul_inl(a.c1, b.c1); t2 = mul_inl(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1)); }
  return fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}

template <int V>
__global__ void __launch_bounds__(64) k(uint32_t* out, int iters) {
  uint32_t id = blockIdx.x * 64 + threadIdx.x;
  fp2 x, y;
  for (int i = 0; i < 12; i++) { x.c0.v[i] = id * 77 + i; x.c1.v[i] = id ^ i; y.c0.v[i] = i * 3 + 1; y.c1.v[i] = id + 5 * i; }
  x.c0.v[11] &= 0xfffffff; x.c1.v[11] &= 0xfffffff; y.c0.v[11] &= 0xfffffff; y.c1.v[11] &= 0xfffffff;
  for (int i = 0; i < iters; i++) x = f2mul<V>(x, y);
  uint32_t s = 0;
  for (int i = 0; i < 12; i++) s ^= x.c0.v[i] ^ x.c1.v[i];
  out[id] = s;
}

template <int V>
static void run(uint32_t* d, int waves, int iters) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<V>, dim3(waves), dim3(64), 0, 0, d, 2);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<V>, dim3(waves), dim3(64), 0, 0, d, iters);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double fpm = 3.0 * iters * waves * 64;
  printf("{\"variant\": %d, \"waves\": %d, \"us_per_fp_mul_per_thread\": %.3f, \"G_fp_mul_s\": %.2f}\n", V, waves,
         ms * 1e3 / (3.0 * iters), fpm / (ms * 1e-3) / 1e9);
}

int main() {
  uint32_t* d; hipMalloc(&d, 4 * 64 * 16384);
  for (int w : {256, 1024, 4096, 16384}) { run<0>(d, w, 200); run<1>(d, w, 200); run<2>(d, w, 200); run<3>(d, w, 200); }
  return 0;
}
