// Correctness + speed of the device Montgomery products against fp_mul_body (tools/, not product
// code): fp_mul28 (14 x 28-bit limbs, what fp_mul runs), fp_sqr28 (what fp_sqr runs) and the
// 32-bit inline-asm form.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "lb_field.h"
#include "lb_fpmul_gfx950.h"

__device__ __forceinline__ fp mul_asm(const fp& a, const fp& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t o[12], top;
  lbm_mont_mul(o, &top, a.v, b.v);
  return fp_reduce_once(o, top);
#else
  return a;
#endif
}
__device__ uint32_t rng(uint32_t& s) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; }

__global__ void k_check(int n, uint32_t* bad) {
  uint32_t s = 0x9e3779b9u ^ (blockIdx.x * 64 + threadIdx.x) * 2654435761u;
  for (int it = 0; it < n; it++) {
    fp a, b;
    for (int j = 0; j < 12; j++) { a.v[j] = rng(s); b.v[j] = rng(s); }
    int mode = it & 3;
    if (mode == 1) for (int j = 0; j < 12; j++) a.v[j] = 0xffffffffu;   // max limbs
    a.v[11] &= 0x1a0111e9u; b.v[11] &= 0x1a0111e9u;                     // < p
    if (mode == 2) { for (int j = 0; j < 12; j++) b.v[j] = 0; b.v[0] = 1; }
    fp r1 = fp_mul_body(a, b), r2 = mul_asm(a, b), r3 = fp_mul28(a, b);
    for (int j = 0; j < 12; j++) if (r1.v[j] != r2.v[j] || r1.v[j] != r3.v[j]) atomicAdd(bad, 1u);
    fp q1 = fp_mul_body(a, a), q2 = fp_sqr28(a);
    for (int j = 0; j < 12; j++) if (q1.v[j] != q2.v[j]) atomicAdd(bad, 1u);
  }
}
template <int V>
__global__ void __launch_bounds__(64) k_speed(uint32_t* out, int iters) {
  fp a, b;
  for (int j = 0; j < 12; j++) { a.v[j] = threadIdx.x * 77 + j; b.v[j] = blockIdx.x + 5 * j; }
  for (int i = 0; i < iters; i++)
    a = V == 3 ? fp_sqr28(a) : V == 2 ? fp_mul28(a, b) : V ? mul_asm(a, b) : fp_mul_body(a, b);
  uint32_t x = 0; for (int j = 0; j < 12; j++) x ^= a.v[j];
  out[blockIdx.x * 64 + threadIdx.x] = x;
}
template <int V> static float run(uint32_t* d, int waves, int iters) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k_speed<V>, dim3(waves), dim3(64), 0, 0, d, 2);
  hipEventRecord(e0); hipLaunchKernelGGL(k_speed<V>, dim3(waves), dim3(64), 0, 0, d, iters); hipEventRecord(e1);
  hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms, e0, e1); return ms;
}
int main() {
  uint32_t *bad, *d; hipMalloc(&bad, 4); hipMemset(bad, 0, 4); hipMalloc(&d, 4 * 64 * 16384);
  hipLaunchKernelGGL(k_check, dim3(256), dim3(64), 0, 0, 1000, bad);
  uint32_t hb; hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
  printf("{\"mismatches\": %u, \"checked\": %d", hb, 256 * 64 * 1000);
  for (int w : {256, 4096}) {
    float t0 = run<0>(d, w, 400), t1 = run<1>(d, w, 400), t2 = run<2>(d, w, 400), t3 = run<3>(d, w, 400);
    printf(", \"w%d_body_Gmul_s\": %.2f, \"w%d_asm32_Gmul_s\": %.2f, \"w%d_mul28_Gmul_s\": %.2f, \"w%d_sqr28_Gsqr_s\": %.2f",
           w, w * 64.0 * 400 / t0 / 1e6, w, w * 64.0 * 400 / t1 / 1e6, w, w * 64.0 * 400 / t2 / 1e6, w,
           w * 64.0 * 400 / t3 / 1e6);
  }
  printf("}\n");
  return hb != 0;
}
