// Microbenchmark of the wave-cooperative engine pieces (tools/, not product code).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "lb_kernels.h"

__global__ void __launch_bounds__(64) k_wmul(int iters, uint32_t* out) {
  __shared__ fp S[LBW_SLOTS];
  const int lane = threadIdx.x;
  w_init_consts(S);
  if (lane < 12) { fp v = fp_one(); v.v[0] += lane; S[LBW_A(0) + lane] = v; S[LBW_A(1) + lane] = v; }
  w_sync();
  for (int i = 0; i < iters; i++) w_mul(S, LBW_A(0), LBW_A(0), LBW_A(1));
  if (lane == 0) out[blockIdx.x] = S[LBW_A(0)].v[0];
}
__global__ void __launch_bounds__(64) k_wsqr(int iters, uint32_t* out) {
  __shared__ fp S[LBW_SLOTS];
  const int lane = threadIdx.x;
  w_init_consts(S);
  if (lane < 12) { fp v = fp_one(); v.v[0] += lane; S[LBW_A(0) + lane] = v; }
  w_sync();
  for (int i = 0; i < iters; i++) w_sqr(S, LBW_A(0), LBW_A(0));
  if (lane == 0) out[blockIdx.x] = S[LBW_A(0)].v[0];
}
__global__ void __launch_bounds__(64) k_inv(uint32_t* out) {
  __shared__ fp S[LBW_SLOTS];
  const int lane = threadIdx.x;
  if (lane < 12) { fp v = fp_one(); v.v[0] += lane; S[LBW_A(0) + lane] = v; }
  w_sync();
  w_inv(S, LBW_A(1), LBW_A(0));
  if (lane == 0) out[blockIdx.x] = S[LBW_A(1)].v[0];
}
__global__ void __launch_bounds__(64) k_fe(uint32_t* out) {
  __shared__ fp S[LBW_SLOTS];
  const int lane = threadIdx.x;
  w_init_consts(S);
  if (lane < 12) { fp v = fp_one(); v.v[0] += lane; S[LBW_A(0) + lane] = v; }
  w_sync();
  w_final_exp(S, LBW_A(0), LBW_A(0));
  if (lane == 0) out[blockIdx.x] = S[LBW_A(0)].v[0];
}
__global__ void __launch_bounds__(64) k_ml(uint32_t* out) {
  __shared__ fp S[LBW_SLOTS];
  const int lane = threadIdx.x;
  w_init_consts(S);
  if (lane < 6) S[LBW_PT + lane] = lane < 2 ? fp_load(lane == 0 ? LB_G1X : LB_G1Y) : fp_load(LB_B2 + 12 * ((lane - 2) & 1));
  w_sync();
  w_miller(S, LBW_A(0));
  if (lane == 0) out[blockIdx.x] = S[LBW_A(0)].v[0];
}
__global__ void __launch_bounds__(64) k_g2aff(uint32_t* out) {
  if (threadIdx.x != 0) return;
  g2j p; p.x = fp2_one(); p.y = fp2_one(); p.z = fp2{fp_one(), fp_one()};
  g2a a; jac_to_aff(a, p);
  out[blockIdx.x] = a.x.c0.v[0];
}

template <class F>
static float timeit(F f) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  f(); hipDeviceSynchronize();
  hipEventRecord(a); f(); hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); return ms;
}

int main() {
  uint32_t* d; hipMalloc(&d, 4 * 4096);
  printf("{\"w_mul_us\": %.2f, ", timeit([&] { hipLaunchKernelGGL(k_wmul, dim3(1), dim3(64), 0, 0, 100, d); }) * 10.f);
  printf("\"w_sqr_us\": %.2f, ", timeit([&] { hipLaunchKernelGGL(k_wsqr, dim3(1), dim3(64), 0, 0, 100, d); }) * 10.f);
  printf("\"fp12_inv_1lane_ms\": %.3f, ", timeit([&] { hipLaunchKernelGGL(k_inv, dim3(1), dim3(64), 0, 0, d); }));
  printf("\"g2_to_affine_1lane_ms\": %.3f, ", timeit([&] { hipLaunchKernelGGL(k_g2aff, dim3(1), dim3(64), 0, 0, d); }));
  printf("\"w_final_exp_ms\": %.3f, ", timeit([&] { hipLaunchKernelGGL(k_fe, dim3(1), dim3(64), 0, 0, d); }));
  printf("\"w_miller_ms\": %.3f, ", timeit([&] { hipLaunchKernelGGL(k_ml, dim3(1), dim3(64), 0, 0, d); }));
  printf("\"w_mul_x1024_blocks_us_per_mul\": %.3f}\n", timeit([&] { hipLaunchKernelGGL(k_wmul, dim3(1024), dim3(64), 0, 0, 100, d); }) * 10.f);
  return 0;
}
