// Cycle costs of the wave engine's linear-combination pieces, one wave (tools/, not product code):
// w_lin over 24 and 8 terms with the record in registers, the LDS slot loads alone, the 64-bit
// accumulation alone, and the conditional-subtraction chain alone.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "lb_kernels.h"

__global__ void __launch_bounds__(64) k_lin(long long* out, const int16_t* rec_g) {
  LBW_SHARED(S0);
  lds_fp* S = (lds_fp*)S0;
  const int lane = threadIdx.x;
  for (int k = lane; k < LBW_SLOTS; k += 64) { fp v = fp_one(); v.v[0] += k; v.v[11] = 0x1000; lds_st(S, k, v); }
  __syncthreads();
  int16_t rec[LBW_LREC];
  // lane-dependent slots, all distinct-ish (like a real phase)
  for (int k = 0; k < LBW_LREC; k++) rec[k] = rec_g[k];
  for (int k = 0; k < 24; k++) rec[1 + 2 * k] = (int16_t)((64 + lane * 3 + k * 5) % (LBW_SLOTS - 1));
  fp acc = fp_zero();
  long long t0 = clock64();
  for (int it = 0; it < 8; it++) {
    fp r = w_lin<LBW_MAXL>(S, rec + 1, 12, 12, false);
    acc.v[it % 12] ^= r.v[0];
    rec[1] ^= (int16_t)(r.v[1] & 1);
  }
  long long t1 = clock64();
  for (int it = 0; it < 8; it++) {
    fp r = w_lin<LBW_MAXP>(S, rec + 1, 8, 0, false);
    acc.v[it % 12] ^= r.v[0];
    rec[1] ^= (int16_t)(r.v[1] & 1);
  }
  long long t2 = clock64();
  // LDS loads alone: 24 slots per iteration
  for (int it = 0; it < 8; it++) {
    LB_UNROLL for (int k = 0; k < 24; k++) {
      fp v = lds_ld(S, rec[1 + 2 * k]);
      acc.v[k % 12] ^= v.v[k % 12];
    }
    rec[1] ^= (int16_t)(acc.v[0] & 1);
  }
  long long t3 = clock64();
  // 64-bit accumulation alone over register values: 24 terms x 12 limbs
  uint64_t pa[12] = {0};
  fp v0 = lds_ld(S, lane), v1 = lds_ld(S, lane + 1);
  for (int it = 0; it < 8; it++) {
    LB_UNROLL for (int k = 0; k < 24; k++) {
      const fp& v = (k & 1) ? v1 : v0;
      const uint32_t c = (uint32_t)rec[2 + 2 * k];
      LB_UNROLL for (int j = 0; j < 12; j++) pa[j] += (uint64_t)v.v[j] * c;
    }
    v0.v[0] ^= (uint32_t)pa[it % 12];
  }
  long long t4 = clock64();
  uint32_t r13[13];
  for (int j = 0; j < 13; j++) r13[j] = (uint32_t)pa[j % 12];
  for (int it = 0; it < 8; it++) {
    LB_UNROLL for (int j = 6; j >= 0; j--) w_csub13(r13, j ? LB_P_X2 : LB_P_X1);
    r13[0] ^= it;
  }
  long long t5 = clock64();
  acc.v[0] ^= r13[3] ^ (uint32_t)pa[5];
  lds_st(S, lane, acc);
  if (lane == 0) {
    out[0] = (t1 - t0) / 8;
    out[1] = (t2 - t1) / 8;
    out[2] = (t3 - t2) / 8;
    out[3] = (t4 - t3) / 8;
    out[4] = (t5 - t4) / 8;
  }
}

int main() {
  long long* d;
  int16_t* rg;
  hipMalloc(&d, 8 * 8);
  hipMalloc(&rg, 2 * LBW_LREC);
  int16_t h_rec[LBW_LREC];
  for (int k = 0; k < LBW_LREC; k++) h_rec[k] = (k % 2 == 0 && k > 0) ? 1 : 0;
  hipMemcpy(rg, h_rec, sizeof(h_rec), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_lin, dim3(1), dim3(64), 0, 0, d, rg);
  hipLaunchKernelGGL(k_lin, dim3(1), dim3(64), 0, 0, d, rg);
  long long h[8];
  hipMemcpy(h, d, 8 * 8, hipMemcpyDeviceToHost);
  printf("{\"w_lin24\": %lld, \"w_lin8\": %lld, \"lds_24_slots\": %lld, \"mad_acc_24x12\": %lld, \"csub_x7\": %lld}\n",
         h[0], h[1], h[2], h[3], h[4]);
  return 0;
}
