// Per-phase cycle timing of one MUL12 program run by one wave (tools/, not product code).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "lb_kernels.h"

__global__ void __launch_bounds__(64) k_phase(long long* out) {
  __shared__ fp S[LBW_SLOTS];
  const int lane = threadIdx.x;
  w_init_consts(S);
  if (lane < 12) { fp v = fp_one(); v.v[0] += lane; S[LBW_A(0) + lane] = v; S[LBW_A(1) + lane] = v; }
  w_sync();
  long long t0 = clock64();
  w_in(S, 24, lane < 12 ? LBW_A(0) + lane : LBW_A(1) + (lane - 12));
  long long t1 = clock64();
  // inline copy of w_exec with timestamps
  const int16_t* prog = LBW_MUL12;
  const int nph = prog[0], nout = prog[2];
  int pos = 3 + nout; pos += (-pos) & 7;
  long long tp[8];
  for (int ph = 0; ph < nph; ph++) {
    const int kind = prog[pos], n = prog[pos + 1];
    pos += 8;
    if (kind == 0) {
      const int k = lane;
      if (k < n) {
        int16_t rec[LBW_PREC];
        w_fetch<LBW_PREC>(rec, prog + pos + k * LBW_PREC);
        fp x = w_lin<LBW_MAXT>(S, rec + 1);
        fp y = w_lin<LBW_MAXT>(S, rec + 1 + 2 * LBW_MAXT);
        S[rec[0]] = fp_mul(x, y);
      }
      pos += n * LBW_PREC;
    } else {
      const int k = lane;
      if (k < n) {
        int16_t rec[LBW_LREC];
        w_fetch<LBW_LREC>(rec, prog + pos + k * LBW_LREC);
        S[rec[0]] = w_lin<LBW_MAXL>(S, rec + 1);
      }
      pos += n * LBW_LREC;
    }
    w_sync();
    tp[ph] = clock64();
  }
  w_out(S, LBW_MUL12, 0, 12, LBW_A(2));
  long long t9 = clock64();
  // fp_mul alone, lin alone
  fp a = S[LBW_A(0) + (lane % 12)], b = S[LBW_A(1) + (lane % 12)];
  long long m0 = clock64();
  for (int i = 0; i < 10; i++) a = fp_mul(a, b);
  long long m1 = clock64();
  S[LBW_A(3) + (lane % 12)] = a;
  if (lane == 0) {
    out[0] = t1 - t0;
    long long prev = t1;
    for (int ph = 0; ph < nph; ph++) { out[1 + ph] = tp[ph] - prev; prev = tp[ph]; }
    out[6] = t9 - prev;
    out[7] = (m1 - m0) / 10;
    out[8] = nph;
  }
}

int main() {
  long long* d; hipMalloc(&d, 8 * 16);
  hipLaunchKernelGGL(k_phase, dim3(1), dim3(64), 0, 0, d);
  hipLaunchKernelGGL(k_phase, dim3(1), dim3(64), 0, 0, d);
  long long h[16]; hipMemcpy(h, d, 8 * 16, hipMemcpyDeviceToHost);
  printf("{\"cycles_w_in\": %lld, \"phase\": [%lld, %lld, %lld, %lld, %lld], \"w_out\": %lld, \"fp_mul\": %lld, \"nph\": %lld}\n",
         h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8]);
  return 0;
}
