// Cycle timing of the wave-cooperative programs run by one wave (tools/, not product code):
// w_mul (MUL12 incl. in/out copies), w_sqr (SQR12), the exec part of one Miller doubling step,
// a full final exponentiation, and one lane's fp_mul for scale.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "lb_kernels.h"

__global__ void __launch_bounds__(64) k_phase(long long* out) {
  LBW_SHARED_ML(S);
  const int lane = threadIdx.x;
  w_init_consts(S, LBW_PROGS_ALL);
  if (lane < 12) { fp v = fp_one(); v.v[0] += lane; w_st(S, LBW_A(0) + lane, v); w_st(S, LBW_A(1) + lane, v); }
  if (lane < 24) { fp v = fp_one(); v.v[1] += lane; w_st(S, LBW_IN + lane, v); }
  w_sync();
  long long t0 = clock64();
  w_mul(S, LBW_A(2), LBW_A(0), LBW_A(1));
  long long t1 = clock64();
  w_sqr(S, LBW_A(3), LBW_A(2));
  long long t2 = clock64();
  w_exec(S, LBW_DBL_STEP);
  long long t3 = clock64();
  w_final_exp(S, LBW_A(0), LBW_A(3));
  long long t4 = clock64();
  fp a = w_ld(S, LBW_A(0) + (lane % 12)), b = w_ld(S, LBW_A(1) + (lane % 12));
  long long m0 = clock64();
  for (int i = 0; i < 10; i++) a = fp_mul(a, b);
  long long m1 = clock64();
  w_st(S, LBW_A(4) + (lane % 12), a);
  // per-phase breakdown of one MUL12 (w_in, each phase of w_exec, w_out); the second of two
  // runs is reported (warm instruction cache and program records)
  long long q0 = 0, q1 = 0, q2 = 0, q3 = 0;
  for (int rep = 0; rep < 2; rep++) {
  q0 = clock64();
  w_in(S, 24, lane < 12 ? LBW_A(0) + lane : LBW_A(1) + (lane - 12));
  q1 = clock64();
  {
    const lds_i16* prog = w_progs(S) + LBW_MUL12;
    const int nph = prog[0], nout = prog[2];
    int pos = 3 + nout;
    pos += (-pos) & 7;
    for (int ph = 0; ph < nph && ph < 4; ph++) {
      const int kind = prog[pos], n = prog[pos + 1];
      const int npa = prog[pos + 2], nna = prog[pos + 3], npb = prog[pos + 4], nnb = prog[pos + 5];
      const int ra = prog[pos + 6], rb = prog[pos + 7];
      pos += 8;
      long long f0 = clock64(), f1 = f0, f2 = f0;
      if (kind == 0) {
        const int k = lane;
        if (k < n) {
          int16_t rec[LBW_PREC];
          w_fetch<LBW_PREC>(rec, prog + pos + k * LBW_PREC);
          f1 = clock64();
          fp x = w_lin<LBW_MAXP>((lds_fp*)S, rec + 1, npa, nna, false);
          fp y = w_lin<LBW_MAXP>((lds_fp*)S, rec + 1 + 2 * LBW_MAXP, npb, nnb, false);
          f2 = clock64();
          w_st(S, rec[0], fp_mul(x, y));
        }
        pos += n * LBW_PREC;
      } else {
        const int k = lane;
        if (k < n) {
          int16_t rec[LBW_LREC];
          w_fetch<LBW_LREC>(rec, prog + pos + k * LBW_LREC);
          f1 = clock64();
          w_st(S, rec[0] & ~LBW_OUT_FLAG, w_lin<LBW_MAXL>((lds_fp*)S, rec + 1, npa, nna, (rec[0] & LBW_OUT_FLAG) != 0));
          f2 = clock64();
        }
        pos += n * LBW_LREC;
      }
      long long f3 = clock64();
      w_sync();
      long long f4 = clock64();
      if (lane == 0) {
        out[8 + 5 * ph] = f1 - f0;  // record fetch
        out[9 + 5 * ph] = f2 - f1;  // linear combinations
        out[10 + 5 * ph] = f3 - f2; // product (+ store)
        out[11 + 5 * ph] = f4 - f3; // barrier
        out[12 + 5 * ph] = kind;
      }
    }
  }
  q2 = clock64();
  w_out(S, LBW_MUL12, 0, 12, LBW_A(6));
  q3 = clock64();
  }
  if (lane == 0) { out[28] = q1 - q0; out[29] = q2 - q1; out[30] = q3 - q2; }
  long long r0 = wall_clock64();
  long long c0 = clock64();
  for (int i = 0; i < 20; i++) a = fp_mul(a, b);
  long long c1 = clock64();
  long long r1 = wall_clock64();
  w_st(S, LBW_A(5) + (lane % 12), a);
  if (lane == 0) {
    out[0] = t1 - t0;
    out[1] = t2 - t1;
    out[2] = t3 - t2;
    out[3] = t4 - t3;
    out[4] = (m1 - m0) / 10;
    out[5] = c1 - c0;
    out[6] = r1 - r0;
  }
}

int main() {
  long long* d; hipMalloc(&d, 8 * 32);
  hipLaunchKernelGGL(k_phase, dim3(1), dim3(64), 0, 0, d);
  hipLaunchKernelGGL(k_phase, dim3(1), dim3(64), 0, 0, d);
  long long h[32]; hipMemcpy(h, d, 8 * 32, hipMemcpyDeviceToHost);
  int wall_khz = 0; hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0);
  double mhz = h[6] > 0 ? (double)h[5] / ((double)h[6] / (wall_khz * 1e3)) / 1e6 : 0.0;
  printf("{\"w_mul\": %lld, \"w_sqr\": %lld, \"dbl_step_exec\": %lld, \"final_exp\": %lld, \"fp_mul_1lane\": %lld, "
         "\"shader_clock_mhz\": %.0f}\n", h[0], h[1], h[2], h[3], h[4], mhz);
  printf("{\"mul12_w_in\": %lld, \"mul12_exec\": %lld, \"mul12_w_out\": %lld, \"phases\": [", h[28], h[29], h[30]);
  for (int ph = 0; ph < 3; ph++)
    printf("%s{\"kind\": %lld, \"fetch\": %lld, \"lin\": %lld, \"mul_store\": %lld, \"barrier\": %lld}", ph ? ", " : "",
           h[12 + 5 * ph], h[8 + 5 * ph], h[9 + 5 * ph], h[10 + 5 * ph], h[11 + 5 * ph]);
  printf("]}\n");
  return 0;
}
