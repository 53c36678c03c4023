// The posdivsteps Jacobi symbol (lb_field.h fp_is_square_sg) against the binary algorithm
// (fp_is_square) on random words below 2^380, p - k for k = 1..1000, values just below p, and
// 0..4.  Host build of the device header (tests/test_jacobi_host.py).
#include <cstdio>
#include <random>
#include "lb_serial.h"
int main() {
  const uint32_t Pl[12] = {LB_P0, LB_P1, LB_P2, LB_P3, LB_P4, LB_P5, LB_P6, LB_P7, LB_P8, LB_P9, LB_P10, LB_P11};
  std::mt19937_64 rng(7);
  int bad = 0, unsettled = 0, sq = 0, n = 0;
  for (int it = 0; it < 12000; it++, n++) {
    fp x;
    for (int w = 0; w < 12; w++) x.v[w] = (uint32_t)rng();
    x.v[11] &= 0x0fffffffu;
    if (it < 5) {
      for (int w = 0; w < 12; w++) x.v[w] = 0;
      x.v[0] = it;
    } else if (it >= 10000 && it < 11000) {  // p - k
      uint64_t br = it - 10000 + 1;
      for (int w = 0; w < 12; w++) {
        const uint64_t d = (uint64_t)Pl[w] - br;
        x.v[w] = (uint32_t)d;
        br = d >> 63;
      }
    } else if (it >= 11000) {
      x.v[11] = Pl[11] - 1;  // top word just below p's
    }
    const bool ref = fp_is_square(x);
    const int r = fp_is_square_sg(x);
    if (r < 0) unsettled++;
    else if ((r == 1) != ref) bad++;
    sq += ref;
  }
  printf("mismatches: %d / %d unsettled %d squares %d\n", bad, n, unsettled, sq);
  return bad != 0 || unsettled != 0;
}
