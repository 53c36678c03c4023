// Host check of the limb-resident exponentiation (lb_field.h fp_pow_const_28, radix 2^392) against
// the 12 x 32-bit chain (fp_pow_const_i<false>) for both square-root exponents; built and run by
// tests/test_pow28_host.py with g++ (the LB_HD functions compile for the host).
#include <cstdio>
#include <random>
#include "lb_field.h"
int main() {
  std::mt19937_64 g(7);
  int bad = 0;
  for (int it = 0; it < 300; it++) {
    fp a;
    for (int k = 0; k < 12; k++) a.v[k] = (uint32_t)g();
    a.v[11] &= 0x0fffffffu;  // < 2^380 < p
    if (it == 0) a = fp_zero();
    if (it == 1) a = fp_one();
    fp x = fp_pow_const_i<false>(a, LB_EXP_SQRT, 378), y = fp_pow_const_28(a, LB_EXP_SQRT, 378);
    fp x2 = fp_pow_const_i<false>(a, LB_EXP_ISQRT, 378), y2 = fp_pow_const_28(a, LB_EXP_ISQRT, 378);
    if (!fp_eq(x, y) || !fp_eq(x2, y2)) bad++;
  }
  printf("mismatches: %d / 300\n", bad);
  return bad != 0;
}
