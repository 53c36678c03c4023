// Operand scanning (fp_mul28, what fp_mul runs: 28 live 64-bit column accumulators) against
// product scanning (finely integrated, FIPS: one running column, NC independent MAD chains per
// column) on the same 14 x 28-bit Montgomery contract (tools/, not product code).
// Prints: mismatches against fp_mul_body, then per variant the lone-wave latency per product and
// the chip-wide throughput (products / s), each inline and through a noinline call.
//   tools/ubench/fpmul_ps
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "lb_field.h"

template <int NC>
__device__ __forceinline__ fp mul_ps(const fp& a, const fp& b) {
  const uint32_t P28[14] = {LB_P28_0, LB_P28_1, LB_P28_2, LB_P28_3, LB_P28_4,  LB_P28_5,  LB_P28_6,
                            LB_P28_7, LB_P28_8, LB_P28_9, LB_P28_10, LB_P28_11, LB_P28_12, LB_P28_13};
  uint32_t A[14], B[14], M[14], R[14];
  LB_UNROLL for (int k = 0; k < 14; k++) A[k] = lb_bits28(a.v, 28 * k);
  B[0] = (b.v[0] << 8) & 0x0fffffffu;
  LB_UNROLL for (int k = 1; k < 14; k++) B[k] = lb_bits28(b.v, 28 * k - 8);
  uint64_t carry = 0;
  LB_UNROLL for (int k = 0; k < 27; k++) {
    uint64_t c[NC];
    c[0] = carry;
    LB_UNROLL for (int q = 1; q < NC; q++) c[q] = 0;
    int t = 0;
    const int lo = k < 14 ? 0 : k - 13, hi = k < 14 ? k : 13;
    LB_UNROLL for (int i = lo; i <= hi; i++) c[(t++) % NC] += (uint64_t)A[i] * B[k - i];
    LB_UNROLL for (int i = lo; i <= hi; i++)
      if (i < k || k >= 14) c[(t++) % NC] += (uint64_t)M[i] * P28[k - i];
    uint64_t s = c[0];
    LB_UNROLL for (int q = 1; q < NC; q++) s += c[q];
    if (k < 14) {
      M[k] = ((uint32_t)s * LB_PINV28) & 0x0fffffffu;
      s += (uint64_t)M[k] * P28[0];
    } else {
      R[k - 14] = (uint32_t)s & 0x0fffffffu;
    }
    carry = s >> 28;
  }
  R[13] = (uint32_t)carry;
  uint32_t o[12];
  LB_UNROLL for (int w = 0; w < 12; w++) {
    const int l = (32 * w) / 28, s = 32 * w - 28 * l;
    o[w] = (R[l] >> s) | (R[l + 1] << (28 - s));
  }
  return fp_reduce_once(o, 0u);
}

typedef uint32_t v16u __attribute__((ext_vector_type(16)));
__device__ __forceinline__ v16u pk(const fp& a) { v16u r; for (int i = 0; i < 12; i++) r[i] = a.v[i]; r[12] = r[13] = r[14] = r[15] = 0; return r; }
__device__ __forceinline__ fp upk(v16u a) { fp r; for (int i = 0; i < 12; i++) r.v[i] = a[i]; return r; }
__device__ __attribute__((noinline)) v16u call_os(v16u a, v16u b) { return pk(fp_mul28(upk(a), upk(b))); }
__device__ __attribute__((noinline)) v16u call_ps2(v16u a, v16u b) { return pk(mul_ps<2>(upk(a), upk(b))); }
__device__ __attribute__((noinline)) v16u call_ps4(v16u a, v16u b) { return pk(mul_ps<4>(upk(a), upk(b))); }

template <int V>
__device__ __forceinline__ fp mulv(const fp& a, const fp& b) {
  if constexpr (V == 0) return fp_mul28(a, b);
  if constexpr (V == 1) return mul_ps<2>(a, b);
  if constexpr (V == 2) return mul_ps<4>(a, b);
  if constexpr (V == 3) return upk(call_os(pk(a), pk(b)));
  if constexpr (V == 4) return upk(call_ps2(pk(a), pk(b)));
  return upk(call_ps4(pk(a), pk(b)));
}

__device__ uint32_t rng(uint32_t& s) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; }
__global__ void k_check(int n, uint32_t* bad) {
  uint32_t s = 0x9e3779b9u ^ (blockIdx.x * 64 + threadIdx.x) * 2654435761u;
  for (int it = 0; it < n; it++) {
    fp a, b;
    for (int j = 0; j < 12; j++) { a.v[j] = rng(s); b.v[j] = rng(s); }
    if ((it & 3) == 1) for (int j = 0; j < 12; j++) a.v[j] = 0xffffffffu;
    a.v[11] &= 0x1a0111e9u; b.v[11] &= 0x1a0111e9u;
    if ((it & 3) == 2) { for (int j = 0; j < 12; j++) b.v[j] = 0; b.v[0] = 1; }
    fp r = fp_mul_body(a, b), x = mul_ps<2>(a, b), y = mul_ps<4>(a, b);
    for (int j = 0; j < 12; j++) if (r.v[j] != x.v[j] || r.v[j] != y.v[j]) atomicAdd(bad, 1u);
  }
}
template <int V>
__global__ void __launch_bounds__(64) k_speed(uint32_t* out, int iters) {
  fp a, b;
  for (int j = 0; j < 12; j++) { a.v[j] = threadIdx.x * 77 + j; b.v[j] = blockIdx.x + 5 * j; }
  for (int i = 0; i < iters; i++) a = mulv<V>(a, b);
  for (int j = 0; j < 12; j++) out[(blockIdx.x * 64 + threadIdx.x) * 12 + j] = a.v[j];
}

int main() {
  uint32_t *bad, *out;
  hipMalloc(&bad, 4); hipMemset(bad, 0, 4);
  hipMalloc(&out, (size_t)16384 * 64 * 48);
  hipLaunchKernelGGL(k_check, dim3(256), dim3(64), 0, 0, 256, bad);
  uint32_t hb = 0; hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
  printf("mismatches vs fp_mul_body: %u (of %d)\n", hb, 256 * 64 * 256);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[6] = {"operand-scan inline", "product-scan x2 inline", "product-scan x4 inline",
                          "operand-scan call", "product-scan x2 call", "product-scan x4 call"};
  void (*ks[6])(uint32_t*, int) = {k_speed<0>, k_speed<1>, k_speed<2>, k_speed<3>, k_speed<4>, k_speed<5>};
  for (int v = 0; v < 6; v++) {
    float lat = 0, thr = 0;
    for (int rep = 0; rep < 2; rep++) {
      const int it1 = 2000;
      hipEventRecord(e0); hipLaunchKernelGGL(ks[v], dim3(1), dim3(64), 0, 0, out, it1); hipEventRecord(e1);
      hipEventSynchronize(e1); hipEventElapsedTime(&lat, e0, e1);
      const int blocks = 256 * 4 * 8, it2 = 400;
      hipEventRecord(e0); hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(64), 0, 0, out, it2); hipEventRecord(e1);
      hipEventSynchronize(e1); hipEventElapsedTime(&thr, e0, e1);
      if (rep) printf("%-24s latency %.0f ns/product   throughput %.2f G products/s\n", names[v], lat * 1e6 / it1,
                      (double)blocks * 64 * it2 / (thr * 1e-3) / 1e9);
    }
  }
  return hb != 0;
}
