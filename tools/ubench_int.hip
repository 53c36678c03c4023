// Integer-VALU roofline calibration for gfx950 (MI355X).
// Measures the chip-wide issue rate of v_mad_u64_u32 (the 32x32+64->64 multiply-add
// every Fp limb product uses), v_add_co_u32/v_addc_co_u32 and v_mov_b32, so that the
// roofline "peak" in bench.py is a measured number, not a guess.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int KIND>
__global__ void __launch_bounds__(256) k_rate(uint64_t* out, int iters, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed, b = a ^ 0x9e3779b9u;
  uint64_t acc[8];
#pragma unroll
  for (int k = 0; k < 8; k++) acc[k] = a + k;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (KIND == 0) {
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[k]) : "v"(a), "v"(b) : "vcc");
      } else if (KIND == 1) {
        uint32_t lo = (uint32_t)acc[k], hi = (uint32_t)(acc[k] >> 32);
        asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc" : "+v"(lo), "+v"(hi) : "v"(a) : "vcc");
        acc[k] = ((uint64_t)hi << 32) | lo;
      } else if (KIND == 2) {
        uint32_t lo = (uint32_t)acc[k];
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(lo) : "v"(b));
        acc[k] = (acc[k] & 0xffffffff00000000ull) | lo;
      } else {
        uint32_t lo = (uint32_t)acc[k];
        asm volatile("v_xor_b32 %0, %0, %1" : "+v"(lo) : "v"(b));
        acc[k] = (acc[k] & 0xffffffff00000000ull) | lo;
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND>
static double run(uint64_t* d, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k_rate<KIND>, dim3(blocks), dim3(256), 0, 0, d, 16, 1u);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_rate<KIND>, dim3(blocks), dim3(256), 0, 0, d, iters, 2u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0; hipEventElapsedTime(&ms, e0, e1);
  double ops = (double)blocks * 256 * iters * 8 * (KIND == 1 ? 2 : 1);
  return ops / (ms * 1e-3) / 1e12;
}

static constexpr uint32_t PP[12] = {0xffffaaab,0xb9feffff,0xb153ffff,0x1eabfffe,0xf6b0f624,0x6730d2a0,0xf38512bf,0x64774b84,0x434bacd7,0x4b1ba7b6,0x397fe69a,0x1a0111ea};
static constexpr uint32_t PINV = 0xfffcfffd;
struct fp { uint32_t v[12]; };

__device__ __forceinline__ fp mul_cios(const fp& a, const fp& b) {
  uint32_t t[14];
#pragma unroll
  for (int j = 0; j < 14; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
      c = (uint64_t)a.v[i] * b.v[j] + t[j] + (c >> 32);
      t[j] = (uint32_t)c;
    }
    c = (uint64_t)t[12] + (c >> 32);
    t[12] = (uint32_t)c; t[13] = (uint32_t)(c >> 32);
    uint32_t m = t[0] * PINV;
    c = (uint64_t)m * PP[0] + t[0];
#pragma unroll
    for (int j = 1; j < 12; j++) {
      c = (uint64_t)m * PP[j] + t[j] + (c >> 32);
      t[j - 1] = (uint32_t)c;
    }
    c = (uint64_t)t[12] + (c >> 32);
    t[11] = (uint32_t)c;
    t[12] = t[13] + (uint32_t)(c >> 32);
  }
  // conditional subtract
  uint32_t s[12]; uint32_t br = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) {
    uint64_t d = (uint64_t)t[j] - PP[j] - br;
    s[j] = (uint32_t)d; br = (uint32_t)(d >> 32) & 1;
  }
  bool ge = (t[12] != 0) || (br == 0);
  fp r;
#pragma unroll
  for (int j = 0; j < 12; j++) r.v[j] = ge ? s[j] : t[j];
  return r;
}


__global__ void __launch_bounds__(256) k_fpmul(fp* x, int iters) {
  int id = blockIdx.x * blockDim.x + threadIdx.x;
  fp a, b;
#pragma unroll
  for (int j = 0; j < 12; j++) { a.v[j] = (id * 7919u + j) & 0x0fffffff; b.v[j] = (id * 104729u + 3 * j) & 0x0fffffff; }
  fp c = b;
  for (int i = 0; i < iters; i++) { a = mul_cios(a, b); c = mul_cios(c, b); }
#pragma unroll
  for (int j = 0; j < 12; j++) a.v[j] ^= c.v[j];
  x[id] = a;
}

static double run_fpmul(int blocks, int iters) {
  fp* d; if (hipMalloc(&d, sizeof(fp) * blocks * 256) != hipSuccess) return -1;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k_fpmul, dim3(blocks), dim3(256), 0, 0, d, 4);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_fpmul, dim3(blocks), dim3(256), 0, 0, d, iters);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms = 0; hipEventElapsedTime(&ms, e0, e1);
  hipFree(d);
  return (double)blocks * 256 * iters * 2 / (ms * 1e-3) / 1e9;
}

int main() {
  int blocks = 256 * 8 * 4;  // 8 blocks/CU-ish worth of waves
  uint64_t* d;
  CHECK(hipMalloc(&d, sizeof(uint64_t) * blocks * 256));
  int iters = 4096;
  printf("{\"v_mad_u64_u32_Tops\": %.3f, ", run<0>(d, blocks, iters));
  printf("\"v_add_co_addc_Tops\": %.3f, ", run<1>(d, blocks, iters));
  printf("\"v_mul_lo_u32_Tops\": %.3f, ", run<2>(d, blocks, iters));
  printf("\"v_xor_b32_Tops\": %.3f, ", run<3>(d, blocks, iters));
  printf("\"fp_mul_cios_Gmul_s\": %.3f}\n", run_fpmul(256 * 8, 512));
  CHECK(hipFree(d));
  return 0;
}
