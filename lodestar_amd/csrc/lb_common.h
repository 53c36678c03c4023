// Common macros for the BLS12-381 engine.  Every arithmetic routine is written once as
// LB_HD (host+device, force-inlined) so the same source runs in the gfx950 kernels and
// in the CPU unit-test harness (tests/harness/), which is how the arithmetic is checked
// against oracle/ without a GPU.  The product path is only ever the HIP build.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define LB_HD __host__ __device__ __forceinline__
#define LB_HDNI __host__ __device__ __attribute__((noinline))
#define LB_CONST static __constant__ const
#else
#define LB_HD static inline
#define LB_HDNI static
#define LB_CONST static const
#endif

#define LB_UNROLL _Pragma("unroll")

// blst error codes (blst.h BLST_ERROR) + the @chainsafe/blst size error, used as
// per-set / per-job status.  Job results in the C ABI are 1 (valid), 0 (invalid) or
// -code (the job rejects with that error, as worker.ts:100-102 does).
enum lb_status {
  LB_OK = 0,
  LB_BAD_ENCODING = 1,
  LB_POINT_NOT_ON_CURVE = 2,
  LB_POINT_NOT_IN_GROUP = 3,
  LB_AGGR_TYPE_MISMATCH = 4,
  LB_VERIFY_FAIL = 5,
  LB_PK_IS_INFINITY = 6,
  LB_BAD_SCALAR = 7,
  LB_INVALID_SIZE = 10,
  LB_EMPTY_AGGREGATE_ARRAY = 11,
  LB_EMPTY_SIGNATURE_SET = 12,
};
