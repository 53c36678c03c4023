// C-ABI engine (include/lodestar_bls.h) driving the gfx950 pipeline of lb_kernels.h.
//
// One engine per GPU, one HIP stream per engine; calls on one engine are serialised by a
// mutex (the reference's worker pool runs one job package per worker at a time,
// multithread/index.ts:290-381).  Inputs are copied into device memory at batch creation
// (the reference structured-clones its BlsWorkReq[], multithread/index.ts:330), so the
// caller never has to keep its buffers alive.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/random.h>

#include <mutex>
#include <string>
#include <vector>

#include "lb_kernels.h"

#define LB_ABI_VERSION 1

namespace {

struct dbuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes + bytes / 4 + 4096;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

const char* const kStageNames[] = {"decode_sigs", "hash_map", "hash_finish", "pk_blind", "miller",
                                   "job_leaves",  "tree_up",  "root_check",  "bisect"};
constexpr int kStages = 9;

}  // namespace

struct lb_batch {
  uint32_t n_jobs = 0, n_sets = 0, n_pks = 0;
  std::vector<uint32_t> job_off;  // host copy (bisection bookkeeping)
  dbuf d_job_off, d_pk_off, d_pks, d_msgs, d_sigs, d_sig_sizes;
  bool has_sizes = false;
  int device = 0;
  ~lb_batch() {
    d_job_off.release();
    d_pk_off.release();
    d_pks.release();
    d_msgs.release();
    d_sigs.release();
    d_sig_sizes.release();
  }
};

struct lb_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  // workspace
  dbuf scalars, sig_aff, sig_inf, sig_status, q, h_aff, rpk, rsig, pk_status, ml, treeP, treeS, job_status,
      nodes, verdict, parts, ok;
  std::vector<uint64_t> h_scalars;
  // profiling
  bool profiling = false;
  hipEvent_t ev[kStages + 1] = {};
  float last_ms[kStages] = {};
  float acc_ms[kStages] = {};
};

#define LB_HIP(call)                                                                        \
  do {                                                                                      \
    hipError_t _e = (call);                                                                 \
    if (_e != hipSuccess) {                                                                 \
      fprintf(stderr, "lodestar_bls: %s failed: %s (%s:%d)\n", #call, hipGetErrorString(_e), \
              __FILE__, __LINE__);                                                          \
      return LB_ERR_DEVICE;                                                                 \
    }                                                                                       \
  } while (0)

static inline uint32_t nblk(uint32_t n) { return (n + LB_TPB - 1) / LB_TPB; }

static int fill_scalars(lb_engine* e, uint32_t n, const uint64_t* user) {
  e->h_scalars.resize(n);
  if (user) {
    for (uint32_t i = 0; i < n; i++)
      if (user[i] == 0) return LB_BAD_SCALAR;
    memcpy(e->h_scalars.data(), user, (size_t)n * 8);
  } else {
    // blst verifyMultipleSignatures: 8 bytes from the CSPRNG per set, forced non-zero
    size_t need = (size_t)n * 8, got = 0;
    uint8_t* dst = reinterpret_cast<uint8_t*>(e->h_scalars.data());
    while (got < need) {
      ssize_t r = getrandom(dst + got, need - got, 0);
      if (r < 0) return LB_ERR_DEVICE;
      got += (size_t)r;
    }
    for (uint32_t i = 0; i < n; i++)
      while (e->h_scalars[i] == 0) getrandom(&e->h_scalars[i], 8, 0);
  }
  return LB_OK;
}

extern "C" {

int32_t lb_abi_version(void) { return LB_ABI_VERSION; }

const char* lb_error_name(int32_t code) {
  switch (code) {
    case LB_OK: return "BLST_SUCCESS";
    case LB_BAD_ENCODING: return "BLST_BAD_ENCODING";
    case LB_POINT_NOT_ON_CURVE: return "BLST_POINT_NOT_ON_CURVE";
    case LB_POINT_NOT_IN_GROUP: return "BLST_POINT_NOT_IN_GROUP";
    case LB_AGGR_TYPE_MISMATCH: return "BLST_AGGR_TYPE_MISMATCH";
    case LB_VERIFY_FAIL: return "BLST_VERIFY_FAIL";
    case LB_PK_IS_INFINITY: return "BLST_PK_IS_INFINITY";
    case LB_BAD_SCALAR: return "BLST_BAD_SCALAR";
    case LB_INVALID_SIZE: return "BLST_INVALID_SIZE";
    case LB_EMPTY_AGGREGATE_ARRAY: return "EMPTY_AGGREGATE_ARRAY";
    case LB_EMPTY_SIGNATURE_SET: return "Empty signature set";
    case LB_ERR_ARGUMENT: return "LB_ERR_ARGUMENT";
    case LB_ERR_DEVICE: return "LB_ERR_DEVICE";
    case LB_ERR_NO_DEVICE: return "LB_ERR_NO_DEVICE";
    default: return "LB_UNKNOWN_ERROR";
  }
}

int32_t lb_engine_create(int32_t device, lb_engine** out) {
  if (!out) return LB_ERR_ARGUMENT;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return LB_ERR_NO_DEVICE;
  if (device < 0) LB_HIP(hipGetDevice(&device));
  if (device >= count) return LB_ERR_NO_DEVICE;
  hipDeviceProp_t prop;
  LB_HIP(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    fprintf(stderr, "lodestar_bls: device %d is %s, this build targets gfx950 only\n", device, prop.gcnArchName);
    return LB_ERR_NO_DEVICE;
  }
  LB_HIP(hipSetDevice(device));
  lb_engine* e = new lb_engine();
  e->device = device;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
    delete e;
    return LB_ERR_DEVICE;
  }
  for (int i = 0; i <= kStages; i++) hipEventCreate(&e->ev[i]);
  *out = e;
  return LB_OK;
}

void lb_engine_destroy(lb_engine* e) {
  if (!e) return;
  hipSetDevice(e->device);
  hipStreamSynchronize(e->stream);
  dbuf* bufs[] = {&e->scalars, &e->sig_aff, &e->sig_inf, &e->sig_status, &e->q, &e->h_aff, &e->rpk, &e->rsig,
                  &e->pk_status, &e->ml, &e->treeP, &e->treeS, &e->job_status, &e->nodes, &e->verdict, &e->parts,
                  &e->ok};
  for (dbuf* b : bufs) b->release();
  for (int i = 0; i <= kStages; i++)
    if (e->ev[i]) hipEventDestroy(e->ev[i]);
  hipStreamDestroy(e->stream);
  delete e;
}

int32_t lb_engine_set_profiling(lb_engine* e, int32_t enable) {
  if (!e) return LB_ERR_ARGUMENT;
  e->profiling = enable != 0;
  return LB_OK;
}

int32_t lb_engine_last_profile(lb_engine* e, const char** names, float* ms, int32_t cap, int32_t* n) {
  if (!e || !n) return LB_ERR_ARGUMENT;
  int k = cap < kStages ? cap : kStages;
  for (int i = 0; i < k; i++) {
    if (names) names[i] = kStageNames[i];
    if (ms) ms[i] = e->last_ms[i];
  }
  *n = k;
  return LB_OK;
}

int32_t lb_batch_create(lb_engine* e, uint32_t n_jobs, const uint32_t* job_offsets, const uint32_t* set_pk_offsets,
                        const uint8_t* pubkeys, const uint8_t* signing_roots, const uint8_t* signatures,
                        const uint32_t* sig_sizes, lb_batch** out) {
  if (!e || !out || !job_offsets || !set_pk_offsets) return LB_ERR_ARGUMENT;
  *out = nullptr;
  if (job_offsets[0] != 0) return LB_ERR_ARGUMENT;
  for (uint32_t j = 0; j < n_jobs; j++)
    if (job_offsets[j + 1] < job_offsets[j]) return LB_ERR_ARGUMENT;
  uint32_t n_sets = job_offsets[n_jobs];
  if (set_pk_offsets[0] != 0) return LB_ERR_ARGUMENT;
  for (uint32_t i = 0; i < n_sets; i++)
    if (set_pk_offsets[i + 1] < set_pk_offsets[i]) return LB_ERR_ARGUMENT;
  uint32_t n_pks = set_pk_offsets[n_sets];
  if ((n_sets && (!signing_roots || !signatures)) || (n_pks && !pubkeys)) return LB_ERR_ARGUMENT;
  std::lock_guard<std::mutex> lk(e->mu);
  LB_HIP(hipSetDevice(e->device));
  lb_batch* b = new lb_batch();
  b->device = e->device;
  b->n_jobs = n_jobs;
  b->n_sets = n_sets;
  b->n_pks = n_pks;
  b->job_off.assign(job_offsets, job_offsets + n_jobs + 1);
  b->has_sizes = sig_sizes != nullptr;
  auto up = [&](dbuf& d, const void* src, size_t bytes) -> hipError_t {
    hipError_t r = d.ensure(bytes ? bytes : 16);
    if (r != hipSuccess || !bytes) return r;
    return hipMemcpyAsync(d.p, src, bytes, hipMemcpyHostToDevice, e->stream);
  };
  hipError_t r = up(b->d_job_off, job_offsets, (size_t)(n_jobs + 1) * 4);
  if (r == hipSuccess) r = up(b->d_pk_off, set_pk_offsets, (size_t)(n_sets + 1) * 4);
  if (r == hipSuccess) r = up(b->d_pks, pubkeys, (size_t)n_pks * 96);
  if (r == hipSuccess) r = up(b->d_msgs, signing_roots, (size_t)n_sets * 32);
  if (r == hipSuccess) r = up(b->d_sigs, signatures, (size_t)n_sets * 96);
  if (r == hipSuccess && sig_sizes) r = up(b->d_sig_sizes, sig_sizes, (size_t)n_sets * 4);
  if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
  if (r != hipSuccess) {
    fprintf(stderr, "lodestar_bls: batch upload failed: %s\n", hipGetErrorString(r));
    delete b;
    return LB_ERR_DEVICE;
  }
  *out = b;
  return LB_OK;
}

void lb_batch_destroy(lb_batch* b) {
  if (!b) return;
  hipSetDevice(b->device);
  delete b;
}
uint32_t lb_batch_num_sets(const lb_batch* b) { return b ? b->n_sets : 0; }
uint32_t lb_batch_num_jobs(const lb_batch* b) { return b ? b->n_jobs : 0; }

}  // extern "C"

// Runs the per-set pipeline and builds the job product tree.  m = tree leaf count (pow2).
static int32_t run_pipeline(lb_engine* e, lb_batch* b, const uint64_t* scalars, uint32_t& m) {
  const uint32_t n = b->n_sets, nj = b->n_jobs;
  int st = fill_scalars(e, n, scalars);
  if (st != LB_OK) return st;
  m = 1;
  while (m < nj) m <<= 1;
  const uint32_t ns = n ? n : 1;
  LB_HIP(e->scalars.ensure((size_t)ns * 8));
  LB_HIP(e->sig_aff.ensure((size_t)ns * sizeof(g2a)));
  LB_HIP(e->sig_inf.ensure((size_t)ns * 4));
  LB_HIP(e->sig_status.ensure((size_t)ns * 4));
  LB_HIP(e->q.ensure((size_t)ns * 2 * sizeof(g2j)));
  LB_HIP(e->h_aff.ensure((size_t)ns * sizeof(g2a)));
  LB_HIP(e->rpk.ensure((size_t)ns * sizeof(g1a)));
  LB_HIP(e->rsig.ensure((size_t)ns * sizeof(g2j)));
  LB_HIP(e->pk_status.ensure((size_t)ns * 4));
  LB_HIP(e->ml.ensure((size_t)ns * sizeof(fp12)));
  LB_HIP(e->treeP.ensure((size_t)2 * m * sizeof(fp12)));
  LB_HIP(e->treeS.ensure((size_t)2 * m * sizeof(g2j)));
  LB_HIP(e->job_status.ensure((size_t)(nj ? nj : 1) * 4));
  hipStream_t s = e->stream;
  if (n) LB_HIP(hipMemcpyAsync(e->scalars.p, e->h_scalars.data(), (size_t)n * 8, hipMemcpyHostToDevice, s));
  auto mark = [&](int k) {
    if (e->profiling) hipEventRecord(e->ev[k], s);
  };
  mark(0);
  if (n) {
    hipLaunchKernelGGL(k_decode_sigs, dim3(nblk(n)), dim3(LB_TPB), 0, s, n, b->d_sigs.as<uint8_t>(),
                       b->has_sizes ? b->d_sig_sizes.as<uint32_t>() : nullptr, e->sig_aff.as<uint32_t>(),
                       e->sig_inf.as<uint32_t>(), e->sig_status.as<int32_t>());
    mark(1);
    hipLaunchKernelGGL(k_hash_map, dim3(nblk(2 * n)), dim3(LB_TPB), 0, s, n, b->d_msgs.as<uint8_t>(),
                       e->q.as<uint32_t>());
    mark(2);
    hipLaunchKernelGGL(k_hash_finish, dim3(nblk(n)), dim3(LB_TPB), 0, s, n, e->q.as<uint32_t>(),
                       e->h_aff.as<uint32_t>());
    mark(3);
    hipLaunchKernelGGL(k_pk_blind, dim3(nblk(n)), dim3(LB_TPB), 0, s, n, b->d_pk_off.as<uint32_t>(),
                       b->d_pks.as<uint8_t>(), e->scalars.as<uint64_t>(), e->sig_aff.as<uint32_t>(),
                       e->sig_inf.as<uint32_t>(), e->sig_status.as<int32_t>(), e->rpk.as<uint32_t>(),
                       e->rsig.as<uint32_t>(), e->pk_status.as<int32_t>());
    mark(4);
    hipLaunchKernelGGL(k_miller, dim3(nblk(n)), dim3(LB_TPB), 0, s, n, e->rpk.as<uint32_t>(),
                       e->h_aff.as<uint32_t>(), e->sig_status.as<int32_t>(), e->pk_status.as<int32_t>(),
                       e->ml.as<uint32_t>());
    mark(5);
  } else {
    for (int k = 1; k <= 5; k++) mark(k);
  }
  hipLaunchKernelGGL(k_job_leaves, dim3(nblk(m)), dim3(LB_TPB), 0, s, nj, n, m, b->d_job_off.as<uint32_t>(),
                     e->sig_status.as<int32_t>(), e->pk_status.as<int32_t>(), e->ml.as<uint32_t>(),
                     e->rsig.as<uint32_t>(), e->treeP.as<uint32_t>(), e->treeS.as<uint32_t>(),
                     e->job_status.as<int32_t>());
  mark(6);
  for (uint32_t lo = m / 2; lo >= 1; lo /= 2)
    hipLaunchKernelGGL(k_tree_up, dim3(lo + nblk(lo)), dim3(64), 0, s, m, lo, e->treeP.as<uint32_t>(),
                       e->treeS.as<uint32_t>());
  mark(7);
  LB_HIP(hipGetLastError());
  return LB_OK;
}

static int32_t check_nodes(lb_engine* e, uint32_t m, const std::vector<uint32_t>& nodes, std::vector<int32_t>& v) {
  uint32_t c = (uint32_t)nodes.size();
  v.assign(c, 0);
  if (!c) return LB_OK;
  LB_HIP(e->nodes.ensure((size_t)c * 4));
  LB_HIP(e->verdict.ensure((size_t)c * 4));
  LB_HIP(hipMemcpyAsync(e->nodes.p, nodes.data(), (size_t)c * 4, hipMemcpyHostToDevice, e->stream));
  hipLaunchKernelGGL(k_node_check, dim3(c), dim3(64), 0, e->stream, m, c, e->nodes.as<uint32_t>(),
                     e->treeP.as<uint32_t>(), e->treeS.as<uint32_t>(), e->verdict.as<int32_t>());
  LB_HIP(hipGetLastError());
  LB_HIP(hipMemcpyAsync(v.data(), e->verdict.p, (size_t)c * 4, hipMemcpyDeviceToHost, e->stream));
  LB_HIP(hipStreamSynchronize(e->stream));
  return LB_OK;
}

static void finish_profile(lb_engine* e, bool bisected) {
  if (!e->profiling) return;
  hipEventSynchronize(e->ev[kStages]);
  for (int k = 0; k < kStages; k++) {
    float ms = 0.f;
    if (k == kStages - 1 && !bisected) {
      e->last_ms[k] = 0.f;
      continue;
    }
    hipEventElapsedTime(&ms, e->ev[k], e->ev[k + 1]);
    e->last_ms[k] = ms;
  }
}

extern "C" int32_t lb_batch_verify(lb_engine* e, lb_batch* b, const uint64_t* scalars, int32_t* out_job) {
  if (!e || !b || (b->n_jobs && !out_job)) return LB_ERR_ARGUMENT;
  std::lock_guard<std::mutex> lk(e->mu);
  LB_HIP(hipSetDevice(e->device));
  const uint32_t nj = b->n_jobs;
  if (nj == 0) return LB_OK;
  uint32_t m = 1;
  int32_t st = run_pipeline(e, b, scalars, m);
  if (st != LB_OK) return st;
  std::vector<int32_t> jst(nj);
  LB_HIP(hipMemcpyAsync(jst.data(), e->job_status.p, (size_t)nj * 4, hipMemcpyDeviceToHost, e->stream));
  // subtree "live job" counts, heap layout (leaves at [m, 2m))
  std::vector<uint32_t> live(2 * m, 0);
  LB_HIP(hipStreamSynchronize(e->stream));
  for (uint32_t j = 0; j < nj; j++) live[m + j] = jst[j] == LB_OK ? 1u : 0u;
  for (uint32_t i = m - 1; i >= 1; i--) live[i] = live[2 * i] + live[2 * i + 1];
  for (uint32_t j = 0; j < nj; j++) out_job[j] = jst[j] == LB_OK ? 1 : -jst[j];
  std::vector<uint32_t> cand;
  std::vector<int32_t> v;
  if (live[1]) cand.push_back(1);
  bool first = true, bisected = false;
  while (!cand.empty()) {
    st = check_nodes(e, m, cand, v);
    if (st != LB_OK) return st;
    if (first) {
      if (e->profiling) hipEventRecord(e->ev[8], e->stream);
      first = false;
    } else {
      bisected = true;
    }
    std::vector<uint32_t> next;
    for (size_t k = 0; k < cand.size(); k++) {
      uint32_t c = cand[k];
      if (v[k]) continue;  // verified: its live jobs stay 1
      if (c >= m) {
        out_job[c - m] = 0;
        continue;
      }
      next.push_back(2 * c);
      next.push_back(2 * c + 1);
    }
    // drop empty subtrees; when the failing subtrees are small, test their leaves directly
    std::vector<uint32_t> nz;
    uint64_t leaves = 0;
    for (uint32_t c : next)
      if (live[c]) {
        nz.push_back(c);
        leaves += live[c];
      }
    if (!nz.empty() && leaves <= 256) {
      std::vector<uint32_t> lv;
      for (uint32_t c : nz) {
        uint32_t lo = c, hi = c;
        while (lo < m) {
          lo = 2 * lo;
          hi = 2 * hi + 1;
        }
        for (uint32_t l = lo; l <= hi; l++)
          if (live[l]) lv.push_back(l);
      }
      nz.swap(lv);
    }
    cand.swap(nz);
  }
  if (e->profiling) hipEventRecord(e->ev[kStages], e->stream);
  finish_profile(e, bisected);
  return LB_OK;
}

extern "C" int32_t lb_batch_partial(lb_engine* e, lb_batch* b, const uint64_t* scalars, uint8_t* out576,
                                    int32_t* out_job) {
  if (!e || !b || !out576 || (b->n_jobs && !out_job)) return LB_ERR_ARGUMENT;
  std::lock_guard<std::mutex> lk(e->mu);
  LB_HIP(hipSetDevice(e->device));
  uint32_t m = 1;
  if (b->n_jobs == 0) {
    fp12_to_be576(out576, fp12_one());
    return LB_OK;
  }
  int32_t st = run_pipeline(e, b, scalars, m);
  if (st != LB_OK) return st;
  LB_HIP(e->parts.ensure(576));
  hipLaunchKernelGGL(k_root_partial, dim3(1), dim3(64), 0, e->stream, m, e->treeP.as<uint32_t>(),
                     e->treeS.as<uint32_t>(), e->parts.as<uint8_t>());
  LB_HIP(hipGetLastError());
  std::vector<int32_t> jst(b->n_jobs);
  LB_HIP(hipMemcpyAsync(out576, e->parts.p, 576, hipMemcpyDeviceToHost, e->stream));
  LB_HIP(hipMemcpyAsync(jst.data(), e->job_status.p, (size_t)b->n_jobs * 4, hipMemcpyDeviceToHost, e->stream));
  if (e->profiling) {
    hipEventRecord(e->ev[8], e->stream);
    hipEventRecord(e->ev[9], e->stream);
  }
  LB_HIP(hipStreamSynchronize(e->stream));
  for (uint32_t j = 0; j < b->n_jobs; j++) out_job[j] = jst[j] == LB_OK ? 1 : -jst[j];
  finish_profile(e, false);
  return LB_OK;
}

extern "C" int32_t lb_fp12_product_is_one(lb_engine* e, const uint8_t* partials576, uint32_t n, int32_t* ok) {
  if (!e || !ok || (n && !partials576)) return LB_ERR_ARGUMENT;
  std::lock_guard<std::mutex> lk(e->mu);
  LB_HIP(hipSetDevice(e->device));
  LB_HIP(e->parts.ensure((size_t)(n ? n : 1) * 576));
  LB_HIP(e->ok.ensure(4));
  if (n) LB_HIP(hipMemcpyAsync(e->parts.p, partials576, (size_t)n * 576, hipMemcpyHostToDevice, e->stream));
  hipLaunchKernelGGL(k_partials_check, dim3(1), dim3(64), 0, e->stream, n, e->parts.as<uint8_t>(),
                     e->ok.as<int32_t>());
  LB_HIP(hipGetLastError());
  LB_HIP(hipMemcpyAsync(ok, e->ok.p, 4, hipMemcpyDeviceToHost, e->stream));
  LB_HIP(hipStreamSynchronize(e->stream));
  return LB_OK;
}

extern "C" int32_t lb_verify_jobs(lb_engine* e, uint32_t n_jobs, const uint32_t* job_offsets,
                                  const uint32_t* set_pk_offsets, const uint8_t* pubkeys,
                                  const uint8_t* signing_roots, const uint8_t* signatures,
                                  const uint32_t* sig_sizes, const uint64_t* scalars, int32_t* out_job) {
  lb_batch* b = nullptr;
  int32_t st = lb_batch_create(e, n_jobs, job_offsets, set_pk_offsets, pubkeys, signing_roots, signatures,
                               sig_sizes, &b);
  if (st != LB_OK) return st;
  st = lb_batch_verify(e, b, scalars, out_job);
  lb_batch_destroy(b);
  return st;
}

extern "C" int32_t lb_aggregate_pubkeys(lb_engine* e, uint32_t n_sets, const uint32_t* set_pk_offsets,
                                        const uint8_t* pubkeys, uint8_t* out96, int32_t* out_status) {
  if (!e || !set_pk_offsets || (n_sets && (!out96 || !out_status))) return LB_ERR_ARGUMENT;
  if (set_pk_offsets[0] != 0) return LB_ERR_ARGUMENT;
  for (uint32_t i = 0; i < n_sets; i++)
    if (set_pk_offsets[i + 1] < set_pk_offsets[i]) return LB_ERR_ARGUMENT;
  uint32_t n_pks = set_pk_offsets[n_sets];
  if (n_pks && !pubkeys) return LB_ERR_ARGUMENT;
  if (!n_sets) return LB_OK;
  std::lock_guard<std::mutex> lk(e->mu);
  LB_HIP(hipSetDevice(e->device));
  dbuf off, pk, out, stat;
  hipError_t r = off.ensure((size_t)(n_sets + 1) * 4);
  if (r == hipSuccess) r = pk.ensure((size_t)(n_pks ? n_pks : 1) * 96);
  if (r == hipSuccess) r = out.ensure((size_t)n_sets * 96);
  if (r == hipSuccess) r = stat.ensure((size_t)n_sets * 4);
  if (r == hipSuccess)
    r = hipMemcpyAsync(off.p, set_pk_offsets, (size_t)(n_sets + 1) * 4, hipMemcpyHostToDevice, e->stream);
  if (r == hipSuccess && n_pks) r = hipMemcpyAsync(pk.p, pubkeys, (size_t)n_pks * 96, hipMemcpyHostToDevice, e->stream);
  if (r == hipSuccess) {
    hipLaunchKernelGGL(k_aggregate, dim3(nblk(n_sets)), dim3(LB_TPB), 0, e->stream, n_sets, off.as<uint32_t>(),
                       pk.as<uint8_t>(), out.as<uint8_t>(), stat.as<int32_t>());
    r = hipGetLastError();
  }
  if (r == hipSuccess) r = hipMemcpyAsync(out96, out.p, (size_t)n_sets * 96, hipMemcpyDeviceToHost, e->stream);
  if (r == hipSuccess) r = hipMemcpyAsync(out_status, stat.p, (size_t)n_sets * 4, hipMemcpyDeviceToHost, e->stream);
  if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
  off.release();
  pk.release();
  out.release();
  stat.release();
  if (r != hipSuccess) {
    fprintf(stderr, "lodestar_bls: aggregate failed: %s\n", hipGetErrorString(r));
    return LB_ERR_DEVICE;
  }
  return LB_OK;
}

// Generic "n items in, per-item outputs back" launcher for the small helper kernels.
namespace {
struct io_spec {
  const void* src;
  size_t bytes;
  bool out;  // copy back after the launch
  void* dst;
};
}  // namespace

template <class Launch>
static int32_t run_simple(lb_engine* e, std::vector<io_spec> io, Launch launch) {
  std::lock_guard<std::mutex> lk(e->mu);
  LB_HIP(hipSetDevice(e->device));
  std::vector<dbuf> bufs(io.size());
  hipError_t r = hipSuccess;
  for (size_t k = 0; k < io.size() && r == hipSuccess; k++) {
    r = bufs[k].ensure(io[k].bytes ? io[k].bytes : 16);
    if (r == hipSuccess && !io[k].out && io[k].bytes)
      r = hipMemcpyAsync(bufs[k].p, io[k].src, io[k].bytes, hipMemcpyHostToDevice, e->stream);
  }
  if (r == hipSuccess) {
    std::vector<void*> ptrs;
    for (auto& b : bufs) ptrs.push_back(b.p);
    launch(ptrs);
    r = hipGetLastError();
  }
  for (size_t k = 0; k < io.size() && r == hipSuccess; k++)
    if (io[k].out && io[k].dst && io[k].bytes)
      r = hipMemcpyAsync(io[k].dst, bufs[k].p, io[k].bytes, hipMemcpyDeviceToHost, e->stream);
  if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
  for (auto& b : bufs) b.release();
  if (r != hipSuccess) {
    fprintf(stderr, "lodestar_bls: helper kernel failed: %s\n", hipGetErrorString(r));
    return LB_ERR_DEVICE;
  }
  return LB_OK;
}

extern "C" int32_t lb_g1_decompress(lb_engine* e, uint32_t n, const uint8_t* in48, uint8_t* out96,
                                    int32_t* out_status, int32_t validate) {
  if (!e || (n && (!in48 || !out96 || !out_status))) return LB_ERR_ARGUMENT;
  if (!n) return LB_OK;
  return run_simple(e, {{in48, (size_t)n * 48, false, nullptr}, {nullptr, (size_t)n * 96, true, out96},
                        {nullptr, (size_t)n * 4, true, out_status}},
                    [&](std::vector<void*>& p) {
                      hipLaunchKernelGGL(k_g1_decompress, dim3(nblk(n)), dim3(LB_TPB), 0, e->stream, n,
                                         (const uint8_t*)p[0], (uint8_t*)p[1], (int32_t*)p[2], validate);
                    });
}

extern "C" int32_t lb_sk_to_pk(lb_engine* e, uint32_t n, const uint8_t* sks32, uint8_t* out48, uint8_t* out96) {
  if (!e || (n && !sks32)) return LB_ERR_ARGUMENT;
  if (!n) return LB_OK;
  return run_simple(e, {{sks32, (size_t)n * 32, false, nullptr}, {nullptr, (size_t)n * 48, true, out48},
                        {nullptr, (size_t)n * 96, true, out96}},
                    [&](std::vector<void*>& p) {
                      hipLaunchKernelGGL(k_sk_to_pk, dim3(nblk(n)), dim3(LB_TPB), 0, e->stream, n,
                                         (const uint8_t*)p[0], (uint8_t*)p[1], (uint8_t*)p[2]);
                    });
}

extern "C" int32_t lb_sign(lb_engine* e, uint32_t n, const uint8_t* sks32, const uint8_t* msgs32, uint8_t* out96) {
  if (!e || (n && (!sks32 || !msgs32 || !out96))) return LB_ERR_ARGUMENT;
  if (!n) return LB_OK;
  return run_simple(e, {{sks32, (size_t)n * 32, false, nullptr}, {msgs32, (size_t)n * 32, false, nullptr},
                        {nullptr, (size_t)n * 96, true, out96}},
                    [&](std::vector<void*>& p) {
                      hipLaunchKernelGGL(k_sign, dim3(nblk(n)), dim3(LB_TPB), 0, e->stream, n,
                                         (const uint8_t*)p[0], (const uint8_t*)p[1], (uint8_t*)p[2]);
                    });
}
