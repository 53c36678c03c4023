// C-ABI engine (include/lodestar_bls.h) driving the gfx950 pipeline of lb_kernels.h.
//
// One engine per GPU, one HIP stream per engine; calls on one engine are serialised by a
// mutex (the reference's worker pool runs one job package per worker at a time,
// multithread/index.ts:290-381).  Inputs are copied into device memory at batch creation
// (the reference structured-clones its BlsWorkReq[], multithread/index.ts:330), so the
// caller never has to keep its buffers alive.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "lb_kernels.h"
#include "lb_kzg.h"
#include "lb_kdecl.h"  // kernels of the other translation units (split build)

#define LB_ABI_VERSION 1

namespace {

struct dbuf {
  void* p = nullptr;
  size_t cap = 0;
  bool view = false;  // p points into another buffer (a batch's upload arena): never freed here
  hipError_t ensure(size_t bytes) {
    if (view) {
      p = nullptr;
      cap = 0;
      view = false;
    }
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
    if (p && !view) hipFree(p);
    p = nullptr;
    cap = 0;
    view = false;
  }
  void set_view(void* q, size_t bytes) {
    if (p && !view) hipFree(p);
    p = q;
    cap = bytes;
    view = true;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

// Pipeline stages; (s1) / (s2) = the HIP stream a stage runs on.  s2 carries signature decode,
// pubkey aggregation + blinding and the whole sum(r_i sig_i) branch; s1 groups the sets by
// signing root, hashes each distinct root, sums r_i PK_i per root and runs one Miller loop per
// root into the message product tree.  They join before the root check.  Only a failing root
// runs the per-set fallback (per-set Miller loops + the job tree) and the bisection.
enum {
  ST_DECODE = 0,  // s2
  ST_DEDUP,       // s1
  ST_HASH_MAP,    // s1
  ST_HASH_FIN,    // s1
  ST_PK_CHUNKS,   // s2
  ST_PK_BLIND,    // s2
  ST_SIG_MSM,     // s2
  ST_GSUM,        // s1
  ST_MILLER,      // s1
  ST_TREE_P,      // s1
  ST_ML_S,        // s2
  ST_ROOT,        // s1 (after joining s2)
  ST_FALLBACK,    // s1: invalid-set search, range MSMs + part sums
  ST_BISECT,      // s1: invalid-set search, node checks
  ST_TOTAL,
  kStages
};
const char* const kStageNames[kStages] = {"decode_sigs", "dedup",   "hash_map", "hash_finish", "pk_chunks",
                                          "pk_blind",    "sig_msm", "group_sum", "miller",    "tree_up_P",
                                          "ml_S",        "root_check", "search_msm", "search_check", "total"};

}  // namespace

struct lb_batch {
  uint32_t n_jobs = 0, n_sets = 0, n_pks = 0;
  // unique per upload (batch_fill): lb_batch_search_after_partial matches on it, not on the
  // address, which a freed batch's successor may reuse
  uint64_t serial = 0;
  std::vector<uint32_t> job_off;  // host copy (bisection bookkeeping)
  std::vector<uint32_t> h_set_chunk_off, h_chunk_lo;  // host staging of the chunk decomposition
  uint32_t n_chunks = 0;           // pubkey aggregation chunks (k_pk_chunks)
  bool indexed = false;            // pubkeys are indices into the engine's resident table
  dbuf d_job_off, d_pk_off, d_pks, d_msgs, d_sigs, d_sig_sizes, d_set_chunk_off, d_chunk_lo;
  dbuf d_arena;  // small uploads: the arrays above as views into one buffer, filled by one copy
  bool has_sizes = false;
  int device = 0;
  ~lb_batch() {
    d_job_off.release();
    d_arena.release();
    d_pk_off.release();
    d_pks.release();
    d_msgs.release();
    d_sigs.release();
    d_sig_sizes.release();
    d_set_chunk_off.release();
    d_chunk_lo.release();
  }
};

#ifndef LB_SEARCH_CHUNK_DEF
#define LB_SEARCH_CHUNK_DEF 8
#endif
struct lb_engine {
  int device = 0;
  // LB_ENGINE_LATENCY (lb_engine_create_ex): streams confined to the device's reserved CUs, the
  // latency forms always (the partition keeps every other engine off those CUs)
  bool latency = false;
  int n_cus = 0;  // CUs its streams may use (the whole device, or one side of the partition)
  hipStream_t stream = nullptr;   // s1
  hipStream_t stream2 = nullptr;  // s2
  hipStream_t stream3 = nullptr;  // s3: pubkey aggregation + blinding, beside the signature decode
  // LB_PRIO_MAX=k: batches of at most k sets run on a second stream trio created at the device's
  // greatest priority (created on first use).  Off by default: measured through the JS drop-in,
  // verifyOnMainThread under a gossip load took 396-758 ms with it against 9.0-9.2 ms without,
  // and the pool's throughput fell 3-5x (profiles/r5_prio_streams_ab.txt)
  hipStream_t hp[3] = {nullptr, nullptr, nullptr};
  uint32_t prio_max = 0;
  hipEvent_t ev_g1 = nullptr, ev_s = nullptr, ev_fork = nullptr, ev_dec = nullptr, ev_pk = nullptr;
  hipEvent_t ev_pkst = nullptr;  // the pubkey statuses (k_pk_blind mode 1), before the ladder
  // small batches alone (round 6): the decoded signatures (s2) -> r_i sig_i on s3 beside the
  // subgroup check (ev_sdec), and the terms ready for the sum on s2 (ev_sblind)
  hipEvent_t ev_sdec = nullptr, ev_sblind = nullptr;
  std::mutex mu;
  // workspace
  dbuf scalars, sig_aff, sig_inf, sig_status, q, h_aff, rpk, rsig, pk_status, ml, treeP, treeS, job_status,
      nodes, verdict, parts, ok, chunk_acc, chunk_status, fS;
  // message grouping (k_msg_*, k_gsum_*)
  dbuf msg_tab, rep_of, uid_of, uniq_set, n_u, set_uid, gcnt, gpos, goff, gch, chunk_beg, chunk_end, members,
      set_live, gacc, gp_aff, gp_inf, chunk_root;
  uint32_t gmax_chunks = 0;  // chunks of the largest root (the k_gsum_tree levels), read back with n_u
  // under load (not alone) the per-root sums fold the blinding in, one Straus chain per chunk
  // (k_gsum_straus over pk3) instead of k_pk_blind's per-set ladder + the chunk sums; the per-set
  // r PK (rpk) are then computed only if a search needs them (rpk_stale).  LB_GSUM_STRAUS=1: on.
  // Off by default: measured 4 % below the per-set ladders at 7 in flight even with the chunks in
  // size order (10.53-10.59 M against 11.01-11.03 M sets/s, profiles/r6_straus_ab.txt)
  bool straus = false, straus_run = false, rpk_stale = false;
  // a batch alone: the per-root sums' chunks combined by a segmented shuffle tree in one launch
  // (k_gsum_wave, chunks of LB_GROUP_CHUNK_WAVE) instead of the k_gsum_tree launches; LB_GSUM_WAVE=0
  bool gsum_wave = true;
  dbuf pk3, corder;  // (x, y, beta x) per set; the Straus lanes' chunk order (+ size counts)
  bool gsum_tree = true;     // LB_GSUM_TREE=0: the chunk sums added serially per root (A/B)
  // this pipeline run's forms: `alone` (device_alone at its start) picks the latency forms -- the
  // row engine (row_fe: LB_ROW_FE=0 disables it) and the per-root sum tree over 8-member chunks
  bool alone = false, row_fe = true;
  int alone_force = -1;  // LB_ALONE=1 / 0 pins device_alone() (tests: the latency forms must run), -1 by load
  uint32_t gchunk = LB_GROUP_CHUNK;
  // bucket MSM for sum r_i sig_i (k_msm_*)
  dbuf sig_aos, bcnt, bcursor, boff, bch, bchunk_beg, bchunk_end, bmembers, bacc, bsum, wsum;
  // parked lone-lane state: k_hash_finish's points (4 x 72 words per launched lane), k_miller_lane's T
  dbuf park;
  // per-root chain on speculative liveness (pubkey statuses only), started after the pubkey side
  // instead of after the signature decode; redone with the full statuses only when a set's
  // signature failed to decode (k_live_mismatch).  LB_SPEC_GSUM=1; off by default: measured no
  // gain, the streams then contend for a chip one batch already fills (profiles/r4_spec_ab.txt)
  bool spec_gsum = false;
  dbuf set_spec, live_flag;
  uint32_t* h_flag = nullptr;
  // serial of the batch upload whose lb_batch_partial left its state (trees, statuses, scalars) in
  // this engine's workspace, for lb_batch_search_after_partial; any other pipeline run clears it
  uint64_t partial_serial = 0;
  uint32_t partial_mu = 0;
  // bucket sums and the bucket reduction by 8-lane groups (k_msm_buckets_g8, k_msm_window_g8,
  // k_msm_horner_g8); LB_MSM_G8=0: the lone-lane kernels (k_msm_buckets, k_msm_reduce)
  bool msm_g8 = true;
  // invalid-set search (search_invalid): node descriptors and per-node results
  dbuf sx[32];   // search round buffers (search_invalid: SX_*)
  dbuf pk_aff;  // affine aggregate pubkey per set (single-set checks of the search)
  dbuf y_root;  // FE value of the root check (the search starts from it)
  uint64_t msg_key = 0;  // keyed probe hash (CSPRNG)
  // batches with at most this many distinct roots run their Miller loops one wave per root
  // (k_miller_wave); larger ones one lane per root (k_miller_lane) while other batches are in
  // flight on the device, else 8 lanes per root (k_miller_g8).  LB_MILLER_WAVE_MAX;
  // LB_MILLER_FORM = lane | g8 pins the large-batch form (default: by device load).
  uint32_t miller_wave_max = 2048;
  // ... and up to this many roots (tree nodes of a level) on the row engine (lb_row.h: one 16-wave
  // workgroup per item, the products split over 16-lane rows; latency).  LB_ROW_MAX.
  uint32_t row_max = 256;
  int miller_form = 0;  // 0 by load, 1 lane, 2 g8
  // one-lane Miller loops with f and a temporary in LDS (two waves per CU) up to this many roots,
  // f alone in LDS (one wave per SIMD) above: LB_MILLER_LDS3_MAX (lb_kernels.h k_miller_lane)
  uint32_t miller_lds3_max = 32768;
  // ... and hash_to_G2's cofactor clearing with 8 lanes per root (k_hash_finish_g8).  LB_HASH_G8_MAX.
  uint32_t hash_g8_max = 2048;
  // ... and with a workgroup per root on the row engine while the device is alone.  LB_HASH_ROW_MAX.
  uint32_t hash_row_max = 256;
  uint32_t hash_row_careful = 0;  // LB_HASH_ROW_CAREFUL=1: the exceptional-case path always (tests)
  // round 6: the row forms' G2 chains (cofactor clearing, the subgroup ladder, r_i sig_i) in
  // projective coordinates with the complete formulas; LB_ROW_PROJ=0: the Jacobian programs
  bool row_proj = true;
  // round 6, small batches alone: the r PK ladder on rows and r_i sig_i on s3 beside the
  // subgroup check; LB_SMALL_PAR=0: both on their round-5 streams and forms (A/B)
  bool small_par = true;
  // ... and the signature decode's square roots on rows up to this many sets.  LB_DEC_ROW_MAX.
  uint32_t dec_row_max = 4096;
  // ... and the signatures' subgroup check with 8 lanes per set (k_sig_subgroup_g8).  LB_SUBGROUP_G8_MAX.
  uint32_t subgroup_g8_max = 4096;
  // ... and S = sum r_i sig_i by per-set 8-lane scalar multiplications + trees instead of the
  // bucket MSM (k_sig_blind_g8).  LB_SMALL_S_MAX.
  uint32_t small_s_max = 32768;
  uint32_t small_s_g8_max = 2048;  // ... with 8 lanes per set up to here, one lane above (LB_SMALL_S_G8_MAX)
  // search rounds whose weighted sums cover at most this many positions skip the bucket MSM
  // (k_smsm_terms_g8 + segmented sums).  LB_SEARCH_SMALL_MAX.
  uint32_t search_small_max = 32768;
  // one launch pair per search round (look-ahead tests not skipped for passing checks)
  bool search_merge = true;
  dbuf s_terms, s_part;
  // per-root signature sums for the search's root-level instances (LB_SEARCH_ROOTSUM)
  dbuf s_root, rs_idx, s_set;
  bool search_rootsum = true;
  bool search_pre = false;  // later rounds take [w] of the kept per-set terms (LB_SEARCH_PRE)
  // the small rounds' per-position terms: 0 by load (8 lanes per position while the device runs no
  // other batch, one lane under load), 1 one lane, 2 eight lanes (LB_SMSM_FORM=lane / g8)
  int smsm_form = 0;
  // members per lane in the search rounds' bucket MSM chunks (k_msm_chunks).  Its buckets hold ~8
  // members (109 instances x 1 024 buckets over ~0.9 M entries), so long chunks leave most lanes
  // of a wave idle behind the longest one; LB_SEARCH_CHUNK
  uint32_t search_chunk = LB_SEARCH_CHUNK_DEF;
  // large batches: the first round checks the root tree's top subtrees directly, their S_j from
  // one 4-window bucket MSM over all sets, without look-ahead tests and without the per-root sums
  // (one GLV ladder per set); LB_SEARCH_BLOCKS=0 restores the per-root sums + look-ahead round
  bool search_blk = true;
  // distinct roots numbered in hash-table order (pseudo-random) rather than input order, so the
  // search's first-round subtrees hold comparable numbers of sets (LB_ROOT_SHUFFLE=0: input order)
  bool root_shuffle = true;
  std::vector<uint64_t> h_scalars;
  // resident pubkey table: one 128-byte record per key (g1a + flag, LB_TABLE_REC words)
  dbuf table;
  uint32_t table_n = 0, table_cap = 0;
  // KZG trusted setup (lb_kzg_load_setup): [tau^i] G1 as g1a SoA (kzg_n entries), [tau^0,1] G2
  dbuf kzg_g1, kzg_g2;
  uint32_t kzg_n = 0;
  // profiling
  bool profiling = false;
  hipEvent_t ev0[kStages] = {}, ev1[kStages] = {};
  bool used[kStages] = {};
  float last_ms[kStages] = {};
  float acc_ms[kStages] = {};  // stages run once per search round: summed over the rounds
  // pinned host word for the distinct-root count read back after grouping: the per-root kernels
  // are launched over that count, not over the set count (their scratch is sized per dispatch)
  uint32_t* h_nu = nullptr;
  void* h_stage = nullptr;  // pinned staging of small batch uploads (batch_fill, under mu)
  size_t h_stage_cap = 0;
  // engine-owned input workspace reused by lb_verify_jobs* (no per-call device allocation)
  lb_batch* scratch = nullptr;
};

// Engines per device are capped so that one process cannot create more concurrently active
// HIP streams than the device can back with queues and scratch (exhaustion aborts the HSA queue
// asynchronously instead of returning an error).  LB_MAX_ENGINES_PER_DEVICE overrides the cap.
// Round 4: 7 -> 10.  Every queue's scratch is reserved for the largest private segment it runs
// times the device's wave capacity; with the per-root kernels at <= 2.7 KB per lane (k_miller_lane
// was 6.7 KB) 8 and 10 engines run without an abort (profiles/r4_engines_ab.txt), and
// lb_engine_create reserves each engine's s1 scratch up front (above).
static std::mutex g_engine_mu;
static int g_engine_count[64];
static std::atomic<uint64_t> g_batch_serial{0};
// Batches currently inside the pipeline per device (all engines of the process).  With more than
// one, the device is throughput-bound and the per-root kernels take their work-efficient forms.
#ifndef LB_HASH_ALONE_G8
#define LB_HASH_ALONE_G8 1  // cofactor clearing by 8-lane groups whenever the device is otherwise idle (0: by root count only)
#endif
static std::atomic<int> g_device_busy[64];
// The two most recent pipeline exits per device by distinct engines (steady-clock ns): exit[0] the
// latest, exit[1] the latest of any other engine than exit[0]'s, so an engine can ask when ANOTHER
// engine last left the pipeline (round-4 ADVICE: one slot let an engine that left 1 ms after
// another see the device as idle while the other was between two batches)
struct exit_rec {
  const void* eng = nullptr;
  int64_t ns = 0;
};
static std::mutex g_exit_mu[64];
static exit_rec g_device_exit[64][2];
static int64_t lb_now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// CUs reserved for latency engines per device (0: no partition); engines created while a
// partition exists run on the complement.  LB_LATENCY_CUS (default 8 of the device's CUs).  The
// partition lives as long as a latency engine does (g_latency_live counts them): after the last
// one is destroyed, engines created later get the whole device again (round-5 ADVICE).
static int g_latency_cus[64];
static int g_latency_live[64];
struct busy_scope {
  int dev;
  const void* eng;
  bool counted;
  busy_scope(int d, const void* e, bool latency = false) : dev(d), eng(e), counted(!latency) {
    if (counted) g_device_busy[dev].fetch_add(1, std::memory_order_relaxed);
  }
  ~busy_scope() {
    if (!counted) return;  // a latency engine's calls run on its own CUs: not load for the others
    {
      std::lock_guard<std::mutex> lk(g_exit_mu[dev]);
      exit_rec* r = g_device_exit[dev];
      if (r[0].eng != eng) r[1] = r[0];
      r[0] = exit_rec{eng, lb_now_ns()};
    }
    g_device_busy[dev].fetch_sub(1, std::memory_order_relaxed);
  }
};
// The device runs no other batch: none inside the pipeline, and no OTHER engine's batch left it
// within the last LB_ALONE_GRACE_MS (an in-flight engine's host thread between two batches is
// still load: at 7 in flight those gaps sent batches to the latency forms, ~2 % of the headline,
// profiles/r4_regress_ab.txt)
#ifndef LB_ALONE_GRACE_MS
#define LB_ALONE_GRACE_MS 20
#endif
template <class E>
static bool device_alone(const E* e) {
  if (e->latency) return true;  // its reserved CUs run nothing else
  if (e->alone_force >= 0) return e->alone_force != 0;
  if (g_device_busy[e->device].load(std::memory_order_relaxed) > 1) return false;
  int64_t other;
  {
    std::lock_guard<std::mutex> lk(g_exit_mu[e->device]);
    const exit_rec* r = g_device_exit[e->device];
    other = r[0].eng != (const void*)e ? r[0].ns : r[1].ns;
  }
  return other == 0 || lb_now_ns() - other > (int64_t)LB_ALONE_GRACE_MS * 1000000;
}
static int max_engines_per_device() {
  const char* v = getenv("LB_MAX_ENGINES_PER_DEVICE");
  int k = v ? atoi(v) : 0;
  return k > 0 ? k : 10;  // the highest engine count measured abort-free (profiles/r4_engines_ab.txt)
}

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
static inline uint32_t nblk_inv(uint32_t n) { return (n + LB_INV_TPB - 1) / LB_INV_TPB; }

// unblinded: the verdict of this run covers exactly this batch (lb_batch_verify / lb_verify_jobs*),
// so a 1-set batch may verify unblinded as Signature.verify does.  A partial product that is
// multiplied with other ranks' partials (lb_batch_partial) is always blinded: two unblinded 1-set
// partials sig_A + D and sig_B - D would cancel in the product (round-5 ADVICE).
static int fill_scalars(lb_engine* e, uint32_t n, const uint64_t* user, bool unblinded) {
  e->h_scalars.resize(n);
  if (!user && n == 1 && unblinded) {
    e->h_scalars[0] = 1;  // one set: verified unblinded (k_sig_unblinded), as Signature.verify
    return LB_OK;
  }
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

int32_t lb_engine_create(int32_t device, lb_engine** out) { return lb_engine_create_ex(device, 0u, out); }
// a CU mask over [lo, hi) of ncu CUs (32 per word)
static std::vector<uint32_t> cu_mask(int ncu, int lo, int hi) {
  std::vector<uint32_t> m((size_t)(ncu + 31) / 32, 0u);
  for (int c = lo; c < hi && c < ncu; c++) m[(size_t)c / 32] |= 1u << (c % 32);
  return m;
}
int32_t lb_engine_create_ex(int32_t device, uint32_t flags, lb_engine** out) {
  if (!out || (flags & ~LB_ENGINE_LATENCY)) return LB_ERR_ARGUMENT;
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
  if (device >= 64) return LB_ERR_NO_DEVICE;
  {
    std::lock_guard<std::mutex> lk(g_engine_mu);
    if (g_engine_count[device] >= max_engines_per_device()) {
      fprintf(stderr, "lodestar_bls: engine limit (%d per device) reached on device %d\n", max_engines_per_device(),
              device);
      return LB_ERR_DEVICE;
    }
    g_engine_count[device]++;
  }
  lb_engine* e = new lb_engine();
  e->device = device;
  while (getrandom(&e->msg_key, 8, 0) != 8) {
  }
  // s1 carries the latency-bound chain (grouping, per-root hashing and Miller loops, the root
  // check, the invalid-set search), created at the least stream priority as measured: the
  // greatest priority for it cost the headline 2-3 % and did not help the search (round 3,
  // profiles/r3_search_split_ab.txt)
  int prio_least = 0, prio_greatest = 0;
  hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest);
  if (const char* mw = getenv("LB_MILLER_WAVE_MAX")) e->miller_wave_max = (uint32_t)strtoul(mw, nullptr, 10);
  if (const char* rm = getenv("LB_ROW_MAX")) e->row_max = (uint32_t)strtoul(rm, nullptr, 10);
  if (const char* gt = getenv("LB_GSUM_TREE")) e->gsum_tree = std::atoi(gt) != 0;
  if (const char* gs = getenv("LB_GSUM_STRAUS")) e->straus = std::atoi(gs) != 0;
  if (const char* gw = getenv("LB_GSUM_WAVE")) e->gsum_wave = std::atoi(gw) != 0;
  if (const char* rf = getenv("LB_ROW_FE")) e->row_fe = std::atoi(rf) != 0;
  if (const char* pm = getenv("LB_PRIO_MAX")) e->prio_max = (uint32_t)strtoul(pm, nullptr, 10);
  if (const char* ml = getenv("LB_MILLER_LDS3_MAX")) e->miller_lds3_max = (uint32_t)strtoul(ml, nullptr, 10);
  if (const char* mf = getenv("LB_MILLER_FORM")) e->miller_form = !strcmp(mf, "lane") ? 1 : !strcmp(mf, "g8") ? 2 : 0;
  if (const char* hg = getenv("LB_HASH_G8_MAX")) e->hash_g8_max = (uint32_t)strtoul(hg, nullptr, 10);
  if (const char* hr = getenv("LB_HASH_ROW_MAX")) e->hash_row_max = (uint32_t)strtoul(hr, nullptr, 10);
  if (const char* dr = getenv("LB_DEC_ROW_MAX")) e->dec_row_max = (uint32_t)strtoul(dr, nullptr, 10);
  if (const char* hc = getenv("LB_HASH_ROW_CAREFUL")) e->hash_row_careful = (uint32_t)strtoul(hc, nullptr, 10);
  if (const char* rp = getenv("LB_ROW_PROJ")) e->row_proj = std::atoi(rp) != 0;
  if (const char* sp = getenv("LB_SMALL_PAR")) e->small_par = std::atoi(sp) != 0;
  if (const char* sg = getenv("LB_SUBGROUP_G8_MAX")) e->subgroup_g8_max = (uint32_t)strtoul(sg, nullptr, 10);
  if (const char* ss = getenv("LB_SMALL_S_MAX")) e->small_s_max = (uint32_t)strtoul(ss, nullptr, 10);
  if (const char* sg8 = getenv("LB_SMALL_S_G8_MAX")) e->small_s_g8_max = (uint32_t)strtoul(sg8, nullptr, 10);
  if (const char* sm = getenv("LB_SEARCH_SMALL_MAX")) e->search_small_max = (uint32_t)strtoul(sm, nullptr, 10);
  if (const char* sm = getenv("LB_SEARCH_MERGE")) e->search_merge = std::atoi(sm) != 0;
  if (const char* sm = getenv("LB_SEARCH_ROOTSUM")) e->search_rootsum = std::atoi(sm) != 0;
  if (const char* sm = getenv("LB_SEARCH_PRE")) e->search_pre = std::atoi(sm) != 0;
  if (const char* sf = getenv("LB_SMSM_FORM")) e->smsm_form = !strcmp(sf, "lane") ? 1 : !strcmp(sf, "g8") ? 2 : 0;
  if (const char* sc = getenv("LB_SEARCH_CHUNK")) {
    const uint32_t v = (uint32_t)strtoul(sc, nullptr, 10);
    if (v >= 1 && v <= 64) e->search_chunk = v;
  }
  if (const char* sm = getenv("LB_SEARCH_BLOCKS")) e->search_blk = std::atoi(sm) != 0;
  if (const char* sm = getenv("LB_ROOT_SHUFFLE")) e->root_shuffle = std::atoi(sm) != 0;
  if (const char* sm = getenv("LB_MSM_G8")) e->msm_g8 = std::atoi(sm) != 0;
  if (const char* sm = getenv("LB_SPEC_GSUM")) e->spec_gsum = std::atoi(sm) != 0;
  if (const char* al = getenv("LB_ALONE")) e->alone_force = std::atoi(al) != 0 ? 1 : 0;
  // CU partition: a latency engine's streams on the reserved CUs [0, R), every engine created
  // while a partition exists on [R, ncu)
  bool masked = false;
  std::vector<uint32_t> mask;
  {
    std::lock_guard<std::mutex> lk(g_engine_mu);
    const int ncu = prop.multiProcessorCount;
    e->n_cus = ncu;
    if (flags & LB_ENGINE_LATENCY) {
      if (g_latency_cus[device] == 0) {
        const char* v = getenv("LB_LATENCY_CUS");
        const int r = v ? atoi(v) : 8;
        g_latency_cus[device] = std::max(1, std::min(r, ncu / 4));
        // engines created before the partition keep the whole device (their streams exist):
        // they share the reserved CUs, which only costs the latency engine its isolation
        if (g_engine_count[device] > 1)
          fprintf(stderr, "lodestar_bls: latency engine created after %d other engine(s) on device %d: "
                  "those still run on every CU (create the latency engine first)\n", g_engine_count[device] - 1, device);
      }
      g_latency_live[device]++;
      e->latency = true;
      mask = cu_mask(ncu, 0, g_latency_cus[device]);
      e->n_cus = g_latency_cus[device];
      masked = true;
    } else if (g_latency_cus[device] > 0) {
      mask = cu_mask(ncu, g_latency_cus[device], ncu);
      e->n_cus = ncu - g_latency_cus[device];
      masked = true;
    }
  }
  auto mk = [&](hipStream_t* st, bool prio) {
    if (masked) return hipExtStreamCreateWithCUMask(st, (uint32_t)mask.size(), mask.data());
    return prio ? hipStreamCreateWithPriority(st, hipStreamNonBlocking, prio_least)
                : hipStreamCreateWithFlags(st, hipStreamNonBlocking);
  };
  if (mk(&e->stream, true) != hipSuccess || mk(&e->stream2, false) != hipSuccess || mk(&e->stream3, false) != hipSuccess ||

      hipHostMalloc((void**)&e->h_nu, 8, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&e->h_flag, 4, hipHostMallocDefault) != hipSuccess) {
    if (e->stream) hipStreamDestroy(e->stream);
    if (e->stream2) hipStreamDestroy(e->stream2);
    if (e->stream3) hipStreamDestroy(e->stream3);
    if (e->h_nu) hipHostFree(e->h_nu);
    std::lock_guard<std::mutex> lk(g_engine_mu);
    g_engine_count[device]--;
    if (e->latency && --g_latency_live[device] == 0) g_latency_cus[device] = 0;
    delete e;
    return LB_ERR_DEVICE;
  }
  hipEventCreateWithFlags(&e->ev_g1, hipEventDisableTiming);
  hipEventCreateWithFlags(&e->ev_s, hipEventDisableTiming);
  hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming);
  hipEventCreateWithFlags(&e->ev_dec, hipEventDisableTiming);
  hipEventCreateWithFlags(&e->ev_pk, hipEventDisableTiming);
  hipEventCreateWithFlags(&e->ev_pkst, hipEventDisableTiming);
  hipEventCreateWithFlags(&e->ev_sdec, hipEventDisableTiming);
  hipEventCreateWithFlags(&e->ev_sblind, hipEventDisableTiming);
  for (int i = 0; i < kStages; i++) {
    hipEventCreate(&e->ev0[i]);
    hipEventCreate(&e->ev1[i]);
  }
  // Reserve the streams' scratch now, one engine at a time, for the largest private segments they
  // can run (s1: k_miller_lane<2>, 2.7 KB per lane): empty dispatches over more waves than the
  // device holds.
  // The runtime sizes a queue's scratch for the largest segment it has run, from one per-process
  // pool, and a queue that cannot grow it mid-run aborts asynchronously; growing it here, with the
  // stream synchronised, turns an exhausted pool into LB_ERR_DEVICE from lb_engine_create.
  {
    bool ok;
    {
      std::lock_guard<std::mutex> lk(g_engine_mu);
      ok = e->n_u.ensure(4) == hipSuccess && hipMemsetAsync(e->n_u.p, 0, 4, e->stream) == hipSuccess;
      if (ok) {
        hipLaunchKernelGGL(k_miller_lane<2>, dim3(4096), dim3(LB_TPB), 0, e->stream, 0u, 1u, e->n_u.as<uint32_t>(),
                           nullptr, nullptr, nullptr, nullptr, nullptr);
        hipLaunchKernelGGL(k_hash_finish, dim3(4096), dim3(LB_INV_TPB), 0, e->stream, 0u, e->n_u.as<uint32_t>(),
                           nullptr, nullptr, nullptr, 0u);
        // s2 and s3 the same way (round 6), each for the kernels with a private segment it runs,
        // at their largest dispatch: s2 the signature decode over the whole device (472 B per
        // lane), the 8-lane subgroup check and r_i sig_i of small batches (616 / 868 B); s3 the
        // 96-byte-key chunk sums (584 B).  The rest of s2 / s3's kernels need less per lane and
        // fewer lanes (resource table: DESIGN.md section 5.2).
        // LB_RESERVE_S23 (A/B): 0 none, 1 the decode + s3 only, 2 (default) all of the above
        const char* rv = getenv("LB_RESERVE_S23");
        const int res23 = rv ? atoi(rv) : 2;
        if (res23 >= 1) {
          hipLaunchKernelGGL(k_decompress_sigs, dim3(4096), dim3(LB_TPB), 0, e->stream2, 0u, nullptr, nullptr, nullptr,
                             nullptr, nullptr, nullptr);
          hipLaunchKernelGGL(k_pk_chunks, dim3(4096), dim3(LB_TPB), 0, e->stream3, 0u, nullptr, nullptr, nullptr, nullptr);
          // the row r PK ladder (one row per set), at the largest small batch
          hipLaunchKernelGGL(k_pk_blind_rowp, dim3(std::max<uint32_t>(1u, e->row_max)), dim3(64), 0, e->stream3,
                             0u, nullptr, nullptr, nullptr, nullptr);
        }
        if (res23 >= 2) {
          // (one wave per 8 sets, at least one wave, at most 16 384: more than the device holds)
          auto g8_waves = [](uint32_t sets) { return dim3(std::min<uint32_t>(16384u, std::max<uint32_t>(1u, sets / 8 + 1))); };
          hipLaunchKernelGGL(k_sig_subgroup_g8, g8_waves(e->subgroup_g8_max), dim3(64), 0, e->stream2, 0u, nullptr,
                             nullptr, nullptr);
          hipLaunchKernelGGL(k_sig_blind_g8, g8_waves(e->small_s_g8_max), dim3(64), 0, e->stream2, 0u, nullptr, nullptr,
                             nullptr, nullptr, nullptr);
        }
        ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(e->stream) == hipSuccess &&
             hipStreamSynchronize(e->stream2) == hipSuccess && hipStreamSynchronize(e->stream3) == hipSuccess;
      }
    }
    if (!ok) {
      fprintf(stderr, "lodestar_bls: engine scratch reservation failed on device %d\n", device);
      lb_engine_destroy(e);
      return LB_ERR_DEVICE;
    }
  }
  *out = e;
  return LB_OK;
}

void lb_engine_destroy(lb_engine* e) {
  if (!e) return;
  hipSetDevice(e->device);
  hipStreamSynchronize(e->stream);
  dbuf* bufs[] = {&e->scalars, &e->sig_aff, &e->sig_inf, &e->sig_status, &e->q, &e->h_aff, &e->rpk, &e->rsig,
                  &e->pk_status, &e->ml, &e->treeP, &e->treeS, &e->job_status, &e->nodes, &e->verdict, &e->parts,
                  &e->ok, &e->chunk_acc, &e->chunk_status, &e->fS, &e->table, &e->msg_tab,
                  &e->rep_of, &e->uid_of, &e->uniq_set, &e->n_u, &e->set_uid, &e->gcnt, &e->gpos, &e->goff,
                  &e->gch, &e->chunk_beg, &e->chunk_end, &e->members, &e->set_live, &e->gacc, &e->gp_aff,
                  &e->gp_inf, &e->chunk_root, &e->sig_aos, &e->bcnt, &e->bcursor, &e->boff, &e->bch, &e->bchunk_beg,
                  &e->bchunk_end, &e->bmembers, &e->bacc, &e->bsum, &e->wsum, &e->park, &e->set_spec, &e->live_flag, &e->pk_aff, &e->y_root, &e->kzg_g1,
                  &e->kzg_g2, &e->s_terms, &e->s_part, &e->s_root, &e->rs_idx, &e->s_set, &e->pk3, &e->corder};
  for (dbuf* b : bufs) b->release();
  for (dbuf& b : e->sx) b.release();
  for (int i = 0; i < kStages; i++) {
    if (e->ev0[i]) hipEventDestroy(e->ev0[i]);
    if (e->ev1[i]) hipEventDestroy(e->ev1[i]);
  }
  hipEventDestroy(e->ev_g1);
  hipEventDestroy(e->ev_s);
  hipEventDestroy(e->ev_fork);
  hipEventDestroy(e->ev_dec);
  hipEventDestroy(e->ev_pk);
  if (e->ev_pkst) hipEventDestroy(e->ev_pkst);
  if (e->ev_sdec) hipEventDestroy(e->ev_sdec);
  if (e->ev_sblind) hipEventDestroy(e->ev_sblind);
  hipStreamSynchronize(e->stream2);
  hipStreamSynchronize(e->stream3);
  if (e->scratch) delete e->scratch;
  if (e->h_nu) hipHostFree(e->h_nu);
  if (e->h_flag) hipHostFree(e->h_flag);
  if (e->h_stage) hipHostFree(e->h_stage);
  hipStreamDestroy(e->stream2);
  hipStreamDestroy(e->stream3);
  hipStreamDestroy(e->stream);
  for (hipStream_t h : e->hp)
    if (h) {
      hipStreamSynchronize(h);
      hipStreamDestroy(h);
    }
  {
    std::lock_guard<std::mutex> lk(g_engine_mu);
    g_engine_count[e->device]--;
    if (e->latency && --g_latency_live[e->device] == 0) g_latency_cus[e->device] = 0;
  }
  delete e;
}

int32_t lb_engine_cu_count(const lb_engine* e) { return e ? e->n_cus : 0; }

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

}  // extern "C"

// Validates the offsets and uploads one batch into b's device buffers (grown, never shrunk, so
// an engine-owned workspace batch is reused across calls without device allocation).  The caller
// holds e->mu.
static constexpr size_t kStageMax = (size_t)1 << 20;  // batch uploads up to this go up as one copy
static int32_t batch_fill(lb_engine* e, lb_batch* b, uint32_t n_jobs, const uint32_t* job_offsets,
                          const uint32_t* set_pk_offsets, const uint8_t* pubkeys, const uint32_t* pk_indices,
                          const uint8_t* signing_roots, const uint8_t* signatures, const uint32_t* sig_sizes) {
  if (!e || !job_offsets || !set_pk_offsets) return LB_ERR_ARGUMENT;
  if (job_offsets[0] != 0) return LB_ERR_ARGUMENT;
  for (uint32_t j = 0; j < n_jobs; j++)
    if (job_offsets[j + 1] < job_offsets[j]) return LB_ERR_ARGUMENT;
  const uint32_t n_sets = job_offsets[n_jobs];
  if (set_pk_offsets[0] != 0) return LB_ERR_ARGUMENT;
  for (uint32_t i = 0; i < n_sets; i++)
    if (set_pk_offsets[i + 1] < set_pk_offsets[i]) return LB_ERR_ARGUMENT;
  const uint32_t n_pks = set_pk_offsets[n_sets];
  if (n_pks & LB_CHUNK_FIRST) return LB_ERR_ARGUMENT;  // key offsets are 31-bit (chunk flags)
  const bool indexed = pk_indices != nullptr;
  if ((n_sets && (!signing_roots || !signatures)) || (n_pks && !pubkeys && !indexed)) return LB_ERR_ARGUMENT;
  LB_HIP(hipSetDevice(e->device));
  b->device = e->device;
  b->serial = g_batch_serial.fetch_add(1, std::memory_order_relaxed) + 1;
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
  // chunk decomposition of every set's pubkey range (<= LB_PK_CHUNK keys per chunk; a small batch,
  // whose aggregation is latency -- a block's 131 sets of ~256 keys --, <= LB_PK_CHUNK_SMALL: its
  // serial chain per lane 16 -> 4 mixed additions before the six-level segmented tree)
  std::vector<uint32_t>& set_chunk_off = b->h_set_chunk_off;
  std::vector<uint32_t>& chunk_lo = b->h_chunk_lo;
  set_chunk_off.resize(n_sets + 1);
  chunk_lo.clear();
  const uint32_t pkc = n_sets <= e->row_max ? LB_PK_CHUNK_SMALL : LB_PK_CHUNK;
  for (uint32_t i = 0; i < n_sets; i++) {
    set_chunk_off[i] = (uint32_t)chunk_lo.size();
    for (uint32_t k = set_pk_offsets[i]; k < set_pk_offsets[i + 1]; k += pkc)
      chunk_lo.push_back(k | (k == set_pk_offsets[i] ? LB_CHUNK_FIRST : 0u));  // flag: the set's first chunk
  }
  set_chunk_off[n_sets] = (uint32_t)chunk_lo.size();
  b->n_chunks = (uint32_t)chunk_lo.size();
  chunk_lo.push_back(n_pks | LB_CHUNK_FIRST);  // chunk c ends where chunk c+1 starts (chunks never
  // span sets: a set's last chunk ends at the next set's first key, which is its own first chunk start)
  b->indexed = indexed;
  struct part {
    dbuf* d;
    const void* src;
    size_t bytes;
  };
  const part parts[] = {{&b->d_job_off, job_offsets, (size_t)(n_jobs + 1) * 4},
                        {&b->d_set_chunk_off, set_chunk_off.data(), set_chunk_off.size() * 4},
                        {&b->d_chunk_lo, chunk_lo.data(), chunk_lo.size() * 4},
                        {&b->d_pk_off, set_pk_offsets, (size_t)(n_sets + 1) * 4},
                        {&b->d_pks, indexed ? (const void*)pk_indices : (const void*)pubkeys,
                         (size_t)n_pks * (indexed ? 4 : 96)},
                        {&b->d_msgs, signing_roots, (size_t)n_sets * 32},
                        {&b->d_sigs, signatures, (size_t)n_sets * 96},
                        {&b->d_sig_sizes, sig_sizes, sig_sizes ? (size_t)n_sets * 4 : 0}};
  // a small batch (a 1-set call, a block) goes up as ONE copy from pinned staging into an arena
  // the arrays are views of: eight pageable copies were ~0.1 ms of a 1-set call's 3.7
  size_t total = 0;
  for (const part& q : parts) total += ((q.bytes > 16 ? q.bytes : 16) + 255) & ~(size_t)255;
  bool staged = total <= kStageMax;
  if (staged && e->h_stage_cap < total) {
    if (e->h_stage) hipHostFree(e->h_stage);
    e->h_stage = nullptr;
    e->h_stage_cap = 0;
    if (hipHostMalloc(&e->h_stage, kStageMax, hipHostMallocDefault) == hipSuccess) e->h_stage_cap = kStageMax;
    else staged = false;
  }
  hipError_t r = hipSuccess;
  if (staged) {
    r = b->d_arena.ensure(total);
    size_t off = 0;
    for (const part& q : parts) {
      if (q.bytes) memcpy(static_cast<uint8_t*>(e->h_stage) + off, q.src, q.bytes);
      off += ((q.bytes > 16 ? q.bytes : 16) + 255) & ~(size_t)255;
    }
    if (r == hipSuccess) r = hipMemcpyAsync(b->d_arena.p, e->h_stage, total, hipMemcpyHostToDevice, e->stream);
    off = 0;
    for (const part& q : parts) {
      const size_t sz = ((q.bytes > 16 ? q.bytes : 16) + 255) & ~(size_t)255;
      if (r == hipSuccess && (q.bytes || q.d != &b->d_sig_sizes)) q.d->set_view(static_cast<uint8_t*>(b->d_arena.p) + off, sz);
      off += sz;
    }
  } else {
    for (const part& q : parts)
      if (r == hipSuccess && (q.bytes || q.d != &b->d_sig_sizes)) r = up(*q.d, q.src, q.bytes);
  }
  if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
  if (r != hipSuccess) {
    // no view may outlive a failed (re)allocation of the arena: the batch is left empty, so a
    // later verify of it reads nothing (round-5 ADVICE)
    for (const part& q : parts) q.d->release();
    b->d_arena.release();
    b->n_jobs = b->n_sets = b->n_pks = b->n_chunks = 0;
    b->job_off.assign(1, 0u);
    fprintf(stderr, "lodestar_bls: batch upload failed: %s\n", hipGetErrorString(r));
    return LB_ERR_DEVICE;
  }
  return LB_OK;
}

static int32_t batch_create(lb_engine* e, uint32_t n_jobs, const uint32_t* job_offsets, const uint32_t* set_pk_offsets,
                            const uint8_t* pubkeys, const uint32_t* pk_indices, const uint8_t* signing_roots,
                            const uint8_t* signatures, const uint32_t* sig_sizes, lb_batch** out) {
  if (!e || !out) return LB_ERR_ARGUMENT;
  *out = nullptr;
  std::lock_guard<std::mutex> lk(e->mu);
  lb_batch* b = new lb_batch();
  int32_t st = batch_fill(e, b, n_jobs, job_offsets, set_pk_offsets, pubkeys, pk_indices, signing_roots, signatures,
                          sig_sizes);
  if (st != LB_OK) {
    delete b;
    return st;
  }
  *out = b;
  return LB_OK;
}

// pk_indices == NULL is only meaningful when no set carries a key (every set then rejects with
// EMPTY_AGGREGATE_ARRAY); it is passed on as a one-word sentinel, never read.
static const uint32_t kNoIndices[1] = {0};
static int32_t check_null_indices(uint32_t n_jobs, const uint32_t* job_offsets, const uint32_t* set_pk_offsets) {
  if (!job_offsets || !set_pk_offsets) return LB_ERR_ARGUMENT;
  return set_pk_offsets[job_offsets[n_jobs]] == 0 ? LB_OK : LB_ERR_ARGUMENT;
}

extern "C" {

int32_t lb_batch_create(lb_engine* e, uint32_t n_jobs, const uint32_t* job_offsets, const uint32_t* set_pk_offsets,
                        const uint8_t* pubkeys, const uint8_t* signing_roots, const uint8_t* signatures,
                        const uint32_t* sig_sizes, lb_batch** out) {
  return batch_create(e, n_jobs, job_offsets, set_pk_offsets, pubkeys, nullptr, signing_roots, signatures, sig_sizes,
                      out);
}

int32_t lb_batch_create_indexed(lb_engine* e, uint32_t n_jobs, const uint32_t* job_offsets,
                                const uint32_t* set_pk_offsets, const uint32_t* pk_indices,
                                const uint8_t* signing_roots, const uint8_t* signatures, const uint32_t* sig_sizes,
                                lb_batch** out) {
  if (!pk_indices) {
    const int32_t st = check_null_indices(n_jobs, job_offsets, set_pk_offsets);
    if (st != LB_OK) return st;
    pk_indices = kNoIndices;
  }
  return batch_create(e, n_jobs, job_offsets, set_pk_offsets, nullptr, pk_indices, signing_roots, signatures,
                      sig_sizes, out);
}

void* lb_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}

void lb_host_free(void* p) {
  if (p) hipHostFree(p);
}

uint32_t lb_pubkey_table_size(const lb_engine* e) { return e ? e->table_n : 0; }

int32_t lb_pubkey_table_append(lb_engine* e, uint32_t n, const uint8_t* keys, uint32_t key_size, int32_t validate,
                               int32_t* out_status, uint32_t* out_first_index) {
  if (!e || (n && (!keys || !out_status)) || (key_size != 48 && key_size != 96)) return LB_ERR_ARGUMENT;
  std::lock_guard<std::mutex> lk(e->mu);
  LB_HIP(hipSetDevice(e->device));
  const uint32_t first = e->table_n;
  if (out_first_index) *out_first_index = first;
  if (!n) return LB_OK;
  const uint32_t need = first + n;
  if (need > e->table_cap) {
    // grow: records keep their layout, one contiguous copy
    uint32_t cap = e->table_cap ? e->table_cap : 1024;
    while (cap < need) cap *= 2;
    dbuf nt;
    LB_HIP(nt.ensure((size_t)cap * LB_TABLE_REC * 4));
    if (first)
      LB_HIP(hipMemcpyAsync(nt.p, e->table.p, (size_t)first * LB_TABLE_REC * 4, hipMemcpyDeviceToDevice, e->stream));
    LB_HIP(hipStreamSynchronize(e->stream));
    e->table.release();
    e->table = nt;
    e->table_cap = cap;
  }
  dbuf kin, st;
  hipError_t r = kin.ensure((size_t)n * key_size);
  if (r == hipSuccess) r = st.ensure((size_t)n * 4);
  if (r == hipSuccess) r = hipMemcpyAsync(kin.p, keys, (size_t)n * key_size, hipMemcpyHostToDevice, e->stream);
  if (r == hipSuccess) {
    hipLaunchKernelGGL(k_table_fill, dim3(nblk(n)), dim3(LB_TPB), 0, e->stream, n, kin.as<uint8_t>(), key_size,
                       validate, first, e->table.as<uint32_t>(), st.as<int32_t>());
    r = hipGetLastError();
  }
  if (r == hipSuccess) r = hipMemcpyAsync(out_status, st.p, (size_t)n * 4, hipMemcpyDeviceToHost, e->stream);
  if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
  kin.release();
  st.release();
  if (r != hipSuccess) {
    fprintf(stderr, "lodestar_bls: pubkey table append failed: %s\n", hipGetErrorString(r));
    return LB_ERR_DEVICE;
  }
  e->table_n = need;
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

// stage timing helpers (HIP events on the stage's own stream)
struct stage_scope {
  lb_engine* e;
  int k;
  hipStream_t st;
  stage_scope(lb_engine* e_, int k_, hipStream_t st_) : e(e_), k(k_), st(st_) {
    if (e->profiling) {
      hipEventRecord(e->ev0[k], st);
      e->used[k] = true;
    }
  }
  ~stage_scope() {
    if (e->profiling) hipEventRecord(e->ev1[k], st);
  }
};

// Bucket sums -> S_j = sum_d d B_d per instance j (n_inst instances of W windows, buckets
// [j W 256, (j+1) W 256) of bsum) -> element out0 + j of `out` (SoA, stride n_out).
// entries: bucket entries (point, window) of the launch, an upper bound.  The bucket sums go by
// 8-lane groups (one wave per bucket) only when buckets hold several chunks on average (the batch
// MSM: ~30 chunk sums per bucket); a search round's many small instances leave ~one chunk per
// bucket, which one lane per bucket sums without the wave's idle groups.
static hipError_t msm_reduce(lb_engine* e, hipStream_t st, uint32_t bcap, uint32_t nb, uint32_t n_inst, int W,
                             uint32_t* out, uint32_t n_out, uint32_t out0, uint64_t entries, uint32_t chunk) {
  if (e->msm_g8) {
    hipError_t r = e->wsum.ensure((size_t)n_inst * W * sizeof(g2j));
    if (r != hipSuccess) return r;
    // 8-lane bucket sums only while the device runs no other batch: they issue ~6x the
    // instructions of one lane per bucket (profiles/r4_r3_valu.txt), which under load is the cost
    if (entries >= (uint64_t)4 * chunk * nb && device_alone(e))
      hipLaunchKernelGGL(k_msm_buckets_g8, dim3(nb), dim3(64), 0, st, e->bch.as<uint32_t>(), e->bacc.as<uint32_t>(),
                         bcap, e->bsum.as<uint32_t>(), nb);
    else
      hipLaunchKernelGGL(k_msm_buckets, dim3(nblk(nb)), dim3(LB_TPB), 0, st, e->bch.as<uint32_t>(),
                         e->bacc.as<uint32_t>(), bcap, e->bsum.as<uint32_t>(), nb);
    hipLaunchKernelGGL(k_msm_window_g8, dim3(n_inst * W), dim3(256), 0, st, e->bsum.as<uint32_t>(), nb,
                       e->wsum.as<uint32_t>(), n_inst * W);
    if (W == LB_MSM_W)
      hipLaunchKernelGGL(k_msm_horner_g8<LB_MSM_W>, dim3((n_inst + 7) / 8), dim3(64), 0, st, e->wsum.as<uint32_t>(),
                         n_inst, out, n_out, out0);
    else
      hipLaunchKernelGGL(k_msm_horner_g8<LB_SMSM_W>, dim3((n_inst + 7) / 8), dim3(64), 0, st, e->wsum.as<uint32_t>(),
                         n_inst, out, n_out, out0);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_msm_buckets, dim3(nblk(nb)), dim3(LB_TPB), 0, st, e->bch.as<uint32_t>(), e->bacc.as<uint32_t>(),
                     bcap, e->bsum.as<uint32_t>(), nb);
  if (W == LB_MSM_W)
    hipLaunchKernelGGL(k_msm_reduce<LB_MSM_W>, dim3(n_inst), dim3(64 * LB_MSM_W), 0, st, e->bsum.as<uint32_t>(), nb, out,
                       n_out, out0);
  else
    hipLaunchKernelGGL(k_msm_reduce<LB_SMSM_W>, dim3(n_inst), dim3(64 * LB_SMSM_W), 0, st, e->bsum.as<uint32_t>(), nb,
                       out, n_out, out0);
  return hipGetLastError();
}

// s1: P_u = sum of r_i PK_i over the sets of root u with live[i] (k_gsum_*), the Miller loops
// (form by root count and device load) into the leaves of the root product tree, the tree.
static hipError_t per_root_chain(lb_engine* e, uint32_t n, uint32_t nuh, uint32_t mu, const uint32_t* live) {
  hipStream_t s1 = e->stream;
  const uint32_t* nu = e->n_u.as<uint32_t>();
  {
    stage_scope sc(e, ST_GSUM, s1);
    // chunks of <= LB_GROUP_CHUNK members: at most nuh + n / LB_GROUP_CHUNK of them
    const uint32_t nch = nuh + n / e->gchunk;
    const bool wave = e->gsum_tree && e->alone && e->gsum_wave;
    if (wave)
      hipLaunchKernelGGL(k_gsum_wave, dim3(nblk(nch)), dim3(LB_TPB), 0, s1, n, nu, e->gch.as<uint32_t>(),
                         e->chunk_beg.as<uint32_t>(), e->chunk_end.as<uint32_t>(), e->chunk_root.as<uint32_t>(),
                         e->members.as<uint32_t>(), live, e->rpk.as<uint32_t>(), e->gacc.as<uint32_t>());
    else if (e->straus_run) {
      hipError_t r = e->corder.ensure((size_t)(nch + 2 * (LB_STRAUS_CHUNK + 1)) * 4);
      if (r != hipSuccess) return r;
      uint32_t* cnt = e->corder.as<uint32_t>() + nch;
      r = hipMemsetAsync(cnt, 0, (size_t)2 * (LB_STRAUS_CHUNK + 1) * 4, s1);
      if (r != hipSuccess) return r;
      for (uint32_t pass = 0; pass < 2; pass++)
        hipLaunchKernelGGL(k_chunk_order, dim3(nblk(nch)), dim3(LB_TPB), 0, s1, nu, e->gch.as<uint32_t>(),
                           e->chunk_beg.as<uint32_t>(), e->chunk_end.as<uint32_t>(), cnt, e->corder.as<uint32_t>(), pass);
      hipLaunchKernelGGL(k_gsum_straus, dim3(nblk(nch)), dim3(LB_TPB), 0, s1, n, nu, e->gch.as<uint32_t>(),
                         e->chunk_beg.as<uint32_t>(), e->chunk_end.as<uint32_t>(), e->corder.as<uint32_t>(),
                         e->members.as<uint32_t>(), live, e->pk3.as<uint32_t>(), e->scalars.as<uint64_t>(),
                         e->gacc.as<uint32_t>());
    }
    else
      hipLaunchKernelGGL(k_gsum_chunks, dim3(nblk(nch)), dim3(LB_TPB), 0, s1, n, nu,
                         e->gch.as<uint32_t>(), e->chunk_beg.as<uint32_t>(), e->chunk_end.as<uint32_t>(),
                         e->members.as<uint32_t>(), live, e->rpk.as<uint32_t>(), e->gacc.as<uint32_t>());
    // the per-root tree over the chunk sums (levels until one partial per root is left)
    const bool tree = e->gsum_tree && e->alone && !wave;  // (the Straus chunks under load are 8 members too)
    for (uint32_t st = 1; tree && st < e->gmax_chunks; st *= LB_GSUM_FAN)
      hipLaunchKernelGGL(k_gsum_tree, dim3(nblk(nch)), dim3(LB_TPB), 0, s1, n, nu, e->gch.as<uint32_t>(),
                         e->chunk_root.as<uint32_t>(), st, e->gacc.as<uint32_t>());
    hipLaunchKernelGGL(k_gsum_final, dim3(nblk_inv(nuh)), dim3(LB_INV_TPB), 0, s1, n, nu, e->gch.as<uint32_t>(),
                       e->gacc.as<uint32_t>(), e->gp_aff.as<uint32_t>(), e->gp_inf.as<uint32_t>(),
                       wave ? 2u : (tree ? 0u : 1u));
  }
  {
    stage_scope sc(e, ST_MILLER, s1);
    const bool shared = e->miller_form == 1 ||
                        (e->miller_form == 0 && !device_alone(e));
    if (nuh <= e->row_max && e->alone && e->row_fe) {
      hipLaunchKernelGGL(k_miller_row, dim3(nuh), dim3(LBR_NT), 0, s1, n, mu, nu, e->gp_aff.as<uint32_t>(),
                         e->gp_inf.as<uint32_t>(), e->h_aff.as<uint32_t>(), e->treeP.as<uint32_t>());
    } else if (nuh <= e->miller_wave_max) {
      hipLaunchKernelGGL(k_miller_wave, dim3(nuh), dim3(64), 0, s1, n, mu, nu, e->gp_aff.as<uint32_t>(),
                         e->gp_inf.as<uint32_t>(), e->h_aff.as<uint32_t>(), e->treeP.as<uint32_t>());
    } else if (shared) {
      hipError_t r = e->park.ensure((size_t)2 * 72 * 4 * n);  // T and a temporary per root
      if (r != hipSuccess) return r;
      if (nuh <= e->miller_lds3_max)
        hipLaunchKernelGGL(k_miller_lane<3>, dim3(nblk(nuh)), dim3(LB_TPB), 0, s1, n, mu, nu, e->gp_aff.as<uint32_t>(),
                           e->gp_inf.as<uint32_t>(), e->h_aff.as<uint32_t>(), e->treeP.as<uint32_t>(),
                           e->park.as<uint32_t>());
      else
        hipLaunchKernelGGL(k_miller_lane<2>, dim3(nblk(nuh)), dim3(LB_TPB), 0, s1, n, mu, nu, e->gp_aff.as<uint32_t>(),
                           e->gp_inf.as<uint32_t>(), e->h_aff.as<uint32_t>(), e->treeP.as<uint32_t>(),
                           e->park.as<uint32_t>());
    } else {
      hipLaunchKernelGGL(k_miller_g8, dim3((nuh + LBG_ROOTS - 1) / LBG_ROOTS), dim3(64 * LBG_WAVES), 0, s1, n, mu, nu,
                         e->gp_aff.as<uint32_t>(), e->gp_inf.as<uint32_t>(), e->h_aff.as<uint32_t>(),
                         e->treeP.as<uint32_t>());
    }
  }
  {
    stage_scope sc(e, ST_TREE_P, s1);
    for (uint32_t lo = mu / 2; lo >= 1; lo /= 2) {
      if (lo <= e->row_max && e->alone && e->row_fe)
        hipLaunchKernelGGL(k_tree_up_row, dim3(lo), dim3(LBR_NT), 0, s1, mu, lo, nu, e->treeP.as<uint32_t>());
      else
        hipLaunchKernelGGL(k_tree_up_U, dim3(lo), dim3(64), 0, s1, mu, lo, nu, e->treeP.as<uint32_t>());
    }
  }
  return hipGetLastError();
}

// Runs the batch pipeline on two streams: the job S tree (leaf count mj = pow2 >= jobs) with
// fS = ML(-G1, S_root) on s2, the message product tree (leaf count mu = pow2 >= sets, leaves
// [0, n_u) live) on s1, joined on s1 ready for the root check.
static int32_t run_pipeline(lb_engine* e, lb_batch* b, const uint64_t* scalars, uint32_t& mj, uint32_t& mu,
                            bool unblinded) {
  const uint32_t n = b->n_sets, nj = b->n_jobs;
  e->partial_serial = 0;
  e->alone = device_alone(e);
  e->straus_run = e->straus && !e->alone;
  e->rpk_stale = e->straus_run;
  e->gchunk = (e->alone && e->gsum_tree) ? (e->gsum_wave ? LB_GROUP_CHUNK_WAVE : LB_GROUP_CHUNK_ALONE)
                                          : (e->straus_run ? LB_STRAUS_CHUNK : LB_GROUP_CHUNK);
  const bool one_unblinded = n == 1 && !scalars && unblinded;
  int st = fill_scalars(e, n, scalars, unblinded);
  if (st != LB_OK) return st;
  mj = 1;
  while (mj < nj) mj <<= 1;
  mu = 1;
  while (mu < n) mu <<= 1;
  const uint32_t mt = mj > mu ? mj : mu;
  const uint32_t ns = n ? n : 1;
  uint32_t cap = 64;
  while (cap < 2 * ns) cap <<= 1;
  LB_HIP(e->scalars.ensure((size_t)ns * 8));
  LB_HIP(e->sig_aff.ensure((size_t)ns * sizeof(g2a)));
  LB_HIP(e->sig_inf.ensure((size_t)ns * 4));
  LB_HIP(e->sig_status.ensure((size_t)ns * 4));
  LB_HIP(e->q.ensure((size_t)ns * 2 * sizeof(g2j)));
  LB_HIP(e->h_aff.ensure((size_t)ns * sizeof(g2a)));
  LB_HIP(e->rpk.ensure((size_t)ns * sizeof(g1j)));
  LB_HIP(e->pk_aff.ensure((size_t)ns * sizeof(g1a)));
  LB_HIP(e->pk_status.ensure((size_t)ns * 4));
  LB_HIP(e->treeP.ensure((size_t)2 * mt * sizeof(fp12)));
  LB_HIP(e->treeS.ensure((size_t)2 * mj * sizeof(g2j)));
  LB_HIP(e->job_status.ensure((size_t)(nj ? nj : 1) * 4));
  LB_HIP(e->fS.ensure(sizeof(fp12)));
  LB_HIP(e->msg_tab.ensure((size_t)cap * 4));
  dbuf* per_set[] = {&e->rep_of, &e->uid_of, &e->uniq_set, &e->set_uid, &e->gcnt, &e->gpos, &e->chunk_beg,
                     &e->chunk_end, &e->members, &e->set_live, &e->gp_inf, &e->chunk_root};
  for (dbuf* d : per_set) LB_HIP(d->ensure((size_t)ns * 4));
  LB_HIP(e->goff.ensure((size_t)(ns + 1) * 4));
  LB_HIP(e->gch.ensure((size_t)(ns + 1) * 4));
  LB_HIP(e->n_u.ensure(8));
  LB_HIP(e->gacc.ensure((size_t)ns * sizeof(g1j)));
  LB_HIP(e->gp_aff.ensure((size_t)ns * sizeof(g1a)));
  const uint32_t bcap = (2 * LB_MSM_W * ns) / LB_MSM_CHUNK + LB_MSM_NB;  // bucket chunks, upper bound
  LB_HIP(e->sig_aos.ensure((size_t)ns * sizeof(g2a)));
  LB_HIP(e->bcnt.ensure((size_t)LB_MSM_NB * 4));
  LB_HIP(e->bcursor.ensure((size_t)LB_MSM_NB * 4));
  LB_HIP(e->boff.ensure((size_t)(LB_MSM_NB + 1) * 4));
  LB_HIP(e->bch.ensure((size_t)(LB_MSM_NB + 1) * 4));
  LB_HIP(e->bchunk_beg.ensure((size_t)bcap * 4));
  LB_HIP(e->bchunk_end.ensure((size_t)bcap * 4));
  LB_HIP(e->bmembers.ensure((size_t)2 * LB_MSM_W * ns * 4));
  LB_HIP(e->bacc.ensure((size_t)bcap * sizeof(g2j)));
  LB_HIP(e->bsum.ensure((size_t)LB_MSM_NB * sizeof(g2j)));
  const uint32_t nc = b->n_chunks;
  LB_HIP(e->chunk_acc.ensure((size_t)(nc ? nc : 1) * sizeof(g1j)));
  LB_HIP(e->chunk_status.ensure((size_t)(nc ? nc : 1) * 4));
  for (int k = 0; k < kStages; k++) {
    e->used[k] = false;
    e->acc_ms[k] = 0.f;
  }
  hipStream_t s1 = e->stream, s2 = e->stream2, s3_ = e->stream3;
  if (e->profiling) {
    hipEventRecord(e->ev0[ST_TOTAL], s1);
    e->used[ST_TOTAL] = true;
  }
  if (n) LB_HIP(hipMemcpyAsync(e->scalars.p, e->h_scalars.data(), (size_t)n * 8, hipMemcpyHostToDevice, s1));
  // fork: s2 starts after s1's scalar upload
  LB_HIP(hipEventRecord(e->ev_fork, s1));
  LB_HIP(hipStreamWaitEvent(s2, e->ev_fork, 0));
  LB_HIP(hipStreamWaitEvent(s3_, e->ev_fork, 0));
  const uint32_t* nu = e->n_u.as<uint32_t>();
  if (n) {
    // ---- pubkeys, r*PK: on s3 beside the signature decode for batches up to small_s_max sets
    // (shortens the signature side's chain); on s2 before the decode for large batches, where the
    // two would contend with the per-root chain on s1 for the whole chip
    // (also for a large batch alone on the device: its s1 chain then slowed by more than the s2
    // chain gained, 5.2 -> 5.1 M sets/s, round-3 A/B)
    // (with the speculative per-root chain the pubkey side always runs on s3: the chain starts
    // when it is done, beside the decode)
    const hipStream_t s3 = (e->spec_gsum || n <= e->small_s_max) ? s3_ : s2;
    {
      stage_scope sc(e, ST_PK_CHUNKS, s3);
      if (nc && b->indexed)
        hipLaunchKernelGGL(k_pk_chunks_idx, dim3(nblk(nc)), dim3(LB_TPB), 0, s3, nc, b->d_chunk_lo.as<uint32_t>(),
                           b->d_pks.as<uint32_t>(), e->table.as<uint32_t>(), e->table_n, e->chunk_acc.as<uint32_t>(),
                           e->chunk_status.as<int32_t>());
      else if (nc)
        hipLaunchKernelGGL(k_pk_chunks, dim3(nblk(nc)), dim3(LB_TPB), 0, s3, nc, b->d_chunk_lo.as<uint32_t>(),
                           b->d_pks.as<uint8_t>(), e->chunk_acc.as<uint32_t>(), e->chunk_status.as<int32_t>());
    }
    // on its own stream the pubkey side splits: the aggregates' statuses (what the job statuses
    // and so the S side need) first, then the r PK ladder (only the per-root sums need it)
    const bool pk_split = s3 != s2;
    // small batches alone: the r PK ladder (k_pk_blind mode 2) with row products, one 16-lane row
    // per set (on s3, before r_i sig_i; a fourth stream per engine, round 6, put 7 engines' 28
    // streams past what the device schedules without stalls: +10 ms on some batches)
    const bool pk_rowp = e->small_par && pk_split && !e->straus_run && n <= e->row_max && e->alone && e->row_fe;
    // r_i sig_i on s3 beside the subgroup check (small batches alone, row forms, one-workgroup sum)
    const bool sb_par = e->small_par && pk_split && !one_unblinded && n <= e->small_s_max && n <= e->small_s_g8_max &&
                        n <= e->row_max && e->alone && e->row_fe && !e->straus_run;
    {
      stage_scope sc(e, ST_PK_BLIND, s3);
      // modes: 0 all, 1 aggregate + status (+ pk3 for the Straus sums), 2 the per-set ladder
      const uint32_t m0 = (pk_split || e->straus_run) ? 1u : 0u;
      const uint32_t m1 = e->straus_run ? 1u : (pk_split ? 2u : 0u);
      if (e->straus_run) LB_HIP(e->pk3.ensure((size_t)ns * sizeof(g1x3)));
      for (uint32_t mode = m0; mode <= m1; mode++) {
        if (mode == 2u && pk_rowp) {
          hipLaunchKernelGGL(k_pk_blind_rowp, dim3(n), dim3(64), 0, s3, n, e->pk_aff.as<uint32_t>(),
                             e->scalars.as<uint64_t>(), e->rpk.as<uint32_t>(), e->pk_status.as<int32_t>());
          continue;
        }
        hipLaunchKernelGGL(k_pk_blind, dim3(nblk_inv(n)), dim3(LB_INV_TPB), 0, s3, n, nc, b->d_set_chunk_off.as<uint32_t>(),
                           e->chunk_acc.as<uint32_t>(), e->chunk_status.as<int32_t>(), e->pk_aff.as<uint32_t>(),
                           e->scalars.as<uint64_t>(), e->rpk.as<uint32_t>(), e->pk_status.as<int32_t>(), mode,
                           (mode == 1u && e->straus_run) ? e->pk3.as<uint32_t>() : nullptr);
        if (mode == 1u) LB_HIP(hipEventRecord(e->ev_pkst, s3));
      }
    }
    LB_HIP(hipEventRecord(e->ev_pk, s3));
    // signatures: decoded while s1 groups and hashes the messages
    {
      stage_scope sc(e, ST_DECODE, s2);
      if (n <= e->dec_row_max && e->alone && e->row_fe)
        hipLaunchKernelGGL(k_decompress_sigs_row, dim3(LB_H2C_FOLD ? (n + 1) / 2 : (n + 3) / 4), dim3(64), 0, s2, n, b->d_sigs.as<uint8_t>(),
                           b->has_sizes ? b->d_sig_sizes.as<uint32_t>() : nullptr, e->sig_aff.as<uint32_t>(),
                           e->sig_aos.as<uint4>(), e->sig_inf.as<uint32_t>(), e->sig_status.as<int32_t>());
      else
        hipLaunchKernelGGL(k_decompress_sigs, dim3(nblk(n)), dim3(LB_TPB), 0, s2, n, b->d_sigs.as<uint8_t>(),
                           b->has_sizes ? b->d_sig_sizes.as<uint32_t>() : nullptr, e->sig_aff.as<uint32_t>(),
                           e->sig_aos.as<uint4>(), e->sig_inf.as<uint32_t>(), e->sig_status.as<int32_t>());
      if (sb_par) LB_HIP(hipEventRecord(e->ev_sdec, s2));
      // (8 lanes per signature also for a slot while the device is otherwise idle ran slower:
      // 13.5 vs 13.0 ms per slot, profiles/r3_idle_forms_ab.txt)
      if (n <= e->row_max && e->alone && e->row_fe && e->small_par)  // one wave per signature (round 6)
        hipLaunchKernelGGL(k_sig_subgroup_w4, dim3(n), dim3(64), 0, s2, n, e->sig_aff.as<uint32_t>(),
                           e->sig_inf.as<uint32_t>(), e->sig_status.as<int32_t>());
      else if (n <= e->row_max && e->alone && e->row_fe)
        hipLaunchKernelGGL(k_sig_subgroup_row, dim3(n), dim3(LBR_NT), 0, s2, n, e->sig_aff.as<uint32_t>(),
                           e->sig_inf.as<uint32_t>(), e->sig_status.as<int32_t>(), e->row_proj ? 1u : 0u);
      else if (n <= e->subgroup_g8_max)
        hipLaunchKernelGGL(k_sig_subgroup_g8, dim3((n + 7) / 8), dim3(64), 0, s2, n, e->sig_aff.as<uint32_t>(),
                           e->sig_inf.as<uint32_t>(), e->sig_status.as<int32_t>());
      else
        hipLaunchKernelGGL(k_sig_subgroup, dim3(nblk(n)), dim3(LB_TPB), 0, s2, n, e->sig_aff.as<uint32_t>(),
                           e->sig_inf.as<uint32_t>(), e->sig_status.as<int32_t>());
      LB_HIP(hipStreamWaitEvent(s2, pk_split ? e->ev_pkst : e->ev_pk, 0));  // job statuses need the pubkey statuses
      hipLaunchKernelGGL(k_job_status, dim3(nblk(nj)), dim3(LB_TPB), 0, s2, nj, b->d_job_off.as<uint32_t>(),
                         e->sig_status.as<int32_t>(), e->pk_status.as<int32_t>(), e->job_status.as<int32_t>(),
                         e->set_live.as<uint32_t>());
    }
    LB_HIP(hipEventRecord(e->ev_dec, s2));
    if (sb_par) {
      // r_i sig_i of every decoded set on s3 (after its pubkey work) beside s2's subgroup check and
      // job statuses; the sum on s2 masks the terms by liveness
      LB_HIP(hipStreamWaitEvent(s3, e->ev_sdec, 0));
      if (e->profiling) {
        hipEventRecord(e->ev0[ST_SIG_MSM], s3);
        e->used[ST_SIG_MSM] = true;
      }
      LB_HIP(e->s_terms.ensure((size_t)n * sizeof(g2j)));
      hipLaunchKernelGGL(k_sig_blind_w4, dim3(n), dim3(64), 0, s3, n, e->sig_aff.as<uint32_t>(),
                         e->scalars.as<uint64_t>(), e->sig_inf.as<uint32_t>(), e->s_terms.as<uint32_t>());
      LB_HIP(hipEventRecord(e->ev_sblind, s3));
    }
    // ---- s1: group the sets by signing root
    {
      stage_scope sc(e, ST_DEDUP, s1);
      if (n == 1) {
        hipLaunchKernelGGL(k_dedup_one, dim3(1), dim3(64), 0, s1, e->rep_of.as<uint32_t>(), e->uid_of.as<uint32_t>(),
                           e->uniq_set.as<uint32_t>(), e->n_u.as<uint32_t>(), e->set_uid.as<uint32_t>(),
                           e->gcnt.as<uint32_t>(), e->gpos.as<uint32_t>(), e->goff.as<uint32_t>(), e->gch.as<uint32_t>(),
                           e->chunk_beg.as<uint32_t>(), e->chunk_end.as<uint32_t>(), e->chunk_root.as<uint32_t>(),
                           e->members.as<uint32_t>());
      } else {
        LB_HIP(hipMemsetAsync(e->msg_tab.p, 0xff, (size_t)cap * 4, s1));
        LB_HIP(hipMemsetAsync(e->n_u.p, 0, 4, s1));
        LB_HIP(hipMemsetAsync(e->gcnt.p, 0, (size_t)n * 4, s1));
        hipLaunchKernelGGL(k_msg_insert, dim3(nblk(n)), dim3(LB_TPB), 0, s1, n, b->d_msgs.as<uint8_t>(), e->msg_key,
                           cap, e->msg_tab.as<uint32_t>(), e->rep_of.as<uint32_t>());
        if (e->root_shuffle)
          hipLaunchKernelGGL(k_msg_uid, dim3(nblk(cap)), dim3(LB_TPB), 0, s1, cap, e->msg_tab.as<uint32_t>(),
                             e->uid_of.as<uint32_t>(), e->uniq_set.as<uint32_t>(), e->n_u.as<uint32_t>());
        else {
          // input order (LB_ROOT_SHUFFLE=0: A/B and the search-trace tests), made deterministic on
          // the host: roots numbered by first occurrence and members in input order within a root
          // (the device form's atomics order both by wave scheduling, so two runs of one batch
          // could build different root trees)
          std::vector<uint32_t> rep(n), uid(n, 0xffffffffu), uniq, suid(n), cnt, pos(n);
          LB_HIP(hipMemcpyAsync(rep.data(), e->rep_of.p, (size_t)n * 4, hipMemcpyDeviceToHost, s1));
          LB_HIP(hipStreamSynchronize(s1));
          for (uint32_t i = 0; i < n; i++) {
            const uint32_t r = rep[i];
            if (uid[r] == 0xffffffffu) {
              uid[r] = (uint32_t)uniq.size();
              uniq.push_back(r);
              cnt.push_back(0);
            }
            suid[i] = uid[r];
            pos[i] = cnt[uid[r]]++;
          }
          const uint32_t nun = (uint32_t)uniq.size();
          LB_HIP(hipMemcpyAsync(e->uid_of.p, uid.data(), (size_t)n * 4, hipMemcpyHostToDevice, s1));
          LB_HIP(hipMemcpyAsync(e->uniq_set.p, uniq.data(), (size_t)nun * 4, hipMemcpyHostToDevice, s1));
          LB_HIP(hipMemcpyAsync(e->set_uid.p, suid.data(), (size_t)n * 4, hipMemcpyHostToDevice, s1));
          LB_HIP(hipMemcpyAsync(e->gcnt.p, cnt.data(), (size_t)nun * 4, hipMemcpyHostToDevice, s1));
          LB_HIP(hipMemcpyAsync(e->gpos.p, pos.data(), (size_t)n * 4, hipMemcpyHostToDevice, s1));
          LB_HIP(hipMemcpyAsync(e->n_u.p, &nun, 4, hipMemcpyHostToDevice, s1));
          LB_HIP(hipStreamSynchronize(s1));
        }
        if (e->root_shuffle)
          hipLaunchKernelGGL(k_msg_count, dim3(nblk(n)), dim3(LB_TPB), 0, s1, n, e->rep_of.as<uint32_t>(),
                             e->uid_of.as<uint32_t>(), e->set_uid.as<uint32_t>(), e->gcnt.as<uint32_t>(),
                             e->gpos.as<uint32_t>());
        hipLaunchKernelGGL(k_msg_scan, dim3(1), dim3(1024), 0, s1, nu, 0u, e->gchunk, e->gcnt.as<uint32_t>(), e->goff.as<uint32_t>(),
                           e->gch.as<uint32_t>(), nullptr, nullptr, nullptr, e->n_u.as<uint32_t>() + 1);
        hipLaunchKernelGGL(k_chunk_fill, dim3(nblk(n + n / e->gchunk + 1)), dim3(LB_TPB), 0, s1, nu,
                           e->gchunk, e->goff.as<uint32_t>(), e->gch.as<uint32_t>(),
                           e->chunk_beg.as<uint32_t>(), e->chunk_end.as<uint32_t>(), e->chunk_root.as<uint32_t>());
        hipLaunchKernelGGL(k_msg_scatter, dim3(nblk(n)), dim3(LB_TPB), 0, s1, n, e->set_uid.as<uint32_t>(),
                           e->gpos.as<uint32_t>(), e->goff.as<uint32_t>(), e->members.as<uint32_t>());
      }
      // distinct-root count to the host: the per-root kernels below are launched over it (a
      // launch over the set count would size their private-segment scratch for n lanes)
      // (one set: one root of one chunk, known without the round trip)
      if (n == 1) {
        e->h_nu[0] = 1;
        e->h_nu[1] = 1;
      } else {
        LB_HIP(hipMemcpyAsync(e->h_nu, e->n_u.p, 8, hipMemcpyDeviceToHost, s1));
        LB_HIP(hipStreamSynchronize(s1));
      }
    }
    const uint32_t nuh = e->h_nu[0];
    e->gmax_chunks = e->h_nu[1];
    if (nuh == 0 || nuh > n) return LB_ERR_DEVICE;
    mu = 1;
    while (mu < nuh) mu <<= 1;
    // ---- s1: hash_to_G2 once per distinct root
    {
      stage_scope sc(e, ST_HASH_MAP, s1);
      if (nuh <= e->hash_row_max && e->alone && e->row_fe)
        hipLaunchKernelGGL(k_hash_map_row, dim3(LB_H2C_FOLD ? (LBR_FP2_W4 ? 2 * nuh : nuh) : (2 * nuh + 3) / 4), dim3(64), 0, s1, n, nuh,
                           e->uniq_set.as<uint32_t>(), b->d_msgs.as<uint8_t>(), e->q.as<uint32_t>());
      else
        hipLaunchKernelGGL(k_hash_map, dim3(nblk(2 * nuh)), dim3(LB_TPB), 0, s1, n, nuh, e->uniq_set.as<uint32_t>(),
                           b->d_msgs.as<uint8_t>(), e->q.as<uint32_t>());
    }
    {
      stage_scope sc(e, ST_HASH_FIN, s1);
      // 8 lanes per root when the device runs no other batch (a few hundred waves on 1 024 SIMDs:
      // latency), one lane per root under load (2.5x less work), as for the Miller loops below
      const bool alone = e->miller_form == 0 && device_alone(e);
      if (nuh <= e->hash_row_max && e->alone && e->row_fe)
        hipLaunchKernelGGL(k_hash_finish_row, dim3(nuh), dim3(LBR_NT), 0, s1, n, nu, e->q.as<uint32_t>(),
                           e->h_aff.as<uint32_t>(), e->hash_row_careful ? 1u : (e->row_proj ? 0u : 2u));
      else if (nuh <= e->hash_g8_max || (LB_HASH_ALONE_G8 && alone))
        hipLaunchKernelGGL(k_hash_finish_g8, dim3((nuh + 7) / 8), dim3(64), 0, s1, n, nu, e->q.as<uint32_t>(),
                           e->h_aff.as<uint32_t>());
      else
      {
        const uint32_t pn = nblk_inv(nuh) * LB_INV_TPB;  // one park column per launched lane
        LB_HIP(e->park.ensure((size_t)4 * 72 * 4 * (pn > n ? pn : n)));
        hipLaunchKernelGGL(k_hash_finish, dim3(nblk_inv(nuh)), dim3(LB_INV_TPB), 0, s1, n, nu, e->q.as<uint32_t>(),
                           e->h_aff.as<uint32_t>(), e->park.as<uint32_t>(), pn);
      }
    }
    // ---- s2: S = sum r_i sig_i by bucket MSM, overlapped with the Miller loops
    if (sb_par) {
      LB_HIP(hipStreamWaitEvent(s2, e->ev_sblind, 0));
      hipLaunchKernelGGL(k_g2_sum_g8, dim3(1), dim3(8 * LB_SUM_G8_GROUPS), 0, s2, n, e->s_terms.as<uint32_t>(),
                         2 * mj, e->treeS.as<uint32_t>(), 1u, e->set_live.as<uint32_t>());
      if (e->profiling) hipEventRecord(e->ev1[ST_SIG_MSM], s2);
    } else if (one_unblinded) {
      stage_scope sc(e, ST_SIG_MSM, s2);
      hipLaunchKernelGGL(k_sig_unblinded, dim3(1), dim3(64), 0, s2, e->sig_aff.as<uint32_t>(),
                         e->set_live.as<uint32_t>(), e->sig_inf.as<uint32_t>(), 2 * mj, e->treeS.as<uint32_t>());
    } else if (n <= e->small_s_max) {
      stage_scope sc(e, ST_SIG_MSM, s2);
      LB_HIP(e->s_terms.ensure((size_t)n * sizeof(g2j)));
      LB_HIP(e->s_part.ensure((size_t)((n + 63) / 64) * sizeof(g2j)));
      if (n <= e->row_max && e->alone && e->row_fe)
        hipLaunchKernelGGL(k_sig_blind_row, dim3(n), dim3(LBR_NT), 0, s2, n, e->sig_aff.as<uint32_t>(),
                           e->scalars.as<uint64_t>(), e->set_live.as<uint32_t>(), e->sig_inf.as<uint32_t>(),
                           e->s_terms.as<uint32_t>(), e->row_proj ? 1u : 0u);
      else if (n <= e->small_s_g8_max)
        hipLaunchKernelGGL(k_sig_blind_g8, dim3((n + 7) / 8), dim3(64), 0, s2, n, e->sig_aff.as<uint32_t>(),
                           e->scalars.as<uint64_t>(), e->set_live.as<uint32_t>(), e->sig_inf.as<uint32_t>(),
                           e->s_terms.as<uint32_t>());
      else
        hipLaunchKernelGGL(k_sig_blind, dim3(nblk_inv(n)), dim3(LB_INV_TPB), 0, s2, n, e->sig_aff.as<uint32_t>(),
                           e->scalars.as<uint64_t>(), e->set_live.as<uint32_t>(), e->sig_inf.as<uint32_t>(),
                           e->s_terms.as<uint32_t>());
      if (n <= e->small_s_g8_max) {  // one workgroup of 8-lane additions
        hipLaunchKernelGGL(k_g2_sum_g8, dim3(1), dim3(8 * LB_SUM_G8_GROUPS), 0, s2, n, e->s_terms.as<uint32_t>(),
                           2 * mj, e->treeS.as<uint32_t>(), 1u, nullptr);
      } else {
        // 64:1 levels, ping-ponging between the two buffers; the last level writes treeS[1]
        uint32_t* bufs[2] = {e->s_terms.as<uint32_t>(), e->s_part.as<uint32_t>()};
        uint32_t m = n;
        int cur = 0;
        while (m > 64) {
          const uint32_t mo = (m + 63) / 64;
          hipLaunchKernelGGL(k_g2_sum64, dim3(mo), dim3(64), 0, s2, m, bufs[cur], mo, bufs[cur ^ 1], 0u);
          m = mo;
          cur ^= 1;
        }
        hipLaunchKernelGGL(k_g2_sum64, dim3(1), dim3(64), 0, s2, m, bufs[cur], 2 * mj, e->treeS.as<uint32_t>(), 1u);
      }
    } else {
      stage_scope sc(e, ST_SIG_MSM, s2);
      LB_HIP(hipMemsetAsync(e->bcnt.p, 0, (size_t)LB_MSM_NB * 4, s2));
      LB_HIP(hipMemsetAsync(e->bcursor.p, 0, (size_t)LB_MSM_NB * 4, s2));
      hipLaunchKernelGGL(k_msm_count, dim3(nblk(n)), dim3(LB_TPB), 0, s2, n, e->scalars.as<uint64_t>(),
                         e->set_live.as<uint32_t>(), e->sig_inf.as<uint32_t>(), e->bcnt.as<uint32_t>());
      hipLaunchKernelGGL(k_msg_scan, dim3(1), dim3(1024), 0, s2, nullptr, (uint32_t)LB_MSM_NB, (uint32_t)LB_MSM_CHUNK,
                         e->bcnt.as<uint32_t>(),
                         e->boff.as<uint32_t>(), e->bch.as<uint32_t>(), e->bchunk_beg.as<uint32_t>(),
                         e->bchunk_end.as<uint32_t>(), nullptr, nullptr);
      hipLaunchKernelGGL(k_msm_scatter, dim3(nblk(n)), dim3(LB_TPB), 0, s2, n, e->scalars.as<uint64_t>(),
                         e->set_live.as<uint32_t>(), e->sig_inf.as<uint32_t>(), e->boff.as<uint32_t>(),
                         e->bcursor.as<uint32_t>(), e->bmembers.as<uint32_t>());
      hipLaunchKernelGGL(k_msm_chunks, dim3(nblk(bcap)), dim3(LB_TPB), 0, s2, e->bch.as<uint32_t>(),
                         e->bchunk_beg.as<uint32_t>(), e->bchunk_end.as<uint32_t>(), e->bmembers.as<uint32_t>(),
                         e->sig_aos.as<uint4>(), bcap, e->bacc.as<uint32_t>(), (uint32_t)LB_MSM_NB);
      LB_HIP(msm_reduce(e, s2, bcap, LB_MSM_NB, 1u, LB_MSM_W, e->treeS.as<uint32_t>(), 2 * mj, 1u,
                        (uint64_t)2 * LB_MSM_W * n, LB_MSM_CHUNK));
    }
    // ---- s1: per-root sums of r_i PK_i and the Miller loops: on speculative liveness (the pubkey
    // side only) as soon as it is done, else after the signature decode
    if (e->spec_gsum) {
      LB_HIP(e->set_spec.ensure((size_t)ns * 4));
      LB_HIP(hipStreamWaitEvent(s1, e->ev_pk, 0));
      hipLaunchKernelGGL(k_spec_live, dim3(nblk(nj)), dim3(LB_TPB), 0, s1, nj, b->d_job_off.as<uint32_t>(),
                         e->pk_status.as<int32_t>(), e->set_spec.as<uint32_t>());
      LB_HIP(per_root_chain(e, n, nuh, mu, e->set_spec.as<uint32_t>()));
    } else {
      LB_HIP(hipStreamWaitEvent(s1, e->ev_dec, 0));
      LB_HIP(hipStreamWaitEvent(s1, e->ev_pk, 0));  // r PK (the decode's wait covered the statuses only)
      LB_HIP(per_root_chain(e, n, nuh, mu, e->set_live.as<uint32_t>()));
    }
  } else {
    // no sets: every job is empty; the message tree is the single identity leaf
    LB_HIP(hipEventRecord(e->ev_dec, s2));
    hipLaunchKernelGGL(k_job_status, dim3(nblk(nj)), dim3(LB_TPB), 0, s1, nj, b->d_job_off.as<uint32_t>(),
                       e->sig_status.as<int32_t>(), e->pk_status.as<int32_t>(), e->job_status.as<int32_t>(),
                       e->set_live.as<uint32_t>());
    hipLaunchKernelGGL(k_set_one, dim3(1), dim3(64), 0, s1, e->treeP.as<uint32_t>(), 2 * mu, mu);
  }
  if (!n) {
    // no sets: S_root = infinity
    hipLaunchKernelGGL(k_g2_set_inf, dim3(1), dim3(64), 0, s2, e->treeS.as<uint32_t>(), 2 * mj, 1u);
  }
  // ---- s2: ML(-G1, S_root)
  {
    stage_scope sc(e, ST_ML_S, s2);
    if (e->alone && e->row_fe)
      hipLaunchKernelGGL(k_ml_S_row, dim3(1), dim3(LBR_NT), 0, s2, mj, e->treeS.as<uint32_t>(), e->fS.as<uint32_t>());
    else
      hipLaunchKernelGGL(k_ml_S, dim3(1), dim3(64), 0, s2, mj, e->treeS.as<uint32_t>(), e->fS.as<uint32_t>());
  }
  LB_HIP(hipEventRecord(e->ev_s, s2));
  LB_HIP(hipStreamWaitEvent(s1, e->ev_s, 0));  // join
  LB_HIP(hipGetLastError());
  if (n && e->spec_gsum) {
    // a set counted in the speculative sums whose signature failed to decode: redo the per-root
    // chain with the full statuses (batches with malformed signatures only)
    LB_HIP(e->live_flag.ensure(4));
    LB_HIP(hipMemsetAsync(e->live_flag.p, 0, 4, s1));
    hipLaunchKernelGGL(k_live_mismatch, dim3(nblk(n)), dim3(LB_TPB), 0, s1, n, e->set_live.as<uint32_t>(),
                       e->set_spec.as<uint32_t>(), e->live_flag.as<uint32_t>());
    LB_HIP(hipMemcpyAsync(e->h_flag, e->live_flag.p, 4, hipMemcpyDeviceToHost, s1));
    LB_HIP(hipStreamSynchronize(s1));
    if (*e->h_flag) LB_HIP(per_root_chain(e, n, *e->h_nu, mu, e->set_live.as<uint32_t>()));
  }
  return LB_OK;
}

// ---------------------------------------------------------------- invalid-set search
// After a failing root check: find the failing SETS (a job fails iff one of its live sets does;
// per-job verdicts then equal the reference's per-job re-verification, worker.ts:76-98, up to
// the 2^-64 soundness of the blinding).  Nodes are ranges of the members array (sets sorted by
// signing root): subtrees of the root product tree (P from the tree), then parts of one root
// (P = one Miller loop of the part's sum r_i PK_i with that root's H(m)).  A failing node
// carries its FE value y.  Two moves (lb_kernels.h k_search_check / k_search_test):
//   direct:   each child c of a node gets its own check, y_c = FE(X_c);
//   weighted: one FE of prod_c X_c^(c+1) names the failing child when exactly one fails.
// A failing node descends by a weighted test (one wave for up to 64 children); if the test finds
// two or more failing children, they are checked directly, each failing child in the same round
// getting a weighted test over its own children.  The root starts with direct checks, so one
// round settles two levels.  Costs: a few waves and range MSMs over the failing ranges per
// round; about four rounds for a batch of ~10^5 sets with a handful of invalid ones.
namespace {
struct snode {
  uint32_t kind;  // 0: node `key` of the root product tree at depth d (d == L: the leaf of root key - mu);
                  // 1: part of root `key`; 2: the single set `key`, checked unblinded
  uint32_t key, lo, len, d;
};
struct fnode {
  snode s;
  bool multi;  // the last weighted test over its children found no single failing child
  std::vector<uint32_t> y;  // FE value (144 words, the k_root_check / k_search_check layout)
};
struct search_ctx {
  uint32_t n, nu, mu, L;
  std::vector<uint32_t> goff, members;
  bool rs = false;  // e->s_root holds the per-root sums S_u
};
enum {
  SX_KIND, SX_KEY, SX_LO, SX_LEN, SX_MIDX, SX_VERDICT, SX_Y, SX_PK,  // direct checks
  SX_MPRE, SX_MLO, SX_MMODE, SX_MWA, SX_MWB, SX_S,                     // MSM instances
  SX_TMODE, SX_TF, SX_TV0, SX_TU, SX_TMIDX, SX_TYIDX, SX_TLO, SX_TLEN, SX_TPER, SX_TOUT, SX_TPK, SX_YUP,
  SX_ML, SX_BLO, SX_BHI, SX_BO, SX_COUNT
};
static_assert(SX_COUNT <= 32, "lb_engine::sx");
struct test_job {
  snode node;
  std::vector<snode> ch;
  bool fresh;    // y from the host (a node failing in an earlier round); else from direct check `d`
  uint32_t src;  // fresh: index into F; else index into D
  int32_t spec = -1;    // a look-ahead test of child `spec_k` of fresh test `spec` (y: the parent's)
  uint32_t spec_k = 0;
};
}  // namespace

// children of a failing node: direct checks fan out to depth max(d + 1, min(d + 7, L - 6)) so a
// weighted test of each failing child can reach the leaves; weighted tests to depth d + 6 (<= 64
// children); a root's members in <= 64 parts for direct checks (one FE each), in <= kWtParts
// parts for a weighted test (one FE whatever f: a root of up to 1024 sets names its failing set
// in one round)
static constexpr uint32_t kWtParts = LB_WT_MAX;
static uint32_t parts_per(uint32_t len, bool direct) {
  const uint32_t f = direct ? 64u : kWtParts;
  return (len + f - 1) / f;
}
#ifndef LB_SEARCH_SPEC
#define LB_SEARCH_SPEC 1  // look-ahead tests over the parts of a fresh test's roots, device idle (0: off; A/B builds)
#endif
static constexpr uint32_t kSpecMaxSets = 16384;  // ... for nodes of at most this many sets
#ifndef LB_SEARCH_BISECT
#define LB_SEARCH_BISECT 0  // 1: the round-2 form (halve such a node), for A/B builds
#endif
static void search_children(const search_ctx& x, const snode& a, bool direct, std::vector<snode>& out) {
  out.clear();
  if (a.kind == 2u || a.len <= 1) return;
  auto parts = [&](uint32_t u, uint32_t lo, uint32_t len) {
    const uint32_t per = parts_per(len, direct);
    for (uint32_t q = 0; q < len; q += per) {
      const uint32_t l = per < len - q ? per : len - q;
      if (l == 1 && direct) out.push_back({2u, x.members[lo + q], lo + q, 1u, 0u});
      else out.push_back({1u, u, lo + q, l, 0u});
    }
  };
  if (a.kind == 1u) return parts(a.key, a.lo, a.len);
  if (a.d == x.L) return parts(a.key - x.mu, a.lo, a.len);
  const int d = (int)a.d, L = (int)x.L;
  // direct children: subtrees of 64 roots (their weighted tests can name one failing root); a
  // node of <= 64 roots whose weighted test matched nothing (>= 2 failing roots) is checked root by
  // root in ONE round (halving it instead took up to six rounds for two wrong roots in a subtree)
  int dd = direct ? (d >= L - 6 && !LB_SEARCH_BISECT ? L : std::max(d + 1, std::min(d + 7, L - 6))) : d + 6;
  if (dd > L) dd = L;
  const uint32_t k = (uint32_t)(dd - d), span = (uint32_t)(L - dd);
  for (uint32_t v = a.key << k; v < (a.key + 1) << k; v++) {
    const uint32_t ulo = (v - (1u << dd)) << span;
    if (ulo >= x.nu) break;
    const uint32_t uhi = std::min(x.nu, ulo + (1u << span));
    out.push_back({0u, v, x.goff[ulo], x.goff[uhi] - x.goff[ulo], (uint32_t)dd});
  }
}

template <class T>
static hipError_t sx_up(lb_engine* e, int k, const std::vector<T>& v, hipStream_t s) {
  hipError_t r = e->sx[k].ensure((v.empty() ? 1 : v.size()) * sizeof(T));
  if (r == hipSuccess && !v.empty()) r = hipMemcpyAsync(e->sx[k].p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
  return r;
}

// One launch set: direct checks D, then weighted tests (fresh ones first).  Outputs the direct
// verdicts and FE values (144 words each) and each test's matched child (1-based, 0: none).
static int32_t search_round(lb_engine* e, const search_ctx& x, const std::vector<fnode>& F, const std::vector<snode>& D,
                            const std::vector<test_job>& tests, uint32_t n_fresh, std::vector<int32_t>& verdict,
                            std::vector<uint32_t>& ydir, std::vector<int32_t>& tout) {
  hipStream_t s1 = e->stream;
  const uint32_t c = (uint32_t)D.size(), nt = (uint32_t)tests.size(), n = x.n;
  std::vector<uint32_t> dk(c), dkey(c), dlo(c), dlen(c), dm(c, 0);
  std::vector<uint32_t> mlo, mpre{0}, mmode, mwa, mwb;
  // the same instances over whole roots (root-level form), while every instance is one
  std::vector<uint32_t> rlo, rpre{0};
  bool root_level = x.rs;
  auto msm = [&](uint32_t lo, uint32_t len, uint32_t mode, uint32_t wa, uint32_t wb, const snode* whole) {
    mlo.push_back(lo);
    mpre.push_back(mpre.back() + len);
    mmode.push_back(mode);
    mwa.push_back(wa);
    mwb.push_back(wb);
    if (whole && whole->kind == 0u) {
      const uint32_t span = x.L - whole->d, ulo = (whole->key - (1u << whole->d)) << span;
      const uint32_t uhi = std::min(x.nu, ulo + (1u << span));
      rlo.push_back(ulo);
      rpre.push_back(rpre.back() + (uhi - ulo));
    } else {
      root_level = false;
    }
    return (uint32_t)mlo.size() - 1;
  };
  for (uint32_t j = 0; j < c; j++) {
    dk[j] = D[j].kind;
    dkey[j] = D[j].key;
    dlo[j] = D[j].lo;
    dlen[j] = D[j].len;
    if (D[j].kind != 2u) dm[j] = msm(D[j].lo, D[j].len, 0u, 1u, 0u, &D[j]);
  }
  std::vector<uint32_t> tmode(nt), tf(nt), tv0(nt), tu(nt), tm(nt), tyi(nt), tlo(nt), tlen(nt), tper(nt);
  std::vector<uint32_t> yup((size_t)144 * (n_fresh ? n_fresh : 1));
  for (uint32_t t = 0; t < nt; t++) {
    const test_job& T = tests[t];
    const snode& a = T.node;
    const snode& c0 = T.ch[0];
    tf[t] = (uint32_t)T.ch.size();
    tlo[t] = a.lo;
    tlen[t] = a.len;
    tyi[t] = T.src;
    if (c0.kind == 0u) {  // subtrees of 2^span roots from root ulo0
      const uint32_t span = x.L - c0.d, ulo0 = (c0.key - (1u << c0.d)) << span;
      tmode[t] = 1u;
      tv0[t] = c0.key;
      tm[t] = msm(a.lo, a.len, 1u, ulo0, span, &a);
    } else {  // parts of one root
      const uint32_t per = parts_per(a.len, false);
      tmode[t] = 2u;
      tu[t] = c0.key;
      tper[t] = per;
      tm[t] = msm(a.lo, a.len, 2u, per, 0u, nullptr);
    }
    if (T.fresh) {
      tyi[t] = t;  // fresh tests come first: y_up element t
      for (int q = 0; q < 144; q++) yup[(size_t)q * n_fresh + t] = F[T.src].y[q];
    }
  }
  // root-level round: every instance covers whole roots and the per-set form would take the
  // bucket MSM; the instances then run over the per-root sums S_u (k_rsm_terms)
  const bool rs_path = root_level && !mlo.empty() && mpre.back() > e->search_small_max;
  if (rs_path) {
    mlo.swap(rlo);
    mpre.swap(rpre);
  }
  // weight-1 instances only: 32-bit GLV halves, 4 windows instead of 6
  const bool w4 = std::all_of(mmode.begin(), mmode.end(), [](uint32_t m) { return m == 0u; });
  const uint32_t nwin = w4 ? (uint32_t)LB_MSM_W : (uint32_t)LB_SMSM_W;
  const uint32_t cm = (uint32_t)mlo.size(), T = mpre.back(), nb = cm * nwin * LB_MSM_B;
  const uint32_t schunk = e->search_chunk;
  const uint32_t bcap = (2 * nwin * T) / schunk + nb;
  LB_HIP(sx_up(e, SX_KIND, dk, s1));
  LB_HIP(sx_up(e, SX_KEY, dkey, s1));
  LB_HIP(sx_up(e, SX_LO, dlo, s1));
  LB_HIP(sx_up(e, SX_LEN, dlen, s1));
  LB_HIP(sx_up(e, SX_MIDX, dm, s1));
  LB_HIP(sx_up(e, SX_MPRE, mpre, s1));
  LB_HIP(sx_up(e, SX_MLO, mlo, s1));
  LB_HIP(sx_up(e, SX_MMODE, mmode, s1));
  LB_HIP(sx_up(e, SX_MWA, mwa, s1));
  LB_HIP(sx_up(e, SX_MWB, mwb, s1));
  LB_HIP(sx_up(e, SX_TMODE, tmode, s1));
  LB_HIP(sx_up(e, SX_TF, tf, s1));
  LB_HIP(sx_up(e, SX_TV0, tv0, s1));
  LB_HIP(sx_up(e, SX_TU, tu, s1));
  LB_HIP(sx_up(e, SX_TMIDX, tm, s1));
  LB_HIP(sx_up(e, SX_TYIDX, tyi, s1));
  LB_HIP(sx_up(e, SX_TLO, tlo, s1));
  LB_HIP(sx_up(e, SX_TLEN, tlen, s1));
  LB_HIP(sx_up(e, SX_TPER, tper, s1));
  LB_HIP(sx_up(e, SX_YUP, yup, s1));
  const uint32_t N = c + nt;
  LB_HIP(e->sx[SX_VERDICT].ensure((c ? c : 1) * 4));
  LB_HIP(e->sx[SX_Y].ensure((size_t)(N ? N : 1) * 576));
  LB_HIP(e->sx[SX_ML].ensure((size_t)(N ? N : 1) * 2 * 576));
  LB_HIP(e->sx[SX_PK].ensure((c ? c : 1) * sizeof(g1j)));
  LB_HIP(e->sx[SX_S].ensure((cm ? cm : 1) * sizeof(g2j)));
  LB_HIP(e->sx[SX_TOUT].ensure((nt ? nt : 1) * 4));
  LB_HIP(e->sx[SX_TPK].ensure((nt ? nt : 1) * sizeof(g1j)));
  auto U = [&](int k) { return e->sx[k].as<uint32_t>(); };
  {
    stage_scope sc(e, ST_FALLBACK, s1);
    const bool pre = x.rs && e->search_pre;
    if (cm && T && (rs_path || pre || T <= e->search_small_max)) {
      // small or root-level round: per-position terms + per-instance segmented sums (no bucket MSM)
      std::vector<uint32_t> blo, bhi, bo{0};
      for (uint32_t j = 0; j < cm; j++) {
        for (uint32_t p = mpre[j]; p < mpre[j + 1]; p += 64) {
          blo.push_back(p);
          bhi.push_back(std::min(p + 64, mpre[j + 1]));
        }
        bo.push_back((uint32_t)blo.size());
      }
      const uint32_t nbk = (uint32_t)blo.size();
      LB_HIP(sx_up(e, SX_BLO, blo, s1));
      LB_HIP(sx_up(e, SX_BHI, bhi, s1));
      LB_HIP(sx_up(e, SX_BO, bo, s1));
      LB_HIP(e->s_terms.ensure((size_t)T * sizeof(g2j)));
      LB_HIP(e->s_part.ensure((size_t)(nbk ? nbk : 1) * sizeof(g2j)));
      const smsm_args ma{U(SX_MPRE), U(SX_MLO), U(SX_MMODE), U(SX_MWA), U(SX_MWB)};
      if (rs_path)
        hipLaunchKernelGGL(k_rsm_terms, dim3(nblk(T)), dim3(LB_TPB), 0, s1, T, cm, ma, e->s_root.as<uint32_t>(), x.nu,
                           e->s_terms.as<uint32_t>());
      else if (pre)  // the per-set terms r_i sig_i are kept from search_root_sums
        hipLaunchKernelGGL(k_smsm_terms_pre, dim3(nblk(T)), dim3(LB_TPB), 0, s1, T, cm, ma, e->members.as<uint32_t>(),
                           e->set_uid.as<uint32_t>(), e->s_set.as<uint32_t>(), n, e->s_terms.as<uint32_t>());
      else if (e->smsm_form == 1 ||
               (e->smsm_form == 0 && !device_alone(e)))
        hipLaunchKernelGGL(k_smsm_terms_lane, dim3(nblk_inv(T)), dim3(LB_INV_TPB), 0, s1, T, cm, ma,
                           e->members.as<uint32_t>(), e->set_uid.as<uint32_t>(), e->scalars.as<uint64_t>(),
                           e->set_live.as<uint32_t>(), e->sig_inf.as<uint32_t>(), e->sig_aff.as<uint32_t>(), n,
                           e->s_terms.as<uint32_t>());
      else
        hipLaunchKernelGGL(k_smsm_terms_g8, dim3((T + 7) / 8), dim3(64), 0, s1, T, cm, ma, e->members.as<uint32_t>(),
                           e->set_uid.as<uint32_t>(), e->scalars.as<uint64_t>(), e->set_live.as<uint32_t>(),
                           e->sig_inf.as<uint32_t>(), e->sig_aff.as<uint32_t>(), n, e->s_terms.as<uint32_t>());
      if (nbk)
        hipLaunchKernelGGL(k_seg_sum64, dim3(nbk), dim3(64), 0, s1, U(SX_BLO), U(SX_BHI), T, e->s_terms.as<uint32_t>(),
                           nbk, e->s_part.as<uint32_t>(), nullptr);
      hipLaunchKernelGGL(k_seg_final, dim3(cm), dim3(64), 0, s1, U(SX_BO), e->s_part.as<uint32_t>(), nbk ? nbk : 1u,
                         U(SX_S), cm);
    } else if (cm) {
      LB_HIP(e->bcnt.ensure((size_t)nb * 4));
      LB_HIP(e->bcursor.ensure((size_t)nb * 4));
      LB_HIP(e->boff.ensure((size_t)(nb + 1) * 4));
      LB_HIP(e->bch.ensure((size_t)(nb + 1) * 4));
      LB_HIP(e->bchunk_beg.ensure((size_t)bcap * 4));
      LB_HIP(e->bchunk_end.ensure((size_t)bcap * 4));
      LB_HIP(e->bmembers.ensure((size_t)2 * nwin * (T ? T : 1) * 4));
      LB_HIP(e->bacc.ensure((size_t)bcap * sizeof(g2j)));
      LB_HIP(e->bsum.ensure((size_t)nb * sizeof(g2j)));
      LB_HIP(hipMemsetAsync(e->bcnt.p, 0, (size_t)nb * 4, s1));
      LB_HIP(hipMemsetAsync(e->bcursor.p, 0, (size_t)nb * 4, s1));
      const smsm_args ma{U(SX_MPRE), U(SX_MLO), U(SX_MMODE), U(SX_MWA), U(SX_MWB)};
      if (T) {
        if (w4)
          hipLaunchKernelGGL(k_smsm_count<LB_MSM_W>, dim3(nblk(T)), dim3(LB_TPB), 0, s1, T, cm, ma,
                             e->members.as<uint32_t>(), e->set_uid.as<uint32_t>(), e->scalars.as<uint64_t>(),
                             e->set_live.as<uint32_t>(), e->sig_inf.as<uint32_t>(), e->bcnt.as<uint32_t>());
        else
          hipLaunchKernelGGL(k_smsm_count<LB_SMSM_W>, dim3(nblk(T)), dim3(LB_TPB), 0, s1, T, cm, ma,
                             e->members.as<uint32_t>(), e->set_uid.as<uint32_t>(), e->scalars.as<uint64_t>(),
                             e->set_live.as<uint32_t>(), e->sig_inf.as<uint32_t>(), e->bcnt.as<uint32_t>());
      }
      hipLaunchKernelGGL(k_msg_scan, dim3(1), dim3(1024), 0, s1, nullptr, nb, schunk, e->bcnt.as<uint32_t>(),
                         e->boff.as<uint32_t>(), e->bch.as<uint32_t>(), e->bchunk_beg.as<uint32_t>(),
                         e->bchunk_end.as<uint32_t>(), nullptr, nullptr);
      if (T) {
        if (w4)
          hipLaunchKernelGGL(k_smsm_scatter<LB_MSM_W>, dim3(nblk(T)), dim3(LB_TPB), 0, s1, T, cm, ma,
                             e->members.as<uint32_t>(), e->set_uid.as<uint32_t>(), e->scalars.as<uint64_t>(),
                             e->set_live.as<uint32_t>(), e->sig_inf.as<uint32_t>(), e->boff.as<uint32_t>(),
                             e->bcursor.as<uint32_t>(), e->bmembers.as<uint32_t>());
        else
          hipLaunchKernelGGL(k_smsm_scatter<LB_SMSM_W>, dim3(nblk(T)), dim3(LB_TPB), 0, s1, T, cm, ma,
                             e->members.as<uint32_t>(), e->set_uid.as<uint32_t>(), e->scalars.as<uint64_t>(),
                             e->set_live.as<uint32_t>(), e->sig_inf.as<uint32_t>(), e->boff.as<uint32_t>(),
                             e->bcursor.as<uint32_t>(), e->bmembers.as<uint32_t>());
      }
      hipLaunchKernelGGL(k_msm_chunks, dim3(nblk(bcap)), dim3(LB_TPB), 0, s1, e->bch.as<uint32_t>(),
                         e->bchunk_beg.as<uint32_t>(), e->bchunk_end.as<uint32_t>(), e->bmembers.as<uint32_t>(),
                         e->sig_aos.as<uint4>(), bcap, e->bacc.as<uint32_t>(), nb);
      LB_HIP(msm_reduce(e, s1, bcap, nb, cm, w4 ? LB_MSM_W : LB_SMSM_W, U(SX_S), cm, 0u, (uint64_t)2 * nwin * T,
                        schunk));
    }
    if (c)
      hipLaunchKernelGGL(k_range_pk, dim3(nblk(c)), dim3(LB_TPB), 0, s1, c, U(SX_KIND), U(SX_LO), U(SX_LEN),
                         e->members.as<uint32_t>(), e->set_live.as<uint32_t>(), n, e->rpk.as<uint32_t>(), U(SX_PK));
    if (nt)
      hipLaunchKernelGGL(k_test_pk, dim3(nt), dim3(64), 0, s1, nt, U(SX_TMODE), U(SX_TLO), U(SX_TLEN), U(SX_TPER),
                         e->members.as<uint32_t>(), e->set_live.as<uint32_t>(), n, e->rpk.as<uint32_t>(), U(SX_TPK));
  }
  {
    stage_scope sc(e, ST_BISECT, s1);
    const srch_items I{c, nt, n_fresh, e->search_merge ? 0u : 1u, U(SX_KIND), U(SX_KEY), U(SX_MIDX), U(SX_TMODE), U(SX_TF), U(SX_TV0),
                       U(SX_TU), U(SX_TMIDX), U(SX_TYIDX)};
    auto stage = [&](uint32_t it0, uint32_t cnt) {
      if (!cnt) return;
      hipLaunchKernelGGL(k_search_ml, dim3(2 * cnt), dim3(64), 0, s1, I, it0, cnt, cm ? cm : 1u, e->treeP.as<uint32_t>(),
                         2 * x.mu, U(SX_PK), U(SX_TPK), e->h_aff.as<uint32_t>(), n, U(SX_S), e->pk_aff.as<uint32_t>(),
                         e->sig_aff.as<uint32_t>(), e->sig_inf.as<uint32_t>(), e->set_live.as<uint32_t>(),
                         e->set_uid.as<uint32_t>(), U(SX_Y), U(SX_ML));
      hipLaunchKernelGGL(k_search_fe, dim3(cnt), dim3(64), 0, s1, I, it0, cnt, U(SX_ML), U(SX_Y),
                         e->sx[SX_VERDICT].as<int32_t>());
    };
    if (e->search_merge) {
      stage(0, c + nt);
    } else {
      stage(0, c + n_fresh);             // direct checks and fresh tests
      stage(c + n_fresh, nt - n_fresh);  // look-ahead tests of the failing direct checks
    }
    if (nt) hipLaunchKernelGGL(k_search_match, dim3(nt), dim3(64), 0, s1, I, U(SX_YUP), U(SX_Y), e->sx[SX_TOUT].as<int32_t>());
  }
  LB_HIP(hipGetLastError());
  verdict.resize(c);
  ydir.resize((size_t)144 * N);  // SoA, stride N = c + nt (direct checks first)
  tout.resize(nt);
  if (c) {
    LB_HIP(hipMemcpyAsync(verdict.data(), e->sx[SX_VERDICT].p, (size_t)c * 4, hipMemcpyDeviceToHost, s1));
    LB_HIP(hipMemcpyAsync(ydir.data(), e->sx[SX_Y].p, (size_t)N * 576, hipMemcpyDeviceToHost, s1));
  }
  if (nt) LB_HIP(hipMemcpyAsync(tout.data(), e->sx[SX_TOUT].p, (size_t)nt * 4, hipMemcpyDeviceToHost, s1));
  LB_HIP(hipStreamSynchronize(s1));
  if (e->profiling)
    for (int k : {(int)ST_FALLBACK, (int)ST_BISECT}) {
      float ms = 0.f;
      if (e->used[k] && hipEventElapsedTime(&ms, e->ev0[k], e->ev1[k]) == hipSuccess) e->acc_ms[k] += ms;
      e->used[k] = false;
    }
  return LB_OK;
}

// S_u = sum r_i sig_i over the live sets of each root u (members order): the per-set terms one
// lane per set (k_sig_blind), then segmented sums over each root's positions (blocks of <= 64 of
// one root, then one wave per root).  Once per search, for large batches: the root-level
// instances of a round (subtrees and weighted subtree tests) then cost a 7-bit multiple per ROOT.
static int32_t search_root_sums(lb_engine* e, const search_ctx& x) {
  hipStream_t s1 = e->stream;
  const uint32_t n = x.n, nu = x.nu;
  std::vector<uint32_t> idx;  // blo[nbk] | bhi[nbk] | bo[nu + 1]
  std::vector<uint32_t> blo, bhi, bo{0};
  for (uint32_t u = 0; u < nu; u++) {
    for (uint32_t p = x.goff[u]; p < x.goff[u + 1]; p += 64) {
      blo.push_back(p);
      bhi.push_back(std::min(p + 64, x.goff[u + 1]));
    }
    bo.push_back((uint32_t)blo.size());
  }
  const uint32_t nbk = (uint32_t)blo.size();
  idx.insert(idx.end(), blo.begin(), blo.end());
  idx.insert(idx.end(), bhi.begin(), bhi.end());
  idx.insert(idx.end(), bo.begin(), bo.end());
  LB_HIP(e->rs_idx.ensure(idx.size() * 4));
  LB_HIP(e->s_set.ensure((size_t)n * sizeof(g2j)));
  LB_HIP(e->s_part.ensure((size_t)(nbk ? nbk : 1) * sizeof(g2j)));
  LB_HIP(e->s_root.ensure((size_t)nu * sizeof(g2j)));
  LB_HIP(hipMemcpyAsync(e->rs_idx.p, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, s1));
  const uint32_t* d_idx = e->rs_idx.as<uint32_t>();
  {
    stage_scope sc(e, ST_FALLBACK, s1);
    hipLaunchKernelGGL(k_sig_blind, dim3(nblk_inv(n)), dim3(LB_INV_TPB), 0, s1, n, e->sig_aff.as<uint32_t>(),
                       e->scalars.as<uint64_t>(), e->set_live.as<uint32_t>(), e->sig_inf.as<uint32_t>(),
                       e->s_set.as<uint32_t>());
    if (nbk)
      hipLaunchKernelGGL(k_seg_sum64, dim3(nbk), dim3(64), 0, s1, d_idx, d_idx + nbk, n, e->s_set.as<uint32_t>(), nbk,
                         e->s_part.as<uint32_t>(), e->members.as<uint32_t>());
    hipLaunchKernelGGL(k_seg_final, dim3(nu), dim3(64), 0, s1, d_idx + 2 * nbk, e->s_part.as<uint32_t>(),
                       nbk ? nbk : 1u, e->s_root.as<uint32_t>(), nu);
  }
  LB_HIP(hipGetLastError());
  LB_HIP(hipStreamSynchronize(s1));
  if (e->profiling) {
    float ms = 0.f;
    if (e->used[ST_FALLBACK] && hipEventElapsedTime(&ms, e->ev0[ST_FALLBACK], e->ev1[ST_FALLBACK]) == hipSuccess)
      e->acc_ms[ST_FALLBACK] += ms;
    e->used[ST_FALLBACK] = false;
  }
  return LB_OK;
}

static int32_t search_invalid(lb_engine* e, lb_batch* b, uint32_t mu, int32_t* out_job) {
  const uint32_t n = b->n_sets, nj = b->n_jobs;
  if (e->rpk_stale && n) {
    // the per-root sums ran the Straus form (no per-set r PK): the search's range sums need them
    hipLaunchKernelGGL(k_pk_blind, dim3(nblk_inv(n)), dim3(LB_INV_TPB), 0, e->stream, n, b->n_chunks,
                       b->d_set_chunk_off.as<uint32_t>(), e->chunk_acc.as<uint32_t>(), e->chunk_status.as<int32_t>(),
                       e->pk_aff.as<uint32_t>(), e->scalars.as<uint64_t>(), e->rpk.as<uint32_t>(),
                       e->pk_status.as<int32_t>(), 2u, nullptr);
    LB_HIP(hipGetLastError());
    e->rpk_stale = false;
  }
  search_ctx x;
  x.n = n;
  x.mu = mu;
  x.L = 0;
  while ((1u << x.L) < mu) x.L++;
  x.nu = *e->h_nu;
  x.goff.resize(x.nu + 1);
  x.members.resize(n);
  fnode root{{0u, 1u, 0u, n, 0u}, true, std::vector<uint32_t>(144)};
  LB_HIP(hipMemcpyAsync(x.goff.data(), e->goff.p, (size_t)(x.nu + 1) * 4, hipMemcpyDeviceToHost, e->stream));
  LB_HIP(hipMemcpyAsync(x.members.data(), e->members.p, (size_t)n * 4, hipMemcpyDeviceToHost, e->stream));
  LB_HIP(hipMemcpyAsync(root.y.data(), e->y_root.p, 576, hipMemcpyDeviceToHost, e->stream));
  LB_HIP(hipStreamSynchronize(e->stream));
  // the first round's form for large batches (see lb_engine::search_blk)
  const bool r1_plain = e->search_blk && x.nu > 1 && n > e->search_small_max;
  if (!r1_plain && e->search_rootsum && x.nu > 1 && n > e->search_small_max) {
    const int32_t st = search_root_sums(e, x);
    if (st != LB_OK) return st;
    x.rs = true;
  }
  std::vector<fnode> F{root};
  std::vector<uint32_t> bad_pos;
  auto condemn = [&](const snode& a) {
    for (uint32_t q = 0; q < a.len; q++) bad_pos.push_back(a.lo + q);
  };
  const bool trace = std::getenv("LB_SEARCH_TRACE") != nullptr;
  const size_t kMaxMsm = 1024;  // MSM instances per launch set (1280 buckets each)
  std::vector<snode> ch;
  for (int round = 1; !F.empty(); round++) {
    if (round > 64) {  // depth is bounded far below this; fail closed if it is ever exceeded
      for (const fnode& f : F) condemn(f.s);
      break;
    }
    std::vector<fnode> next;
    // settle single-child chains and terminals on the host
    std::vector<fnode> work;
    for (fnode& f : F) {
      while (true) {
        if (f.s.len <= 1) {
          bad_pos.push_back(f.s.lo);
          break;
        }
        search_children(x, f.s, f.multi, ch);
        if (ch.size() == 1) {
          f.s = ch[0];
          f.multi = false;
          continue;
        }
        if (ch.empty()) condemn(f.s);
        else work.push_back(f);
        break;
      }
    }
    const bool spec_on = LB_SEARCH_SPEC && device_alone(e);
    for (size_t a = 0; a < work.size();) {
      // a launch set: whole failing nodes until the MSM instance budget is reached
      std::vector<fnode> Fs;
      std::vector<snode> D;
      std::vector<uint32_t> d_owner;  // D index -> Fs index
      std::vector<test_job> fresh, spec, ahead;
      size_t inst = 0;
      while (a < work.size() && (Fs.empty() || inst < kMaxMsm)) {
        const fnode& f = work[a++];
        const uint32_t fi = (uint32_t)Fs.size();
        Fs.push_back(f);
        if (!f.multi) {
          test_job t{f.s, {}, true, fi};
          search_children(x, f.s, false, t.ch);
          // a weighted test over <= 64 ROOTS: in the same round, a weighted test over each root's
          // parts, matched against the node's own y (if the node's test names root k, root k is the
          // node's one failing child and y_k = y).  The named root's test then names the set, one
          // round earlier; the other roots' tests are discarded.  Only while the device runs no
          // other batch: under load their Miller loops and final exponentiations cost more than
          // the round they save (profiles/r3_search_spec_ab.txt).
          if (spec_on && !t.ch.empty() && t.ch[0].kind == 0u && t.ch[0].d == x.L && f.s.len <= kSpecMaxSets)
            for (uint32_t k = 0; k < (uint32_t)t.ch.size(); k++) {
              test_job g{t.ch[k], {}, true, fi};
              search_children(x, t.ch[k], false, g.ch);
              if (g.ch.size() < 2) continue;
              g.spec = (int32_t)fresh.size();
              g.spec_k = k;
              spec.push_back(std::move(g));
              inst++;
            }
          fresh.push_back(std::move(t));
          inst++;
          continue;
        }
        std::vector<snode> dch;
        search_children(x, f.s, true, dch);
        for (const snode& c : dch) {
          const uint32_t di = (uint32_t)D.size();
          D.push_back(c);
          d_owner.push_back(fi);
          inst += c.kind != 2u;
          test_job t{c, {}, false, di};
          search_children(x, c, false, t.ch);
          if (t.ch.size() >= 2 && !(r1_plain && round == 1)) {
            ahead.push_back(std::move(t));
            inst++;
          }
        }
      }
      std::vector<test_job> tests(fresh);
      const uint32_t n_own = (uint32_t)fresh.size();
      tests.insert(tests.end(), spec.begin(), spec.end());  // fresh too: y from the host
      const uint32_t n_fresh = (uint32_t)tests.size();
      tests.insert(tests.end(), ahead.begin(), ahead.end());
      std::vector<int32_t> verdict, tout;
      std::vector<uint32_t> ydir;
      const auto t0 = std::chrono::steady_clock::now();
      const int32_t st = search_round(e, x, Fs, D, tests, n_fresh, verdict, ydir, tout);
      if (st != LB_OK) return st;
      if (trace)
        std::fprintf(stderr, "[lb search] round %d: %zu failing nodes, %zu direct checks, %zu weighted tests: %.3f ms\n",
                     round, Fs.size(), D.size(), tests.size(),
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
      // fresh tests: the named child (or, by its look-ahead test, the named child's named part),
      // or the node again with its children to check directly
      std::vector<int32_t> spec_of;  // (own test, child) -> look-ahead test
      std::vector<uint32_t> spec_base(n_own + 1, 0);
      for (uint32_t t = n_own; t < n_fresh; t++) spec_base[tests[t].spec + 1]++;
      for (uint32_t t = 0; t < n_own; t++) spec_base[t + 1] += spec_base[t];
      for (uint32_t t = n_own; t < n_fresh; t++) spec_of.push_back((int32_t)t);  // grouped by own test, child order
      for (uint32_t t = 0; t < n_own; t++) {
        const fnode& f = Fs[tests[t].src];
        const int k = tout[t];
        if (k < 1 || (size_t)k > tests[t].ch.size()) {
          next.push_back({f.s, true, f.y});
          continue;
        }
        int32_t st = -1;
        for (uint32_t q = spec_base[t]; q < spec_base[t + 1]; q++)
          if (tests[spec_of[q]].spec_k == (uint32_t)(k - 1)) st = spec_of[q];
        if (st < 0) {
          next.push_back({tests[t].ch[k - 1], false, f.y});
          continue;
        }
        const int k2 = tout[st];
        if (k2 >= 1 && (size_t)k2 <= tests[st].ch.size()) next.push_back({tests[st].ch[k2 - 1], false, f.y});
        else next.push_back({tests[t].ch[k - 1], true, f.y});
      }
      // direct checks: each failing child goes on by its weighted test
      std::vector<int> any_fail(Fs.size(), 0);
      std::vector<int32_t> ahead_of(D.size(), -1);
      for (uint32_t t = n_fresh; t < tests.size(); t++) ahead_of[tests[t].src] = (int32_t)t;
      for (uint32_t j = 0; j < D.size(); j++) {
        if (verdict[j]) continue;
        any_fail[d_owner[j]] = 1;
        std::vector<uint32_t> yc(144);  // y_out is SoA with stride c: gather this node's 144 words
        for (int q = 0; q < 144; q++) yc[q] = ydir[(size_t)q * (D.size() + tests.size()) + j];
        const int32_t t = ahead_of[j];
        if (t < 0) {
          next.push_back({D[j], false, yc});  // terminal or a single child: settled next round
          continue;
        }
        const int k = tout[t];
        if (k >= 1 && (size_t)k <= tests[t].ch.size()) next.push_back({tests[t].ch[k - 1], false, yc});
        else next.push_back({D[j], true, yc});
      }
      // fail closed: a multi node none of whose children fails (impossible for exact arithmetic)
      for (size_t fi = 0; fi < Fs.size(); fi++)
        if (Fs[fi].multi && !any_fail[fi]) condemn(Fs[fi].s);
    }
    F.swap(next);
  }
  // failing sets -> their jobs (set_live makes every failing set belong to a live job)
  for (uint32_t pos : bad_pos) {
    const uint32_t i = x.members[pos];
    const uint32_t j = (uint32_t)(std::upper_bound(b->job_off.begin(), b->job_off.end(), i) - b->job_off.begin()) - 1;
    if (j < nj && out_job[j] == 1) out_job[j] = 0;
  }
  return LB_OK;
}

static void finish_profile(lb_engine* e) {
  if (!e->profiling) return;
  hipStreamSynchronize(e->stream3);
  hipStreamSynchronize(e->stream2);
  hipStreamSynchronize(e->stream);
  for (int k = 0; k < kStages; k++) {
    float ms = 0.f;
    if (e->used[k]) hipEventElapsedTime(&ms, e->ev0[k], e->ev1[k]);
    e->last_ms[k] = ms + e->acc_ms[k];
  }
}

// The engine's streams for the duration of one call: the high-priority trio for small batches
// (created once, at the greatest priority), the normal trio otherwise.  The caller holds e->mu.
struct stream_choice {
  lb_engine* e;
  bool swapped = false;
  stream_choice(lb_engine* e_, uint32_t n_sets) : e(e_) {
    if (!e->prio_max || n_sets > e->prio_max) return;
    if (!e->hp[0]) {
      int least = 0, greatest = 0;
      hipDeviceGetStreamPriorityRange(&least, &greatest);
      for (int k = 0; k < 3; k++)
        if (hipStreamCreateWithPriority(&e->hp[k], hipStreamNonBlocking, greatest) != hipSuccess) {
          for (int j = 0; j <= k; j++)
            if (e->hp[j]) hipStreamDestroy(e->hp[j]);
          e->hp[0] = e->hp[1] = e->hp[2] = nullptr;
          return;  // the normal streams still work
        }
    }
    std::swap(e->stream, e->hp[0]);
    std::swap(e->stream2, e->hp[1]);
    std::swap(e->stream3, e->hp[2]);
    swapped = true;
  }
  ~stream_choice() {
    if (!swapped) return;
    std::swap(e->stream, e->hp[0]);
    std::swap(e->stream2, e->hp[1]);
    std::swap(e->stream3, e->hp[2]);
  }
};

// caller holds e->mu
static int32_t verify_locked(lb_engine* e, lb_batch* b, const uint64_t* scalars, int32_t* out_job) {
  LB_HIP(hipSetDevice(e->device));
  stream_choice sch(e, b->n_sets);
  const uint32_t nj = b->n_jobs;
  if (nj == 0) return LB_OK;
  uint32_t m = 1, mu = 1;
  busy_scope busy(e->device, e, e->latency);
  int32_t st = run_pipeline(e, b, scalars, m, mu, true);
  if (st != LB_OK) return st;
  // root verdict on s1 (after the join)
  LB_HIP(e->verdict.ensure(4));
  {
    stage_scope sc(e, ST_ROOT, e->stream);
    LB_HIP(e->y_root.ensure(576));
    hipLaunchKernelGGL((e->alone && e->row_fe) ? k_root_check_row : k_root_check, dim3(1), dim3((e->alone && e->row_fe) ? LBR_NT : 64), 0, e->stream, mu, e->treeP.as<uint32_t>(),
                       e->fS.as<uint32_t>(), e->verdict.as<int32_t>(), e->y_root.as<uint32_t>());
  }
  LB_HIP(hipGetLastError());
  std::vector<int32_t> jst(nj);
  int32_t root_ok = 0;
  LB_HIP(hipMemcpyAsync(jst.data(), e->job_status.p, (size_t)nj * 4, hipMemcpyDeviceToHost, e->stream));
  LB_HIP(hipMemcpyAsync(&root_ok, e->verdict.p, 4, hipMemcpyDeviceToHost, e->stream));
  LB_HIP(hipStreamSynchronize(e->stream));
  bool any_live = false;
  for (uint32_t j = 0; j < nj; j++) {
    out_job[j] = jst[j] == LB_OK ? 1 : -jst[j];
    any_live |= jst[j] == LB_OK;
  }
  if (any_live && !root_ok) {
    st = search_invalid(e, b, mu, out_job);
    if (st != LB_OK) return st;
  }
  if (e->profiling) hipEventRecord(e->ev1[ST_TOTAL], e->stream);
  finish_profile(e);
  return LB_OK;
}

extern "C" int32_t lb_batch_verify(lb_engine* e, lb_batch* b, const uint64_t* scalars, int32_t* out_job) {
  if (!e || !b || (b->n_jobs && !out_job)) return LB_ERR_ARGUMENT;
  std::lock_guard<std::mutex> lk(e->mu);
  return verify_locked(e, b, scalars, out_job);
}

extern "C" int32_t lb_batch_partial(lb_engine* e, lb_batch* b, const uint64_t* scalars, uint8_t* out576,
                                    int32_t* out_job) {
  if (!e || !b || !out576 || (b->n_jobs && !out_job)) return LB_ERR_ARGUMENT;
  std::lock_guard<std::mutex> lk(e->mu);
  LB_HIP(hipSetDevice(e->device));
  uint32_t m = 1, mu = 1;
  if (b->n_jobs == 0) {
    fp12_to_be576(out576, fp12_one());
    return LB_OK;
  }
  busy_scope busy(e->device, e, e->latency);
  int32_t st = run_pipeline(e, b, scalars, m, mu, false);  // always blinded: multiplied with other partials
  if (st != LB_OK) return st;
  LB_HIP(e->parts.ensure(576));
  {
    stage_scope sc(e, ST_ROOT, e->stream);
    hipLaunchKernelGGL((e->alone && e->row_fe) ? k_root_partial_row : k_root_partial, dim3(1), dim3((e->alone && e->row_fe) ? LBR_NT : 64), 0, e->stream, mu, e->treeP.as<uint32_t>(),
                       e->fS.as<uint32_t>(), e->parts.as<uint8_t>());
  }
  LB_HIP(hipGetLastError());
  std::vector<int32_t> jst(b->n_jobs);
  LB_HIP(hipMemcpyAsync(out576, e->parts.p, 576, hipMemcpyDeviceToHost, e->stream));
  LB_HIP(hipMemcpyAsync(jst.data(), e->job_status.p, (size_t)b->n_jobs * 4, hipMemcpyDeviceToHost, e->stream));
  if (e->profiling) hipEventRecord(e->ev1[ST_TOTAL], e->stream);
  LB_HIP(hipStreamSynchronize(e->stream));
  for (uint32_t j = 0; j < b->n_jobs; j++) out_job[j] = jst[j] == LB_OK ? 1 : -jst[j];
  finish_profile(e);
  e->partial_serial = b->serial;
  e->partial_mu = mu;
  return LB_OK;
}

extern "C" int32_t lb_batch_search_after_partial(lb_engine* e, lb_batch* b, int32_t* out_job) {
  if (!e || !b || (b->n_jobs && !out_job)) return LB_ERR_ARGUMENT;
  std::lock_guard<std::mutex> lk(e->mu);
  if (b->n_jobs == 0) return LB_OK;
  if (e->partial_serial == 0 || e->partial_serial != b->serial) return LB_ERR_ARGUMENT;  // another call ran since
  LB_HIP(hipSetDevice(e->device));
  busy_scope busy(e->device, e, e->latency);
  const uint32_t mu = e->partial_mu, nj = b->n_jobs;
  LB_HIP(e->verdict.ensure(4));
  LB_HIP(e->y_root.ensure(576));
  // this shard's own root check: a passing shard is done, a failing one searches from it
  hipLaunchKernelGGL((e->alone && e->row_fe) ? k_root_check_row : k_root_check, dim3(1), dim3((e->alone && e->row_fe) ? LBR_NT : 64), 0, e->stream, mu, e->treeP.as<uint32_t>(), e->fS.as<uint32_t>(),
                     e->verdict.as<int32_t>(), e->y_root.as<uint32_t>());
  LB_HIP(hipGetLastError());
  std::vector<int32_t> jst(nj);
  int32_t root_ok = 0;
  LB_HIP(hipMemcpyAsync(jst.data(), e->job_status.p, (size_t)nj * 4, hipMemcpyDeviceToHost, e->stream));
  LB_HIP(hipMemcpyAsync(&root_ok, e->verdict.p, 4, hipMemcpyDeviceToHost, e->stream));
  LB_HIP(hipStreamSynchronize(e->stream));
  bool any_live = false;
  for (uint32_t j = 0; j < nj; j++) {
    out_job[j] = jst[j] == LB_OK ? 1 : -jst[j];
    any_live |= jst[j] == LB_OK;
  }
  int32_t st = LB_OK;
  if (any_live && !root_ok) st = search_invalid(e, b, mu, out_job);
  e->partial_serial = 0;
  return st;
}

extern "C" int32_t lb_fp12_product_is_one(lb_engine* e, const uint8_t* partials576, uint32_t n, int32_t* ok) {
  if (!e || !ok || (n && !partials576)) return LB_ERR_ARGUMENT;
  std::lock_guard<std::mutex> lk(e->mu);
  LB_HIP(hipSetDevice(e->device));
  LB_HIP(e->parts.ensure((size_t)(n ? n : 1) * 576));
  LB_HIP(e->ok.ensure(4));
  if (n) LB_HIP(hipMemcpyAsync(e->parts.p, partials576, (size_t)n * 576, hipMemcpyHostToDevice, e->stream));
  const bool prow = e->row_fe && device_alone(e);
  hipLaunchKernelGGL(prow ? k_partials_check_row : k_partials_check, dim3(1), dim3(prow ? LBR_NT : 64), 0, e->stream, n, e->parts.as<uint8_t>(),
                     e->ok.as<int32_t>());
  LB_HIP(hipGetLastError());
  LB_HIP(hipMemcpyAsync(ok, e->ok.p, 4, hipMemcpyDeviceToHost, e->stream));
  LB_HIP(hipStreamSynchronize(e->stream));
  return LB_OK;
}

// upload into the engine-owned workspace batch + verify, under one hold of the engine lock
static int32_t verify_jobs_ws(lb_engine* e, uint32_t n_jobs, const uint32_t* job_offsets,
                              const uint32_t* set_pk_offsets, const uint8_t* pubkeys, const uint32_t* pk_indices,
                              const uint8_t* signing_roots, const uint8_t* signatures, const uint32_t* sig_sizes,
                              const uint64_t* scalars, int32_t* out_job) {
  if (!e || !job_offsets || (n_jobs && !out_job)) return LB_ERR_ARGUMENT;
  std::lock_guard<std::mutex> lk(e->mu);
  if (!e->scratch) e->scratch = new lb_batch();
  int32_t st = batch_fill(e, e->scratch, n_jobs, job_offsets, set_pk_offsets, pubkeys, pk_indices, signing_roots,
                          signatures, sig_sizes);
  if (st != LB_OK) return st;
  return verify_locked(e, e->scratch, scalars, out_job);
}

extern "C" int32_t lb_verify_jobs(lb_engine* e, uint32_t n_jobs, const uint32_t* job_offsets,
                                  const uint32_t* set_pk_offsets, const uint8_t* pubkeys,
                                  const uint8_t* signing_roots, const uint8_t* signatures,
                                  const uint32_t* sig_sizes, const uint64_t* scalars, int32_t* out_job) {
  return verify_jobs_ws(e, n_jobs, job_offsets, set_pk_offsets, pubkeys, nullptr, signing_roots, signatures,
                        sig_sizes, scalars, out_job);
}

extern "C" int32_t lb_verify_jobs_indexed(lb_engine* e, uint32_t n_jobs, const uint32_t* job_offsets,
                                          const uint32_t* set_pk_offsets, const uint32_t* pk_indices,
                                          const uint8_t* signing_roots, const uint8_t* signatures,
                                          const uint32_t* sig_sizes, const uint64_t* scalars, int32_t* out_job) {
  if (!pk_indices) {
    const int32_t st = check_null_indices(n_jobs, job_offsets, set_pk_offsets);
    if (st != LB_OK) return st;
    pk_indices = kNoIndices;
  }
  return verify_jobs_ws(e, n_jobs, job_offsets, set_pk_offsets, nullptr, pk_indices, signing_roots, signatures,
                        sig_sizes, scalars, out_job);
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
  if (n_pks & LB_CHUNK_FIRST) return LB_ERR_ARGUMENT;
  std::lock_guard<std::mutex> lk(e->mu);
  LB_HIP(hipSetDevice(e->device));
  // the batch pipeline's chunk decomposition (<= LB_PK_CHUNK keys, flagged set starts): chunk sums
  // combined by the wave tree in k_pk_chunks, then k_pk_out96 per set
  std::vector<uint32_t> sco(n_sets + 1), clo;
  for (uint32_t i = 0; i < n_sets; i++) {
    sco[i] = (uint32_t)clo.size();
    for (uint32_t k = set_pk_offsets[i]; k < set_pk_offsets[i + 1]; k += LB_PK_CHUNK)
      clo.push_back(k | (k == set_pk_offsets[i] ? LB_CHUNK_FIRST : 0u));
  }
  sco[n_sets] = (uint32_t)clo.size();
  const uint32_t nc = (uint32_t)clo.size();
  clo.push_back(n_pks | LB_CHUNK_FIRST);
  dbuf dsco, dclo, pk, acc, cst, out, stat;
  hipError_t r = dsco.ensure(sco.size() * 4);
  if (r == hipSuccess) r = dclo.ensure(clo.size() * 4);
  if (r == hipSuccess) r = pk.ensure((size_t)(n_pks ? n_pks : 1) * 96);
  if (r == hipSuccess) r = acc.ensure((size_t)(nc ? nc : 1) * sizeof(g1j));
  if (r == hipSuccess) r = cst.ensure((size_t)(nc ? nc : 1) * 4);
  if (r == hipSuccess) r = out.ensure((size_t)n_sets * 96);
  if (r == hipSuccess) r = stat.ensure((size_t)n_sets * 4);
  if (r == hipSuccess) r = hipMemcpyAsync(dsco.p, sco.data(), sco.size() * 4, hipMemcpyHostToDevice, e->stream);
  if (r == hipSuccess) r = hipMemcpyAsync(dclo.p, clo.data(), clo.size() * 4, hipMemcpyHostToDevice, e->stream);
  if (r == hipSuccess && n_pks) r = hipMemcpyAsync(pk.p, pubkeys, (size_t)n_pks * 96, hipMemcpyHostToDevice, e->stream);
  if (r == hipSuccess) {
    if (nc)
      hipLaunchKernelGGL(k_pk_chunks, dim3(nblk(nc)), dim3(LB_TPB), 0, e->stream, nc, dclo.as<uint32_t>(), pk.as<uint8_t>(),
                         acc.as<uint32_t>(), cst.as<int32_t>());
    hipLaunchKernelGGL(k_pk_out96, dim3(nblk(n_sets)), dim3(LB_TPB), 0, e->stream, n_sets, nc, dsco.as<uint32_t>(),
                       acc.as<uint32_t>(), cst.as<int32_t>(), out.as<uint8_t>(), stat.as<int32_t>());
    r = hipGetLastError();
  }
  if (r == hipSuccess) r = hipMemcpyAsync(out96, out.p, (size_t)n_sets * 96, hipMemcpyDeviceToHost, e->stream);
  if (r == hipSuccess) r = hipMemcpyAsync(out_status, stat.p, (size_t)n_sets * 4, hipMemcpyDeviceToHost, e->stream);
  if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
  dbuf* tmp[] = {&dsco, &dclo, &pk, &acc, &cst, &out, &stat};
  for (dbuf* d : tmp) d->release();
  if (r != hipSuccess) {
    fprintf(stderr, "lodestar_bls: aggregate failed: %s\n", hipGetErrorString(r));
    return LB_ERR_DEVICE;
  }
  return LB_OK;
}

extern "C" int32_t lb_aggregate_signatures(lb_engine* e, uint32_t n_groups, const uint32_t* group_offsets,
                                           const uint8_t* sigs96, const uint32_t* sig_sizes, int32_t validate,
                                           uint8_t* out96, int32_t* out_status) {
  if (!e || !group_offsets || (n_groups && (!out96 || !out_status))) return LB_ERR_ARGUMENT;
  if (group_offsets[0] != 0) return LB_ERR_ARGUMENT;
  for (uint32_t g = 0; g < n_groups; g++)
    if (group_offsets[g + 1] < group_offsets[g]) return LB_ERR_ARGUMENT;
  const uint32_t n = group_offsets[n_groups];
  if (n && !sigs96) return LB_ERR_ARGUMENT;
  if (!n_groups) return LB_OK;
  // chunks of <= LB_PK_CHUNK signatures, never spanning groups
  std::vector<uint32_t> chunk_lo, group_chunk_off(n_groups + 1);
  for (uint32_t g = 0; g < n_groups; g++) {
    group_chunk_off[g] = (uint32_t)chunk_lo.size();
    for (uint32_t i = group_offsets[g]; i < group_offsets[g + 1]; i += LB_PK_CHUNK) chunk_lo.push_back(i);
  }
  group_chunk_off[n_groups] = (uint32_t)chunk_lo.size();
  const uint32_t nc = (uint32_t)chunk_lo.size();
  chunk_lo.push_back(n);
  std::lock_guard<std::mutex> lk(e->mu);
  LB_HIP(hipSetDevice(e->device));
  const uint32_t ns = n ? n : 1, ncs = nc ? nc : 1;
  dbuf in, sizes, aff, aos, inf, st, clo, goff, acc, cst, out, ost;
  hipError_t r = in.ensure((size_t)ns * 96);
  if (r == hipSuccess) r = sizes.ensure((size_t)ns * 4);
  if (r == hipSuccess) r = aff.ensure((size_t)ns * sizeof(g2a));
  if (r == hipSuccess) r = aos.ensure((size_t)ns * sizeof(g2a));
  if (r == hipSuccess) r = inf.ensure((size_t)ns * 4);
  if (r == hipSuccess) r = st.ensure((size_t)ns * 4);
  if (r == hipSuccess) r = clo.ensure((size_t)(nc + 1) * 4);
  if (r == hipSuccess) r = goff.ensure((size_t)(n_groups + 1) * 4);
  if (r == hipSuccess) r = acc.ensure((size_t)ncs * sizeof(g2j));
  if (r == hipSuccess) r = cst.ensure((size_t)ncs * 4);
  if (r == hipSuccess) r = out.ensure((size_t)n_groups * 96);
  if (r == hipSuccess) r = ost.ensure((size_t)n_groups * 4);
  hipStream_t s1 = e->stream;
  if (r == hipSuccess && n) r = hipMemcpyAsync(in.p, sigs96, (size_t)n * 96, hipMemcpyHostToDevice, s1);
  if (r == hipSuccess && n && sig_sizes) r = hipMemcpyAsync(sizes.p, sig_sizes, (size_t)n * 4, hipMemcpyHostToDevice, s1);
  if (r == hipSuccess) r = hipMemcpyAsync(clo.p, chunk_lo.data(), (size_t)(nc + 1) * 4, hipMemcpyHostToDevice, s1);
  if (r == hipSuccess)
    r = hipMemcpyAsync(goff.p, group_chunk_off.data(), (size_t)(n_groups + 1) * 4, hipMemcpyHostToDevice, s1);
  if (r == hipSuccess) {
    if (n) {
      hipLaunchKernelGGL(k_decompress_sigs, dim3(nblk(n)), dim3(LB_TPB), 0, s1, n, in.as<uint8_t>(),
                         sig_sizes ? sizes.as<uint32_t>() : nullptr, aff.as<uint32_t>(), aos.as<uint4>(),
                         inf.as<uint32_t>(), st.as<int32_t>());
      if (validate)
        hipLaunchKernelGGL(k_sig_subgroup, dim3(nblk(n)), dim3(LB_TPB), 0, s1, n, aff.as<uint32_t>(),
                           inf.as<uint32_t>(), st.as<int32_t>());
    }
    if (nc)
      hipLaunchKernelGGL(k_sig_agg_chunks, dim3(nblk(nc)), dim3(LB_TPB), 0, s1, nc, clo.as<uint32_t>(),
                         aff.as<uint32_t>(), n, inf.as<uint32_t>(), st.as<int32_t>(), acc.as<uint32_t>(),
                         cst.as<int32_t>());
    hipLaunchKernelGGL(k_sig_agg_groups, dim3(nblk(n_groups)), dim3(LB_TPB), 0, s1, n_groups, goff.as<uint32_t>(),
                       acc.as<uint32_t>(), nc, cst.as<int32_t>(), out.as<uint8_t>(), ost.as<int32_t>());
    r = hipGetLastError();
  }
  if (r == hipSuccess) r = hipMemcpyAsync(out96, out.p, (size_t)n_groups * 96, hipMemcpyDeviceToHost, s1);
  if (r == hipSuccess) r = hipMemcpyAsync(out_status, ost.p, (size_t)n_groups * 4, hipMemcpyDeviceToHost, s1);
  if (r == hipSuccess) r = hipStreamSynchronize(s1);
  dbuf* all[] = {&in, &sizes, &aff, &aos, &inf, &st, &clo, &goff, &acc, &cst, &out, &ost};
  for (dbuf* d : all) d->release();
  if (r != hipSuccess) {
    fprintf(stderr, "lodestar_bls: signature aggregation failed: %s\n", hipGetErrorString(r));
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

extern "C" int32_t lb_merkleize(lb_engine* e, uint32_t n_trees, const uint32_t* chunk_offsets, const uint8_t* chunks32,
                                const uint32_t* depths, const uint64_t* mix_lengths, uint8_t* out_roots32) {
  if (!e || !chunk_offsets || (n_trees && (!depths || !mix_lengths || !out_roots32))) return LB_ERR_ARGUMENT;
  if (chunk_offsets[0] != 0) return LB_ERR_ARGUMENT;
  for (uint32_t t = 0; t < n_trees; t++) {
    const uint32_t len = chunk_offsets[t + 1] - chunk_offsets[t];
    if (chunk_offsets[t + 1] < chunk_offsets[t] || depths[t] > 63 || (depths[t] < 32 && len > (1u << depths[t])))
      return LB_ERR_ARGUMENT;
  }
  const uint32_t nc = chunk_offsets[n_trees];
  if (nc && !chunks32) return LB_ERR_ARGUMENT;
  if (!n_trees) return LB_OK;
  return run_simple(e, {{chunk_offsets, (size_t)(n_trees + 1) * 4, false, nullptr},
                        {depths, (size_t)n_trees * 4, false, nullptr},
                        {mix_lengths, (size_t)n_trees * 8, false, nullptr},
                        {chunks32, (size_t)nc * 32, false, nullptr},
                        {nullptr, 64 * 32, true, nullptr},  // zero-subtree roots (device scratch)
                        {nullptr, (size_t)n_trees * 32, true, out_roots32}},
                    [&](std::vector<void*>& p) {
                      hipLaunchKernelGGL(k_ssz_zero_hashes, dim3(1), dim3(64), 0, e->stream, (uint8_t*)p[4]);
                      hipLaunchKernelGGL(k_merkleize, dim3(nblk(n_trees)), dim3(LB_TPB), 0, e->stream, n_trees,
                                         (const uint32_t*)p[0], (const uint32_t*)p[1], (const uint64_t*)p[2],
                                         (uint8_t*)p[3], (const uint8_t*)p[4], (uint8_t*)p[5]);
                    });
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

// ---------------------------------------------------------------- KZG (lb_kzg.h)
extern "C" int32_t lb_kzg_load_setup(lb_engine* e, const uint8_t* g1_48, uint32_t n_g1, const uint8_t* g2_96,
                                     uint32_t n_g2, int32_t* out_status) {
  if (!e || !n_g1 || !g1_48 || !g2_96 || n_g2 < 2 || !out_status) return LB_ERR_ARGUMENT;
  std::vector<int32_t> st2(2, LB_OK);
  int32_t r;
  {
    std::lock_guard<std::mutex> lk(e->mu);
    LB_HIP(hipSetDevice(e->device));
    LB_HIP(e->kzg_g1.ensure((size_t)n_g1 * sizeof(g1a)));
    LB_HIP(e->kzg_g2.ensure(2 * sizeof(g2a)));
  }
  lb_engine* ee = e;
  r = run_simple(e, {{g1_48, (size_t)n_g1 * 48, false, nullptr}, {nullptr, (size_t)n_g1 * 4, true, out_status},
                     {g2_96, 2 * 96, false, nullptr}, {nullptr, 2 * 4, true, st2.data()}},
                 [&](std::vector<void*>& p) {
                   hipLaunchKernelGGL(k_kzg_setup_g1, dim3(nblk(n_g1)), dim3(LB_TPB), 0, ee->stream, n_g1,
                                      (const uint8_t*)p[0], ee->kzg_g1.as<uint32_t>(), n_g1, (int32_t*)p[1]);
                   hipLaunchKernelGGL(k_kzg_setup_g2, dim3(1), dim3(64), 0, ee->stream, (const uint8_t*)p[2],
                                      ee->kzg_g2.as<uint32_t>(), (int32_t*)p[3]);
                 });
  if (r != LB_OK) return r;
  if (st2[0] != LB_OK || st2[1] != LB_OK) {
    e->kzg_n = 0;
    return st2[0] != LB_OK ? st2[0] : st2[1];
  }
  for (uint32_t i = 0; i < n_g1; i++)
    if (out_status[i] != LB_OK) {
      e->kzg_n = 0;
      return out_status[i];
    }
  e->kzg_n = n_g1;
  return LB_OK;
}

extern "C" int32_t lb_g1_lincomb(lb_engine* e, uint32_t n, const uint8_t* points48, const uint8_t* scalars32,
                                 uint8_t* out48) {
  if (!e || !out48 || (n && !scalars32)) return LB_ERR_ARGUMENT;
  if (!points48 && n > e->kzg_n) return LB_ERR_ARGUMENT;
  if (!n) {  // empty sum: infinity
    memset(out48, 0, 48);
    out48[0] = 0xc0;
    return LB_OK;
  }
  uint32_t levels = 0;
  for (uint32_t m = n; m > 1; m = (m + 63) / 64) levels++;
  const uint32_t n1 = (n + 63) / 64;
  std::vector<int32_t> st(n, LB_OK);
  lb_engine* ee = e;
  const int32_t r = run_simple(
      e, {{points48, points48 ? (size_t)n * 48 : 0, false, nullptr}, {scalars32, (size_t)n * 32, false, nullptr},
          {nullptr, (size_t)n * sizeof(g1j), true, nullptr}, {nullptr, (size_t)n1 * sizeof(g1j), true, nullptr},
          {nullptr, (size_t)n * 4, true, st.data()}, {nullptr, 48, true, out48}},
      [&](std::vector<void*>& p) {
        hipLaunchKernelGGL(k_g1_terms, dim3(nblk(n)), dim3(LB_TPB), 0, ee->stream, n,
                           points48 ? (const uint8_t*)p[0] : nullptr, ee->kzg_g1.as<uint32_t>(), ee->kzg_n,
                           (const uint32_t*)p[1], (uint32_t*)p[2], (int32_t*)p[4]);
        // reduce 64:1 per level, ping-ponging between the term buffer and the partials buffer
        uint32_t* bufs[2] = {(uint32_t*)p[2], (uint32_t*)p[3]};
        uint32_t m = n;
        int cur = 0;
        for (uint32_t l = 0; l < levels; l++) {
          const uint32_t mo = (m + 63) / 64;
          hipLaunchKernelGGL(k_g1_sum64, dim3(mo), dim3(64), 0, ee->stream, m, bufs[cur], mo, bufs[cur ^ 1]);
          m = mo;
          cur ^= 1;
        }
        hipLaunchKernelGGL(k_g1_out48, dim3(1), dim3(64), 0, ee->stream, bufs[cur], m, (uint8_t*)p[5]);
      });
  if (r != LB_OK) return r;
  for (uint32_t i = 0; i < n; i++)
    if (st[i] != LB_OK) return st[i];
  return LB_OK;
}

extern "C" int32_t lb_kzg_verify_proof(lb_engine* e, const uint8_t* commitment48, const uint8_t* z32,
                                       const uint8_t* y32, const uint8_t* proof48, int32_t* ok) {
  if (!e || !commitment48 || !z32 || !y32 || !proof48 || !ok) return LB_ERR_ARGUMENT;
  if (e->kzg_n == 0) return LB_ERR_ARGUMENT;  // no setup loaded
  uint8_t io[96];
  memcpy(io, commitment48, 48);
  memcpy(io + 48, proof48, 48);
  uint8_t yz[64];
  memcpy(yz, y32, 32);
  memcpy(yz + 32, z32, 32);
  lb_engine* ee = e;
  return run_simple(e, {{io, 96, false, nullptr}, {yz, 64, false, nullptr}, {nullptr, 4, true, ok}},
                    [&](std::vector<void*>& p) {
                      hipLaunchKernelGGL(k_kzg_check, dim3(1), dim3(64), 0, ee->stream, (const uint8_t*)p[0],
                                         (const uint32_t*)p[1], ee->kzg_g2.as<uint32_t>(), (int32_t*)p[2]);
                    });
}
