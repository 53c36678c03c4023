// CPU BASELINE POOL — test / benchmark infrastructure only, never on the product path.
//
// Restates the reference's worker-pool verification policy:
//   * the main thread fills a worker package with jobs until it holds >= 128 sets
//     (prepareWork, packages/beacon-node/src/chain/bls/multithread/index.ts:386-401); idle workers
//     take packages (index.ts:290-330) — here: threads pulling packages from a shared counter;
//   * the worker splits the batchable jobs of a package into chunks of >= 16 jobs
//     (chunkifyMaximizeChunkSize(batchableJobs, BATCHABLE_MIN_PER_CHUNK), worker.ts:17,56), and
//     verifies each chunk's flattened sets as ONE batch (worker.ts:68); if the chunk is false or
//     throws, every job of the chunk is re-verified on its own (worker.ts:76-98);
//   * a non-batchable job is verified on its own (worker.ts:91-98);
//   * verifying a job = verifySignatureSetsMaybeBatch (maybeBatch.ts:16-39): >= 2 sets -> the
//     random-scalar batch equation with one final exponentiation (verifyMultipleSignatures);
//     1 set -> Signature.verify, e(PK, H(m)) e(-G1, sig) == 1 without blinding; 0 -> throw.
// blst itself (@chainsafe/blst 0.2.7) is un-vendored and cannot be built here (SURVEY.md
// §8(c)), so the arithmetic is the engine's own Fp..Fp12 / curve / hash_to_G2 / pairing code
// (lodestar_amd/csrc/*.h) compiled for x86-64 — a "CPU stand-in, not blst"; bench.py reports
// it as cpu_baseline.kind = "port" next to the blst anchor (0.9 ms/set/core,
// packages/beacon-node/src/metrics/metrics/lodestar.ts:505).
#include <stdint.h>
#include <string.h>
#include <sys/random.h>

#include <atomic>
#include <thread>
#include <vector>

#include "lb_serial.h"
#include "lb_h2c.h"
#include "lb_pairing.h"

namespace {

struct Inputs {
  const uint32_t* job_off;
  const uint32_t* pk_off;
  const uint8_t* pks;
  const uint8_t* msgs;
  const uint8_t* sigs;
};

struct Decoded {
  g1a pk;
  bool pk_inf;
  g2a sig;
  bool sig_inf;
};

// Reference precedence inside one verifySignatureSetsMaybeBatch call: every pubkey aggregate was
// formed on the main thread first (getAggregatedPubkey), then every signature is decoded
// (maybeBatch.ts:18-25), then blst rejects an infinite aggregate pubkey.
int decode_sets(const Inputs& in, const std::vector<uint32_t>& sets, std::vector<Decoded>& out) {
  out.resize(sets.size());
  for (size_t k = 0; k < sets.size(); k++) {
    const uint32_t i = sets[k];
    if (in.pk_off[i] == in.pk_off[i + 1]) return LB_EMPTY_AGGREGATE_ARRAY;
    g1j acc = jac_infinity<fp>();
    for (uint32_t q = in.pk_off[i]; q < in.pk_off[i + 1]; q++) {
      g1a p;
      bool inf;
      const int st = g1_deserialize96(in.pks + (size_t)96 * q, p, inf);
      if (st) return st;
      if (!inf) acc = jac_add_aff(acc, p);
    }
    out[k].pk_inf = jac_is_inf(acc);
    jac_to_aff(out[k].pk, acc);
  }
  for (size_t k = 0; k < sets.size(); k++) {
    bool inf;
    int st = g2_decompress96(in.sigs + (size_t)96 * sets[k], out[k].sig, inf);
    if (st == LB_OK && !inf && !g2_in_subgroup(jac_from_aff(out[k].sig))) st = LB_POINT_NOT_IN_GROUP;
    if (st) return st;
    out[k].sig_inf = inf;
  }
  for (size_t k = 0; k < sets.size(); k++)
    if (out[k].pk_inf) return LB_PK_IS_INFINITY;
  return LB_OK;
}

// verifySignatureSetsMaybeBatch over `sets`: 1 / 0 / -code
int maybe_batch(const Inputs& in, const std::vector<uint32_t>& sets, uint64_t& rng) {
  if (sets.empty()) return -LB_EMPTY_SIGNATURE_SET;
  std::vector<Decoded> d;
  const int st = decode_sets(in, sets, d);
  if (st) return -st;
  const g1a ng1{fp_load(LB_G1X), fp_load(LB_G1NEGY)};
  if (sets.size() == 1) {
    // Signature.verify: e(PK, H(m)) * e(-G1, sig) == 1, no blinding
    g2a h;
    jac_to_aff(h, hash_to_g2(in.msgs + (size_t)32 * sets[0]));
    fp12 f = miller_loop(d[0].pk, h);
    if (!d[0].sig_inf) f = fp12_mul(f, miller_loop(ng1, d[0].sig));
    return fp12_is_one(final_exponentiation(f)) ? 1 : 0;
  }
  // verifyMultipleSignatures: 64-bit random blinding per set, one final exponentiation
  fp12 f = fp12_one();
  g2j S = jac_infinity<fp2>();
  for (size_t k = 0; k < sets.size(); k++) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    const uint64_t r = rng | 1;
    g1a rp;
    jac_to_aff(rp, jac_mul_u64(d[k].pk, r));
    if (!d[k].sig_inf) S = jac_add(S, jac_mul_u64(d[k].sig, r));
    g2a h;
    jac_to_aff(h, hash_to_g2(in.msgs + (size_t)32 * sets[k]));
    f = fp12_mul(f, miller_loop(rp, h));
  }
  if (!jac_is_inf(S)) {
    g2a sa;
    jac_to_aff(sa, S);
    f = fp12_mul(f, miller_loop(ng1, sa));
  }
  return fp12_is_one(final_exponentiation(f)) ? 1 : 0;
}

std::vector<uint32_t> job_sets(const Inputs& in, uint32_t j) {
  std::vector<uint32_t> v;
  for (uint32_t i = in.job_off[j]; i < in.job_off[j + 1]; i++) v.push_back(i);
  return v;
}

// chunkifyMaximizeChunkSize (multithread/utils.ts:4-19) over job indices [a, e)
std::vector<std::pair<uint32_t, uint32_t>> chunkify(uint32_t a, uint32_t e, uint32_t min_per_chunk) {
  const uint32_t n = e - a, count = n / min_per_chunk;
  std::vector<std::pair<uint32_t, uint32_t>> out;
  if (count <= 1) {
    out.push_back({a, e});
    return out;
  }
  const uint32_t per = (n + count - 1) / count;
  for (uint32_t i = a; i < e; i += per) out.push_back({i, i + per < e ? i + per : e});
  return out;
}

// one worker package: jobs [a, e) (worker.ts:32-108)
void run_package(const Inputs& in, uint32_t a, uint32_t e, bool batchable, uint64_t& rng, int32_t* out) {
  if (!batchable) {
    for (uint32_t j = a; j < e; j++) out[j] = maybe_batch(in, job_sets(in, j), rng);
    return;
  }
  for (auto [c0, c1] : chunkify(a, e, 16)) {
    std::vector<uint32_t> all;
    for (uint32_t j = c0; j < c1; j++)
      for (uint32_t i = in.job_off[j]; i < in.job_off[j + 1]; i++) all.push_back(i);
    const int r = all.empty() ? -LB_EMPTY_SIGNATURE_SET : maybe_batch(in, all, rng);
    if (r == 1) {
      for (uint32_t j = c0; j < c1; j++) out[j] = 1;
    } else {
      for (uint32_t j = c0; j < c1; j++) out[j] = maybe_batch(in, job_sets(in, j), rng);  // batchRetries
    }
  }
}

}  // namespace

// Verifies n_jobs jobs with the reference pool's policy on n_threads worker threads; out[j] =
// 1 / 0 / -code.  batchable = the jobs came from verifySignatureSets(.., {batchable: true}).
extern "C" int cpu_verify_jobs_policy(uint32_t n_jobs, const uint32_t* job_off, const uint32_t* pk_off,
                                      const uint8_t* pks, const uint8_t* msgs, const uint8_t* sigs, int batchable,
                                      int n_threads, int32_t* out) {
  const Inputs in{job_off, pk_off, pks, msgs, sigs};
  // packages of >= 128 sets (prepareWork, MAX_SIGNATURE_SETS_PER_JOB)
  std::vector<uint32_t> pkg{0};
  uint32_t sets = 0;
  for (uint32_t j = 0; j < n_jobs; j++) {
    sets += job_off[j + 1] - job_off[j];
    if (sets >= 128) {
      pkg.push_back(j + 1);
      sets = 0;
    }
  }
  if (pkg.back() != n_jobs) pkg.push_back(n_jobs);
  std::atomic<uint32_t> next{0};
  auto work = [&]() {
    uint64_t rng = 0;
    while (!rng)
      if (getrandom(&rng, 8, 0) != 8) rng = 0;
    for (;;) {
      const uint32_t p = next.fetch_add(1);
      if (p + 1 >= pkg.size()) break;
      run_package(in, pkg[p], pkg[p + 1], batchable != 0, rng, out);
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < (n_threads > 0 ? n_threads : 1); t++) th.emplace_back(work);
  for (auto& t : th) t.join();
  return 0;
}

// Each job verified on its own (verifySignatureSetsMaybeBatch per job): the test checker.
extern "C" int cpu_verify_jobs(uint32_t n_jobs, const uint32_t* job_off, const uint32_t* pk_off,
                               const uint8_t* pks, const uint8_t* msgs, const uint8_t* sigs, int n_threads,
                               int32_t* out) {
  const Inputs in{job_off, pk_off, pks, msgs, sigs};
  std::atomic<uint32_t> next{0};
  auto work = [&]() {
    uint64_t rng = 0;
    while (!rng)
      if (getrandom(&rng, 8, 0) != 8) rng = 0;
    for (;;) {
      const uint32_t j = next.fetch_add(1);
      if (j >= n_jobs) break;
      out[j] = maybe_batch(in, job_sets(in, j), rng);
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < (n_threads > 0 ? n_threads : 1); t++) th.emplace_back(work);
  for (auto& t : th) t.join();
  return 0;
}

// ---- multi-GPU protocol checker (CPU): the 576-byte partial of a shard and the product check,
// the CPU counterparts of lb_batch_partial / lb_fp12_product_is_one (tests/test_distributed.py).
extern "C" int cpu_partial(uint32_t n_jobs, const uint32_t* job_off, const uint32_t* pk_off, const uint8_t* pks,
                           const uint8_t* msgs, const uint8_t* sigs, uint64_t seed, uint8_t* out576,
                           int32_t* out_status) {
  uint64_t rng = seed | 1;
  fp12 f = fp12_one();
  g2j S = jac_infinity<fp2>();
  for (uint32_t j = 0; j < n_jobs; j++) {
    uint32_t a = job_off[j], e = job_off[j + 1];
    int st = a == e ? LB_EMPTY_SIGNATURE_SET : LB_OK;
    std::vector<g1a> agg;
    std::vector<g2a> sg;
    std::vector<bool> sinf;
    for (uint32_t i = a; i < e && st == LB_OK; i++) {
      if (pk_off[i] == pk_off[i + 1]) { st = LB_EMPTY_AGGREGATE_ARRAY; break; }
      g1j acc = jac_infinity<fp>();
      for (uint32_t k = pk_off[i]; k < pk_off[i + 1] && st == LB_OK; k++) {
        g1a p; bool inf;
        st = g1_deserialize96(pks + (size_t)96 * k, p, inf);
        if (st == LB_OK && !inf) acc = jac_add_aff(acc, p);
      }
      g1a pa; jac_to_aff(pa, acc);
      agg.push_back(jac_is_inf(acc) ? g1a{fp_zero(), fp_zero()} : pa);
      if (jac_is_inf(acc) && st == LB_OK) st = -1;  // marker: infinity, resolved after sig decode
    }
    int pk_inf = st == -1;
    if (pk_inf) st = LB_OK;
    for (uint32_t i = a; i < e && st == LB_OK; i++) {
      g2a s; bool inf;
      st = g2_decompress96(sigs + (size_t)96 * i, s, inf);
      if (st == LB_OK && !inf && !g2_in_subgroup(jac_from_aff(s))) st = LB_POINT_NOT_IN_GROUP;
      sg.push_back(s); sinf.push_back(inf);
    }
    if (st == LB_OK && pk_inf) st = LB_PK_IS_INFINITY;
    out_status[j] = st == LB_OK ? 1 : -st;
    if (st != LB_OK) continue;
    for (uint32_t i = a; i < e; i++) {
      rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
      uint64_t r = rng | 1;
      g1a rp;
      jac_to_aff(rp, jac_mul_u64(agg[i - a], r));
      if (!sinf[i - a]) S = jac_add(S, jac_mul_u64(sg[i - a], r));
      g2a h;
      jac_to_aff(h, hash_to_g2(msgs + (size_t)32 * i));
      f = fp12_mul(f, miller_loop(rp, h));
    }
  }
  if (!jac_is_inf(S)) {
    g2a sa;
    jac_to_aff(sa, S);
    g1a ng1{fp_load(LB_G1X), fp_load(LB_G1NEGY)};
    f = fp12_mul(f, miller_loop(ng1, sa));
  }
  fp12_to_be576(out576, f);
  return 0;
}

extern "C" int cpu_product_is_one(const uint8_t* parts, uint32_t n) {
  fp12 acc = fp12_one();
  for (uint32_t i = 0; i < n; i++) {
    fp12 f;
    if (!fp12_from_be576(f, parts + (size_t)576 * i)) return 0;
    acc = fp12_mul(acc, f);
  }
  return fp12_is_one(final_exponentiation(acc)) ? 1 : 0;
}
