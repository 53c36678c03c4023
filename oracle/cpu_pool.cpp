// CPU BASELINE POOL — test / benchmark infrastructure only, never on the product path.
//
// Restates the reference's worker-pool verification (packages/beacon-node/src/chain/bls/
// multithread/worker.ts:32-108 + maybeBatch.ts:16-39): every job (BlsWorkReq) is verified on
// one CPU thread with ONE random-scalar batch equation and its own final exponentiation,
// threads pulling jobs from a shared queue like the pool's idle workers (index.ts:290-330).
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

static int verify_job(uint32_t a, uint32_t e, const uint32_t* pk_off, const uint8_t* pks, const uint8_t* msgs,
                      const uint8_t* sigs, uint64_t& rng) {
  if (a == e) return -LB_EMPTY_SIGNATURE_SET;
  std::vector<g1a> agg(e - a);
  std::vector<bool> agg_inf(e - a);
  for (uint32_t i = a; i < e; i++) {
    if (pk_off[i] == pk_off[i + 1]) return -LB_EMPTY_AGGREGATE_ARRAY;
    g1j acc = jac_infinity<fp>();
    for (uint32_t k = pk_off[i]; k < pk_off[i + 1]; k++) {
      g1a p;
      bool inf;
      int st = g1_deserialize96(pks + (size_t)96 * k, p, inf);
      if (st) return -st;
      if (!inf) acc = jac_add_aff(acc, p);
    }
    agg_inf[i - a] = jac_is_inf(acc);
    jac_to_aff(agg[i - a], acc);
  }
  std::vector<g2a> sg(e - a);
  std::vector<bool> sg_inf(e - a);
  for (uint32_t i = a; i < e; i++) {
    bool inf;
    int st = g2_decompress96(sigs + (size_t)96 * i, sg[i - a], inf);
    if (st == LB_OK && !inf && !g2_in_subgroup(jac_from_aff(sg[i - a]))) st = LB_POINT_NOT_IN_GROUP;
    if (st) return -st;
    sg_inf[i - a] = inf;
  }
  for (uint32_t i = a; i < e; i++)
    if (agg_inf[i - a]) return -LB_PK_IS_INFINITY;
  fp12 f = fp12_one();
  g2j S = jac_infinity<fp2>();
  for (uint32_t i = a; i < e; i++) {
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    uint64_t r = rng | 1;
    g1a rp;
    jac_to_aff(rp, jac_mul_u64(agg[i - a], r));
    if (!sg_inf[i - a]) S = jac_add(S, jac_mul_u64(sg[i - a], r));
    g2a h;
    jac_to_aff(h, hash_to_g2(msgs + (size_t)32 * i));
    f = fp12_mul(f, miller_loop(rp, h));
  }
  if (!jac_is_inf(S)) {
    g2a sa;
    jac_to_aff(sa, S);
    g1a ng1{fp_load(LB_G1X), fp_load(LB_G1NEGY)};
    f = fp12_mul(f, miller_loop(ng1, sa));
  }
  return fp12_is_one(final_exponentiation(f)) ? 1 : 0;
}

extern "C" int cpu_verify_jobs(uint32_t n_jobs, const uint32_t* job_off, const uint32_t* pk_off,
                               const uint8_t* pks, const uint8_t* msgs, const uint8_t* sigs, int n_threads,
                               int32_t* out) {
  std::atomic<uint32_t> next{0};
  auto work = [&]() {
    uint64_t rng = 0;
    while (!rng) getrandom(&rng, 8, 0);
    for (;;) {
      uint32_t j = next.fetch_add(1);
      if (j >= n_jobs) break;
      out[j] = verify_job(job_off[j], job_off[j + 1], pk_off, pks, msgs, sigs, rng);
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
