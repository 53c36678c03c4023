// Operation counter: the device pipeline's per-stage work, replayed on the CPU build of the same
// headers with every fp_mul counted (build: g++ -DLB_COUNT_OPS).  Test/measurement
// infrastructure for the roofline figures in bench.py; mirrors lb_kernels.h stage by stage.
#define LB_COUNT_OPS 1
#include <string.h>
unsigned long long lb_count_mul = 0;
#include "lb_serial.h"
#include "lb_h2c.h"
#include "lb_pairing.h"

// fp_inv_block (lb_kernels.h): per element 6 + 6 shuffle-scan multiplications and 2 to combine;
// the one inversion per wave is a binary EEA (no multiplications) shared by 64 lanes.
static const unsigned long long INV_BLOCK_MULS = 14;
// Jacobian -> affine through one fp_inv_block, as k_pk_blind does it (zi^2, x zi^2, y zi^2 zi)
static void g1_to_aff_block(g1a& out, const g1j& p) {
  const unsigned long long c = lb_count_mul;
  jac_to_aff(out, p);
  lb_count_mul = c + INV_BLOCK_MULS + 4;
}
// r * PK / r * sig as k_pk_blind / k_sig_blind compute them (r = lo + hi * lambda, jac_mul_glv)
static g1j g1_blind(const g1a& pk, uint64_t r) {
  const g1a t2{fp_mul(pk.x, fp_load(LB_GLV_BETA)), pk.y};
  const g1a t3{fp_mul(pk.x, fp_load(LB_GLV_BETA2)), fp_neg(pk.y)};
  return jac_mul_glv(pk, t2, t3, r);
}
static g2j g2_blind(const g2a& s, uint64_t r) {
  const g2a t2{fp2_mul_fp(s.x, fp_load(LB_PSI2_CX)), fp2_neg(fp2_mul_fp(s.y, fp_load(LB_PSI2_CY)))};
  const g2a t3{fp2_mul_fp(s.x, fp_load(LB_PSI4_CX)), fp2_neg(fp2_mul_fp(s.y, fp_load(LB_PSI4_CY)))};
  return jac_mul_glv(s, t2, t3, r);
}

extern "C" {
unsigned long long cnt_decode(const uint8_t* sig96) {
  lb_count_mul = 0;
  g2a a; bool inf;
  int st = g2_decompress96(sig96, a, inf);
  if (st == 0 && !inf) g2_aff_in_subgroup_i(a);  // as k_decode_sigs
  return lb_count_mul;
}
unsigned long long cnt_hash_map(const uint8_t* msg, int which) {
  lb_count_mul = 0;
  uint32_t ub[64];
  expand_message_xmd_256(ub, msg);
  const uint32_t* w = ub + 32 * which;
  fp2 u{fp_from_be64_words(w), fp_from_be64_words(w + 16)};
  map_to_curve_g2(u);
  return lb_count_mul;
}
unsigned long long cnt_hash_finish(const uint8_t* msg) {
  uint32_t ub[64];
  expand_message_xmd_256(ub, msg);
  g2j q0 = map_to_curve_g2(fp2{fp_from_be64_words(ub), fp_from_be64_words(ub + 16)});
  g2j q1 = map_to_curve_g2(fp2{fp_from_be64_words(ub + 32), fp_from_be64_words(ub + 48)});
  lb_count_mul = 0;
  const g2j h = g2_clear_cofactor(jac_add(q0, q1));
  const unsigned long long c = lb_count_mul;
  g2a a;
  jac_to_aff(a, h);
  lb_count_mul = c + 2 + INV_BLOCK_MULS + 2 + 2 + 3 * 3;  // fp2_sqr = 2, fp2_mul = 3 fp muls
  return lb_count_mul;
}
// k pubkeys (96 B each), scalar r, signature (for r*sig)
unsigned long long cnt_pk_blind(const uint8_t* pks, int k, uint64_t r, const uint8_t* sig96) {
  g2a s; bool sinf;
  g2_decompress96(sig96, s, sinf);
  lb_count_mul = 0;
  g1j acc = jac_infinity<fp>();
  g1a first;
  for (int i = 0; i < k; i++) {
    g1a p; bool inf;
    g1_deserialize96(pks + 96 * i, p, inf);
    acc = jac_add_aff(acc, p);
    if (i == 0) first = p;
  }
  (void)first;
  g1a pk, rp;
  g1_to_aff_block(pk, acc);
  g1_to_aff_block(rp, g1_blind(pk, r));
  g2_blind(s, r);
  return lb_count_mul;
}
// the two halves of blinding (k_pk_blind: r*PK + affine; k_sig_blind: r*sig)
unsigned long long cnt_g1_blind(const uint8_t* pk96, uint64_t r) {
  g1a p; bool inf;
  g1_deserialize96(pk96, p, inf);
  lb_count_mul = 0;
  g1a pk, rp;
  g1_to_aff_block(pk, jac_from_aff(p));
  g1_to_aff_block(rp, g1_blind(pk, r));
  return lb_count_mul;
}
unsigned long long cnt_g2_blind(const uint8_t* sig96, uint64_t r) {
  g2a s; bool inf;
  g2_decompress96(sig96, s, inf);
  lb_count_mul = 0;
  g2_blind(s, r);
  return lb_count_mul;
}
unsigned long long cnt_pk_key(const uint8_t* pks, int k) {
  lb_count_mul = 0;
  g1j acc = jac_infinity<fp>();
  for (int i = 0; i < k; i++) {
    g1a p; bool inf;
    g1_deserialize96(pks + 96 * i, p, inf);
    acc = jac_add_aff(acc, p);
  }
  return lb_count_mul;
}
unsigned long long cnt_fe(void) {
  fp12 f = fp12_one();
  f.c1.c2.c0 = fp_one();
  lb_count_mul = 0;
  final_exponentiation(f);
  return lb_count_mul;
}
unsigned long long cnt_miller(const uint8_t* pk96, const uint8_t* msg) {
  g1a p; bool inf;
  g1_deserialize96(pk96, p, inf);
  g2a h;
  jac_to_aff(h, hash_to_g2(msg));
  lb_count_mul = 0;
  miller_loop(p, h);
  return lb_count_mul;
}
unsigned long long cnt_fp12_mul(void) {
  fp12 a = fp12_one();
  lb_count_mul = 0;
  fp12_mul(a, a);
  return lb_count_mul;
}
unsigned long long cnt_g2_add(const uint8_t* sig96) {
  g2a s; bool inf;
  g2_decompress96(sig96, s, inf);
  g2j p = jac_from_aff(s), q = jac_dbl(p);
  lb_count_mul = 0;
  jac_add(p, q);
  return lb_count_mul;
}
unsigned long long cnt_node_check(const uint8_t* sig96) {
  g2a s; bool inf;
  g2_decompress96(sig96, s, inf);
  g2j S = jac_dbl(jac_from_aff(s));
  fp12 P = fp12_one();
  lb_count_mul = 0;
  g2a sa;
  jac_to_aff(sa, S);
  g1a ng1{fp_load(LB_G1X), fp_load(LB_G1NEGY)};
  fp12 f = fp12_mul(P, miller_loop(ng1, sa));
  final_exponentiation(f);
  return lb_count_mul;
}
}
