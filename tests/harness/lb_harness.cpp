// CPU unit-test harness: compiles the device arithmetic headers (lodestar_amd/csrc/*.h)
// as plain C++ so tests/test_arith_cpu.py can check every stage against oracle/ without
// a GPU.  Test infrastructure only; the product path is the HIP build.
#include <string.h>
#include "lb_serial.h"
#include "lb_h2c.h"
#include "lb_pairing.h"

static fp rd(const uint8_t* b) { fp x; fp_plain_from_be48(x, b, 0xff); return fp_to_mont(x); }
static void wr(uint8_t* b, const fp& a) { fp_plain_to_be48(b, fp_from_mont(a)); }
static fp2 rd2(const uint8_t* b) { return fp2{rd(b), rd(b + 48)}; }   // c0 || c1
static void wr2(uint8_t* b, const fp2& a) { wr(b, a.c0); wr(b + 48, a.c1); }
static g2a rdg2(const uint8_t* b) { return g2a{rd2(b), rd2(b + 96)}; }
static int wrg2(uint8_t* b, const g2j& p) { g2a a; bool ok = jac_to_aff(a, p); wr2(b, a.x); wr2(b + 96, a.y); return ok; }
static g1a rdg1(const uint8_t* b) { return g1a{rd(b), rd(b + 48)}; }
static int wrg1(uint8_t* b, const g1j& p) { g1a a; bool ok = jac_to_aff(a, p); wr(b, a.x); wr(b + 48, a.y); return ok; }

extern "C" {
void h_fp_mul(const uint8_t* a, const uint8_t* b, uint8_t* o) { wr(o, fp_mul(rd(a), rd(b))); }
void h_fp_add(const uint8_t* a, const uint8_t* b, uint8_t* o) { wr(o, fp_add(rd(a), rd(b))); }
void h_fp_sub(const uint8_t* a, const uint8_t* b, uint8_t* o) { wr(o, fp_sub(rd(a), rd(b))); }
void h_fp_inv(const uint8_t* a, uint8_t* o) { wr(o, fp_inv(rd(a))); }
int h_fp_is_square(const uint8_t* a) { return fp_is_square(rd(a)); }
void h_fp2_mul(const uint8_t* a, const uint8_t* b, uint8_t* o) { wr2(o, fp2_mul(rd2(a), rd2(b))); }
void h_fp2_sqr(const uint8_t* a, uint8_t* o) { wr2(o, fp2_sqr(rd2(a))); }
void h_fp2_inv(const uint8_t* a, uint8_t* o) { wr2(o, fp2_inv(rd2(a))); }
int h_fp2_sqrt(const uint8_t* a, uint8_t* o) { fp2 r; int ok = fp2_sqrt(r, rd2(a)); wr2(o, r); return ok; }
int h_fp2_sgn0(const uint8_t* a) { return fp2_sgn0(rd2(a)); }
void h_expand_xmd(const uint8_t* msg, uint8_t* out256) {
  uint32_t w[64]; expand_message_xmd_256(w, msg);
  for (int i = 0; i < 64; i++) { out256[4*i] = w[i] >> 24; out256[4*i+1] = w[i] >> 16; out256[4*i+2] = w[i] >> 8; out256[4*i+3] = w[i]; }
}
void h_hash_to_field(const uint8_t* msg, uint8_t* out192) {
  uint32_t ub[64]; expand_message_xmd_256(ub, msg);
  for (int k = 0; k < 4; k++) wr(out192 + 48 * k, fp_from_be64_words(ub + 16 * k));
}
int h_map_to_curve(const uint8_t* u96, uint8_t* out192) { return wrg2(out192, map_to_curve_g2(rd2(u96))); }
int h_map_to_curve_fold(const uint8_t* u96, uint8_t* out192) {
  return wrg2(out192, map_to_curve_g2_fold(rd2(u96), [](const fp& a, const uint32_t* e, int top) { return fp_pow_const(a, e, top); }));
}
int h_hash_to_g2(const uint8_t* msg, uint8_t* out192) { return wrg2(out192, hash_to_g2(msg)); }
int h_g2_clear_cofactor(const uint8_t* p192, uint8_t* out192) { return wrg2(out192, g2_clear_cofactor(jac_from_aff(rdg2(p192)))); }
int h_g2_in_subgroup(const uint8_t* p192) { return g2_in_subgroup(jac_from_aff(rdg2(p192))); }
int h_g2_aff_in_subgroup(const uint8_t* p192) { return g2_aff_in_subgroup_i(rdg2(p192)); }
int h_g2_psi(const uint8_t* p192, uint8_t* out192) { return wrg2(out192, g2_psi(jac_from_aff(rdg2(p192)))); }
int h_g2_mul(const uint8_t* p192, uint64_t k, uint8_t* out192) { return wrg2(out192, jac_mul_u64(rdg2(p192), k)); }
int h_g2_add(const uint8_t* p, const uint8_t* q, uint8_t* o) { return wrg2(o, jac_add(jac_from_aff(rdg2(p)), jac_from_aff(rdg2(q)))); }
int h_g2_dbl(const uint8_t* p, uint8_t* o) { return wrg2(o, jac_dbl(jac_from_aff(rdg2(p)))); }
int h_g1_mul(const uint8_t* p96, uint64_t k, uint8_t* out96) { return wrg1(out96, jac_mul_u64(rdg1(p96), k)); }
int h_g1_add(const uint8_t* p, const uint8_t* q, uint8_t* o) { return wrg1(o, jac_add(jac_from_aff(rdg1(p)), jac_from_aff(rdg1(q)))); }
int h_g1_add_aff(const uint8_t* p, const uint8_t* q, uint8_t* o) { return wrg1(o, jac_add_aff(jac_from_aff(rdg1(p)), rdg1(q))); }
int h_g2_decompress(const uint8_t* b96, uint8_t* out192, int* inf) { g2a a; bool i; int st = g2_decompress96(b96, a, i); wr2(out192, a.x); wr2(out192 + 96, a.y); *inf = i; return st; }
int h_g1_decompress(const uint8_t* b48, uint8_t* out96, int* inf) { g1a a; bool i; int st = g1_decompress48(b48, a, i); wr(out96, a.x); wr(out96 + 48, a.y); *inf = i; return st; }
int h_g1_deserialize(const uint8_t* b96, uint8_t* out96, int* inf) { g1a a; bool i; int st = g1_deserialize96(b96, a, i); wr(out96, a.x); wr(out96 + 48, a.y); *inf = i; return st; }
void h_g2_compress(const uint8_t* p192, uint8_t* out96) { g2_compress96(out96, rdg2(p192), false); }
void h_g1_compress(const uint8_t* p96, uint8_t* out48) { g1_compress48(out48, rdg1(p96), false); }
void h_miller(const uint8_t* p96, const uint8_t* q192, uint8_t* out576) { fp12_to_be576(out576, miller_loop(rdg1(p96), rdg2(q192))); }
void h_miller_fe(const uint8_t* p96, const uint8_t* q192, uint8_t* out576) { fp12_to_be576(out576, final_exponentiation(miller_loop(rdg1(p96), rdg2(q192)))); }
// FE(ML(P1,Q1) * ML(P2,Q2)) == 1 ?
int h_pairing_check2(const uint8_t* p1, const uint8_t* q1, const uint8_t* p2, const uint8_t* q2) {
  fp12 f = fp12_mul(miller_loop(rdg1(p1), rdg2(q1)), miller_loop(rdg1(p2), rdg2(q2)));
  return fp12_is_one(final_exponentiation(f));
}
}
