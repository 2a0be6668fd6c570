// TEST HARNESS ONLY: host build of the device arithmetic headers so the
// field/curve/hash/pairing code can be unit-tested against the oracle in a
// container without a GPU.  Never linked into libblsmi355x.so, never loaded
// by the product shim.  All values cross the boundary as canonical
// big-endian integers (48 bytes per Fp).
#include "bls_ops.h"
#include "bls_lane.h"
#include "bls_tower_inline.h"
#include "bls_pp_lane.h"
#include "bls_fp_inv.h"
#include <string.h>
using namespace bls;

static Fp in_fp(const uint8_t* b) { return fp_to_mont(raw_from_be48(b)); }
static void out_fp(uint8_t* b, const Fp& a) { raw_to_be48(fp_from_mont(a), b); }
static Fp2 in_fp2(const uint8_t* b) { return Fp2{in_fp(b), in_fp(b + 48)}; }
static void out_fp2(uint8_t* b, const Fp2& a) { out_fp(b, a.c0); out_fp(b + 48, a.c1); }
static Fp12 in_fp12(const uint8_t* b) {
  Fp12 r;
  r.c0.c0 = in_fp2(b + 0 * 96); r.c1.c0 = in_fp2(b + 1 * 96);
  r.c0.c1 = in_fp2(b + 2 * 96); r.c1.c1 = in_fp2(b + 3 * 96);
  r.c0.c2 = in_fp2(b + 4 * 96); r.c1.c2 = in_fp2(b + 5 * 96);
  return r;
}
static void out_fp12(uint8_t* b, const Fp12& r) {
  out_fp2(b + 0 * 96, r.c0.c0); out_fp2(b + 1 * 96, r.c1.c0);
  out_fp2(b + 2 * 96, r.c0.c1); out_fp2(b + 3 * 96, r.c1.c1);
  out_fp2(b + 4 * 96, r.c0.c2); out_fp2(b + 5 * 96, r.c1.c2);
}

extern "C" {
// inline tower of the lane kernels (bls_tower_inline.h): Fp2 product with unreduced operand sums, Fp12 steps
void hc_f2mul_i(const uint8_t* a, const uint8_t* b, uint8_t* o) { out_fp2(o, f2mul(in_fp2(a), in_fp2(b))); }
void hc_f12sqr_i(const uint8_t* a, uint8_t* o) { out_fp12(o, f12sqr(in_fp12(a))); }
void hc_f12line_i(const uint8_t* f, const uint8_t* l0, const uint8_t* l2, const uint8_t* l3, uint8_t* o) {
  out_fp12(o, f12line(in_fp12(f), in_fp2(l0), in_fp2(l2), in_fp2(l3)));
}
void hc_fp_mul(const uint8_t* a, const uint8_t* b, uint8_t* o) { out_fp(o, fp_mul(in_fp(a), in_fp(b))); }
void hc_fp_add(const uint8_t* a, const uint8_t* b, uint8_t* o) { out_fp(o, fp_add(in_fp(a), in_fp(b))); }
void hc_fp_sub(const uint8_t* a, const uint8_t* b, uint8_t* o) { out_fp(o, fp_sub(in_fp(a), in_fp(b))); }
void hc_fp_inv(const uint8_t* a, uint8_t* o) { out_fp(o, fp_inv(in_fp(a))); }
void hc_fp_inv_sg(const uint8_t* a, uint8_t* o) { out_fp(o, fp_inv_sg(in_fp(a))); }
void hc_fp2_mul(const uint8_t* a, const uint8_t* b, uint8_t* o) { out_fp2(o, fp2_mul(in_fp2(a), in_fp2(b))); }
void hc_fp2_sqr(const uint8_t* a, uint8_t* o) { out_fp2(o, fp2_sqr(in_fp2(a))); }
void hc_fp2_inv(const uint8_t* a, uint8_t* o) { out_fp2(o, fp2_inv(in_fp2(a))); }
int hc_fp2_sqrt(const uint8_t* a, uint8_t* o) { Fp2 r; int ok = fp2_sqrt(r, in_fp2(a)); out_fp2(o, r); return ok; }
void hc_fp12_mul(const uint8_t* a, const uint8_t* b, uint8_t* o) { out_fp12(o, fp12_mul(in_fp12(a), in_fp12(b))); }
void hc_fp12_sqr(const uint8_t* a, uint8_t* o) { out_fp12(o, fp12_sqr(in_fp12(a))); }
void hc_fp12_inv(const uint8_t* a, uint8_t* o) { out_fp12(o, fp12_inv(in_fp12(a))); }
void hc_fp12_frob1(const uint8_t* a, uint8_t* o) { out_fp12(o, fp12_frob1(in_fp12(a))); }
void hc_fp12_frob2(const uint8_t* a, uint8_t* o) { out_fp12(o, fp12_frob2(in_fp12(a))); }
void hc_fp12_mul_line(const uint8_t* f, const uint8_t* l0, const uint8_t* l2, const uint8_t* l3, uint8_t* o) {
  out_fp12(o, fp12_mul_line(in_fp12(f), in_fp2(l0), in_fp2(l2), in_fp2(l3)));
}
void hc_final_exp(const uint8_t* a, uint8_t* o) { out_fp12(o, final_exponentiation(in_fp12(a))); }
// P: x||y (96 bytes), Q: x0||x1||y0||y1 (192 bytes)
void hc_miller_loop(const uint8_t* p, const uint8_t* q, uint8_t* o) {
  G1A P{in_fp(p), in_fp(p + 48), false};
  G2A Q{in_fp2(q), in_fp2(q + 96), false};
  out_fp12(o, miller_loop(P, Q));
}
int hc_g1_decompress(const uint8_t* b, uint8_t* o) {
  G1A a; int st = g1_decompress(a, b);
  if (st == DEC_OK) { out_fp(o, a.x); out_fp(o + 48, a.y); }
  return st;
}
int hc_g2_decompress(const uint8_t* b, uint8_t* o) {
  G2A a; int st = g2_decompress(a, b);
  if (st == DEC_OK) { out_fp2(o, a.x); out_fp2(o + 96, a.y); }
  return st;
}
int hc_g1_in_subgroup(const uint8_t* p) { G1J j{in_fp(p), in_fp(p + 48), FP_ONE}; return g1_in_subgroup(j); }
int hc_g2_in_subgroup(const uint8_t* q) { G2J j{in_fp2(q), in_fp2(q + 96), fp2_one()}; return g2_in_subgroup(j); }
void hc_expand_message_xmd(const uint8_t* m, uint32_t ml, const uint8_t* d, uint32_t dl, uint8_t* o) {
  expand_message_xmd_256(o, m, ml, d, dl);
}
void hc_hash_to_field(const uint8_t* m, uint32_t ml, const uint8_t* d, uint32_t dl, uint8_t* o) {
  Fp2 u[2]; hash_to_field_fp2(u, m, ml, d, dl); out_fp2(o, u[0]); out_fp2(o + 96, u[1]);
}
void hc_map_to_curve(const uint8_t* u, uint8_t* o) {
  Fp2 x, y; map_to_curve_sswu(x, y, in_fp2(u)); out_fp2(o, x); out_fp2(o + 96, y);
}
void hc_hash_to_g2(const uint8_t* m, uint32_t ml, const uint8_t* d, uint32_t dl, uint8_t* o96) {
  g2_compress(o96, jac_to_aff(hash_to_g2(m, ml, d, dl)));
}
int hc_key_validate(const uint8_t* pk) { G1A a; return key_validate(a, pk); }
int hc_sig_validate(const uint8_t* s) { G2A a; return sig_validate(a, s); }
int hc_core_verify(const uint8_t* pk, const uint8_t* m, uint32_t ml, const uint8_t* d, uint32_t dl, const uint8_t* sig) {
  G1A a; if (!key_validate(a, pk)) return 0;
  return core_verify_point(a, m, ml, d, dl, sig);
}
void hc_g2_mul_u256(const uint8_t* q, const uint32_t* k, uint8_t* o96) {
  G2J j{in_fp2(q), in_fp2(q + 96), fp2_one()};
  g2_compress(o96, jac_to_aff(jac_mul_u256(j, k)));
}
void hc_g1_mul_u256(const uint8_t* p, const uint32_t* k, uint8_t* o48) {
  G1J j{in_fp(p), in_fp(p + 48), FP_ONE};
  g1_compress(o48, jac_to_aff(jac_mul_u256(j, k)));
}
}
extern "C" int hc_fp_is_square(const uint8_t* a) { return fp_is_square(in_fp(a)); }
extern "C" void hc_fp_sqr(const uint8_t* a, uint8_t* o) { out_fp(o, fp_sqr(in_fp(a))); }
// per-lane chain math (bls_lane.h)
extern "C" int hc_fp2_sqrt_lane(const uint8_t* a, uint8_t* o) { Fp2 r; int ok = fp2_sqrt_lane(r, in_fp2(a)); out_fp2(o, r); return ok; }
extern "C" void hc_map_to_curve_lane(const uint8_t* u, uint8_t* o) {
  Fp2 x, y; map_to_curve_sswu_lane(x, y, in_fp2(u)); out_fp2(o, x); out_fp2(o + 96, y);
}
extern "C" int hc_g2_decompress_lane(const uint8_t* b, uint8_t* o) {
  G2A a; int st = g2_decompress_lane(a, b);
  if (st == DEC_OK) { out_fp2(o, a.x); out_fp2(o + 96, a.y); }
  return st;
}
extern "C" void hc_fp_pow_w3(const uint8_t* a, const uint32_t* e, int nbits, uint8_t* o) { out_fp(o, fp_pow_w3(in_fp(a), e, nbits)); }

// Jacobian [|x|] chain of the hash_to_G2 lane kernels (bls_pp_lane.h j2_*), from and back to homogeneous
// projective: q affine (x0||x1||y0||y1, 192 bytes) -> affine [|x|] q; returns the exception flag
extern "C" int hc_j2_mul_xabs(const uint8_t* q, uint8_t* o) {
  const PP<Fp2> Q{in_fp2(q), in_fp2(q + 96), fp2_one()};
  bool exc = false;
  const PP<Fp2> M = j2_to_pp(j2_mul_xabs(j2_from_pp(Q), exc));
  const Fp2 zi = fp2_inv(M.z);
  out_fp2(o, fp2_mul(M.x, zi));
  out_fp2(o + 96, fp2_mul(M.y, zi));
  return exc ? 1 : 0;
}
// madd chain step: affine p + affine q through j2_add_aff (p as Jacobian with Z = 1)
extern "C" int hc_j2_add_aff(const uint8_t* p, const uint8_t* q, uint8_t* o) {
  const G2J P{in_fp2(p), in_fp2(p + 96), fp2_one()};
  bool exc = false;
  const G2J R = j2_add_aff(j2_dbl(P), in_fp2(q), in_fp2(q + 96), exc);  // 2p + q
  const PP<Fp2> S = j2_to_pp(R);
  const Fp2 zi = fp2_inv(S.z);
  out_fp2(o, fp2_mul(S.x, zi));
  out_fp2(o + 96, fp2_mul(S.y, zi));
  return exc ? 1 : 0;
}

// register-resident hash_to_field of the FAV h2c kernel (bls_xmd32.h): 32-byte message, POP DST
#include "bls_xmd32.h"
extern "C" void hc_hash_to_field_m32(const uint8_t* m32, uint8_t* o) {
  Fp2 u[2];
  hash_to_field_fp2_m32(u, m32);
  out_fp2(o, u[0]);
  out_fp2(o + 96, u[1]);
}
// the inline SSWU of the FAV h2c kernel (bls_lane.h map_to_curve_sswu_lane_i); returns its `rare` flag
extern "C" int hc_map_to_curve_lane_i(const uint8_t* u, uint8_t* o) {
  Fp2 x, y;
  bool rare = false;
  map_to_curve_sswu_lane_i(x, y, in_fp2(u), rare);
  out_fp2(o, x);
  out_fp2(o + 96, y);
  return rare ? 1 : 0;
}
