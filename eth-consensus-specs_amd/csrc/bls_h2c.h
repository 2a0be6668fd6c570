// hash_to_G2 for BLS12381G2_XMD:SHA-256_SSWU_RO_ (RFC 9380):
//   expand_message_xmd -> hash_to_field (2 x Fp2) -> simplified SWU on E2'
//   -> 3-isogeny to E2 -> add -> clear_cofactor (Budroni-Pintore, psi-based).
// The isogeny is evaluated straight into Jacobian coordinates, so the only
// inversions on the path are the SWU inv0 and the field square roots.
#pragma once
#include "bls_curve.h"
#include "bls_sha256.h"

namespace bls {

// 64 big-endian bytes mod p -> Montgomery form: lo*R^2/R + hi*(2^384 R^2)/R
BLS_HDNI Fp fp_from_be64_mod(const uint8_t* b) {
  Fp lo = raw_from_be48(b + 16);
  Fp hi = fp_zero();
  for (int i = 0; i < 4; i++) {
    const uint8_t* q = b + 12 - 4 * i;
    hi.l[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
  return fp_add(fp_mul(lo, FP_R2), fp_mul(hi, FP_2P384_R2));
}

BLS_HDNI void hash_to_field_fp2(Fp2 u[2], const uint8_t* msg, uint32_t msg_len, const uint8_t* dst, uint32_t dst_len) {
  uint8_t ub[256];
  expand_message_xmd_256(ub, msg, msg_len, dst, dst_len);
  u[0].c0 = fp_from_be64_mod(ub);
  u[0].c1 = fp_from_be64_mod(ub + 64);
  u[1].c0 = fp_from_be64_mod(ub + 128);
  u[1].c1 = fp_from_be64_mod(ub + 192);
}

BLS_HDNI int fp2_sgn0(const Fp2& a_mont) {
  Fp a0 = fp_from_mont(a_mont.c0), a1 = fp_from_mont(a_mont.c1);
  int sign0 = a0.l[0] & 1;
  int zero0 = fp_is_zero(a0);
  int sign1 = a1.l[0] & 1;
  return sign0 | (zero0 & sign1);
}

// RFC 9380 §6.6.2 (straight-line form) -> affine point on E2'
BLS_HDNI void map_to_curve_sswu(Fp2& x, Fp2& y, const Fp2& u) {
  Fp2 zu2 = fp2_mul(SSWU_Z, fp2_sqr(u));
  Fp2 den = fp2_add(fp2_sqr(zu2), zu2);
  Fp2 x1;
  if (fp2_is_zero(den)) {
    x1 = SSWU_B_OVER_ZA;
  } else {
    x1 = fp2_mul(SSWU_MINUS_B_OVER_A, fp2_add(fp2_one(), fp2_inv(den)));
  }
  Fp2 gx1 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1), SSWU_A), x1), SSWU_B);
  Fp2 yy;
  if (fp2_is_square(gx1)) {
    x = x1;
    fp2_sqrt(yy, gx1);
  } else {
    Fp2 x2 = fp2_mul(zu2, x1);
    Fp2 gx2 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x2), SSWU_A), x2), SSWU_B);
    x = x2;
    fp2_sqrt(yy, gx2);
  }
  if (fp2_sgn0(u) != fp2_sgn0(yy)) yy = fp2_neg(yy);
  y = yy;
}

// 3-isogeny E2' -> E2, output Jacobian with Z = xden*yden
BLS_HDNI G2J iso_map_jac(const Fp2& x, const Fp2& y) {
  Fp2 xx = fp2_sqr(x);
  Fp2 xxx = fp2_mul(xx, x);
  Fp2 xnum = fp2_add(fp2_add(fp2_mul(ISO_XNUM_3, xxx), fp2_mul(ISO_XNUM_2, xx)), fp2_add(fp2_mul(ISO_XNUM_1, x), ISO_XNUM_0));
  Fp2 xden = fp2_add(fp2_add(xx, fp2_mul(ISO_XDEN_1, x)), ISO_XDEN_0);
  Fp2 ynum = fp2_add(fp2_add(fp2_mul(ISO_YNUM_3, xxx), fp2_mul(ISO_YNUM_2, xx)), fp2_add(fp2_mul(ISO_YNUM_1, x), ISO_YNUM_0));
  Fp2 yden = fp2_add(fp2_add(xxx, fp2_mul(ISO_YDEN_2, xx)), fp2_add(fp2_mul(ISO_YDEN_1, x), ISO_YDEN_0));
  if (fp2_is_zero(xden) || fp2_is_zero(yden)) return jac_identity<Fp2>();
  // x = xnum/xden, y = y*ynum/yden ; Z = xden*yden, X = x Z^2, Y = y Z^3
  G2J r;
  r.z = fp2_mul(xden, yden);
  Fp2 yden2 = fp2_sqr(yden);
  r.x = fp2_mul(fp2_mul(xnum, xden), yden2);
  Fp2 xden3 = fp2_mul(fp2_sqr(xden), xden);
  r.y = fp2_mul(fp2_mul(fp2_mul(y, ynum), xden3), yden2);
  return r;
}

// RFC 9380 Appendix G.3: h_eff * P = [x^2-x-1]P + [x-1]psi(P) + psi^2(2P)
BLS_HDNI G2J clear_cofactor_g2(const G2J& p) {
  G2J t1 = jac_neg(jac_mul_xabs(p));                 // [x]P
  G2J t2 = g2_psi(p);                                 // psi(P)
  G2J t3 = g2_psi2(jac_dbl(p));                       // psi^2(2P)
  t3 = jac_add(t3, jac_neg(t2));                      // t3 - t2
  t2 = jac_add(t1, t2);                               // t1 + t2
  t2 = jac_neg(jac_mul_xabs(t2));                     // [x](t1 + t2)
  t3 = jac_add(t3, t2);
  t3 = jac_add(t3, jac_neg(t1));
  return jac_add(t3, jac_neg(p));
}

BLS_HDNI G2J hash_to_g2_from_u(const Fp2 u[2]) {
  Fp2 x0, y0, x1, y1;
  map_to_curve_sswu(x0, y0, u[0]);
  map_to_curve_sswu(x1, y1, u[1]);
  G2J q = jac_add(iso_map_jac(x0, y0), iso_map_jac(x1, y1));
  return clear_cofactor_g2(q);
}

BLS_HDNI G2J hash_to_g2(const uint8_t* msg, uint32_t msg_len, const uint8_t* dst, uint32_t dst_len) {
  Fp2 u[2];
  hash_to_field_fp2(u, msg, msg_len, dst, dst_len);
  return hash_to_g2_from_u(u);
}

}  // namespace bls
