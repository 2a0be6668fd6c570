// Per-lane arithmetic for the long sequential chains of the FAV batch (one
// lane owns one value; no cross-lane traffic):
//   - fp_pow_w3: fixed-exponent sliding-window (w = 3) exponentiation with the
//     multiplications inlined in one loop body, so the 379-bit square-root
//     exponents cost ~379 squarings + ~95 products with operands in VGPRs;
//   - fp2_sqrt_lane: square root in Fp2 with two Fp exponentiations and no
//     inversion or Jacobi symbol (see below);
//   - map_to_curve_sswu_lane: RFC 9380 simplified SWU with two exponentiations
//     (x1's inversion is folded into the norm root's, see below);
//   - g2_decompress_lane: ZCash signature decoding with fp2_sqrt_lane.
// Results are identical to bls_h2c.h / bls_curve.h (the same canonical
// points; tests/hostcheck compares both with the oracle).
#pragma once
#include "bls_curve.h"
#include "bls_fq.h"
#include "bls_sha256.h"
#include "bls_tower_inline.h"

namespace bls {

// a^e, e given as little-endian u32 limbs with bit nbits-1 set: sliding
// window w = 3 in the digit form of bls_fq.h (every operand is a product
// output, so no bound bookkeeping; ~1.4x the packed products' rate and
// squarings at 315 instead of 390 mads), canonical packed result.  Control
// flow depends only on e (uniform across lanes).
BLS_HD Fp fp_pow_w3(const Fp& a, const uint32_t* e, int nbits) { return fq_pack_n(fq_pow_w3(fq_unpack(a), e, nbits)); }

// a^(p-2): inversion with uniform control flow (no divergent GCD loop)
BLS_HD Fp fp_inv_fermat_w3(const Fp& a) { return fp_pow_w3(a, EXP_P_MINUS_2, EXP_P_MINUS_2_BITS); }

BLS_HD Fp2 fp2_inv_lane(const Fp2& a) {
  const Fp ni = fp_inv_fermat_w3(fp_add(fp_sqr_i(a.c0), fp_sqr_i(a.c1)));
  return Fp2{fp_mul_i(a.c0, ni), fp_neg(fp_mul_i(a.c1, ni))};
}

BLS_HD Fp fp_sqrt_cand(const Fp& a) { return fp_pow_w3(a, EXP_SQRT, EXP_SQRT_BITS); }      // a^((p+1)/4)
BLS_HD Fp fp_pow_pm3_4(const Fp& a) { return fp_pow_w3(a, EXP_SQRT_M3, EXP_SQRT_M3_BITS); }  // a^((p-3)/4)

// Square root of a = a0 + a1 i with a1 != 0, given n with n^2 = a0^2 + a1^2.
// t = (a0 + n)/2 and s = t^((p-3)/4):
//   t a square:      x0 = t s,        x1 = a1 s / 2     (x0 = sqrt t, 1/x0 = s)
//   t a non-square:  x0 = a1 s / 2,   x1 = -t s         (p = 3 mod 8 makes
//                    s^2 = -1/t, i.e. s = sqrt(-1/t), and x0^2 - x1^2 = a0)
// Both cases satisfy (x0 + x1 i)^2 = a; the caller picks the sign.
BLS_HD Fp2 fp2_sqrt_from_norm_root(const Fp2& a, const Fp& n) {
  const Fp t = fp_mul_i(fp_add(a.c0, n), FP_INV2);
  const Fp s = fp_pow_pm3_4(t);
  const Fp ts = fp_mul_i(t, s);
  const Fp hs = fp_mul_i(fp_mul_i(a.c1, FP_INV2), s);
  if (fp_is_one(fp_mul_i(ts, s))) return Fp2{ts, hs};
  return Fp2{hs, fp_neg(ts)};
}

// Some square root of a; false if a is not a square in Fp2.
BLS_HDNI bool fp2_sqrt_lane(Fp2& out, const Fp2& a) {
  if (fp_is_zero(a.c1)) {  // a in Fp: s = a0^((p+1)/4), s^2 = a0 or -a0
    const Fp s = fp_sqrt_cand(a.c0);
    out = fp_eq(fp_sqr_i(s), a.c0) ? Fp2{s, fp_zero()} : Fp2{fp_zero(), s};
    return true;  // every element of Fp is a square in Fp2
  }
  const Fp nrm = fp_add(fp_sqr_i(a.c0), fp_sqr_i(a.c1));
  const Fp n = fp_sqrt_cand(nrm);
  if (!fp_eq(fp_sqr_i(n), nrm)) return false;
  out = fp2_sqrt_from_norm_root(a, n);
  return true;
}

// fp2_sqrt_lane inlined (the signature-decode kernel: the out-of-line call cost it a call frame of private memory)
BLS_HD bool fp2_sqrt_lane_i(Fp2& out, const Fp2& a) {
  if (fp_is_zero(a.c1)) {
    const Fp s = fp_sqrt_cand(a.c0);
    out = fp_eq(fp_sqr_i(s), a.c0) ? Fp2{s, fp_zero()} : Fp2{fp_zero(), s};
    return true;
  }
  const Fp nrm = fp_add(fp_sqr_i(a.c0), fp_sqr_i(a.c1));
  const Fp n = fp_sqrt_cand(nrm);
  if (!fp_eq(fp_sqr_i(n), nrm)) return false;
  out = fp2_sqrt_from_norm_root(a, n);
  return true;
}

BLS_HD int fp2_sgn0_lane(const Fp2& a_mont) {
  Fp one = fp_zero();
  one.l[0] = 1;
  const Fp a0 = fp_mul_i(a_mont.c0, one), a1 = fp_mul_i(a_mont.c1, one);  // out of Montgomery form, inline
  return (int)(a0.l[0] & 1u) | ((int)fp_is_zero(a0) & (int)(a1.l[0] & 1u));
}

// RFC 9380 simplified SWU on E2' -> affine (x, y), with ONE exponentiation
// before the final square root instead of an inversion plus an
// exponentiation.  x1 = xn / xd (xn = -B/A (den + 1), xd = den), D = norm(xd),
// g(x1) = gxn / xd^3 and norm(g(x1)) = Ag / D^3 with Ag = norm(gxn).  For
// w = Ag D^5 and z = w^((p-3)/4) (p = 3 mod 4), z^2 = chi(w) / w, where
// chi(w) = chi(norm(g(x1))) says whether g(x1) is a square in Fp2.  Hence
//   1 / D = chi z^2 Ag D^4      (the inversion of x1)
//   c = Ag D z,  c^2 = chi norm(g(x1))
// -- c is a root of +-norm(g(x1)), which is all the two branches below need
// (round 1 took c = norm(g(x1))^((p+1)/4), the same up to sign; the root's sign
// does not matter to fp2_sqrt_from_norm_root, and y's sign is fixed by sgn0).
// If g(x2) is used, g(x2) = Z^3 u^6 g(x1) and its norm root is K c norm(u)^3
// with K = sqrt(-norm(Z)^3) (SSWU_K_NORM).  Ag = 0 (g(x1) = 0) keeps 1/D by a
// Fermat inversion (unreachable for hash outputs in practice).
// Inline form for the hash_to_G2 lane kernel: inline products (f2mul / f2sqr of bls_tower_inline.h; each
// out-of-line fp2_mul / fp2_sqr call cost the kernel a call frame of private memory), everything used after an
// exponentiation folded before it, so few values live across the exponentiation loops (zu2, xn conj(xd), ag d^4,
// ag d, K norm(u)^3 and sgn0(u)), and no call: the two cases that need another exponentiation -- g(x1) = 0 and
// g(x) in Fp -- are returned as `rare` (the caller's item goes to its reference-path fallback; neither occurs for
// hash outputs in practice).  Otherwise the same x, y as map_to_curve_sswu_lane.
BLS_HD void map_to_curve_sswu_lane_i(Fp2& x, Fp2& y, const Fp2& u, bool& rare) {
  const int sgn_u = fp2_sgn0_lane(u);
  const Fp2 zu2 = f2mul(SSWU_Z, f2sqr(u));
  const Fp nu = fp_add(fp_sqr_i(u.c0), fp_sqr_i(u.c1));
  const Fp knu3 = fp_mul_i(SSWU_K_NORM, fp_mul_i(fp_sqr_i(nu), nu));  // K norm(u)^3 (the g(x2) branch)
  const Fp2 den = fp2_add(f2sqr(zu2), zu2);
  const bool exc = fp2_is_zero(den);
  const Fp2 xn = exc ? SSWU_B_OVER_ZA : f2mul(SSWU_MINUS_B_OVER_A, fp2_add(fp2_one(), den));
  const Fp2 xd = exc ? fp2_one() : den;
  const Fp2 xd2 = f2sqr(xd);
  // gxn = xn^3 + A xn xd^2 + B xd^3
  const Fp2 gxn = fp2_add(f2mul(fp2_add(f2sqr(xn), f2mul(SSWU_A, xd2)), xn), f2mul(SSWU_B, f2mul(xd2, xd)));
  const Fp ag = fp_add(fp_sqr_i(gxn.c0), fp_sqr_i(gxn.c1));
  const Fp d = fp_add(fp_sqr_i(xd.c0), fp_sqr_i(xd.c1));
  const Fp d4 = fp_sqr_i(fp_sqr_i(d));
  const Fp w = fp_mul_i(ag, fp_mul_i(d4, d));
  const Fp2 xnc = f2mul(xn, fp2_conj(xd));
  const Fp agd4 = fp_mul_i(ag, d4), agd = fp_mul_i(ag, d);
  const bool ag0 = fp_is_zero(ag);
  const Fp z = fp_pow_pm3_4(w);
  const Fp z2 = fp_sqr_i(z);
  const bool square = ag0 || fp_is_one(fp_mul_i(z2, w));  // chi(w) = 1 (or g(x1) = 0: y = 0)
  Fp dinv = fp_mul_i(z2, agd4);  // chi / D
  if (!square) dinv = fp_neg(dinv);
  const Fp2 x1{fp_mul_i(xnc.c0, dinv), fp_mul_i(xnc.c1, dinv)};
  const Fp c = fp_mul_i(agd, z);
  x = square ? x1 : f2mul(zu2, x1);
  const Fp2 gx = fp2_add(f2mul(fp2_add(f2sqr(x), SSWU_A), x), SSWU_B);
  const Fp n = square ? c : fp_mul_i(knu3, c);
  rare = ag0 || fp_is_zero(gx.c1);
  Fp2 yy = fp2_sqrt_from_norm_root(gx, n);
  if (sgn_u != fp2_sgn0_lane(yy)) yy = fp2_neg(yy);
  y = yy;
}
BLS_HDNI void map_to_curve_sswu_lane(Fp2& x, Fp2& y, const Fp2& u) {
  const Fp2 u2 = fp2_sqr(u);
  const Fp2 zu2 = fp2_mul(SSWU_Z, u2);
  const Fp2 den = fp2_add(fp2_sqr(zu2), zu2);
  const bool exc = fp2_is_zero(den);
  const Fp2 xn = exc ? SSWU_B_OVER_ZA : fp2_mul(SSWU_MINUS_B_OVER_A, fp2_add(fp2_one(), den));
  const Fp2 xd = exc ? fp2_one() : den;
  const Fp2 xd2 = fp2_sqr(xd);
  // gxn = xn^3 + A xn xd^2 + B xd^3
  const Fp2 gxn = fp2_add(fp2_mul(fp2_add(fp2_sqr(xn), fp2_mul(SSWU_A, xd2)), xn), fp2_mul(SSWU_B, fp2_mul(xd2, xd)));
  const Fp ag = fp_add(fp_sqr_i(gxn.c0), fp_sqr_i(gxn.c1));
  const Fp d = fp_add(fp_sqr_i(xd.c0), fp_sqr_i(xd.c1));
  const Fp d2 = fp_sqr_i(d), d4 = fp_sqr_i(d2);
  const Fp w = fp_mul_i(ag, fp_mul_i(d4, d));
  const Fp z = fp_pow_pm3_4(w);
  const Fp z2 = fp_sqr_i(z);
  const bool square = fp_is_zero(ag) || fp_is_one(fp_mul_i(z2, w));  // chi(w) = 1 (or g(x1) = 0: y = 0)
  Fp dinv = fp_mul_i(fp_mul_i(z2, ag), d4);  // chi / D
  if (!square) dinv = fp_neg(dinv);
  if (fp_is_zero(ag)) dinv = fp_inv_fermat_w3(d);
  const Fp2 xnc = fp2_mul(xn, fp2_conj(xd));
  const Fp2 x1{fp_mul_i(xnc.c0, dinv), fp_mul_i(xnc.c1, dinv)};
  const Fp c = fp_mul_i(fp_mul_i(ag, d), z);
  Fp2 gx;
  Fp n;
  if (square) {
    x = x1;
    gx = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1), SSWU_A), x1), SSWU_B);
    n = c;
  } else {
    x = fp2_mul(zu2, x1);
    gx = fp2_add(fp2_mul(fp2_add(fp2_sqr(x), SSWU_A), x), SSWU_B);
    const Fp nu = fp_add(fp_sqr_i(u.c0), fp_sqr_i(u.c1));
    n = fp_mul_i(fp_mul_i(SSWU_K_NORM, c), fp_mul_i(fp_sqr_i(nu), nu));
  }
  Fp2 yy;
  if (fp_is_zero(gx.c1)) {
    fp2_sqrt_lane(yy, gx);
  } else {
    yy = fp2_sqrt_from_norm_root(gx, n);
  }
  if (fp2_sgn0_lane(u) != fp2_sgn0_lane(yy)) yy = fp2_neg(yy);
  y = yy;
}


// 96 bytes (x.c1 || x.c0) -> affine G2 (py_ecc signature_to_G2 rules); no
// subgroup check.
BLS_HDNI int g2_decompress_lane(G2A& out, const uint8_t* b) {
  const uint8_t f = b[0];
  const bool c_flag = f & 0x80, b_flag = f & 0x40, a_flag = f & 0x20;
  out.inf = false;
  if (!c_flag) return DEC_BAD_FLAGS;
  uint8_t tmp[48];
  for (int i = 0; i < 48; i++) tmp[i] = b[i];
  tmp[0] &= 0x1f;
  const Fp x1 = raw_from_be48(tmp);
  const Fp x0 = raw_from_be48(b + 48);
  const bool x_zero = fp_is_zero(x1) && fp_is_zero(x0);
  if (b_flag != x_zero) return DEC_BAD_FLAGS;
  if (x_zero) {
    if (a_flag) return DEC_BAD_FLAGS;
    out.inf = true;
    out.x = fp2_zero();
    out.y = fp2_zero();
    return DEC_INFINITY;
  }
  if (!raw_lt_p(x1) || !raw_lt_p(x0)) return DEC_NOT_FIELD;
  const Fp2 xm{fp_to_mont(x0), fp_to_mont(x1)};
  const Fp2 rhs = fp2_add(fp2_mul(fp2_sqr(xm), xm), FP2_B2);
  Fp2 y;
  if (!fp2_sqrt_lane(y, rhs)) return DEC_NOT_ON_CURVE;
  if (fp2_lex_largest(y) != a_flag) y = fp2_neg(y);
  out.x = xm;
  out.y = y;
  return DEC_OK;
}

constexpr Fp FP_RAW_ONE = {{1u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}};  // a R^-1 = a out of Montgomery form

// g2_decompress_lane for 4-byte-aligned signatures, inline and call-free: word loads instead of a byte buffer,
// fp_mul_i by R^2 instead of the out-of-line fp_to_mont, fp2_sqrt_lane_i.  Same statuses and points.
__device__ __forceinline__ int g2_decompress_lane_w(G2A& out, const uint8_t* b) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(b);
  Fp x1, x0;
#pragma unroll
  for (int k = 0; k < 12; k++) {
    x1.l[11 - k] = __builtin_bswap32(w[k]);
    x0.l[11 - k] = __builtin_bswap32(w[12 + k]);
  }
  const uint32_t f = x1.l[11] >> 24;
  const bool c_flag = f & 0x80, b_flag = f & 0x40, a_flag = f & 0x20;
  x1.l[11] &= 0x1fffffffu;
  out.inf = false;
  if (!c_flag) return DEC_BAD_FLAGS;
  const bool x_zero = fp_is_zero(x1) && fp_is_zero(x0);
  if (b_flag != x_zero) return DEC_BAD_FLAGS;
  if (x_zero) {
    if (a_flag) return DEC_BAD_FLAGS;
    out.inf = true;
    out.x = fp2_zero();
    out.y = fp2_zero();
    return DEC_INFINITY;
  }
  if (!raw_lt_p(x1) || !raw_lt_p(x0)) return DEC_NOT_FIELD;
  const Fp2 xm{fp_mul_i(x0, FP_R2), fp_mul_i(x1, FP_R2)};
  const Fp2 rhs = fp2_add(f2mul(f2sqr(xm), xm), FP2_B2);
  Fp2 y;
  if (!fp2_sqrt_lane_i(y, rhs)) return DEC_NOT_ON_CURVE;
  // fp2_lex_largest inline (the out-of-line one is a call frame of private memory)
  const Fp y0 = fp_mul_i(y.c0, FP_RAW_ONE), y1 = fp_mul_i(y.c1, FP_RAW_ONE);
  const bool largest = !fp_is_zero(y1) ? raw_gt_half(y1) : raw_gt_half(y0);
  if (largest != a_flag) y = fp2_neg(y);
  out.x = xm;
  out.y = y;
  return DEC_OK;
}

}  // namespace bls
