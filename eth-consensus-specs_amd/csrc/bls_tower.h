// Extension-field tower Fp2 = Fp[i]/(i^2+1), Fp6 = Fp2[v]/(v^3-xi),
// Fp12 = Fp6[w]/(w^2-v), xi = 1+i.  Karatsuba throughout; the Fp12 line
// multiplication is sparse (w-basis positions 0, 2, 3, see bls_pairing.h).
#pragma once
#include "bls_fp.h"

namespace bls {

// ---------------------------------------------------------------- Fp2 ----
BLS_HD Fp2 fp2_zero() { return Fp2{fp_zero(), fp_zero()}; }
BLS_HD Fp2 fp2_one() { return Fp2{FP_ONE, fp_zero()}; }
BLS_HD bool fp2_is_zero(const Fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
BLS_HD bool fp2_eq(const Fp2& a, const Fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
BLS_HD bool fp2_is_one(const Fp2& a) { return fp_is_one(a.c0) && fp_is_zero(a.c1); }
BLS_HD Fp2 fp2_select(bool c, const Fp2& a, const Fp2& b) {
  return Fp2{fp_select(c, a.c0, b.c0), fp_select(c, a.c1, b.c1)};
}
BLS_HD Fp2 fp2_add(const Fp2& a, const Fp2& b) { return Fp2{fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
BLS_HD Fp2 fp2_sub(const Fp2& a, const Fp2& b) { return Fp2{fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
BLS_HD Fp2 fp2_dbl(const Fp2& a) { return Fp2{fp_dbl(a.c0), fp_dbl(a.c1)}; }
BLS_HD Fp2 fp2_neg(const Fp2& a) { return Fp2{fp_neg(a.c0), fp_neg(a.c1)}; }
BLS_HD Fp2 fp2_conj(const Fp2& a) { return Fp2{a.c0, fp_neg(a.c1)}; }

BLS_HDNI Fp2 fp2_mul(const Fp2& a, const Fp2& b) {
  Fp t0 = fp_mul(a.c0, b.c0);
  Fp t1 = fp_mul(a.c1, b.c1);
  Fp t2 = fp_mul(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
  return Fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}

BLS_HDNI Fp2 fp2_sqr(const Fp2& a) {
  Fp t0 = fp_mul(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1));
  Fp t1 = fp_mul(a.c0, a.c1);
  return Fp2{t0, fp_dbl(t1)};
}

BLS_HDNI Fp2 fp2_mul_fp(const Fp2& a, const Fp& b) { return Fp2{fp_mul(a.c0, b), fp_mul(a.c1, b)}; }

// a * (1 + i)
BLS_HD Fp2 fp2_mul_xi(const Fp2& a) { return Fp2{fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; }

BLS_HD Fp fp2_norm(const Fp2& a) { return fp_add(fp_sqr(a.c0), fp_sqr(a.c1)); }

BLS_HDNI Fp2 fp2_inv(const Fp2& a) {
  Fp ni = fp_inv(fp2_norm(a));
  return Fp2{fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni))};
}

BLS_HD Fp2 fp2_mul_small(const Fp2& a, int k) { return Fp2{fp_mul_small(a.c0, k), fp_mul_small(a.c1, k)}; }

// a is a square in Fp2 iff its norm is a square in Fp
BLS_HDNI bool fp2_is_square(const Fp2& a) { return fp_is_square(fp2_norm(a)); }

// Some square root of a (norm method); returns false if none exists.
// Cost: two Fp square-root exponentiations, one Jacobi symbol, one binary
// inversion (the Jacobi symbol picks the right half-norm candidate first).
BLS_HDNI bool fp2_sqrt(Fp2& out, const Fp2& a) {
  if (fp_is_zero(a.c1)) {
    Fp s;
    if (fp_is_square(a.c0)) {
      fp_sqrt(s, a.c0);
      out = Fp2{s, fp_zero()};
      return true;
    }
    if (fp_sqrt(s, fp_neg(a.c0))) {
      out = Fp2{fp_zero(), s};
      return true;
    }
    return false;
  }
  Fp n;
  if (!fp_sqrt(n, fp2_norm(a))) return false;
  Fp t = fp_mul(fp_add(a.c0, n), FP_INV2);
  if (!fp_is_square(t)) t = fp_mul(fp_sub(a.c0, n), FP_INV2);
  Fp x0;
  if (!fp_sqrt(x0, t)) return false;
  Fp x1 = fp_mul(a.c1, fp_inv(fp_dbl(x0)));
  Fp2 r{x0, x1};
  out = r;
  return fp2_eq(fp2_sqr(r), a);
}

// ---------------------------------------------------------------- Fp6 ----
BLS_HD Fp6 fp6_zero() { return Fp6{fp2_zero(), fp2_zero(), fp2_zero()}; }
BLS_HD Fp6 fp6_one() { return Fp6{fp2_one(), fp2_zero(), fp2_zero()}; }
BLS_HDNI Fp6 fp6_add(const Fp6& a, const Fp6& b) {
  return Fp6{fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)};
}
BLS_HDNI Fp6 fp6_sub(const Fp6& a, const Fp6& b) {
  return Fp6{fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)};
}
BLS_HDNI Fp6 fp6_neg(const Fp6& a) { return Fp6{fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)}; }
BLS_HD bool fp6_is_zero(const Fp6& a) { return fp2_is_zero(a.c0) && fp2_is_zero(a.c1) && fp2_is_zero(a.c2); }

BLS_HDNI Fp6 fp6_mul(const Fp6& a, const Fp6& b) {
  Fp2 t0 = fp2_mul(a.c0, b.c0);
  Fp2 t1 = fp2_mul(a.c1, b.c1);
  Fp2 t2 = fp2_mul(a.c2, b.c2);
  Fp2 c0 = fp2_add(fp2_mul_xi(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c1, a.c2), fp2_add(b.c1, b.c2)), t1), t2)), t0);
  Fp2 c1 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b.c0, b.c1)), t0), t1), fp2_mul_xi(t2));
  Fp2 c2 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c2), fp2_add(b.c0, b.c2)), t0), t2), t1);
  return Fp6{c0, c1, c2};
}

// Chung-Hasan SQR2
BLS_HDNI Fp6 fp6_sqr(const Fp6& a) {
  Fp2 s0 = fp2_sqr(a.c0);
  Fp2 ab = fp2_mul(a.c0, a.c1);
  Fp2 s1 = fp2_dbl(ab);
  Fp2 s2 = fp2_sqr(fp2_add(fp2_sub(a.c0, a.c1), a.c2));
  Fp2 bc = fp2_mul(a.c1, a.c2);
  Fp2 s3 = fp2_dbl(bc);
  Fp2 s4 = fp2_sqr(a.c2);
  Fp2 c0 = fp2_add(s0, fp2_mul_xi(s3));
  Fp2 c1 = fp2_add(s1, fp2_mul_xi(s4));
  Fp2 c2 = fp2_sub(fp2_sub(fp2_add(fp2_add(s1, s2), s3), s0), s4);
  return Fp6{c0, c1, c2};
}

// a * v
BLS_HDNI Fp6 fp6_mul_v(const Fp6& a) { return Fp6{fp2_mul_xi(a.c2), a.c0, a.c1}; }

// a * (b0 + b1 v)
BLS_HDNI Fp6 fp6_mul_01(const Fp6& a, const Fp2& b0, const Fp2& b1) {
  Fp2 t0 = fp2_mul(a.c0, b0);
  Fp2 t1 = fp2_mul(a.c1, b1);
  Fp2 c0 = fp2_add(t0, fp2_mul_xi(fp2_mul(a.c2, b1)));
  Fp2 c1 = fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b0, b1)), t0), t1);
  Fp2 c2 = fp2_add(t1, fp2_mul(a.c2, b0));
  return Fp6{c0, c1, c2};
}

// a * (b1 v)
BLS_HDNI Fp6 fp6_mul_1(const Fp6& a, const Fp2& b1) {
  return Fp6{fp2_mul_xi(fp2_mul(a.c2, b1)), fp2_mul(a.c0, b1), fp2_mul(a.c1, b1)};
}

BLS_HDNI Fp6 fp6_inv(const Fp6& a) {
  Fp2 t0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  Fp2 t1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  Fp2 t2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  Fp2 det = fp2_add(fp2_mul(a.c0, t0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, t1), fp2_mul(a.c1, t2))));
  Fp2 di = fp2_inv(det);
  return Fp6{fp2_mul(t0, di), fp2_mul(t1, di), fp2_mul(t2, di)};
}

// --------------------------------------------------------------- Fp12 ----
BLS_HD Fp12 fp12_one() { return Fp12{fp6_one(), fp6_zero()}; }
BLS_HD bool fp12_is_one(const Fp12& a) {
  return fp2_is_one(a.c0.c0) && fp2_is_zero(a.c0.c1) && fp2_is_zero(a.c0.c2) && fp6_is_zero(a.c1);
}

BLS_HDNI Fp12 fp12_mul(const Fp12& a, const Fp12& b) {
  Fp6 t0 = fp6_mul(a.c0, b.c0);
  Fp6 t1 = fp6_mul(a.c1, b.c1);
  Fp6 c1 = fp6_sub(fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), t0), t1);
  return Fp12{fp6_add(t0, fp6_mul_v(t1)), c1};
}

// complex squaring: 2 Fp6 multiplications
BLS_HDNI Fp12 fp12_sqr(const Fp12& a) {
  Fp6 t = fp6_mul(a.c0, a.c1);
  Fp6 c0 = fp6_sub(fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1))), t), fp6_mul_v(t));
  return Fp12{c0, fp6_add(t, t)};
}

BLS_HDNI Fp12 fp12_conj(const Fp12& a) { return Fp12{a.c0, fp6_neg(a.c1)}; }

BLS_HDNI Fp12 fp12_inv(const Fp12& a) {
  Fp6 d = fp6_sub(fp6_sqr(a.c0), fp6_mul_v(fp6_sqr(a.c1)));
  Fp6 di = fp6_inv(d);
  return Fp12{fp6_mul(a.c0, di), fp6_neg(fp6_mul(a.c1, di))};
}

// Sparse line l = l0 + l2 w^2 + l3 w^3  ==  ((l0, l2, 0), (0, l3, 0)) in the tower.
BLS_HDNI Fp12 fp12_mul_line(const Fp12& f, const Fp2& l0, const Fp2& l2, const Fp2& l3) {
  Fp6 t0 = fp6_mul_01(f.c0, l0, l2);
  Fp6 t1 = fp6_mul_1(f.c1, l3);
  Fp6 s = fp6_mul_01(fp6_add(f.c0, f.c1), l0, fp2_add(l2, l3));
  return Fp12{fp6_add(t0, fp6_mul_v(t1)), fp6_sub(fp6_sub(s, t0), t1)};
}

// Frobenius maps on the w-basis: coefficient k (w^k) -> conj^n(c_k) * gamma_{n,k}.
// Tower position of w^k: k even -> c0.c(k/2), k odd -> c1.c(k/2).
BLS_HDNI Fp12 fp12_frob1(const Fp12& a) {
  Fp12 r;
  r.c0.c0 = fp2_conj(a.c0.c0);
  r.c1.c0 = fp2_mul(fp2_conj(a.c1.c0), FROB1_1);
  r.c0.c1 = fp2_mul(fp2_conj(a.c0.c1), FROB1_2);
  r.c1.c1 = fp2_mul(fp2_conj(a.c1.c1), FROB1_3);
  r.c0.c2 = fp2_mul(fp2_conj(a.c0.c2), FROB1_4);
  r.c1.c2 = fp2_mul(fp2_conj(a.c1.c2), FROB1_5);
  return r;
}

BLS_HDNI Fp12 fp12_frob2(const Fp12& a) {  // gamma_{2,k} lie in Fp
  Fp12 r;
  r.c0.c0 = a.c0.c0;
  r.c1.c0 = fp2_mul_fp(a.c1.c0, FROB2_1.c0);
  r.c0.c1 = fp2_mul_fp(a.c0.c1, FROB2_2.c0);
  r.c1.c1 = fp2_mul_fp(a.c1.c1, FROB2_3.c0);
  r.c0.c2 = fp2_mul_fp(a.c0.c2, FROB2_4.c0);
  r.c1.c2 = fp2_mul_fp(a.c1.c2, FROB2_5.c0);
  return r;
}

}  // namespace bls
