// Optimal-ate pairing pieces for BLS12-381 (x = -0xd201000000010000).
//
// Miller loop: T runs in Jacobian coordinates on the twist E2; each step
// yields a line scaled by an Fp2 factor (killed by the final exponentiation)
// with only three non-zero w-basis coefficients:
//   line = l0 + l2 w^2 + l3 w^3,
// tangent at T=(X,Y,Z):  l0 = 3X^3 - 2Y^2, l2 = -3X^2 Z^2 xP, l3 = 2YZ^3 yP
// chord T,Q (Q affine):  l0 = r xQ - yQ Z3, l2 = -r xP,     l3 = Z3 yP
// (r, Z3 from madd-2007-bl).  Derivation: untwist (x,y) -> (x w^-2, y w^-3)
// and multiply the affine line by w^3 and the Fp2 denominator.
//
// Final exponentiation: easy part (p^6-1)(p^2+1), hard part via
//   3 (p^4-p^2+1)/r = (x-1)^2 (x+p) (x^2+p^2-1) + 3,
// i.e. this returns e^3; e == 1 <=> e^3 == 1 because gcd(3, r) = 1.
#pragma once
#include "bls_curve.h"

namespace bls {

struct Line {
  Fp2 l0, l2, l3;
};

// T <- 2T, returns the tangent line evaluated at P = (xP, yP); nxP = -xP.
BLS_HDNI Line ml_dbl_step(G2J& t, const Fp& nxP, const Fp& yP) {
  Fp2 A = fp2_sqr(t.x);
  Fp2 B = fp2_sqr(t.y);
  Fp2 C = fp2_sqr(B);
  Fp2 D = fp2_dbl(fp2_sub(fp2_sub(fp2_sqr(fp2_add(t.x, B)), A), C));
  Fp2 E = fp2_add(fp2_dbl(A), A);
  Fp2 F = fp2_sqr(E);
  Fp2 ZZ = fp2_sqr(t.z);
  Line L;
  L.l0 = fp2_sub(fp2_mul(E, t.x), fp2_dbl(B));
  L.l2 = fp2_mul_fp(fp2_mul(E, ZZ), nxP);
  Fp2 z3 = fp2_sub(fp2_sub(fp2_sqr(fp2_add(t.y, t.z)), B), ZZ);  // 2YZ
  L.l3 = fp2_mul_fp(fp2_mul(z3, ZZ), yP);
  Fp2 x3 = fp2_sub(F, fp2_dbl(D));
  Fp2 C8 = fp2_dbl(fp2_dbl(fp2_dbl(C)));
  t.y = fp2_sub(fp2_mul(E, fp2_sub(D, x3)), C8);
  t.x = x3;
  t.z = z3;
  return L;
}

// T <- T + Q (Q affine, T != +-Q), returns the chord line evaluated at P.
BLS_HDNI Line ml_add_step(G2J& t, const Fp2& xQ, const Fp2& yQ, const Fp& nxP, const Fp& yP) {
  Fp2 z1z1 = fp2_sqr(t.z);
  Fp2 u2 = fp2_mul(xQ, z1z1);
  Fp2 s2 = fp2_mul(fp2_mul(yQ, t.z), z1z1);
  Fp2 h = fp2_sub(u2, t.x);
  Fp2 hh = fp2_sqr(h);
  Fp2 i = fp2_dbl(fp2_dbl(hh));
  Fp2 j = fp2_mul(h, i);
  Fp2 r = fp2_dbl(fp2_sub(s2, t.y));
  Fp2 v = fp2_mul(t.x, i);
  Fp2 x3 = fp2_sub(fp2_sub(fp2_sqr(r), j), fp2_dbl(v));
  Fp2 y3 = fp2_sub(fp2_mul(r, fp2_sub(v, x3)), fp2_dbl(fp2_mul(t.y, j)));
  Fp2 z3 = fp2_sub(fp2_sub(fp2_sqr(fp2_add(t.z, h)), z1z1), hh);
  Line L;
  L.l0 = fp2_sub(fp2_mul(r, xQ), fp2_mul(yQ, z3));
  L.l2 = fp2_mul_fp(r, nxP);
  L.l3 = fp2_mul_fp(z3, yP);
  t.x = x3;
  t.y = y3;
  t.z = z3;
  return L;
}

// f_{|x|,Q}(P) conjugated (x < 0).  Returns 1 if P or Q is the identity.
BLS_HDNI Fp12 miller_loop(const G1A& P, const G2A& Q) {
  if (P.inf || Q.inf) return fp12_one();
  const Fp nxP = fp_neg(P.x);
  G2J T{Q.x, Q.y, fp2_one()};
  Fp12 f = fp12_one();
  bool first = true;
  for (int i = 62; i >= 0; --i) {
    if (!first) f = fp12_sqr(f);
    first = false;
    Line L = ml_dbl_step(T, nxP, P.y);
    f = fp12_mul_line(f, L.l0, L.l2, L.l3);
    if ((X_ABS >> i) & 1ull) {
      L = ml_add_step(T, Q.x, Q.y, nxP, P.y);
      f = fp12_mul_line(f, L.l0, L.l2, L.l3);
    }
  }
  return fp12_conj(f);
}

// a^|x| (plain square-and-multiply; input in the cyclotomic subgroup)
BLS_HDNI Fp12 fp12_pow_xabs(const Fp12& a) {
  Fp12 r = a;
  for (int i = 62; i >= 0; --i) {
    r = fp12_sqr(r);
    if ((X_ABS >> i) & 1ull) r = fp12_mul(r, a);
  }
  return r;
}

// a^x for x = -|x| (inverse = conjugate in the cyclotomic subgroup)
BLS_HDNI Fp12 fp12_pow_x(const Fp12& a) { return fp12_conj(fp12_pow_xabs(a)); }

BLS_HDNI Fp12 final_exponentiation(const Fp12& f) {
  // easy part
  Fp12 t = fp12_mul(fp12_conj(f), fp12_inv(f));  // f^(p^6-1)
  t = fp12_mul(fp12_frob2(t), t);                 // ^(p^2+1)
  // hard part (times 3)
  Fp12 a = fp12_mul(fp12_pow_x(t), fp12_conj(t));  // t^(x-1)
  a = fp12_mul(fp12_pow_x(a), fp12_conj(a));       // t^((x-1)^2)
  Fp12 b = fp12_mul(fp12_pow_x(a), fp12_frob1(a)); // a^(x+p)
  Fp12 c = fp12_pow_x(fp12_pow_x(b));              // b^(x^2)
  c = fp12_mul(fp12_mul(c, fp12_frob2(b)), fp12_conj(b));  // b^(x^2+p^2-1)
  Fp12 t3 = fp12_mul(fp12_sqr(t), t);
  return fp12_mul(c, t3);
}

}  // namespace bls
