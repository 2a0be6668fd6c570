// Inlined extension-field tower and Miller-loop steps for one-lane-per-pair
// kernels (bls_miller_lane.hip).  Same formulas, operation order and
// canonical outputs as the out-of-line versions in bls_tower.h /
// bls_pairing.h, so results are bit-identical; every Montgomery product is
// inlined (fp_mul_i), which keeps the v_mad_u64_u32 chains free of call
// overhead at the cost of code size (profiles/r01_s2_fmerate_microbench.txt:
// inline products reach ~73 % of the mad rate at one wave per SIMD, calls ~43 %).
#pragma once
#include "bls_pairing.h"

namespace bls {

// a + b without the final reduction (< 2p < 2^382: fits 12 limbs; a valid
// Montgomery operand, which only needs to stay below 2^406)
BLS_HD Fp fp_add_raw(const Fp& a, const Fp& b) {
  Fp s;
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) s.l[i] = __builtin_addc(a.l[i], b.l[i], c, &c);
  return s;
}

// Karatsuba with three reduced products.  Operands may be unreduced sums
// (< 8p): a Montgomery product only needs x y < p 2^406, and its output is
// canonical; the sums feeding products are therefore left unreduced
// (fp_add_raw), which saves the conditional subtraction of each.  (A
// lazy-reduction variant -- one fused column pass with two reductions, 952
// instead of 1,134 mads -- held too many digits live and made the pair Miller
// kernel spill: 12x slower.)
BLS_HD Fp2 f2mul(const Fp2& a, const Fp2& b) {
  const Fp t0 = fp_mul_i(a.c0, b.c0), t1 = fp_mul_i(a.c1, b.c1);
  const Fp t2 = fp_mul_i(fp_add_raw(a.c0, a.c1), fp_add_raw(b.c0, b.c1));
  return Fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}
// unreduced Fp2 sum, only as a product operand
BLS_HD Fp2 f2add_raw(const Fp2& a, const Fp2& b) { return Fp2{fp_add_raw(a.c0, b.c0), fp_add_raw(a.c1, b.c1)}; }
BLS_HD Fp2 f2sqr(const Fp2& a) {
  const Fp t0 = fp_mul_i(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1));
  const Fp t1 = fp_mul_i(a.c0, a.c1);
  return Fp2{t0, fp_dbl(t1)};
}
BLS_HD Fp2 f2mulfp(const Fp2& a, const Fp& b) { return Fp2{fp_mul_i(a.c0, b), fp_mul_i(a.c1, b)}; }
BLS_HD Fp2 f2add(const Fp2& a, const Fp2& b) { return fp2_add(a, b); }
BLS_HD Fp2 f2sub(const Fp2& a, const Fp2& b) { return fp2_sub(a, b); }
BLS_HD Fp2 f2xi(const Fp2& a) { return fp2_mul_xi(a); }

BLS_HD Fp6 f6add(const Fp6& a, const Fp6& b) { return Fp6{f2add(a.c0, b.c0), f2add(a.c1, b.c1), f2add(a.c2, b.c2)}; }
BLS_HD Fp6 f6sub(const Fp6& a, const Fp6& b) { return Fp6{f2sub(a.c0, b.c0), f2sub(a.c1, b.c1), f2sub(a.c2, b.c2)}; }
BLS_HD Fp6 f6v(const Fp6& a) { return Fp6{f2xi(a.c2), a.c0, a.c1}; }
BLS_HD Fp6 f6mul(const Fp6& a, const Fp6& b) {
  const Fp2 t0 = f2mul(a.c0, b.c0), t1 = f2mul(a.c1, b.c1), t2 = f2mul(a.c2, b.c2);
  const Fp2 c0 = f2add(f2xi(f2sub(f2sub(f2mul(f2add(a.c1, a.c2), f2add(b.c1, b.c2)), t1), t2)), t0);
  const Fp2 c1 = f2add(f2sub(f2sub(f2mul(f2add(a.c0, a.c1), f2add(b.c0, b.c1)), t0), t1), f2xi(t2));
  const Fp2 c2 = f2add(f2sub(f2sub(f2mul(f2add(a.c0, a.c2), f2add(b.c0, b.c2)), t0), t2), t1);
  return Fp6{c0, c1, c2};
}
BLS_HD Fp6 f6mul01(const Fp6& a, const Fp2& b0, const Fp2& b1) {
  const Fp2 t0 = f2mul(a.c0, b0), t1 = f2mul(a.c1, b1);
  const Fp2 c0 = f2add(t0, f2xi(f2mul(a.c2, b1)));
  const Fp2 c1 = f2sub(f2sub(f2mul(f2add(a.c0, a.c1), f2add(b0, b1)), t0), t1);
  const Fp2 c2 = f2add(t1, f2mul(a.c2, b0));
  return Fp6{c0, c1, c2};
}
BLS_HD Fp6 f6mul1(const Fp6& a, const Fp2& b1) {
  return Fp6{f2xi(f2mul(a.c2, b1)), f2mul(a.c0, b1), f2mul(a.c1, b1)};
}
BLS_HD Fp12 f12sqr(const Fp12& a) {
  const Fp6 t = f6mul(a.c0, a.c1);
  const Fp6 c0 = f6sub(f6sub(f6mul(f6add(a.c0, a.c1), f6add(a.c0, f6v(a.c1))), t), f6v(t));
  return Fp12{c0, f6add(t, t)};
}
BLS_HD Fp12 f12line(const Fp12& f, const Fp2& l0, const Fp2& l2, const Fp2& l3) {
  const Fp6 t0 = f6mul01(f.c0, l0, l2);
  const Fp6 t1 = f6mul1(f.c1, l3);
  const Fp6 s = f6mul01(f6add(f.c0, f.c1), l0, f2add(l2, l3));
  return Fp12{f6add(t0, f6v(t1)), f6sub(f6sub(s, t0), t1)};
}

BLS_HD void ml_dbl_i(G2J& t, const Fp& nxP, const Fp& yP, Fp2& l0, Fp2& l2, Fp2& l3) {
  const Fp2 A = f2sqr(t.x), Bq = f2sqr(t.y), C = f2sqr(Bq);
  const Fp2 D = fp2_dbl(f2sub(f2sub(f2sqr(f2add(t.x, Bq)), A), C));
  const Fp2 E = f2add(fp2_dbl(A), A);
  const Fp2 F = f2sqr(E);
  const Fp2 ZZ = f2sqr(t.z);
  l0 = f2sub(f2mul(E, t.x), fp2_dbl(Bq));
  l2 = f2mulfp(f2mul(E, ZZ), nxP);
  const Fp2 z3 = f2sub(f2sub(f2sqr(f2add(t.y, t.z)), Bq), ZZ);
  l3 = f2mulfp(f2mul(z3, ZZ), yP);
  const Fp2 x3 = f2sub(F, fp2_dbl(D));
  const Fp2 C8 = fp2_dbl(fp2_dbl(fp2_dbl(C)));
  t.y = f2sub(f2mul(E, f2sub(D, x3)), C8);
  t.x = x3;
  t.z = z3;
}

BLS_HD void ml_add_i(G2J& t, const Fp2& xQ, const Fp2& yQ, const Fp& nxP, const Fp& yP, Fp2& l0, Fp2& l2,
                     Fp2& l3) {
  const Fp2 z1z1 = f2sqr(t.z);
  const Fp2 u2 = f2mul(xQ, z1z1);
  const Fp2 s2 = f2mul(f2mul(yQ, t.z), z1z1);
  const Fp2 h = f2sub(u2, t.x);
  const Fp2 hh = f2sqr(h);
  const Fp2 i = fp2_dbl(fp2_dbl(hh));
  const Fp2 j = f2mul(h, i);
  const Fp2 r = fp2_dbl(f2sub(s2, t.y));
  const Fp2 v = f2mul(t.x, i);
  const Fp2 x3 = f2sub(f2sub(f2sqr(r), j), fp2_dbl(v));
  const Fp2 y3 = f2sub(f2mul(r, f2sub(v, x3)), fp2_dbl(f2mul(t.y, j)));
  const Fp2 z3 = f2sub(f2sub(f2sqr(f2add(t.z, h)), z1z1), hh);
  l0 = f2sub(f2mul(r, xQ), f2mul(yQ, z3));
  l2 = f2mulfp(r, nxP);
  l3 = f2mulfp(z3, yP);
  t.x = x3;
  t.y = y3;
  t.z = z3;
}

}  // namespace bls
