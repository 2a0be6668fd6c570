// Complete projective G1 additions (Renes-Costello-Batina alg. 7 / 8, a = 0,
// b3 = 12) in the redundant digit form of bls_fq.h, for the registry gather
// (k_fav_gather_q, bls_kernels.hip).
#pragma once
#include "bls_fq.h"

namespace bls {

// The registry gather in the redundant digit form (bls_fq.h): the accumulator
// stays in digits between additions (no unpack / repack / final subtraction
// per product), additions and subtractions are digit-wise, and the products by
// 3b = 12 are one pass of 64-bit digit products.  Bounds, for the L-form
// accumulator (digits <= 2^29 + 2^4; value X < 66p, Y, Z < 4p):
//   (x2 + y2)(X + Y): digits <= 2^30 x 2^30 + ...; t3 = that - (t0 + t1) + 128p
//   is normalised; t1' = t1 - 12 Z + 64p (digits <= 3 * 2^29) only meets
//   L-form partners; every product's value is far below p R (R / p ~ 2^25.3).
// The host test (tests/test_hostcheck.py::test_fq_gather_formulas) runs these
// formulas with the 128-bit column checks of bls_fq.h.
struct G1Q {
  Fq x, y, z;
};
BLS_HD G1Q g1q_add_aff(const G1Q& p, const Fq& x2, const Fq& y2) {
  const Fq t0 = fq_mul(p.x, x2);
  const Fq t1 = fq_mul(p.y, y2);
  const Fq t3 = fq_norm(fq_sub2(fq_mul(fq_add(x2, y2), fq_add(p.x, p.y)), fq_add(t0, t1)));
  const Fq t4 = fq_add(fq_mul(y2, p.z), p.y);
  const Fq y3 = fq_mul_small(fq_add(fq_mul(x2, p.z), p.x), 12);
  const Fq t0p = fq_add(fq_add(t0, t0), t0);
  const Fq t2 = fq_mul_small(p.z, 12);
  const Fq z3 = fq_norm(fq_add(t1, t2));
  const Fq t1p = fq_sub(t1, t2);
  G1Q r;
  r.x = fq_norm(fq_sub(fq_mul(t3, t1p), fq_mul(t4, y3)));
  r.y = fq_norm(fq_add(fq_mul(t1p, z3), fq_mul(y3, t0p)));
  r.z = fq_norm(fq_add(fq_mul(z3, t4), fq_mul(t0p, t3)));
  return r;
}
// complete projective addition (RCB alg. 7) of two accumulators in L form
BLS_HD G1Q g1q_add(const G1Q& p, const G1Q& q) {
  const Fq t0 = fq_mul(p.x, q.x), t1 = fq_mul(p.y, q.y), t2 = fq_mul(p.z, q.z);
  const Fq t3 = fq_norm(fq_sub2(fq_mul(fq_add(p.x, p.y), fq_add(q.x, q.y)), fq_add(t0, t1)));
  const Fq t4 = fq_norm(fq_sub2(fq_mul(fq_add(p.y, p.z), fq_add(q.y, q.z)), fq_add(t1, t2)));
  const Fq y3 = fq_mul_small(fq_sub2(fq_mul(fq_add(p.x, p.z), fq_add(q.x, q.z)), fq_add(t0, t2)), 12);
  const Fq t0p = fq_add(fq_add(t0, t0), t0);
  const Fq t2p = fq_mul_small(t2, 12);
  const Fq z3 = fq_norm(fq_add(t1, t2p));
  const Fq t1p = fq_sub(t1, t2p);
  G1Q r;
  r.x = fq_norm(fq_sub(fq_mul(t3, t1p), fq_mul(t4, y3)));
  r.y = fq_norm(fq_add(fq_mul(t1p, z3), fq_mul(y3, t0p)));
  r.z = fq_norm(fq_add(fq_mul(z3, t4), fq_mul(t0p, t3)));
  return r;
}

// complete doubling (RCB alg. 9) of an L-form point; outputs X, Y < 4p, Z < 2p in L form
BLS_HD G1Q g1q_dbl(const G1Q& p) {
  const Fq t0 = fq_mul(p.y, p.y);
  const Fq t1 = fq_mul(p.y, p.z);
  const Fq t2 = fq_mul_small(fq_mul(p.z, p.z), 12);                 // 3b Z^2, < 24p
  const Fq u = fq_mul(p.x, p.y);
  const Fq z8 = fq_mul_small(t0, 8);
  const Fq x3a = fq_mul(t2, z8);
  G1Q r;
  r.z = fq_mul(t1, z8);
  const Fq w = fq_norm(fq_sub2(t0, fq_mul_small(t2, 3)));           // t0 - 3 t2 + 128p
  r.y = fq_norm(fq_add(fq_mul(w, fq_add(t0, t2)), x3a));
  r.x = fq_mul_small(fq_mul(w, u), 2);
  return r;
}

}  // namespace bls
