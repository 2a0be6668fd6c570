// Fp2 products and the Jacobian [|x|] chain of the cofactor clearing in the
// redundant digit form of bls_fq.h.
//
// Every stored value is in L form (carry-save normalised digits); the
// subtraction constant of each step is the smallest multiple of p (64p ..
// 2048p, bls_fq_constants.h) that covers its subtrahend's digits and value,
// and every product's operand values stay far enough below p R (R / p ~ 2^25.3)
// -- the bounds written beside each step are in units of p, for the chain's
// state X < 1030p, Y < 650p, Z < 270p.  The host tests
// (tests/test_hostcheck.py::test_fq_g2_chain) run the whole chain with the
// 128-bit column, value and subtraction checks of bls_fq.h compiled in.
#pragma once
#include "bls_fq.h"
#include "bls_fqb.h"
#include "bls_tower.h"

namespace bls {

// Order the Fq2 products of a chain step one after another on the device: the scheduler interleaved the
// independent products of a doubling / addition and held so many digit columns live that an inlined chain
// spilled ~300 VGPRs (the host build has nothing to order).
#if defined(__HIP_DEVICE_COMPILE__)
#define FQ_SEQ() __builtin_amdgcn_sched_barrier(0)
#else
#define FQ_SEQ() ((void)0)
#endif

template <const uint32_t* K>
BLS_HD Fq fq_subk(const Fq& a, const Fq& b) {
  FQ_CHECK_SUB(b, K);
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = a.d[i] + (K[i] - b.d[i]);
  return r;
}
template <const uint32_t* K>
BLS_HD Fq2 fq2_subk(const Fq2& a, const Fq2& b) {
  return Fq2{fq_subk<K>(a.c0, b.c0), fq_subk<K>(a.c1, b.c1)};
}
BLS_HD Fq2 fq2_add(const Fq2& a, const Fq2& b) { return Fq2{fq_add(a.c0, b.c0), fq_add(a.c1, b.c1)}; }
BLS_HD Fq2 fq2_norm(const Fq2& a) { return Fq2{fq_norm(a.c0), fq_norm(a.c1)}; }
BLS_HD Fq2 fq2_mul_small(const Fq2& a, uint32_t k) { return Fq2{fq_mul_small(a.c0, k), fq_mul_small(a.c1, k)}; }

// -b1 for fq2_mul: K = 4096p in borrowed digits covering any L-form digit (the chain's operands stay below 2312p)
constexpr fqb_detail::KConst Q29_KNEG = fqb_detail::k_for(4096, fqb_detail::MASK + 64);
static_assert(Q29_KNEG.ok && Q29_KNEG.c >= 4096 && Q29_KNEG.c <= 4200, "fq2_mul negation constant");
// PRECONDITION (every call site; checked only by the BLS_FQ_CHECK host build): both operands in L or N form,
// i.e. the output of a product or fq_norm -- digits <= 2^29 + 64 and values < 4096p.  An unnormalised fq_add
// sum (digits up to 2^30) can overflow a 28-product column of fq_mul_dot2 on the device with no error.
// Chains that need compile-time proofs use the bound-typed Fq2B product of bls_fqb.h instead.
// c0 = a0 b0 + a1 (K - b1), c1 = a0 b1 + a1 b0, one reduction each (fq_mul_dot2), operands in L form with
// b1 < 4096p and a0, a1, b0 < 4096p (a0 b0 + a1 (K - b1) < 4096 (4096 + 4200) p^2 < p R): both coefficients in N form (< 2p).  The Karatsuba form
// it replaced ran three products, three reductions, two subtractions and two normalisations.
BLS_HD Fq2 fq2_mul(const Fq2& a, const Fq2& b) {
  FQ_CHECK_SUB(b.c1, Q29_KNEG.d);
  Fq nb;
#pragma unroll
  for (int i = 0; i < 14; i++) nb.d[i] = Q29_KNEG.d[i] - b.c1.d[i];
  return Fq2{fq_mul_dot2(a.c0, b.c0, a.c1, fq_norm(nb)), fq_mul_dot2(a.c0, b.c1, a.c1, b.c0)};
}
// (a0 + a1)(a0 - a1), 2 a0 a1 for a in L form with a1 < 2046p: c0 < 2p, c1 < 4p
BLS_HD Fq2 fq2_sqr(const Fq2& a) {
  const Fq t0 = fq_mul(fq_add(a.c0, a.c1), fq_norm(fq_subk<Q29_K2048_2>(a.c0, a.c1)));
  const Fq t1 = fq_mul(a.c0, a.c1);
  return Fq2{t0, fq_mul_small(t1, 2)};
}
BLS_HD Fq2 fq2_unpack(const Fp2& a) { return Fq2{fq_unpack(a.c0), fq_unpack(a.c1)}; }
BLS_HD Fp2 fq2_pack(const Fq2& a) { return Fp2{fq_pack(a.c0), fq_pack(a.c1)}; }

struct J2Q {
  Fq2 x, y, z;
};

// dbl-2009-l: X < 1030p, Y < 650p, Z < 270p in -> X3 < 1028p, Y3 < 194p, Z3 < 260p
BLS_HD J2Q j2q_dbl(const J2Q& p) {
  const Fq2 A = fq2_sqr(p.x);                                      // (2, 4)
  FQ_SEQ();
  const Fq2 Bq = fq2_sqr(p.y);
  FQ_SEQ();
  const Fq2 C = fq2_sqr(Bq);
  FQ_SEQ();
  const Fq2 XB2 = fq2_sqr(fq2_norm(fq2_add(p.x, Bq)));
  FQ_SEQ();
  const Fq2 D = fq2_mul_small(fq2_subk<Q29_K2>(XB2, fq2_add(A, C)), 2);  // 2 (XB2 - A - C + 128p) < 264p
  const Fq2 E = fq2_mul_small(A, 3);                               // < 12p
  J2Q r;
  r.x = fq2_norm(fq2_subk<Q29_K1024>(fq2_sqr(E), fq2_mul_small(D, 2)));  // F - 2D + 1024p < 1028p
  FQ_SEQ();
  const Fq2 DX = fq2_norm(fq2_subk<Q29_K2048_2>(D, r.x));         // < 2312p
  r.y = fq2_norm(fq2_subk<Q29_K1>(fq2_mul(E, DX), fq2_mul_small(C, 8)));  // < 194p
  FQ_SEQ();
  r.z = fq2_mul_small(fq2_mul(p.y, p.z), 2);                       // < 260p
  FQ_SEQ();
  return r;
}

// add-2007-bl (incomplete): exc |= the exceptional cases (h = 0, an identity operand), checked on canonical values
BLS_HD J2Q j2q_add(const J2Q& p, const J2Q& q, bool& exc) {
  const Fq2 z1z1 = fq2_sqr(p.z);
  FQ_SEQ();
  const Fq2 z2z2 = fq2_sqr(q.z);
  FQ_SEQ();
  const Fq2 u1 = fq2_mul(p.x, z2z2);
  FQ_SEQ();
  const Fq2 u2 = fq2_mul(q.x, z1z1);        // N form (< 2p)
  FQ_SEQ();
  const Fq2 s1 = fq2_mul(fq2_mul(p.y, q.z), z2z2);
  FQ_SEQ();
  const Fq2 s2 = fq2_mul(fq2_mul(q.y, p.z), z1z1);
  FQ_SEQ();
  const Fq2 h = fq2_norm(fq2_subk<Q29_K256>(u2, u1));              // < 386p
  exc = exc || fp2_is_zero(fq2_pack(h)) || fp2_is_zero(fq2_pack(p.z)) || fp2_is_zero(fq2_pack(q.z));
  FQ_SEQ();
  const Fq2 rr = fq2_mul_small(fq2_subk<Q29_K256>(s2, s1), 2);     // < 772p
  const Fq2 i = fq2_sqr(fq2_mul_small(h, 2));
  FQ_SEQ();
  const Fq2 j = fq2_mul(h, i);
  FQ_SEQ();
  const Fq2 v = fq2_mul(u1, i);
  FQ_SEQ();
  J2Q r;
  r.x = fq2_norm(fq2_subk<Q29_K512_2>(fq2_sqr(rr), fq2_add(j, fq2_mul_small(v, 2))));  // < 516p
  FQ_SEQ();
  const Fq2 vx = fq2_norm(fq2_subk<Q29_K1024>(v, r.x));           // < 1154p
  r.y = fq2_norm(fq2_subk<Q29_K512_2>(fq2_mul(rr, vx), fq2_mul_small(fq2_mul(s1, j), 2)));  // < 642p
  FQ_SEQ();
  const Fq2 zz = fq2_norm(fq2_subk<Q29_K2>(fq2_sqr(fq2_norm(fq2_add(p.z, q.z))), fq2_add(z1z1, z2z2)));
  FQ_SEQ();
  r.z = fq2_mul(zz, h);                                              // N form (< 2p)
  FQ_SEQ();
  return r;
}

// [|x|] p with the base point parked in LDS during the chain (lds: 84 words x 64 lanes, [word][lane]): it is read
// only by the 5 additions, and the 84 registers it held pushed an inlined chain past the register file (~300
// spilled VGPRs) -- in registers the chain had to be a separate call with a ~1.8 KB private segment.
__device__ __forceinline__ J2Q j2q_mul_xabs_lds(const J2Q& p, bool& exc, uint32_t* lds) {
  const int lane = threadIdx.x & 63;
  const uint32_t* pw = reinterpret_cast<const uint32_t*>(&p);
#pragma unroll
  for (int w = 0; w < 84; w++) lds[w * 64 + lane] = pw[w];
  J2Q m = p;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    m = j2q_dbl(m);
    if ((X_ABS >> b) & 1ull) {
      J2Q q;
      uint32_t* qw = reinterpret_cast<uint32_t*>(&q);
#pragma unroll
      for (int w = 0; w < 84; w++) qw[w] = lds[w * 64 + lane];
      m = j2q_add(m, q, exc);
    }
  }
  return m;
}

// [|x|] p (the leading bit of |x| is bit 63)
BLS_HD J2Q j2q_mul_xabs(const J2Q& p, bool& exc) {
  J2Q m = p;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    m = j2q_dbl(m);
    if ((X_ABS >> b) & 1ull) m = j2q_add(m, p, exc);
  }
  return m;
}

}  // namespace bls
