// The Jacobian [|x|] chain of the cofactor clearing (bls_fq_g2.h j2q_*) on a
// LANE PAIR per item in the F2 layout: lanes 2k / 2k+1 (hi = lane & 1) hold
// coefficient c_hi of every Fp2 value of the chain, in the same redundant digit
// form.  A product first swaps the operands' other coefficients in from the
// partner lane (one DPP quad_perm [1,0,3,2] per digit, bls_pp_lane.h cl_swap),
// then each lane forms its own coefficient with exactly the expression the
// one-lane code uses for it:
//   a b:  c0 = dot2(a0, b0, a1, K - b1)      c1 = dot2(a0, b1, a1, b0)
//   a^2:  c0 = (a0 + a1)(a0 - a1)            c1 = 2 a0 a1
// so every value -- and every bound the host tests prove for j2q_dbl /
// j2q_add -- is the one-lane chain's, bit for bit.  Linear steps act on each
// coefficient alone (no exchange).  A doubling is 16 FME on one lane and 8
// per lane here: the chain's latency halves for the same total products plus
// 14 DPP moves per operand exchange, and a lane holds half the point.
#pragma once
#include "bls_fq_g2.h"
#include "bls_pp_lane.h"

namespace bls {

__device__ __forceinline__ Fq fq_swap(const Fq& a) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = cl_swap(a.d[i]);
  return r;
}

// this lane's coefficient of a b (fq2_mul)
__device__ __forceinline__ Fq q2p_mul(const Fq& a, const Fq& b, bool hi) {
  const Fq ao = fq_swap(a), bo = fq_swap(b);
  Fq nb;
#pragma unroll
  for (int i = 0; i < 14; i++) nb.d[i] = Q29_KNEG.d[i] - bo.d[i];  // lane 0: K - b1 (lane 1 discards it)
  return fq_mul_dot2(fq_select(hi, ao, a), b, fq_select(hi, a, ao), fq_select(hi, bo, fq_norm(nb)));
}
// this lane's coefficient of a^2 (fq2_sqr)
__device__ __forceinline__ Fq q2p_sqr(const Fq& a, bool hi) {
  const Fq ao = fq_swap(a);
  const Fq t = fq_mul(fq_select(hi, ao, fq_add(a, ao)), fq_select(hi, a, fq_norm(fq_subk<Q29_K2048_2>(a, ao))));
  return fq_select(hi, fq_mul_small(t, 2), t);
}
// an Fp2 is zero iff both lanes' coefficients are
__device__ __forceinline__ bool q2p_is_zero(const Fq& a) {
  const uint32_t z = fp_is_zero(fq_pack(a)) ? 1u : 0u;
  return (z & cl_swap(z)) != 0;
}

struct J2P {
  Fq x, y, z;  // this lane's coefficients
};

// j2q_dbl, coefficient-wise (the bounds of j2q_dbl: X < 1030p, Y < 650p, Z < 270p in -> X3 < 1028p, Y3 < 194p,
// Z3 < 260p)
__device__ __forceinline__ J2P j2p_dbl(const J2P& p, bool hi) {
  const Fq A = q2p_sqr(p.x, hi);
  FQ_SEQ();
  const Fq Bq = q2p_sqr(p.y, hi);
  FQ_SEQ();
  const Fq C = q2p_sqr(Bq, hi);
  FQ_SEQ();
  const Fq XB2 = q2p_sqr(fq_norm(fq_add(p.x, Bq)), hi);
  FQ_SEQ();
  const Fq D = fq_mul_small(fq_subk<Q29_K2>(XB2, fq_add(A, C)), 2);
  const Fq E = fq_mul_small(A, 3);
  J2P r;
  r.x = fq_norm(fq_subk<Q29_K1024>(q2p_sqr(E, hi), fq_mul_small(D, 2)));
  FQ_SEQ();
  const Fq DX = fq_norm(fq_subk<Q29_K2048_2>(D, r.x));
  r.y = fq_norm(fq_subk<Q29_K1>(q2p_mul(E, DX, hi), fq_mul_small(C, 8)));
  FQ_SEQ();
  r.z = fq_mul_small(q2p_mul(p.y, p.z, hi), 2);
  FQ_SEQ();
  return r;
}

// j2q_add, coefficient-wise; exc |= the exceptional cases (h = 0, an identity operand) of the whole Fp2 values
__device__ __forceinline__ J2P j2p_add(const J2P& p, const J2P& q, bool& exc, bool hi) {
  const Fq z1z1 = q2p_sqr(p.z, hi);
  FQ_SEQ();
  const Fq z2z2 = q2p_sqr(q.z, hi);
  FQ_SEQ();
  const Fq u1 = q2p_mul(p.x, z2z2, hi);
  FQ_SEQ();
  const Fq u2 = q2p_mul(q.x, z1z1, hi);
  FQ_SEQ();
  const Fq s1 = q2p_mul(q2p_mul(p.y, q.z, hi), z2z2, hi);
  FQ_SEQ();
  const Fq s2 = q2p_mul(q2p_mul(q.y, p.z, hi), z1z1, hi);
  FQ_SEQ();
  const Fq h = fq_norm(fq_subk<Q29_K256>(u2, u1));
  exc = exc || q2p_is_zero(h) || q2p_is_zero(p.z) || q2p_is_zero(q.z);
  FQ_SEQ();
  const Fq rr = fq_mul_small(fq_subk<Q29_K256>(s2, s1), 2);
  const Fq i = q2p_sqr(fq_mul_small(h, 2), hi);
  FQ_SEQ();
  const Fq j = q2p_mul(h, i, hi);
  FQ_SEQ();
  const Fq v = q2p_mul(u1, i, hi);
  FQ_SEQ();
  J2P r;
  r.x = fq_norm(fq_subk<Q29_K512_2>(q2p_sqr(rr, hi), fq_add(j, fq_mul_small(v, 2))));
  FQ_SEQ();
  const Fq vx = fq_norm(fq_subk<Q29_K1024>(v, r.x));
  r.y = fq_norm(fq_subk<Q29_K512_2>(q2p_mul(rr, vx, hi), fq_mul_small(q2p_mul(s1, j, hi), 2)));
  FQ_SEQ();
  const Fq zz = fq_norm(fq_subk<Q29_K2>(q2p_sqr(fq_norm(fq_add(p.z, q.z)), hi), fq_add(z1z1, z2z2)));
  FQ_SEQ();
  r.z = q2p_mul(zz, h, hi);
  FQ_SEQ();
  return r;
}

// [|x|] p, the base point parked in LDS (42 words x 64 lanes, [word][lane]) while the chain runs
__device__ __forceinline__ J2P j2p_mul_xabs_lds(const J2P& p, bool& exc, uint32_t* lds, bool hi) {
  const int lane = threadIdx.x & 63;
  const uint32_t* pw = reinterpret_cast<const uint32_t*>(&p);
#pragma unroll
  for (int w = 0; w < 42; w++) lds[w * 64 + lane] = pw[w];
  J2P m = p;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    m = j2p_dbl(m, hi);
    if ((X_ABS >> b) & 1ull) {
      J2P q;
      uint32_t* qw = reinterpret_cast<uint32_t*>(&q);
#pragma unroll
      for (int w = 0; w < 42; w++) qw[w] = lds[w * 64 + lane];
      m = j2p_add(m, q, exc, hi);
    }
  }
  return m;
}

// this lane's coefficient of a packed Fp2, and the packed Fp2 from both lanes' canonical coefficients
__device__ __forceinline__ Fq q2p_own(const Fp2& a, bool hi) { return fq_unpack(fp_select(hi, a.c1, a.c0)); }
__device__ __forceinline__ Fp2 q2p_join(const Fq& a, bool hi) {
  const Fp mine = fq_pack(a);
  Fp other;
#pragma unroll
  for (int i = 0; i < 12; i++) other.l[i] = cl_swap(mine.l[i]);
  return Fp2{fp_select(hi, other, mine), fp_select(hi, mine, other)};
}

}  // namespace bls
