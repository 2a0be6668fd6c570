// Complete projective point arithmetic for lane kernels (Renes-Costello-Batina
// for a = 0, the formulas of tools/wavec.py rcb_dbl / rcb_add / rcb_add_aff)
// with one lane per point (pp_*) or a lane pair per point (pp2_*: each
// dependency level split between lanes 2k / 2k+1, products exchanged by one
// DPP swap).  Used by bls_chain_lane.hip and the hash_to_G2 lane kernels of
// bls_fav_kernels.hip.
#pragma once
#include "bls_tower_inline.h"

namespace bls {

// Products of a one-lane chain are issued one after another: letting the
// scheduler interleave the independent Fp2 products of a formula held several
// products' digit columns live at once and pushed the one-lane kernels past
// the 512-register file (measured: 770 spilled VGPRs in the cofactor chain).
#if defined(__HIP_DEVICE_COMPILE__)
#define LANE_SEQ() __builtin_amdgcn_sched_barrier(0)
#else
#define LANE_SEQ() ((void)0)
#endif

// multiplication by 3b: b = 4 on E1, b = 4(1 + i) on E2
BLS_HD Fp ln_b3(const Fp& a) {
  const Fp a4 = fp_dbl(fp_dbl(a));
  return fp_add(fp_dbl(a4), a4);
}
BLS_HD Fp2 ln_b3(const Fp2& t) { return Fp2{ln_b3(fp_sub(t.c0, t.c1)), ln_b3(fp_add(t.c0, t.c1))}; }
BLS_HD Fp ln_mul(const Fp& a, const Fp& b) { return fp_mul_i(a, b); }
BLS_HD Fp2 ln_mul(const Fp2& a, const Fp2& b) { return f2mul(a, b); }
BLS_HD Fp ln_sqr(const Fp& a) { return fp_sqr_i(a); }
BLS_HD Fp2 ln_sqr(const Fp2& a) { return f2sqr(a); }

template <class F>
struct PP {
  F x, y, z;
};

template <class F>
BLS_HD PP<F> pp_dbl(const PP<F>& p) {
  const F t0 = ln_sqr(p.y);
  LANE_SEQ();
  const F t1 = ln_mul(p.y, p.z);
  LANE_SEQ();
  const F t2 = ln_b3(ln_sqr(p.z));
  LANE_SEQ();
  const F u = ln_mul(p.x, p.y);
  LANE_SEQ();
  const F z8 = fdbl(fdbl(fdbl(t0)));
  const F x3a = ln_mul(t2, z8);
  LANE_SEQ();
  PP<F> r;
  r.z = ln_mul(t1, z8);
  LANE_SEQ();
  const F w = fsub(t0, fadd(fdbl(t2), t2));
  r.y = fadd(ln_mul(w, fadd(t0, t2)), x3a);
  LANE_SEQ();
  r.x = fdbl(ln_mul(w, u));
  return r;
}

template <class F>
BLS_HD PP<F> pp_finish(F t0, F t1, const F& t2, const F& t3, const F& t4, F y3) {
  t0 = fadd(fdbl(t0), t0);
  const F z3 = fadd(t1, t2);
  t1 = fsub(t1, t2);
  y3 = ln_b3(y3);
  const F a = ln_mul(t3, t1);
  LANE_SEQ();
  const F b = ln_mul(t4, y3);
  LANE_SEQ();
  const F c = ln_mul(t1, z3);
  LANE_SEQ();
  const F d = ln_mul(y3, t0);
  LANE_SEQ();
  const F e = ln_mul(z3, t4);
  LANE_SEQ();
  const F g = ln_mul(t0, t3);
  PP<F> r;
  r.x = fsub(a, b);
  r.y = fadd(c, d);
  r.z = fadd(e, g);
  return r;
}

template <class F>
BLS_HD PP<F> pp_add(const PP<F>& p, const PP<F>& q) {
  const F t0 = ln_mul(p.x, q.x);
  LANE_SEQ();
  const F t1 = ln_mul(p.y, q.y);
  LANE_SEQ();
  const F t2 = ln_mul(p.z, q.z);
  LANE_SEQ();
  const F t3 = fsub(fsub(ln_mul(fadd(p.x, p.y), fadd(q.x, q.y)), t0), t1);
  LANE_SEQ();
  const F t4 = fsub(fsub(ln_mul(fadd(p.y, p.z), fadd(q.y, q.z)), t1), t2);
  LANE_SEQ();
  const F y3 = fsub(fsub(ln_mul(fadd(p.x, p.z), fadd(q.x, q.z)), t0), t2);
  LANE_SEQ();
  return pp_finish(t0, t1, ln_b3(t2), t3, t4, y3);
}

// p + (x2, y2) with (x2, y2) affine, not the identity
template <class F>
BLS_HD PP<F> pp_add_aff(const PP<F>& p, const F& x2, const F& y2) {
  const F t0 = ln_mul(p.x, x2);
  LANE_SEQ();
  const F t1 = ln_mul(p.y, y2);
  LANE_SEQ();
  const F t3 = fsub(fsub(ln_mul(fadd(x2, y2), fadd(p.x, p.y)), t0), t1);
  LANE_SEQ();
  const F t4 = fadd(ln_mul(y2, p.z), p.y);
  LANE_SEQ();
  const F y3 = fadd(ln_mul(x2, p.z), p.x);
  LANE_SEQ();
  return pp_finish(t0, t1, ln_b3(p.z), t3, t4, y3);
}

// ---------------------------------------------------------------------------
// G2 chains on TWO lanes per item.  Both lanes of a pair hold the running
// point; each dependency level of a complete formula is split between them
// and the products are exchanged by one DPP swap (quad_perm [1,0,3,2]):
//   doubling   level 1  lane 0: y^2, z^2          lane 1: y z, x y
//              level 2  lane 0: t2 z8, w (t0+t2)  lane 1: t1 z8, w u
//   addition   level 1  lane 0: x1x2, y1y2, z1z2  lane 1: the three Karatsuba cross sums
//              level 2  (pp_finish) three of its six products per lane
// 12 instead of 22 FME per doubling and lane (squarings run as products so
// the instruction stream is uniform).  Every value is the canonical residue
// pp_dbl / pp_add / pp_add_aff produce, so the chains are bit-identical.
__device__ __forceinline__ uint32_t cl_swap(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ Fp2 cl_swap2(const Fp2& a) {
  Fp2 r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.l[i] = cl_swap(a.c0.l[i]);
    r.c1.l[i] = cl_swap(a.c1.l[i]);
  }
  return r;
}
__device__ __forceinline__ Fp2 cl_sel(bool c, const Fp2& a, const Fp2& b) {
  return Fp2{fp_select(c, a.c0, b.c0), fp_select(c, a.c1, b.c1)};
}
// (own product, partner's product) -> (lane 0's value, lane 1's value) on both lanes
__device__ __forceinline__ void cl_xchg(bool hi, const Fp2& mine, Fp2& v0, Fp2& v1) {
  const Fp2 o = cl_swap2(mine);
  v0 = cl_sel(hi, o, mine);
  v1 = cl_sel(hi, mine, o);
}

__device__ __forceinline__ PP<Fp2> pp2_dbl(const PP<Fp2>& p, bool hi) {
  Fp2 t0, t1, zz, u;
  cl_xchg(hi, f2mul(p.y, cl_sel(hi, p.z, p.y)), t0, t1);              // y^2 | y z
  cl_xchg(hi, f2mul(cl_sel(hi, p.x, p.z), cl_sel(hi, p.y, p.z)), zz, u);  // z^2 | x y
  const Fp2 t2 = ln_b3(zz);
  const Fp2 z8 = fdbl(fdbl(fdbl(t0)));
  const Fp2 w = fsub(t0, fadd(fdbl(t2), t2));
  Fp2 x3a, z3, ws, wu;
  cl_xchg(hi, f2mul(cl_sel(hi, t1, t2), z8), x3a, z3);               // t2 z8 | t1 z8
  cl_xchg(hi, f2mul(w, cl_sel(hi, u, fadd(t0, t2))), ws, wu);        // w (t0 + t2) | w u
  PP<Fp2> r;
  r.z = z3;
  r.y = fadd(ws, x3a);
  r.x = fdbl(wu);
  return r;
}

// pp_finish with its six products three per lane
__device__ __forceinline__ PP<Fp2> pp2_finish(bool hi, Fp2 t0, Fp2 t1, const Fp2& t2, const Fp2& t3, const Fp2& t4,
                                              Fp2 y3) {
  t0 = fadd(fdbl(t0), t0);
  const Fp2 z3 = fadd(t1, t2);
  t1 = fsub(t1, t2);
  y3 = ln_b3(y3);
  Fp2 a0, a1, b0, b1, c0, c1;
  cl_xchg(hi, f2mul(cl_sel(hi, t4, t3), cl_sel(hi, y3, t1)), a0, a1);  // t3 t1 | t4 y3
  cl_xchg(hi, f2mul(cl_sel(hi, y3, t1), cl_sel(hi, t0, z3)), b0, b1);  // t1 z3 | y3 t0
  cl_xchg(hi, f2mul(cl_sel(hi, t0, z3), cl_sel(hi, t3, t4)), c0, c1);  // z3 t4 | t0 t3
  PP<Fp2> r;
  r.x = fsub(a0, a1);
  r.y = fadd(b0, b1);
  r.z = fadd(c0, c1);
  return r;
}

__device__ __forceinline__ PP<Fp2> pp2_add(const PP<Fp2>& p, const PP<Fp2>& q, bool hi) {
  Fp2 t0, m3, t1, m4, t2, m5;
  cl_xchg(hi, f2mul(cl_sel(hi, fadd(p.x, p.y), p.x), cl_sel(hi, fadd(q.x, q.y), q.x)), t0, m3);
  cl_xchg(hi, f2mul(cl_sel(hi, fadd(p.y, p.z), p.y), cl_sel(hi, fadd(q.y, q.z), q.y)), t1, m4);
  cl_xchg(hi, f2mul(cl_sel(hi, fadd(p.x, p.z), p.z), cl_sel(hi, fadd(q.x, q.z), q.z)), t2, m5);
  const Fp2 t3 = fsub(fsub(m3, t0), t1);
  const Fp2 t4 = fsub(fsub(m4, t1), t2);
  const Fp2 y3 = fsub(fsub(m5, t0), t2);
  return pp2_finish(hi, t0, t1, ln_b3(t2), t3, t4, y3);
}

__device__ __forceinline__ PP<Fp2> pp2_add_aff(const PP<Fp2>& p, const Fp2& x2, const Fp2& y2, bool hi) {
  Fp2 t0, m3, t1, m5;
  cl_xchg(hi, f2mul(cl_sel(hi, fadd(x2, y2), p.x), cl_sel(hi, fadd(p.x, p.y), x2)), t0, m3);
  cl_xchg(hi, f2mul(cl_sel(hi, x2, p.y), cl_sel(hi, p.z, y2)), t1, m5);
  const Fp2 m4 = f2mul(y2, p.z);  // both lanes
  const Fp2 t3 = fsub(fsub(m3, t0), t1);
  const Fp2 t4 = fadd(m4, p.y);
  const Fp2 y3 = fadd(m5, p.x);
  return pp2_finish(hi, t0, t1, ln_b3(p.z), t3, t4, y3);
}

// ---------------------------------------------------------------------------
// Jacobian chains on ONE lane per item (x = X/Z^2, y = Y/Z^3), for scalar
// multiplications by |x| where the complete projective formulas cost more:
// a doubling (dbl-2009-l) is 5 squarings + 2 products in Fp2 = 16 FME per item
// against 22 for pp_dbl on one lane and 2 x 12 on a lane pair (pp2_dbl), and
// it needs fewer live temporaries.  The addition (add-2007-bl) is incomplete:
// it is wrong when the two points are equal, opposite or the identity, so it
// raises `exc` whenever h = U2 - U1 or a Z is zero (the caller routes the item
// to its complete-formula fallback).  No branch depends on the data.
BLS_HD G2J j2_dbl(const G2J& p) {
  const Fp2 A = f2sqr(p.x);
  LANE_SEQ();
  const Fp2 Bq = f2sqr(p.y);
  LANE_SEQ();
  const Fp2 C = f2sqr(Bq);
  LANE_SEQ();
  const Fp2 D = fp2_dbl(fp2_sub(fp2_sub(f2sqr(fp2_add(p.x, Bq)), A), C));
  LANE_SEQ();
  const Fp2 E = fp2_add(fp2_dbl(A), A);
  G2J r;
  r.x = fp2_sub(f2sqr(E), fp2_dbl(D));
  LANE_SEQ();
  r.y = fp2_sub(f2mul(E, fp2_sub(D, r.x)), fp2_dbl(fp2_dbl(fp2_dbl(C))));
  LANE_SEQ();
  r.z = fp2_dbl(f2mul(p.y, p.z));
  return r;
}
BLS_HD G2J j2_add(const G2J& p, const G2J& q, bool& exc) {
  const Fp2 z1z1 = f2sqr(p.z);
  LANE_SEQ();
  const Fp2 z2z2 = f2sqr(q.z);
  LANE_SEQ();
  const Fp2 u1 = f2mul(p.x, z2z2);
  LANE_SEQ();
  const Fp2 u2 = f2mul(q.x, z1z1);
  LANE_SEQ();
  const Fp2 s1 = f2mul(f2mul(p.y, q.z), z2z2);
  LANE_SEQ();
  const Fp2 s2 = f2mul(f2mul(q.y, p.z), z1z1);
  LANE_SEQ();
  const Fp2 h = fp2_sub(u2, u1);
  exc = exc || fp2_is_zero(h) || fp2_is_zero(p.z) || fp2_is_zero(q.z);
  const Fp2 rr = fp2_dbl(fp2_sub(s2, s1));
  const Fp2 i = f2sqr(fp2_dbl(h));
  LANE_SEQ();
  const Fp2 j = f2mul(h, i);
  LANE_SEQ();
  const Fp2 v = f2mul(u1, i);
  LANE_SEQ();
  G2J r;
  r.x = fp2_sub(fp2_sub(f2sqr(rr), j), fp2_dbl(v));
  LANE_SEQ();
  r.y = fp2_sub(f2mul(rr, fp2_sub(v, r.x)), fp2_dbl(f2mul(s1, j)));
  LANE_SEQ();
  r.z = f2mul(fp2_sub(fp2_sub(f2sqr(fp2_add(p.z, q.z)), z1z1), z2z2), h);
  return r;
}
// p + affine (x2, y2) (madd-2007-bl), same exception rule (p.z = 0 or h = 0)
BLS_HD G2J j2_add_aff(const G2J& p, const Fp2& x2, const Fp2& y2, bool& exc) {
  const Fp2 z1z1 = f2sqr(p.z);
  LANE_SEQ();
  const Fp2 u2 = f2mul(x2, z1z1);
  LANE_SEQ();
  const Fp2 s2 = f2mul(f2mul(y2, p.z), z1z1);
  LANE_SEQ();
  const Fp2 h = fp2_sub(u2, p.x);
  exc = exc || fp2_is_zero(h) || fp2_is_zero(p.z);
  const Fp2 hh = f2sqr(h);
  LANE_SEQ();
  const Fp2 i = fp2_dbl(fp2_dbl(hh));
  const Fp2 j = f2mul(h, i);
  LANE_SEQ();
  const Fp2 rr = fp2_dbl(fp2_sub(s2, p.y));
  const Fp2 v = f2mul(p.x, i);
  LANE_SEQ();
  G2J r;
  r.x = fp2_sub(fp2_sub(f2sqr(rr), j), fp2_dbl(v));
  LANE_SEQ();
  r.y = fp2_sub(f2mul(rr, fp2_sub(v, r.x)), fp2_dbl(f2mul(p.y, j)));
  LANE_SEQ();
  r.z = fp2_sub(fp2_sub(f2sqr(fp2_add(p.z, h)), z1z1), hh);
  return r;
}
// homogeneous projective (X : Y : Z) <-> Jacobian: (X Z, Y Z^2, Z) and (X Z, Y, Z^3)
BLS_HD G2J j2_from_pp(const PP<Fp2>& p) {
  const Fp2 zz = f2sqr(p.z);
  return G2J{f2mul(p.x, p.z), f2mul(p.y, zz), p.z};
}
BLS_HD PP<Fp2> j2_to_pp(const G2J& p) { return PP<Fp2>{f2mul(p.x, p.z), p.y, f2mul(f2sqr(p.z), p.z)}; }
// [|x|] p (the leading bit of |x| is bit 63)
BLS_HD G2J j2_mul_xabs(const G2J& p, bool& exc) {
  G2J m = p;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    m = j2_dbl(m);
    if ((X_ABS >> b) & 1ull) m = j2_add(m, p, exc);
  }
  return m;
}

}  // namespace bls
