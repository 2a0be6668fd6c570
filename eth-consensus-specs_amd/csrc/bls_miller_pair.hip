// f accumulation of the split Miller loop (the G2 side, k_miller_lines2 in
// bls_miller_lane.hip, writes the line records) with four lanes per f.
#include "bls_kernels.h"
#include "bls_tower_inline.h"

namespace bls {

namespace {

constexpr int ML_WORDS2 = 72;  // line record: three Fp2 (l0, E*ZZ or r, z3*ZZ or z3), as k_miller_lines2 writes

__device__ __forceinline__ Fp sel_fp(bool c, const Fp& a, const Fp& b) { return fp_select(c, a, b); }
__device__ __forceinline__ Fp2 sel_fp2(bool c, const Fp2& a, const Fp2& b) {
  return Fp2{sel_fp(c, a.c0, b.c0), sel_fp(c, a.c1, b.c1)};
}
__device__ __forceinline__ Fp6 sel_fp6(bool c, const Fp6& a, const Fp6& b) {
  return Fp6{sel_fp2(c, a.c0, b.c0), sel_fp2(c, a.c1, b.c1), sel_fp2(c, a.c2, b.c2)};
}

__device__ __forceinline__ Fp2 ml_load2(const uint32_t* L, size_t n, int w0) {
  Fp2 a;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    a.c0.l[j] = L[(size_t)(w0 + j) * n];
    a.c1.l[j] = L[(size_t)(w0 + 12 + j) * n];
  }
  return a;
}

// The Fp2 products of each Fp6 product run one after another (sched_barrier):
// each lazy Fp2 product already has three independent mad chains; letting the
// scheduler interleave six of them held ~6 x 140 registers live and spilled
// (measured 5.0 ms per 10,000 pairs against 5.7 ms interleaved).
#define SEQ() __builtin_amdgcn_sched_barrier(0)

__device__ __forceinline__ Fp6 f6add_raw(const Fp6& a, const Fp6& b) {
  return Fp6{f2add_raw(a.c0, b.c0), f2add_raw(a.c1, b.c1), f2add_raw(a.c2, b.c2)};
}

}  // namespace

// ---------------------------------------------------------------------------
// f accumulation with FOUR lanes per f, shared by G pairs.
//
// Lane 4k + 2h + q: h selects the half of f it owns (h = 0: a = f.c0, h = 1:
// b = f.c1, f = a + b w with w^2 = v; the two q lanes of one h hold the same half),
// q selects which Fp2 products of each Fp6 product it forms:
//   full Fp6 product   q = 0: t_k = X_k Y_k;  q = 1: the three Karatsuba cross
//                      products -- three Fp2 products per lane instead of six
//   line product       q = 0: a_0 l0, a_1 l2, a_2 l2, a_2 l0;  q = 1:
//                      (a_0 + a_1)(l0 + l2), o_2 l3, o_0 l3, o_1 l3  (o: the
//                      other half) -- four instead of eight
//   line P factors     lane (h, q) forms component q of its Fp2 x Fp product
// followed by one DPP exchange (quad_perm [1,0,3,2] between q lanes, [2,3,0,1]
// between h lanes); both q lanes then hold the same combined result, so the
// instruction stream is uniform and every lane-dependent choice is a select.
// With G = 2 the pairs (2k, 2k+1) share one f: one squaring per step for two
// Miller loops (f^2 l_A l_B), the multi-pairing form of SURVEY.md §8(d)'s
// shared-squaring model.  The output is one Fp12 per group; the batch product
// over groups equals the product over pairs, so the verdict and every
// downstream value are unchanged.
namespace {

__device__ __forceinline__ uint32_t dpp_q(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ uint32_t dpp_h(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
}
__device__ __forceinline__ Fp q_fp(const Fp& a) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = dpp_q(a.l[i]);
  return r;
}
__device__ __forceinline__ Fp h_fp(const Fp& a) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = dpp_h(a.l[i]);
  return r;
}
__device__ __forceinline__ Fp2 q_fp2(const Fp2& a) { return Fp2{q_fp(a.c0), q_fp(a.c1)}; }
__device__ __forceinline__ Fp2 h_fp2(const Fp2& a) { return Fp2{h_fp(a.c0), h_fp(a.c1)}; }
__device__ __forceinline__ Fp6 h_fp6(const Fp6& a) { return Fp6{h_fp2(a.c0), h_fp2(a.c1), h_fp2(a.c2)}; }

// X * Y in Fp6, three of its six Fp2 products on each q lane
__device__ __forceinline__ Fp6 q6mul(const Fp6& X, const Fp6& Y, bool q) {
  const Fp2 p0 = f2mul(sel_fp2(q, f2add_raw(X.c1, X.c2), X.c0), sel_fp2(q, f2add_raw(Y.c1, Y.c2), Y.c0));
  SEQ();
  const Fp2 p1 = f2mul(sel_fp2(q, f2add_raw(X.c0, X.c1), X.c1), sel_fp2(q, f2add_raw(Y.c0, Y.c1), Y.c1));
  SEQ();
  const Fp2 p2 = f2mul(sel_fp2(q, f2add_raw(X.c0, X.c2), X.c2), sel_fp2(q, f2add_raw(Y.c0, Y.c2), Y.c2));
  SEQ();
  const Fp2 o0 = q_fp2(p0), o1 = q_fp2(p1), o2 = q_fp2(p2);
  const Fp2 t0 = sel_fp2(q, o0, p0), t1 = sel_fp2(q, o1, p1), t2 = sel_fp2(q, o2, p2);
  const Fp2 u0 = sel_fp2(q, p0, o0), u1 = sel_fp2(q, p1, o1), u2 = sel_fp2(q, p2, o2);
  const Fp2 c0 = f2add(f2xi(f2sub(f2sub(u0, t1), t2)), t0);
  const Fp2 c1 = f2add(f2sub(f2sub(u1, t0), t1), f2xi(t2));
  const Fp2 c2 = f2add(f2sub(f2sub(u2, t0), t2), t1);
  return Fp6{c0, c1, c2};
}

// one Fp12 squaring (a + b w)^2 = (a^2 + v b^2) + 2ab w: h = 0 forms u = (a + b)(a + v b), h = 1 forms
// t = a b; then a' = u - t - v t, b' = 2 t
__device__ __forceinline__ Fp6 q_sqr(const Fp6& own, bool h, bool q) {
  const Fp6 oth = h_fp6(own);
  const Fp6 A = sel_fp6(h, oth, own), Bv = sel_fp6(h, own, oth);
  const Fp6 X = sel_fp6(h, A, f6add_raw(A, Bv));
  const Fp6 Y = sel_fp6(h, Bv, f6add_raw(A, f6v(Bv)));
  const Fp6 P = q6mul(X, Y, q);
  const Fp6 t = h_fp6(P);
  return sel_fp6(h, f6add(P, P), f6sub(f6sub(P, t), f6v(t)));
}

// own *= line: h = 0: a' = a (l0, l2) + v (b l3 v);  h = 1: b' = b (l0, l2) + a (l3 v)
__device__ __forceinline__ Fp6 q_line(const Fp6& own, bool h, bool q, const Fp2& l0, const Fp2& l2, const Fp2& l3) {
  const Fp6 oth = h_fp6(own);
  const Fp2 p1 = f2mul(sel_fp2(q, f2add_raw(own.c0, own.c1), own.c0), sel_fp2(q, f2add_raw(l0, l2), l0));
  SEQ();
  const Fp2 p2 = f2mul(sel_fp2(q, oth.c2, own.c1), sel_fp2(q, l3, l2));
  SEQ();
  const Fp2 p3 = f2mul(sel_fp2(q, oth.c0, own.c2), sel_fp2(q, l3, l2));
  SEQ();
  const Fp2 p4 = f2mul(sel_fp2(q, oth.c1, own.c2), sel_fp2(q, l3, l0));
  SEQ();
  const Fp2 o1 = q_fp2(p1), o2 = q_fp2(p2), o3 = q_fp2(p3), o4 = q_fp2(p4);
  // q = 0 products: t0 = a_0 l0, t1 = a_1 l2, u0 = a_2 l2, u2 = a_2 l0
  const Fp2 t0 = sel_fp2(q, o1, p1), t1 = sel_fp2(q, o2, p2), u0 = sel_fp2(q, o3, p3), u2 = sel_fp2(q, o4, p4);
  // q = 1 products: u1 = (a_0 + a_1)(l0 + l2), v_k = o_{k-1} l3
  const Fp2 u1 = sel_fp2(q, p1, o1), v0 = sel_fp2(q, p2, o2), v1 = sel_fp2(q, p3, o3), v2 = sel_fp2(q, p4, o4);
  const Fp6 m01{f2add(t0, f2xi(u0)), f2sub(f2sub(u1, t0), t1), f2add(t1, u2)};
  const Fp6 m1{f2xi(v0), v1, v2};
  return f6add(m01, sel_fp6(h, m1, f6v(m1)));
}

// line record of pair p at its step pointer Li: (l0, E*ZZ or r, z3*ZZ or z3); lane (h, q) forms
// component q of (h ? z3*ZZ * y_P : E*ZZ * (-x_P)), then two exchanges give l2, l3 on every lane
__device__ __forceinline__ void q_line_p(const uint32_t* Li, size_t n, bool h, bool q, const Fp& nxP, const Fp& yP,
                                         Fp2& l2, Fp2& l3) {
  Fp c;
  const int w0 = (h ? 48 : 24) + (q ? 12 : 0);
#pragma unroll
  for (int j = 0; j < 12; ++j) c.l[j] = Li[(size_t)(w0 + j) * n];
  const Fp mine = fp_mul_i(c, h ? yP : nxP);
  const Fp part = q_fp(mine);
  const Fp2 m{sel_fp(q, part, mine), sel_fp(q, mine, part)};
  const Fp2 o = h_fp2(m);
  l2 = sel_fp2(h, o, m);
  l3 = sel_fp2(h, m, o);
}

}  // namespace

template <int G>
__global__ void __launch_bounds__(64) k_miller_acc4(const G1A* P, const G2A* Q, const int* ok, size_t n,
                                                    const uint32_t* L, Fp12* out) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t grp = t >> 2;
  const bool h = (t & 2) != 0, q = (t & 1) != 0;
  const size_t ngrp = (n + G - 1) / G;
  if (grp >= ngrp) return;  // the four lanes of a group leave together
  bool live[G];
  size_t pi[G];
  bool any = false;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const size_t p = grp * G + g;
    pi[g] = p < n ? p : n - 1;  // clamped: loads stay inside the batch's line buffer
    live[g] = p < n && (!ok || ok[p]) && !P[p].inf && !Q[p].inf;
    any = any || live[g];
  }
  if (!any) {
    if (!q) {
      Fp6* o = h ? &out[grp].c1 : &out[grp].c0;
      *o = h ? Fp6{fp2_zero(), fp2_zero(), fp2_zero()} : Fp6{fp2_one(), fp2_zero(), fp2_zero()};
    }
    return;
  }
  const size_t step = (size_t)ML_WORDS2 * n;
  const uint32_t* Li[G];
#pragma unroll
  for (int g = 0; g < G; ++g) Li[g] = L + pi[g];
  Fp6 f{h ? fp2_zero() : fp2_one(), fp2_zero(), fp2_zero()};
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = q_sqr(f, h, q);
    const int nl = ((X_ABS >> b) & 1ull) ? 2 : 1;
#pragma unroll 1
    for (int s = 0; s < nl; ++s) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        // P coordinates re-read per step (cached; keeps them out of the live registers)
        const G1A* pp = P + pi[g];
        const Fp nxP = fp_neg(pp->x), yP = pp->y;
        Fp2 l2, l3;
        q_line_p(Li[g], n, h, q, nxP, yP, l2, l3);
        const Fp6 fl = q_line(f, h, q, ml_load2(Li[g], n, 0), l2, l3);
        f = G == 1 ? fl : sel_fp6(live[g], fl, f);
        Li[g] += step;
      }
    }
  }
  if (!q) {
    if (h)
      out[grp].c1 = Fp6{fp2_neg(f.c0), fp2_neg(f.c1), fp2_neg(f.c2)};
    else
      out[grp].c0 = f;
  }
}

hipError_t launch_miller_acc4(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, const uint32_t* L,
                              Fp12* f, int G) {
  if (!n) return hipSuccess;
  const size_t ngrp = (n + G - 1) / G;
  const dim3 grid((unsigned)((4 * ngrp + 63) / 64));
  if (G == 2)
    hipLaunchKernelGGL(k_miller_acc4<2>, grid, dim3(64), 0, st, P, Q, ok, n, L, f);
  else
    hipLaunchKernelGGL(k_miller_acc4<1>, grid, dim3(64), 0, st, P, Q, ok, n, L, f);
  return hipGetLastError();
}

}  // namespace bls
