// f accumulation of the split Miller loop with TWO lanes per pair.
//
// k_miller_acc (bls_miller_lane.hip) runs a whole pair on one lane: f (144
// words), one line (72) and the Fp6 temporaries of the Fp12 squaring exceed
// the 512-entry register file, so it spills ~1.4 KB per lane and a 10,000-pair
// launch is only 157 waves (15 % of the SIMDs).  Here lane 2k+0 owns
// f.c0 = a and lane 2k+1 owns f.c1 = b (f = a + b w, w^2 = v); the partner's
// half arrives by one DPP lane swap (quad_perm [1,0,3,2]) per use:
//   squaring   (a + b w)^2 = (a^2 + v b^2) + 2ab w
//              lane 0: u = (a + b)(a + v b),   lane 1: t = a b    (one Fp6 product each)
//              then lane 0 takes t from lane 1:  a' = u - t - v t,   b' = 2 t
//   line       l = (l0 + l2 v) + (l3 v) w  (l2, l3 already times -x_P, y_P)
//              lane 0: a' = a (l0, l2) + v (b l3 v),  lane 1: b' = b (l0, l2) + a (l3 v)
//              (five + three Fp2 products per lane instead of 13 on one lane; the
//              line's P factors: one Fp2 x Fp product per lane, then a swap)
// The Fp2 products of each Fp6 product run one after another (sched_barrier):
// measured 5.0 ms per 10,000 pairs against 5.7 ms when the scheduler
// interleaves them, and sums that only feed products stay unreduced.
// Both lanes run the same instruction stream: every lane-dependent choice is a
// select, never a branch.  Each lane keeps ~half the state, so nothing
// spills, and a launch is twice the waves.  The values are the same field
// elements as k_miller_acc's (canonical residues), so the Miller outputs are
// bit-identical.
#include "bls_kernels.h"
#include "bls_tower_inline.h"

namespace bls {

namespace {

constexpr int ML_WORDS2 = 72;  // line record: three Fp2 (l0, E*ZZ or r, z3*ZZ or z3), as k_miller_lines writes

__device__ __forceinline__ uint32_t swap_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ Fp swap_fp(const Fp& a) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = swap_lane(a.l[i]);
  return r;
}
__device__ __forceinline__ Fp2 swap_fp2(const Fp2& a) { return Fp2{swap_fp(a.c0), swap_fp(a.c1)}; }
__device__ __forceinline__ Fp6 swap_fp6(const Fp6& a) { return Fp6{swap_fp2(a.c0), swap_fp2(a.c1), swap_fp2(a.c2)}; }

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

// Fp6 products of the pair kernel: the Fp2 products one after another
// (sched_barrier between them).  Each lazy Fp2 product already has three
// independent mad chains; letting the scheduler interleave six of them held
// ~6 x 140 registers live and spilled.
#if !defined(PAIR_SEQ) || PAIR_SEQ
#define SEQ() __builtin_amdgcn_sched_barrier(0)
#else
#define SEQ() ((void)0)
#endif

__device__ __forceinline__ Fp6 p6mul(const Fp6& a, const Fp6& b) {
  const Fp2 t0 = f2mul(a.c0, b.c0);
  SEQ();
  const Fp2 t1 = f2mul(a.c1, b.c1);
  SEQ();
  const Fp2 t2 = f2mul(a.c2, b.c2);
  SEQ();
  const Fp2 u0 = f2mul(f2add_raw(a.c1, a.c2), f2add_raw(b.c1, b.c2));
  SEQ();
  const Fp2 u1 = f2mul(f2add_raw(a.c0, a.c1), f2add_raw(b.c0, b.c1));
  SEQ();
  const Fp2 u2 = f2mul(f2add_raw(a.c0, a.c2), f2add_raw(b.c0, b.c2));
  SEQ();
  const Fp2 c0 = f2add(f2xi(f2sub(f2sub(u0, t1), t2)), t0);
  const Fp2 c1 = f2add(f2sub(f2sub(u1, t0), t1), f2xi(t2));
  const Fp2 c2 = f2add(f2sub(f2sub(u2, t0), t2), t1);
  return Fp6{c0, c1, c2};
}
__device__ __forceinline__ Fp6 p6mul01(const Fp6& a, const Fp2& b0, const Fp2& b1) {
  const Fp2 t0 = f2mul(a.c0, b0);
  SEQ();
  const Fp2 t1 = f2mul(a.c1, b1);
  SEQ();
  const Fp2 u0 = f2mul(a.c2, b1);
  SEQ();
  const Fp2 u1 = f2mul(f2add_raw(a.c0, a.c1), f2add_raw(b0, b1));
  SEQ();
  const Fp2 u2 = f2mul(a.c2, b0);
  SEQ();
  return Fp6{f2add(t0, f2xi(u0)), f2sub(f2sub(u1, t0), t1), f2add(t1, u2)};
}
__device__ __forceinline__ Fp6 p6mul1(const Fp6& a, const Fp2& b1) {
  const Fp2 u0 = f2mul(a.c2, b1);
  SEQ();
  const Fp2 u1 = f2mul(a.c0, b1);
  SEQ();
  const Fp2 u2 = f2mul(a.c1, b1);
  SEQ();
  return Fp6{f2xi(u0), u1, u2};
}

__device__ __forceinline__ Fp6 f6add_raw(const Fp6& a, const Fp6& b) {
  return Fp6{f2add_raw(a.c0, b.c0), f2add_raw(a.c1, b.c1), f2add_raw(a.c2, b.c2)};
}

// one Fp12 squaring of the lane pair's f; `own` is this lane's half
__device__ __forceinline__ Fp6 pair_sqr(const Fp6& own, bool hi) {
  const Fp6 oth = swap_fp6(own);
  const Fp6 A = sel_fp6(hi, oth, own), Bv = sel_fp6(hi, own, oth);  // (a, b) on both lanes
  // lane 0: (a + b)(a + v b);  lane 1: a b
  const Fp6 X = sel_fp6(hi, A, f6add_raw(A, Bv));  // product operands: sums left unreduced
  const Fp6 Y = sel_fp6(hi, Bv, f6add_raw(A, f6v(Bv)));
  const Fp6 P = p6mul(X, Y);
  const Fp6 t = swap_fp6(P);  // lane 0 receives t = a b
  // lane 0: u - t - v t;  lane 1: 2 t (its own P)
  return sel_fp6(hi, f6add(P, P), f6sub(f6sub(P, t), f6v(t)));
}

// f *= (l0 + l2 v) + (l3 v) w
__device__ __forceinline__ Fp6 pair_line(const Fp6& own, bool hi, const Fp2& l0, const Fp2& l2, const Fp2& l3) {
  const Fp6 oth = swap_fp6(own);
  const Fp6 m01 = p6mul01(own, l0, l2);  // a (l0, l2) on lane 0, b (l0, l2) on lane 1
  const Fp6 m1 = p6mul1(oth, l3);        // b (l3 v) on lane 0, a (l3 v) on lane 1
  return f6add(m01, sel_fp6(hi, m1, f6v(m1)));
}

// the P factors of a line record: lane 0 forms E*ZZ * (-x_P), lane 1 z3*ZZ * y_P, then they swap
__device__ __forceinline__ void pair_line_p(const uint32_t* Li, size_t n, bool hi, const Fp& nxP, const Fp& yP,
                                            Fp2& l2, Fp2& l3) {
  const Fp2 mine = f2mulfp(ml_load2(Li, n, hi ? 48 : 24), hi ? yP : nxP);
  const Fp2 other = swap_fp2(mine);
  l2 = sel_fp2(hi, other, mine);
  l3 = sel_fp2(hi, mine, other);
}

}  // namespace

__global__ void __launch_bounds__(64) k_miller_acc2(const G1A* P, const G2A* Q, const int* ok, size_t n,
                                                    const uint32_t* L, Fp12* out) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = t >> 1;
  const bool hi = (t & 1) != 0;
  if (i >= n) return;  // both lanes of a pair leave together
  const G1A p = P[i];
  if ((ok && !ok[i]) || p.inf || Q[i].inf) {
    Fp6* o = hi ? &out[i].c1 : &out[i].c0;
    *o = hi ? Fp6{fp2_zero(), fp2_zero(), fp2_zero()} : Fp6{fp2_one(), fp2_zero(), fp2_zero()};
    return;
  }
  const Fp nxP = fp_neg(p.x);
  const Fp yP = p.y;
  const uint32_t* Li = L + i;
  const size_t step = (size_t)ML_WORDS2 * n;
  // f = 1: lane 0 holds 1, lane 1 holds 0
  Fp6 f{hi ? fp2_zero() : fp2_one(), fp2_zero(), fp2_zero()};
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = pair_sqr(f, hi);
#if !defined(PAIR_PSPLIT) || PAIR_PSPLIT
    Fp2 l2, l3;
    pair_line_p(Li, n, hi, nxP, yP, l2, l3);
    f = pair_line(f, hi, ml_load2(Li, n, 0), l2, l3);
    Li += step;
    if ((X_ABS >> b) & 1ull) {
      pair_line_p(Li, n, hi, nxP, yP, l2, l3);
      f = pair_line(f, hi, ml_load2(Li, n, 0), l2, l3);
      Li += step;
    }
#else
    f = pair_line(f, hi, ml_load2(Li, n, 0), f2mulfp(ml_load2(Li, n, 24), nxP), f2mulfp(ml_load2(Li, n, 48), yP));
    Li += step;
    if ((X_ABS >> b) & 1ull) {
      f = pair_line(f, hi, ml_load2(Li, n, 0), f2mulfp(ml_load2(Li, n, 24), nxP), f2mulfp(ml_load2(Li, n, 48), yP));
      Li += step;
    }
#endif
  }
  // out = conj(f) = a - b w
  if (hi)
    out[i].c1 = Fp6{fp2_neg(f.c0), fp2_neg(f.c1), fp2_neg(f.c2)};
  else
    out[i].c0 = f;
}

hipError_t launch_miller_acc2(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, const uint32_t* L,
                              Fp12* f) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_miller_acc2, dim3((unsigned)((2 * n + 63) / 64)), dim3(64), 0, st, P, Q, ok, n, L, f);
  return hipGetLastError();
}

}  // namespace bls
