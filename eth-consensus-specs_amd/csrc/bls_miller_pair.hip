// f accumulation of the split Miller loop (the G2 side, k_miller_lines2 in
// bls_miller_lane.hip, writes the line records) with four lanes per f, in the
// bound-typed redundant digit form (bls_fqb.h).
#include <type_traits>

#include "bls_fqb.h"
#include "bls_kernels.h"
#include "bls_miller_lines.h"
#include "bls_tower_inline.h"

namespace bls {

namespace {

// loop-carried bound of the digit-form f halves: value < ML_QF_V p, digits <= ML_QF_D (every step's output is
// relaxed to it at compile time: qq_sqr ends below 211 p, qq_line below ML_QF_V p)
constexpr uint64_t ML_QF_V = 256, ML_QF_D = 0x20000000ull + 64;

// The Fp2 products of each Fp6 product run one after another (sched_barrier): letting the scheduler
// interleave them held too many products live and spilled (the packed-form kernel measured 5.0 ms per
// 10,000 pairs sequenced against 5.7 ms interleaved).
#define SEQ() __builtin_amdgcn_sched_barrier(0)

__device__ __forceinline__ uint32_t dpp_q(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ uint32_t dpp_h(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
}
// quad broadcasts (lane 4k + 2h + q): the value of the q = 0 / q = 1 lane of the same h, of the h = 0 / h = 1 lane
// of the same q -- one DPP move where an exchange plus a lane select took three instructions
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_b(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
constexpr int BQ0 = 0xA0, BQ1 = 0xF5, BH0 = 0x44, BH1 = 0xEE;  // quad_perm [0,0,2,2] [1,1,3,3] [0,1,0,1] [2,3,2,3]

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
//
// f's halves stay in 14 redundant radix-2^29 digits for the whole loop:
// additions and subtractions are digit-wise (no carry chains, no conditional
// subtractions) and no product unpacks or repacks its operands (the packed
// 12-limb kernel this replaces: 4.39 -> 3.68 ms per 10,000 pairs).  Every
// digit and value bound is checked at compile time (bls_fqb.h).
namespace {

template <uint64_t V, uint64_t D>
__device__ __forceinline__ FqB<V, D> dq(const FqB<V, D>& a) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = dpp_q(a.x.d[i]);
  return {r};
}
template <uint64_t V, uint64_t D>
__device__ __forceinline__ FqB<V, D> dh(const FqB<V, D>& a) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = dpp_h(a.x.d[i]);
  return {r};
}
template <uint64_t V, uint64_t D>
__device__ __forceinline__ Fq2B<V, D> dq2(const Fq2B<V, D>& a) {
  return {dq(a.c0), dq(a.c1)};
}
template <uint64_t V, uint64_t D>
__device__ __forceinline__ Fq2B<V, D> dh2(const Fq2B<V, D>& a) {
  return {dh(a.c0), dh(a.c1)};
}
template <uint64_t V, uint64_t D>
__device__ __forceinline__ Fq6B<V, D> dh6(const Fq6B<V, D>& a) {
  return {dh2(a.c0), dh2(a.c1), dh2(a.c2)};
}
template <int CTRL, uint64_t V, uint64_t D>
__device__ __forceinline__ FqB<V, D> bc(const FqB<V, D>& a) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = dpp_b<CTRL>(a.x.d[i]);
  return {r};
}
template <int CTRL, uint64_t V, uint64_t D>
__device__ __forceinline__ Fq2B<V, D> bc2(const Fq2B<V, D>& a) {
  return {bc<CTRL>(a.c0), bc<CTRL>(a.c1)};
}
template <int CTRL, uint64_t V, uint64_t D>
__device__ __forceinline__ Fq6B<V, D> bc6(const Fq6B<V, D>& a) {
  return {bc2<CTRL>(a.c0), bc2<CTRL>(a.c1), bc2<CTRL>(a.c2)};
}

// X * Y in Fp6, three of its six Fp2 products on each q lane (as q6mul)
template <uint64_t VX, uint64_t DX, uint64_t VY, uint64_t DY>
__device__ __forceinline__ auto qq6mul(const Fq6B<VX, DX>& X, const Fq6B<VY, DY>& Y, bool q) {
  const auto p0 = sel(q, norm(X.c1 + X.c2), X.c0) * sel(q, norm(Y.c1 + Y.c2), Y.c0);
  SEQ();
  const auto p1 = sel(q, norm(X.c0 + X.c1), X.c1) * sel(q, norm(Y.c0 + Y.c1), Y.c1);
  SEQ();
  const auto p2 = sel(q, norm(X.c0 + X.c2), X.c2) * sel(q, norm(Y.c0 + Y.c2), Y.c2);
  SEQ();
  const auto t0 = bc2<BQ0>(p0), t1 = bc2<BQ0>(p1), t2 = bc2<BQ0>(p2);  // the q = 0 lane's products
  const auto u0 = bc2<BQ1>(p0), u1 = bc2<BQ1>(p1), u2 = bc2<BQ1>(p2);  // the q = 1 lane's
  const auto c0 = norm(xi(norm(u0 - (t1 + t2))) + t0);
  const auto c1 = norm((u1 - (t0 + t1)) + xi(t2));
  const auto c2 = norm((u2 - (t0 + t2)) + t1);
  return fq6b(c0, c1, c2);
}

// one Fp12 squaring on the (h, q) lanes, as q_sqr
template <uint64_t V, uint64_t D>
__device__ __forceinline__ auto qq_sqr(const Fq6B<V, D>& own, bool h, bool q) {
  const auto o = dh6(own);  // the other half: b on h = 0, a on h = 1
  const auto X = norm(sel(h, o, own + o));
  const auto Y = norm(sel(h, own, own + f6v(o)));
  const auto P = qq6mul(X, Y, q);
  const auto t = bc6<BH1>(P);  // a b (the h = 1 lanes' product)
  return norm(sel(h, P + P, (P - t) - f6v(t)));
}

// own *= line, as q_line
template <uint64_t V, uint64_t D, uint64_t VL, uint64_t DL, uint64_t VM, uint64_t DM>
__device__ __forceinline__ auto qq_line(const Fq6B<V, D>& own, bool h, bool q, const Fq2B<VL, DL>& l0,
                                        const Fq2B<VM, DM>& l2, const Fq2B<VM, DM>& l3) {
  // the other half's coefficients are exchanged one at a time, right before their product (live range)
  const auto p1 = sel(q, norm(own.c0 + own.c1), own.c0) * sel(q, norm(l0 + l2), l0);
  SEQ();
  const auto p2 = sel(q, dh2(own.c2), own.c1) * sel(q, l3, l2);
  SEQ();
  const auto p3 = sel(q, dh2(own.c0), own.c2) * sel(q, l3, l2);
  SEQ();
  const auto p4 = sel(q, dh2(own.c1), own.c2) * sel(q, l3, l0);
  SEQ();
  const auto t0 = bc2<BQ0>(p1), t1 = bc2<BQ0>(p2), u0 = bc2<BQ0>(p3), u2 = bc2<BQ0>(p4);  // q = 0 products
  const auto u1 = bc2<BQ1>(p1), v0 = bc2<BQ1>(p2), v1 = bc2<BQ1>(p3), v2 = bc2<BQ1>(p4);  // q = 1 products
  const auto m01 = fq6b(t0 + xi(u0), (u1 - (t0 + t1)), t1 + u2);
  const auto m1 = fq6b(xi(v0), v1, v2);
  return norm(norm(m01) + sel(h, m1, f6v(m1)));
}

// one line's inputs on lane (h, q): l0 and the coefficient this lane scales (component q of E ZZ for h = 0, of
// z3 ZZ for h = 1).  (Loading them one line ahead of use measured 3.72 ms per launch against 3.68 ms without, and
// the 512-register allocation it needed cost ~15 % of pipelined throughput.)
struct LineIn {
  Fq2B<ML_LV, ML_LD> l0;
  FqB<ML_LV, ML_LD> c;
};
__device__ __forceinline__ LineIn ld_line(const uint32_t* Li, size_t n, bool h, bool q) {
  LineIn r;
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    r.l0.c0.x.d[j] = Li[(size_t)j * n];
    r.l0.c1.x.d[j] = Li[(size_t)(14 + j) * n];
  }
  const uint32_t* Lc = Li + (size_t)((h ? 56 : 28) + (q ? 14 : 0)) * n;  // per-lane row base: uniform row offsets
#pragma unroll
  for (int j = 0; j < 14; ++j) r.c.x.d[j] = Lc[(size_t)j * n];
  return r;
}

// a P-scaled record of k_miller_fused's line wave (mlines::Line1/Line2<true>): l0, l2 = E ZZ (-x_P), l3 = z3 ZZ y_P
// (l2 and l3 are products -- mlines::scale -- so their words are N-form digits)
struct LineS {
  Fq2B<ML_LV, ML_LD> l0;
  Fq2B<2, fqb_detail::MASK> l2, l3;
};
__device__ __forceinline__ LineS ld_line_s(const uint32_t* Li, size_t n) {
  LineS r;
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    r.l0.c0.x.d[j] = Li[(size_t)j * n];
    r.l0.c1.x.d[j] = Li[(size_t)(14 + j) * n];
    r.l2.c0.x.d[j] = Li[(size_t)(28 + j) * n];
    r.l2.c1.x.d[j] = Li[(size_t)(42 + j) * n];
    r.l3.c0.x.d[j] = Li[(size_t)(56 + j) * n];
    r.l3.c1.x.d[j] = Li[(size_t)(70 + j) * n];
  }
  return r;
}

// the line's P factors, as q_line_p: l2 = E ZZ (-x_P), l3 = z3 ZZ y_P in N form
template <uint64_t VP, uint64_t DP>
__device__ __forceinline__ void qq_line_p(const LineIn& in, const FqB<VP, DP>& pc, bool q, Fq2B<2, fqb_detail::MASK>& l2,
                                          Fq2B<2, fqb_detail::MASK>& l3) {
  const FqN mine = in.c * pc;
  const Fq2B<2, fqb_detail::MASK> m{bc<BQ0>(mine), bc<BQ1>(mine)};  // (component 0, component 1) of this h's product
  l2 = bc2<BH0>(m);                                                  // E ZZ (-x_P), from the h = 0 lanes
  l3 = bc2<BH1>(m);                                                  // z3 ZZ y_P, from the h = 1 lanes
}

}  // namespace

// n pairs; their line records with leading dimension ld >= n (word w of line k of pair i at L[(k ML_WORDS + w) ld
// + i]: the bisection re-reads the first B records of a batch written for B + 64 pairs)
template <int G>
__global__ void __launch_bounds__(64) k_miller_acc4q(const G1A* P, const G2A* Q, const int* ok, size_t n,
                                                     const uint32_t* L, size_t ld, Fp12* out) {
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
  constexpr uint64_t VF = ML_QF_V, DF = ML_QF_D;
  using F = Fq6B<VF, DF>;
  const size_t step = (size_t)ML_WORDS * ld;
  const uint32_t* Lb[G];
#pragma unroll
  for (int g = 0; g < G; ++g) Lb[g] = L + pi[g];
  const FqC one = fqb_canon(FP_ONE), zero{fq_zero()};
  const Fq2B<1, fqb_detail::MASK> z2{zero, zero};
  F f = relax<VF, DF>(Fq6B<1, fqb_detail::MASK>{{sel(h, zero, one), zero}, z2, z2});
  // the P coordinate each lane scales its line coefficient by: -x_P (h = 0, as K - x_P) or y_P (h = 1), formed once
  // and parked in LDS (word-major, this lane's column): held in registers, G of them pushed the kernel past the
  // register file (G = 4 ran at 256 VGPR + 256 AGPR, the AGPRs a spill space paid in accvgpr moves)
  using PcT = decltype(sel(h, zero, zero - zero));
  __shared__ uint32_t pcs[G][14][64];
  const int lane = (int)threadIdx.x;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const FqC pv = fqb_canon(h ? P[pi[g]].y : P[pi[g]].x);
    const PcT pcg = sel(h, pv, zero - pv);
#pragma unroll
    for (int w = 0; w < 14; ++w) pcs[g][w][lane] = pcg.x.d[w];
  }
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = relax<VF, DF>(qq_sqr(f, h, q));
    const int nl = ((X_ABS >> b) & 1ull) ? 2 : 1;
#pragma unroll 1
    for (int s = 0; s < nl; ++s) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const LineIn cur = ld_line(Lb[g], ld, h, q);
        PcT pcg;
#pragma unroll
        for (int w = 0; w < 14; ++w) pcg.x.d[w] = pcs[g][w][lane];
        Fq2B<2, fqb_detail::MASK> l2, l3;
        qq_line_p(cur, pcg, q, l2, l3);
        const auto fl = relax<VF, DF>(qq_line(f, h, q, cur.l0, l2, l3));
        f = G == 1 ? fl : sel(live[g], fl, f);
        Lb[g] += step;
      }
    }
  }
  if (!q) {
    Fp6 r{fq2b_pack(f.c0), fq2b_pack(f.c1), fq2b_pack(f.c2)};
    if (h)
      out[grp].c1 = Fp6{fp2_neg(r.c0), fp2_neg(r.c1), fp2_neg(r.c2)};
    else
      out[grp].c0 = r;
  }
}

// ---------------------------------------------------------------------------
// k_miller_acc4l: four pairs per f with the step's lines multiplied together
// before they meet f (lines first).  A line is L = C + D w with C = (l0, l2, 0)
// and D = (0, l3, 0); per round of four lines (one per pair) each lane forms
//   LL = L_a L_b for two of the pairs (q = 0: pairs 0, 1; q = 1: pairs 2, 3):
//        6 Fp2 products, the Karatsuba set of (l0, l2, l3) x (m0, m2, n3),
//        three per h lane -- LL = (C0, C1, C2) + (0, D1, D2) w
//   M = LL_0 LL_1: CC' (h = 0) and (C + D)(C' + D') (h = 1) as Fp6 products
//        split over q, plus DD' (3 products, one per lane 0..2): 15 products
//   f M: a M0 (h = 0) and b M1 (h = 1) split over q, then (a + b)(M0 + M1)
//        over all four lanes: 18 products
// -- 12 Fp2 products per lane per round against 16 for four f x line
// products (k_miller_acc4q<4>: 4 per line).  The exchanges are quad DPP moves
// as in k_miller_acc4q (broadcast from quad lane j: quad_perm [j, j, j, j]).
namespace {

constexpr int BL0 = 0x00, BL1 = 0x55, BL2 = 0xAA, BL3 = 0xFF;

// one line on this lane: l0, l2 = E ZZ (-x_P), l3 = z3 ZZ y_P; the lane scales its h's coefficient (both
// components: h = 0 E ZZ by -x_P, h = 1 z3 ZZ by y_P) and takes the other from its h partner.  A pair that is not
// live is the line 1.
struct LineF {
  Fq2B<ML_LV, ML_LD> l0;
  Fq2B<2, fqb_detail::MASK> l2, l3;
};
struct LineRaw {
  Fq2B<ML_LV, ML_LD> l0, e;
};
__device__ __forceinline__ LineRaw ld_line_raw(const uint32_t* Li, size_t n, bool h) {
  LineRaw r;
  // the lane's coefficient rows start at a per-lane pointer, so every row offset is uniform (per-lane offsets
  // were hoisted out of the loop as 28 64-bit registers and spilled)
  const uint32_t* Le = Li + (size_t)(h ? 56 : 28) * n;
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    r.l0.c0.x.d[j] = Li[(size_t)j * n];
    r.l0.c1.x.d[j] = Li[(size_t)(14 + j) * n];
    r.e.c0.x.d[j] = Le[(size_t)j * n];
    r.e.c1.x.d[j] = Le[(size_t)(14 + j) * n];
  }
  return r;
}
template <class PcT>
__device__ __forceinline__ LineF line_f(const LineRaw& in, bool h, const PcT& pc, bool live) {
  const Fq2B<2, fqb_detail::MASK> mine{in.e.c0 * pc, in.e.c1 * pc};
  SEQ();
  const auto other = dh2(mine);
  const FqC one = fqb_canon(FP_ONE), zero{fq_zero()};
  const Fq2B<1, fqb_detail::MASK> one2{one, zero}, zero2{zero, zero};
  LineF r;
  r.l0 = relax<ML_LV, ML_LD>(sel(live, in.l0, one2));
  r.l2 = relax<2, fqb_detail::MASK>(sel(live, sel(h, other, mine), zero2));
  r.l3 = relax<2, fqb_detail::MASK>(sel(live, sel(h, mine, other), zero2));
  return r;
}

// M = LL_0 LL_1 for the round's four lines A, B (this q's two pairs); M0 on the h = 0 lanes, M1 on h = 1
__device__ __forceinline__ auto ll_m(const LineF& A, const LineF& B, bool h, bool q) {
  // LL = L_a L_b = (C0, C1, C2) + (0, D1, D2) w on both h lanes of this q:
  //   C0 = l0 m0 + xi l3 n3, C1 = (l0 + l2)(m0 + m2) - l0 m0 - l2 m2, C2 = l2 m2,
  //   D1 = (l0 + l3)(m0 + n3) - l0 m0 - l3 n3, D2 = (l2 + l3)(m2 + n3) - l2 m2 - l3 n3
  // (h = 0 forms the three diagonal products, h = 1 the three sums')
  const auto p0 = sel(h, norm(A.l0 + A.l2), A.l0) * sel(h, norm(B.l0 + B.l2), B.l0);
  SEQ();
  const auto p1 = sel(h, norm(A.l0 + A.l3), A.l2) * sel(h, norm(B.l0 + B.l3), B.l2);
  SEQ();
  const auto p2 = sel(h, norm(A.l2 + A.l3), A.l3) * sel(h, norm(B.l2 + B.l3), B.l3);
  SEQ();
  const auto t0 = bc2<BH0>(p0), t1 = bc2<BH0>(p1), t2 = bc2<BH0>(p2);  // l0 m0, l2 m2, l3 n3
  const auto u0 = bc2<BH1>(p0), u1 = bc2<BH1>(p1), u2 = bc2<BH1>(p2);  // the sums' products
  const auto c0 = norm(t0 + xi(t2));
  const auto c1 = norm(u0 - (t0 + t1));
  const auto d1 = norm(u1 - (t0 + t2));
  const auto d2 = norm(u2 - (t1 + t2));
  // M = LL_0 LL_1 = CC' + v DD' + ((C + D)(C' + D') - CC' - DD') w  (LL_q on the q lanes, the other by a q
  // exchange).  DD' = (D1 v + D2 v^2)(D1' v + D2' v^2) = (xi (e2 - e0 - e1), xi e1, e0) with e0 = D1 D1',
  // e1 = D2 D2', e2 = (D1 + D2)(D1' + D2'): one product on each of lanes 0, 1, 2 (lane 3 repeats lane 2's)
  const auto od1 = dq2(d1);
  const auto od2 = dq2(d2);
  const auto xd1 = sel(q, od1, d1);  // LL_0's
  const auto xd2 = sel(q, od2, d2);
  const auto yd1 = sel(q, d1, od1);  // LL_1's
  const auto yd2 = sel(q, d2, od2);
  const auto e = sel(h, norm(xd1 + xd2), sel(q, xd2, xd1)) * sel(h, norm(yd1 + yd2), sel(q, yd2, yd1));
  SEQ();
  // this q's operand of CC' (h = 0) or (C + D)(C' + D') (h = 1), then the other q's
  const auto x0 = c0;
  const auto x1 = sel(h, norm(c1 + d1), c1);
  const auto x2 = sel(h, norm(t1 + d2), t1);
  const auto y0 = dq2(x0);
  const auto y1 = dq2(x1);
  const auto y2 = dq2(x2);
  const auto X = fq6b(sel(q, y0, x0), sel(q, y1, x1), sel(q, y2, x2));
  const auto Y = fq6b(sel(q, x0, y0), sel(q, x1, y1), sel(q, x2, y2));
  const auto K = qq6mul(X, Y, q);  // CC' on h = 0, (C + D)(C' + D') on h = 1
  const auto e0 = bc2<BL0>(e);
  const auto e1 = bc2<BL1>(e);
  const auto e2 = bc2<BL2>(e);
  const auto DD = fq6b(xi(norm(e2 - (e0 + e1))), xi(e1), e0);
  const auto K0 = bc6<BH0>(K);
  return norm(sel(h, norm(K - norm(K0 + DD)), norm(K0 + f6v(DD))));
}

// f's half parked in LDS ([word][lane], 84 words) while the lines are multiplied together
template <uint64_t V, uint64_t D>
__device__ __forceinline__ void park6(uint32_t* lds, const Fq6B<V, D>& f, int lane) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&f);
#pragma unroll
  for (int i = 0; i < 84; ++i) lds[i * 64 + lane] = w[i];
}
template <uint64_t V, uint64_t D>
__device__ __forceinline__ Fq6B<V, D> unpark6(const uint32_t* lds, int lane) {
  Fq6B<V, D> f;
  uint32_t* w = reinterpret_cast<uint32_t*>(&f);
  __asm__ volatile("" ::: "memory");  // read the LDS copy: no store-to-load forwarding of the parked words
#pragma unroll
  for (int i = 0; i < 84; ++i) w[i] = lds[i * 64 + lane];
  return f;
}

// f M with f's half (a on h = 0, b on h = 1) read back from LDS:
//   a' = a M0 + v b M1, b' = (a + b)(M0 + M1) - a M0 - b M1
// a M0 / b M1 split over q; (a + b)(M0 + M1)'s six products over the four quad lanes in two rounds (lane j =
// 2h + q: {X0 Y0, X1 Y1, X2 Y2, (X1 + X2)(Y1 + Y2)}[j], then lanes 0 / 1 (2 / 3 as copies) (X0 + X1)(Y0 + Y1),
// (X0 + X2)(Y0 + Y2))
template <uint64_t V, uint64_t D, uint64_t VM, uint64_t DM>
__device__ __forceinline__ auto ll_fm(const uint32_t* fpark, const Fq6B<VM, DM>& M, bool h, bool q, int lane) {
  auto f = unpark6<V, D>(fpark, lane);
  const auto Z = qq6mul(f, M, q);  // a M0 on h = 0, b M1 on h = 1
  SEQ();
  const auto X = norm(f + dh6(f));  // a + b
  const auto xa = sel(h, sel(q, norm(X.c1 + X.c2), X.c2), sel(q, X.c1, X.c0));
  const auto xb = sel(q, norm(X.c0 + X.c2), norm(X.c0 + X.c1));
  const auto Y = norm(M + dh6(M));  // M0 + M1
  const auto ya = sel(h, sel(q, norm(Y.c1 + Y.c2), Y.c2), sel(q, Y.c1, Y.c0));
  const auto yb = sel(q, norm(Y.c0 + Y.c2), norm(Y.c0 + Y.c1));
  const auto pa = xa * ya;
  SEQ();
  const auto pb = xb * yb;
  SEQ();
  const auto r0 = bc2<BL0>(pa), r1 = bc2<BL1>(pa), r2 = bc2<BL2>(pa), r3 = bc2<BL3>(pa);
  const auto s0 = bc2<BL0>(pb), s1 = bc2<BL1>(pb);
  const auto S = fq6b(norm(xi(norm(r3 - (r1 + r2))) + r0), norm((s0 - (r0 + r1)) + xi(r2)),
                      norm((s1 - (r0 + r2)) + r1));
  const auto Zo = dh6(Z);
  return norm(sel(h, S - norm(Z + Zo), Z + f6v(Zo)));
}

}  // namespace

// four pairs per f, lines first; the records and the output as k_miller_acc4q<4>
__global__ void __launch_bounds__(64) k_miller_acc4l(const G1A* P, const G2A* Q, const int* ok, size_t n,
                                                     const uint32_t* L, size_t ld, Fp12* out) {
  constexpr int G = 4;
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t grp = t >> 2;
  const bool h = (t & 2) != 0, q = (t & 1) != 0;
  const size_t ngrp = (n + G - 1) / G;
  if (grp >= ngrp) return;  // the four lanes of a group leave together
  bool any = false, live[2];
  size_t pi[2];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const size_t p = grp * G + g;
    const size_t pc = p < n ? p : n - 1;  // clamped: loads stay inside the batch's line buffer
    const bool lv = p < n && (!ok || ok[p]) && !P[p].inf && !Q[p].inf;
    any = any || lv;
    if ((g >> 1) == (int)q) {  // this lane's pairs: 2q, 2q + 1
      live[g & 1] = lv;
      pi[g & 1] = pc;
    }
  }
  if (!any) {
    if (!q) {
      Fp6* o = h ? &out[grp].c1 : &out[grp].c0;
      *o = h ? Fp6{fp2_zero(), fp2_zero(), fp2_zero()} : Fp6{fp2_one(), fp2_zero(), fp2_zero()};
    }
    return;
  }
  constexpr uint64_t VF = ML_QF_V, DF = ML_QF_D;
  using F = Fq6B<VF, DF>;
  const size_t step = (size_t)ML_WORDS * ld;
  const uint32_t* La = L + pi[0];
  const uint32_t* Lb = L + pi[1];
  const FqC one = fqb_canon(FP_ONE), zero{fq_zero()};
  const Fq2B<1, fqb_detail::MASK> z2{zero, zero};
  F f = relax<VF, DF>(Fq6B<1, fqb_detail::MASK>{{sel(h, zero, one), zero}, z2, z2});
  // this lane's P coordinate of each of its two pairs (-x_P as K - x_P on h = 0, y_P on h = 1), parked in LDS
  using PcT = decltype(sel(h, zero, zero - zero));
  __shared__ uint32_t pcs[2][14][64];
  __shared__ uint32_t fpark[84 * 64];
  const int lane = (int)threadIdx.x;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const FqC pv = fqb_canon(h ? P[pi[s]].y : P[pi[s]].x);
    const PcT pcg = sel(h, pv, zero - pv);
#pragma unroll
    for (int w = 0; w < 14; ++w) pcs[s][w][lane] = pcg.x.d[w];
  }
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = relax<VF, DF>(qq_sqr(f, h, q));
    const int nl = ((X_ABS >> b) & 1ull) ? 2 : 1;
#pragma unroll 1
    for (int s = 0; s < nl; ++s) {
      // opaque line pointers: otherwise loop strength reduction keeps one 64-bit induction pointer per record
      // row (56 per pair) across the loop, and they spill
      __asm__ volatile("" : "+v"(La), "+v"(Lb));
      const LineRaw ra = ld_line_raw(La, ld, h);  // both pairs' loads in flight while f is parked
      const LineRaw rb = ld_line_raw(Lb, ld, h);
      park6(fpark, f, lane);
      SEQ();
      PcT pa, pb;
#pragma unroll
      for (int w = 0; w < 14; ++w) pa.x.d[w] = pcs[0][w][lane];
      const LineF A = line_f(ra, h, pa, live[0]);
      SEQ();
#pragma unroll
      for (int w = 0; w < 14; ++w) pb.x.d[w] = pcs[1][w][lane];
      const LineF B = line_f(rb, h, pb, live[1]);
      SEQ();
      const auto M = ll_m(A, B, h, q);
      SEQ();
      f = relax<VF, DF>(ll_fm<VF, DF>(fpark, M, h, q, lane));
      SEQ();
      La += step;
      Lb += step;
    }
  }
  if (!q) {
    Fp6 r{fq2b_pack(f.c0), fq2b_pack(f.c1), fq2b_pack(f.c2)};
    if (h)
      out[grp].c1 = Fp6{fp2_neg(r.c0), fp2_neg(r.c1), fp2_neg(r.c2)};
    else
      out[grp].c0 = r;
  }
}

// ---------------------------------------------------------------------------
// k_miller_acc8: one pair per f on EIGHT lanes -- the latency form for small
// batches.  Lane 8k + 4h + j: h selects the half of f (a = f.c0 / b = f.c1) and
// the quad of lanes that owns it; j (0..3) which products of each step the lane
// forms:
//   squaring   each half's Fp6 product ((a + b)(a + v b) / a b) with its six
//              Fp2 products over the quad in two rounds (q4_6mul): 2 products
//              per lane instead of 3
//   line       the eight Fp2 products of the half's line product two per lane
//              (k_miller_acc4q<1>: four)
// The other half of a quad-uniform value comes from the mirrored lane of the
// other quad (DPP row_half_mirror: lane 4h + j <- lane 4(1 - h) + 3 - j, which
// holds the same value as every lane of its quad), a product of the quad from
// one quad broadcast.  Twice the waves of k_miller_acc4q<1> for ~40 % fewer
// product rounds per step.
namespace {

__device__ __forceinline__ uint32_t dpp_m(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
}
template <uint64_t V, uint64_t D>
__device__ __forceinline__ FqB<V, D> dm(const FqB<V, D>& a) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = dpp_m(a.x.d[i]);
  return {r};
}
template <uint64_t V, uint64_t D>
__device__ __forceinline__ Fq2B<V, D> dm2(const Fq2B<V, D>& a) {
  return {dm(a.c0), dm(a.c1)};
}
template <uint64_t V, uint64_t D>
__device__ __forceinline__ Fq6B<V, D> dm6(const Fq6B<V, D>& a) {
  return {dm2(a.c0), dm2(a.c1), dm2(a.c2)};
}

// the Fp6 product X Y with its six Fp2 products over the four quad lanes in two rounds (lane j = 2 j1 + j0 forms
// {X0 Y0, X1 Y1, X2 Y2, (X1 + X2)(Y1 + Y2)}[j], then lanes 0 / 1 (and, as copies, 2 / 3) (X0 + X1)(Y0 + Y1) /
// (X0 + X2)(Y0 + Y2)); X and Y are the same on every lane of the quad, and so is the result
template <uint64_t VX, uint64_t DX, uint64_t VY, uint64_t DY>
__device__ __forceinline__ auto q4_6mul(const Fq6B<VX, DX>& X, const Fq6B<VY, DY>& Y, bool j1, bool j0) {
  const auto p1 = sel(j1, sel(j0, norm(X.c1 + X.c2), X.c2), sel(j0, X.c1, X.c0)) *
                  sel(j1, sel(j0, norm(Y.c1 + Y.c2), Y.c2), sel(j0, Y.c1, Y.c0));
  SEQ();
  const auto p2 = sel(j0, norm(X.c0 + X.c2), norm(X.c0 + X.c1)) * sel(j0, norm(Y.c0 + Y.c2), norm(Y.c0 + Y.c1));
  SEQ();
  const auto r0 = bc2<BL0>(p1), r1 = bc2<BL1>(p1), r2 = bc2<BL2>(p1), r3 = bc2<BL3>(p1);
  const auto s0 = bc2<BL0>(p2), s1 = bc2<BL1>(p2);
  const auto c0 = norm(xi(norm(r3 - (r1 + r2))) + r0);
  const auto c1 = norm((s0 - (r0 + r1)) + xi(r2));
  const auto c2 = norm((s1 - (r0 + r2)) + r1);
  return fq6b(c0, c1, c2);
}

// one Fp12 squaring on the eight lanes (j1 j0 = j)
template <uint64_t V, uint64_t D>
__device__ __forceinline__ auto q8_sqr(const Fq6B<V, D>& own, bool h, bool j1, bool j0) {
  const auto o = dm6(own);  // the other half
  const auto X = norm(sel(h, o, own + o));
  const auto Y = norm(sel(h, own, own + f6v(o)));
  const auto P = q4_6mul(X, Y, j1, j0);  // (a + b)(a + v b) on h = 0, a b on h = 1
  const auto t = dm6(P);                 // a b on the h = 0 lanes
  return norm(sel(h, P + P, (P - t) - f6v(t)));
}

// own *= line (l0 + l2 v) + l3 v w, the eight products of qq_line two per lane:
//   round 1: a0 l0, a1 l2, a2 l2, a2 l0;  round 2: (a0 + a1)(l0 + l2), o2 l3, o0 l3, o1 l3  (lane j: the j-th)
template <uint64_t V, uint64_t D, uint64_t VL, uint64_t DL, uint64_t VM, uint64_t DM>
__device__ __forceinline__ auto q8_line(const Fq6B<V, D>& own, bool h, bool j1, bool j0, const Fq2B<VL, DL>& l0,
                                        const Fq2B<VM, DM>& l2, const Fq2B<VM, DM>& l3) {
  const auto pa = sel(j1, own.c2, sel(j0, own.c1, own.c0)) * sel(j1, sel(j0, l0, l2), sel(j0, l2, l0));
  SEQ();
  const auto o = dm6(own);
  const auto pb = sel(j1, sel(j0, o.c1, o.c0), sel(j0, o.c2, norm(own.c0 + own.c1))) *
                  sel(j1, l3, sel(j0, l3, norm(l0 + l2)));
  SEQ();
  const auto t0 = bc2<BL0>(pa), t1 = bc2<BL1>(pa), u0 = bc2<BL2>(pa), u2 = bc2<BL3>(pa);
  const auto u1 = bc2<BL0>(pb), v0 = bc2<BL1>(pb), v1 = bc2<BL2>(pb), v2 = bc2<BL3>(pb);
  const auto m01 = fq6b(t0 + xi(u0), (u1 - (t0 + t1)), t1 + u2);
  const auto m1 = fq6b(xi(v0), v1, v2);
  return norm(norm(m01) + sel(h, m1, f6v(m1)));
}

}  // namespace

__global__ void __launch_bounds__(64) k_miller_acc8(const G1A* P, const G2A* Q, const int* ok, size_t n,
                                                    const uint32_t* L, size_t ld, Fp12* out) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t pi = t >> 3;
  const bool h = (t & 4) != 0, j1 = (t & 2) != 0, j0 = (t & 1) != 0;
  if (pi >= n) return;  // the eight lanes of a pair leave together
  const bool live = (!ok || ok[pi]) && !P[pi].inf && !Q[pi].inf;
  if (!live) {
    if (!j1 && !j0) {
      Fp6* o = h ? &out[pi].c1 : &out[pi].c0;
      *o = h ? Fp6{fp2_zero(), fp2_zero(), fp2_zero()} : Fp6{fp2_one(), fp2_zero(), fp2_zero()};
    }
    return;
  }
  constexpr uint64_t VF = ML_QF_V, DF = ML_QF_D;
  using F = Fq6B<VF, DF>;
  const size_t step = (size_t)ML_WORDS * ld;
  const uint32_t* Lp = L + pi;
  const FqC one = fqb_canon(FP_ONE), zero{fq_zero()};
  const Fq2B<1, fqb_detail::MASK> z2{zero, zero};
  F f = relax<VF, DF>(Fq6B<1, fqb_detail::MASK>{{sel(h, zero, one), zero}, z2, z2});
  const FqC pv = fqb_canon(h ? P[pi].y : P[pi].x);
  const auto pc = sel(h, pv, zero - pv);  // -x_P (h = 0) or y_P (h = 1)
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = relax<VF, DF>(q8_sqr(f, h, j1, j0));
    const int nl = ((X_ABS >> b) & 1ull) ? 2 : 1;
#pragma unroll 1
    for (int s = 0; s < nl; ++s) {
      const LineIn cur = ld_line(Lp, ld, h, j0);  // l0 and component j0 of this h's coefficient
      const FqN mine = cur.c * pc;
      const Fq2B<2, fqb_detail::MASK> m{bc<BL0>(mine), bc<BL1>(mine)};  // this h's coefficient times its P factor
      const auto mo = dm2(m);
      const auto l2 = sel(h, mo, m), l3 = sel(h, m, mo);
      f = relax<VF, DF>(q8_line(f, h, j1, j0, cur.l0, l2, l3));
      Lp += step;
    }
  }
  if (!j1 && !j0) {
    Fp6 r{fq2b_pack(f.c0), fq2b_pack(f.c1), fq2b_pack(f.c2)};
    if (h)
      out[pi].c1 = Fp6{fp2_neg(r.c0), fp2_neg(r.c1), fp2_neg(r.c2)};
    else
      out[pi].c0 = r;
  }
}

// ---------------------------------------------------------------------------
// k_miller_fused<G>: both halves of the split Miller loop in ONE workgroup per MF_PAIRS<G> pairs.  Wave 0 runs
// the G2 side and writes each line record into an LDS double buffer; waves 1 and 2 run the f accumulation (four
// lanes per f, G pairs per f, the code of k_miller_acc4q) and read the record of line k while wave 0 forms line k
// + 1 -- one workgroup barrier per line (68).  The line wave is sized to keep up with the accumulation waves:
//   G = 2: 64 pairs, mlines::Line1 (one lane per pair); two accumulation waves of 16 f x 2 pairs
//   G = 1: 32 pairs, mlines::Line2 (two lanes per pair); two accumulation waves of 16 f x 1 pair
// (G = 2 with two lanes per pair and one accumulation wave waited at the barrier half the time: C2 -12 %.)
// Three waves per workgroup: each keeps the whole register file of its SIMD.  The records never touch
// HBM (split into k_miller_lines2 + k_miller_acc4q, a C2 batch wrote and read 84 words x 68 lines per pair, 228
// MB each way), the line kernel's latency leaves the batch's chain, and the launch puts twice the waves of the
// accumulation alone on the chip.
template <int G>
constexpr int MF_PAIRS = G == 2 ? 64 : 32;
template <int G>
constexpr int MF_ACC = 4 * MF_PAIRS<G> / G / 64;  // f-accumulation waves per workgroup (two)

template <int G>
__global__ void __launch_bounds__(64 * (1 + MF_ACC<G>)) k_miller_fused(const G1A* P, const G2A* Q, const int* ok,
                                                                       size_t n, Fp12* out) {
  constexpr int PW = MF_PAIRS<G>;
  __shared__ uint32_t rec[2][ML_WORDS * PW];
  __shared__ uint32_t qlds[56 * 64];
  const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  const size_t pair0 = (size_t)blockIdx.x * PW;
  if (wave == 0) {  // ---- G2 side: line k + 1 while the accumulation reads line k
    constexpr int LPP = 64 / PW;  // lanes per pair
    const int pl = lane / LPP;
    const size_t i = pair0 + pl < n ? pair0 + pl : n - 1;
    G2A q = Q[i];
    if (q.inf) q = g2_generator();  // its records are read but not used (the pair is not live)
    using LT = typename std::conditional<LPP == 1, mlines::Line1<true>, mlines::Line2<true>>::type;
    LT T;
    if constexpr (LPP == 1)
      T.init(q, qlds, lane);
    else
      T.init(q, (lane & 1) != 0, qlds, lane);
    T.pf.init(P[i]);  // the records carry l2, l3 with the pair's P factors applied
    uint32_t* const r0 = &rec[0][pl];
    uint32_t* const r1 = &rec[1][pl];
    T.dbl(r0, PW);  // line 0: the doubling at b = 62
    __syncthreads();
    int b = 62;
    bool added = false;  // whether the record of bit b's addition step has been written
#pragma unroll 1
    for (int k = 1; k <= MILLER_NLINES; ++k) {
      if (k < MILLER_NLINES) {
        uint32_t* dst = (k & 1) ? r1 : r0;
        if (!added && ((X_ABS >> b) & 1ull)) {
          T.add(dst, PW, qlds, lane);
          added = true;
        } else {
          --b;
          added = false;
          T.dbl(dst, PW);
        }
      }
      __syncthreads();
    }
    return;
  }
  // ---- f accumulation: lanes 4k + 2h + q of the accumulation waves own f k of the workgroup (pairs G k .. G k +
  // G - 1 of its MF_PAIRS); every lane runs the whole loop (the barriers), out-of-range groups write nothing
  const int at = (wave - 1) * 64 + lane;
  const int grp = at >> 2;
  const bool h = (at & 2) != 0, q = (at & 1) != 0;
  bool live[G];
  int pl[G];
  size_t pi[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    pl[g] = grp * G + g;
    const size_t p = pair0 + pl[g];
    pi[g] = p < n ? p : n - 1;
    live[g] = p < n && (!ok || ok[p]) && !P[pi[g]].inf && !Q[pi[g]].inf;
  }
  constexpr uint64_t VF = ML_QF_V, DF = ML_QF_D;
  using F = Fq6B<VF, DF>;
  const FqC one = fqb_canon(FP_ONE), zero{fq_zero()};
  const Fq2B<1, fqb_detail::MASK> z2{zero, zero};
  F f = relax<VF, DF>(Fq6B<1, fqb_detail::MASK>{{sel(h, zero, one), zero}, z2, z2});
  __syncthreads();  // line 0 is in rec[0]
  int k = 0;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = relax<VF, DF>(qq_sqr(f, h, q));
    const int nl = ((X_ABS >> b) & 1ull) ? 2 : 1;
#pragma unroll 1
    for (int s = 0; s < nl; ++s, ++k) {
      const uint32_t* buf = rec[k & 1];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const LineS cur = ld_line_s(buf + pl[g], PW);
        const auto fl = relax<VF, DF>(qq_line(f, h, q, cur.l0, cur.l2, cur.l3));
        f = sel(live[g], fl, f);
      }
      __syncthreads();
    }
  }
  const size_t og = pair0 / G + grp;
  if (q || og >= (n + G - 1) / G) return;
  bool any = false;
#pragma unroll
  for (int g = 0; g < G; ++g) any = any || live[g];
  Fp6 r{fq2b_pack(f.c0), fq2b_pack(f.c1), fq2b_pack(f.c2)};
  if (!any) r = h ? Fp6{fp2_zero(), fp2_zero(), fp2_zero()} : Fp6{fp2_one(), fp2_zero(), fp2_zero()};
  if (h)
    out[og].c1 = Fp6{fp2_neg(r.c0), fp2_neg(r.c1), fp2_neg(r.c2)};
  else
    out[og].c0 = r;
}

hipError_t launch_miller_fused(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, Fp12* f, int G) {
  if (!n) return hipSuccess;
  if (G == 2)
    hipLaunchKernelGGL(k_miller_fused<2>, dim3((unsigned)((n + MF_PAIRS<2> - 1) / MF_PAIRS<2>)),
                       dim3(64 * (1 + MF_ACC<2>)), 0, st, P, Q, ok, n, f);
  else
    hipLaunchKernelGGL(k_miller_fused<1>, dim3((unsigned)((n + MF_PAIRS<1> - 1) / MF_PAIRS<1>)),
                       dim3(64 * (1 + MF_ACC<1>)), 0, st, P, Q, ok, n, f);
  return hipGetLastError();
}

hipError_t launch_miller_acc4(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, const uint32_t* L,
                              size_t ld, Fp12* f, int G) {
  if (!n) return hipSuccess;
  if (ld < n) return hipErrorInvalidValue;
  const size_t ngrp = (n + G - 1) / G;
  const dim3 grid((unsigned)((4 * ngrp + 63) / 64));
  if (G == 8)
    hipLaunchKernelGGL(k_miller_acc4q<8>, grid, dim3(64), 0, st, P, Q, ok, n, L, ld, f);
  else if (G == 4)
    hipLaunchKernelGGL(k_miller_acc4q<4>, grid, dim3(64), 0, st, P, Q, ok, n, L, ld, f);
  else if (G == 2)
    hipLaunchKernelGGL(k_miller_acc4q<2>, grid, dim3(64), 0, st, P, Q, ok, n, L, ld, f);
  else
    hipLaunchKernelGGL(k_miller_acc4q<1>, grid, dim3(64), 0, st, P, Q, ok, n, L, ld, f);
  return hipGetLastError();
}

hipError_t launch_miller_acc8(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, const uint32_t* L,
                              size_t ld, Fp12* f) {
  if (!n) return hipSuccess;
  if (ld < n) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_miller_acc8, dim3((unsigned)((8 * n + 63) / 64)), dim3(64), 0, st, P, Q, ok, n, L, ld, f);
  return hipGetLastError();
}

hipError_t launch_miller_acc4l(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, const uint32_t* L,
                               size_t ld, Fp12* f) {
  if (!n) return hipSuccess;
  if (ld < n) return hipErrorInvalidValue;
  const size_t ngrp = (n + 3) / 4;
  hipLaunchKernelGGL(k_miller_acc4l, dim3((unsigned)((4 * ngrp + 63) / 64)), dim3(64), 0, st, P, Q, ok, n, L, ld, f);
  return hipGetLastError();
}

}  // namespace bls
