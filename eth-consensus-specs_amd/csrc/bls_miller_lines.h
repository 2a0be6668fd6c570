// G2 side of the split Miller loop, TWO lanes per pair (k_miller_lines2 in bls_miller_lane.hip, and the line
// waves of k_miller_fused in bls_miller_pair.hip): T's doubling / addition steps and the P-independent parts of
// the line coefficients, each step's line record written to L (word w at L[w * n]).
//
// A doubling step is 7 squarings + 4 products in Fp2 in three dependency levels; lanes 2k / 2k+1 split each level
// and broadcast results by DPP:
//   level 1   lane 0: A = x^2, ZZ = z^2          lane 1: B = y^2, YZ = (y + z)^2
//   level 2   lane 0: C = B^2, XB = (x + B)^2,   lane 1: F = E^2, z3 ZZ, E ZZ
//                     E x  (l0 = E x - 2B)       (E = 3A, z3 = YZ - B - ZZ)
//   level 3   both: y3 = E (D - x3) - 8C         (D = 2(XB - A - C), x3 = F - 2D)
// Each lane stores the line words it formed (lane 0: l0, lane 1: E ZZ and z3 ZZ).  The five addition steps run on
// both lanes (lane 0 stores l0, lane 1 the rest).  T stays in the bound-typed digit form for the whole loop
// (declared FqB<LN_TV, LN_TD>; every step is relaxed to it, so its bounds are checked by induction at compile
// time): no product unpacks or repacks, additions are digit-wise (the packed kernel: 12-limb carry chains and a
// conditional subtraction per addition and per product).
#pragma once
#include "bls_fqb.h"
#include "bls_kernels.h"

namespace bls {
namespace mlines {

// products one after another (interleaved, their digit columns spilled ~140 VGPRs)
#define LN_SEQ() __builtin_amdgcn_sched_barrier(0)
constexpr uint64_t LN_TV = 1024, LN_TD = 0x20000000ull + 64;  // loop-carried bound of T's coordinates

__device__ __forceinline__ uint32_t dpp_bc(uint32_t v, bool odd) {  // lane 2k's value (odd = false) or lane 2k+1's
  return odd ? (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xF5, 0xF, 0xF, false)   // quad_perm [1,1,3,3]
             : (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xA0, 0xF, 0xF, false);  // quad_perm [0,0,2,2]
}
template <bool ODD, uint64_t V, uint64_t D>
__device__ __forceinline__ Fq2B<V, D> bcp(const Fq2B<V, D>& a) {
  Fq2B<V, D> r;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    r.c0.x.d[i] = dpp_bc(a.c0.x.d[i], ODD);
    r.c1.x.d[i] = dpp_bc(a.c1.x.d[i], ODD);
  }
  return r;
}
template <uint64_t V, uint64_t D>
__device__ __forceinline__ void ml_store_q(uint32_t* L, size_t n, int w0, const Fq2B<V, D>& v) {
  const Fq2B<ML_LV, ML_LD> a = relax<ML_LV, ML_LD>(v);
  uint32_t* const Lw = L + (size_t)w0 * n;  // a per-lane row base, so the row offsets are uniform
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    Lw[(size_t)j * n] = a.c0.x.d[j];
    Lw[(size_t)(14 + j) * n] = a.c1.x.d[j];
  }
}

// The line's P factors (k_miller_fused's line waves apply them, so the accumulation reads l0, l2, l3 ready to
// multiply): l2 = E ZZ (-x_P) (addition: r (-x_P)), l3 = z3 ZZ y_P (addition: z3 y_P).  nx = -x_P as K - x_P.
struct PFac {
  FqC y;
  decltype(FqC{} - FqC{}) nx;
  __device__ __forceinline__ void init(const G1A& p) {
    const FqC zero{fq_zero()};
    y = fqb_canon(p.y);
    nx = zero - fqb_canon(p.x);
  }
};
using FqN2 = Fq2B<2, fqb_detail::MASK>;
template <uint64_t V, uint64_t D, uint64_t VS, uint64_t DS>
__device__ __forceinline__ Fq2B<2, fqb_detail::MASK> scale(const Fq2B<V, D>& a, const FqB<VS, DS>& s) {
  return {a.c0 * s, a.c1 * s};
}

// T of one pair on lanes (2k, 2k+1); Q's affine coordinates wait in qlds ([word][lane], 56 x 64 words) for the five
// addition steps (held in registers across the 63 doublings they pushed the kernel into spills)
// SC: the records carry l2, l3 with their P factors applied (PFac); otherwise (l0, E ZZ, z3 ZZ) / (l0, r, z3)
template <bool SC = false>
struct Line2 {
  using TF = Fq2B<LN_TV, LN_TD>;
  using QF = Fq2B<1, fqb_detail::MASK>;
  TF X, Y, Z;
  bool hi;
  PFac pf;  // SC only

  __device__ __forceinline__ void init(const G2A& q, bool hi_, uint32_t* qlds, int lane) {
    hi = hi_;
    const QF qx = fq2b_canon(q.x), qy = fq2b_canon(q.y);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&qx);
    const uint32_t* w2 = reinterpret_cast<const uint32_t*>(&qy);
#pragma unroll
    for (int k = 0; k < 28; k++) {
      qlds[k * 64 + lane] = w[k];
      qlds[(28 + k) * 64 + lane] = w2[k];
    }
    const FqC one = fqb_canon(FP_ONE), zero{fq_zero()};
    X = relax<LN_TV, LN_TD>(qx);
    Y = relax<LN_TV, LN_TD>(qy);
    Z = relax<LN_TV, LN_TD>(QF{one, zero});
  }

  // doubling step: T = 2T, the record (l0, E ZZ, z3 ZZ) at L
  __device__ __forceinline__ void dbl(uint32_t* L, size_t n) {
    const auto s0 = sqr(sel(hi, Y, X));
    LN_SEQ();
    const auto s1 = sqr(sel(hi, norm(Y + Z), Z));
    LN_SEQ();
    const auto A = bcp<false>(s0);
    const auto Bq = bcp<true>(s0);
    const auto ZZ = bcp<false>(s1);
    const auto YZ = bcp<true>(s1);
    const auto E = small<3>(A);
    const auto z3 = norm(YZ - (Bq + ZZ));
    const auto r0 = sqr(sel(hi, E, Bq));                        // lane 0: C;   lane 1: F
    LN_SEQ();
    const auto xb = norm(X + Bq);
    const auto r1 = sel(hi, z3, xb) * sel(hi, ZZ, xb);          // lane 0: XB;  lane 1: z3 ZZ
    LN_SEQ();
    const auto r2 = E * sel(hi, ZZ, X);                         // lane 0: E x; lane 1: E ZZ
    LN_SEQ();
    if constexpr (SC) {
      if (!hi) ml_store_q(L, n, 0, norm(r2 - small<2>(Bq)));  // lane 0: l0 = E x - 2B
      LN_SEQ();
      // lane 1: l2 = E ZZ (-x_P);  lane 0: l3 = z3 ZZ y_P (z3 ZZ from lane 1)
      const auto z3zz = bcp<true>(r1);
      const auto pl = scale(sel(hi, r2, z3zz), sel(hi, pf.nx, pf.y));
      ml_store_q(L, n, hi ? 28 : 56, pl);
      LN_SEQ();
    } else {
      ml_store_q(L, n, hi ? 28 : 0, sel(hi, r2, norm(r2 - small<2>(Bq))));  // lane 0: l0 = E x - 2B
      LN_SEQ();
      if (hi) ml_store_q(L, n, 56, r1);
      LN_SEQ();
    }
    const auto C = bcp<false>(r0);
    const auto XB = bcp<false>(r1);
    const auto F = bcp<true>(r0);
    const auto D = small<2>(norm(XB - (A + C)));
    const auto x3 = norm(F - small<2>(D));
    const auto y3 = norm(E * norm(D - x3) - small<8>(C));
    LN_SEQ();
    X = relax<LN_TV, LN_TD>(x3);
    Y = relax<LN_TV, LN_TD>(y3);
    Z = relax<LN_TV, LN_TD>(z3);
  }

  // addition step on both lanes (T + Q, Q affine): the record (l0, r, z3) at L
  __device__ __forceinline__ void add(uint32_t* L, size_t n, const uint32_t* qlds, int lane) {
    QF qx, qy;
    uint32_t* w = reinterpret_cast<uint32_t*>(&qx);
    uint32_t* w2 = reinterpret_cast<uint32_t*>(&qy);
#pragma unroll
    for (int k = 0; k < 28; k++) {
      w[k] = qlds[k * 64 + lane];
      w2[k] = qlds[(28 + k) * 64 + lane];
    }
    const auto z1z1 = sqr(Z);
    LN_SEQ();
    const auto u2 = qx * z1z1;
    LN_SEQ();
    const auto s2 = (qy * Z) * z1z1;
    LN_SEQ();
    const auto h = norm(u2 - X);
    const auto hh = sqr(h);
    LN_SEQ();
    const auto i4 = small<4>(hh);
    const auto j = h * i4;
    LN_SEQ();
    const auto r = small<2>(norm(s2 - Y));
    const auto v = X * i4;
    LN_SEQ();
    const auto x3 = norm(sqr(r) - (j + small<2>(v)));
    LN_SEQ();
    const auto y3 = norm(r * norm(v - x3) - small<2>(Y * j));
    LN_SEQ();
    const auto z3 = norm(sqr(norm(Z + h)) - (z1z1 + hh));
    LN_SEQ();
    if constexpr (SC) {  // lane 1: l2 = r (-x_P); lane 0: l0 and l3 = z3 y_P
      ml_store_q(L, n, hi ? 28 : 56, scale(sel(hi, r, z3), sel(hi, pf.nx, pf.y)));
      if (!hi) ml_store_q(L, n, 0, norm(r * qx - qy * z3));
    } else if (hi) {
      ml_store_q(L, n, 28, r);
      ml_store_q(L, n, 56, z3);
    } else {
      ml_store_q(L, n, 0, norm(r * qx - qy * z3));
    }
    X = relax<LN_TV, LN_TD>(x3);
    Y = relax<LN_TV, LN_TD>(y3);
    Z = relax<LN_TV, LN_TD>(z3);
  }
};

// The same steps with ONE lane per pair (k_miller_fused's line wave: 64 pairs per wave, so one wave keeps up with
// the two f-accumulation waves of a workgroup): every product of the step on the lane, no DPP exchange and no
// selects; the same formulas, bounds and record words as Line2.
template <bool SC = false>
struct Line1 {
  using TF = Fq2B<LN_TV, LN_TD>;
  using QF = Fq2B<1, fqb_detail::MASK>;
  TF X, Y, Z;
  PFac pf;  // SC only

  __device__ __forceinline__ void init(const G2A& q, uint32_t* qlds, int lane) {
    const QF qx = fq2b_canon(q.x), qy = fq2b_canon(q.y);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&qx);
    const uint32_t* w2 = reinterpret_cast<const uint32_t*>(&qy);
#pragma unroll
    for (int k = 0; k < 28; k++) {
      qlds[k * 64 + lane] = w[k];
      qlds[(28 + k) * 64 + lane] = w2[k];
    }
    const FqC one = fqb_canon(FP_ONE), zero{fq_zero()};
    X = relax<LN_TV, LN_TD>(qx);
    Y = relax<LN_TV, LN_TD>(qy);
    Z = relax<LN_TV, LN_TD>(QF{one, zero});
  }

  __device__ __forceinline__ void dbl(uint32_t* L, size_t n) {
    const auto A = sqr(X);
    LN_SEQ();
    const auto B = sqr(Y);
    LN_SEQ();
    const auto ZZ = sqr(Z);
    LN_SEQ();
    const auto YZ = sqr(norm(Y + Z));
    LN_SEQ();
    const auto E = small<3>(A);
    const auto z3 = norm(YZ - (B + ZZ));
    ml_store_q(L, n, 0, norm(E * X - small<2>(B)));  // l0 = E x - 2B
    LN_SEQ();
    if constexpr (SC) {
      ml_store_q(L, n, 28, scale(FqN2(E * ZZ), pf.nx));
      LN_SEQ();
      ml_store_q(L, n, 56, scale(FqN2(z3 * ZZ), pf.y));
    } else {
      ml_store_q(L, n, 28, E * ZZ);
      LN_SEQ();
      ml_store_q(L, n, 56, z3 * ZZ);
    }
    LN_SEQ();
    const auto C = sqr(B);
    LN_SEQ();
    const auto XB = sqr(norm(X + B));
    LN_SEQ();
    const auto D = small<2>(norm(XB - (A + C)));
    const auto x3 = norm(sqr(E) - small<2>(D));
    LN_SEQ();
    const auto y3 = norm(E * norm(D - x3) - small<8>(C));
    LN_SEQ();
    X = relax<LN_TV, LN_TD>(x3);
    Y = relax<LN_TV, LN_TD>(y3);
    Z = relax<LN_TV, LN_TD>(z3);
  }

  __device__ __forceinline__ void add(uint32_t* L, size_t n, const uint32_t* qlds, int lane) {
    QF qx, qy;
    uint32_t* w = reinterpret_cast<uint32_t*>(&qx);
    uint32_t* w2 = reinterpret_cast<uint32_t*>(&qy);
#pragma unroll
    for (int k = 0; k < 28; k++) {
      w[k] = qlds[k * 64 + lane];
      w2[k] = qlds[(28 + k) * 64 + lane];
    }
    const auto z1z1 = sqr(Z);
    LN_SEQ();
    const auto u2 = qx * z1z1;
    LN_SEQ();
    const auto s2 = (qy * Z) * z1z1;
    LN_SEQ();
    const auto h = norm(u2 - X);
    const auto hh = sqr(h);
    LN_SEQ();
    const auto i4 = small<4>(hh);
    const auto j = h * i4;
    LN_SEQ();
    const auto r = small<2>(norm(s2 - Y));
    const auto v = X * i4;
    LN_SEQ();
    const auto x3 = norm(sqr(r) - (j + small<2>(v)));
    LN_SEQ();
    const auto y3 = norm(r * norm(v - x3) - small<2>(Y * j));
    LN_SEQ();
    const auto z3 = norm(sqr(norm(Z + h)) - (z1z1 + hh));
    LN_SEQ();
    if constexpr (SC) {
      ml_store_q(L, n, 28, scale(r, pf.nx));
      ml_store_q(L, n, 56, scale(z3, pf.y));
    } else {
      ml_store_q(L, n, 28, r);
      ml_store_q(L, n, 56, z3);
    }
    ml_store_q(L, n, 0, norm(r * qx - qy * z3));
    X = relax<LN_TV, LN_TD>(x3);
    Y = relax<LN_TV, LN_TD>(y3);
    Z = relax<LN_TV, LN_TD>(z3);
  }
};

}  // namespace mlines
}  // namespace bls
