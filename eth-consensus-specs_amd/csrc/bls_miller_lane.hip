// Miller loop with one lane per pair (SURVEY.md §8(a) internal piece (6)).
//
// The wave-program Miller kernels (bls_wave_kernels.hip) spread one pair's
// step over the 64 lanes of a workgroup; their operand linear combinations,
// LDS traffic and per-level barriers cost more than the products themselves.
// Here each lane runs a whole pair with inlined arithmetic.  The kernel needs
// the full register file (512 VGPR+AGPR, one wave per SIMD) and spills some
// to scratch, so a launch of B pairs occupies only B/64 SIMDs -- for a
// 10,000-pair batch about 15 % of the chip for ~11 ms -- and the rest of the
// GPU runs the other streams' kernels.  Per pair it is ~4.5x less SIMD time
// than the wave-program version (tools/microbench/miller_lane.hip).
#include "bls_fqb.h"
#include "bls_kernels.h"
#include "bls_tower_inline.h"

namespace bls {


// The Miller loop in two kernels: the G2 side here (doubling/addition steps of T and the P-independent parts of
// the line coefficients) and the f accumulation (k_miller_acc4q, bls_miller_pair.hip).  Lines are stored unscaled
// -- (l0, E*ZZ, z3*ZZ) for a doubling, (l0, r, z3) for an addition -- and the accumulation multiplies the last two
// by -x_P and y_P.  Layout: word w of line k of pair i at L[(k * ML_WORDS + w) * n + i] (bls_kernels.h), so the
// 64 lanes of a wave read and write consecutive words; the words are the 14 digits of bound-typed values
// FqB<ML_LV, ML_LD> (bls_fqb.h), which the accumulation multiplies without unpacking.
//
// TWO lanes per pair.  A doubling step is 7 squarings + 4 products in Fp2 in three dependency levels; lanes
// 2k / 2k+1 split each level and broadcast results by DPP:
//   level 1   lane 0: A = x^2, ZZ = z^2          lane 1: B = y^2, YZ = (y + z)^2
//   level 2   lane 0: C = B^2, XB = (x + B)^2,   lane 1: F = E^2, z3 ZZ, E ZZ
//                     E x  (l0 = E x - 2B)       (E = 3A, z3 = YZ - B - ZZ)
//   level 3   both: y3 = E (D - x3) - 8C         (D = 2(XB - A - C), x3 = F - 2D)
// Each lane stores the line words it formed (lane 0: l0, lane 1: E ZZ and z3 ZZ).  The five addition steps run on
// both lanes (lane 0 stores l0, lane 1 the rest).  T stays in the bound-typed digit form for the whole loop
// (declared FqB<LN_TV, LN_TD>; every step is relaxed to it, so its bounds are checked by induction at compile
// time): no product unpacks or repacks, additions are digit-wise (the packed kernel: 12-limb carry chains and a
// conditional subtraction per addition and per product).
// products one after another (interleaved, their digit columns spilled ~140 VGPRs)
#define LN_SEQ() __builtin_amdgcn_sched_barrier(0)
namespace {
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
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    L[(size_t)(w0 + j) * n] = a.c0.x.d[j];
    L[(size_t)(w0 + 14 + j) * n] = a.c1.x.d[j];
  }
}
}  // namespace

__global__ void __launch_bounds__(64) k_miller_lines2(const G2A* Q, size_t n, uint32_t* L) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = t >> 1;
  const bool hi = (t & 1) != 0;
  if (i >= n) return;  // both lanes of a pair leave together
  const G2A q = Q[i];
  if (q.inf) return;
  using TF = Fq2B<LN_TV, LN_TD>;
  using QF = Fq2B<1, fqb_detail::MASK>;
  // Q's coordinates wait in LDS ([word][lane]) for the five addition steps: held in registers across the 63
  // doublings they pushed the kernel into spills
  __shared__ uint32_t qlds[56 * 64];
  {
    const QF qx = fq2b_canon(q.x), qy = fq2b_canon(q.y);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&qx);
    const uint32_t* w2 = reinterpret_cast<const uint32_t*>(&qy);
#pragma unroll
    for (int k = 0; k < 28; k++) {
      qlds[k * 64 + threadIdx.x] = w[k];
      qlds[(28 + k) * 64 + threadIdx.x] = w2[k];
    }
  }
  const FqC one = fqb_canon(FP_ONE), zero{fq_zero()};
  TF X = relax<LN_TV, LN_TD>(fq2b_canon(q.x)), Y = relax<LN_TV, LN_TD>(fq2b_canon(q.y));
  TF Z = relax<LN_TV, LN_TD>(QF{one, zero});
  uint32_t* Li = L + i;
  const size_t step = (size_t)ML_WORDS * n;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    {
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
      ml_store_q(Li, n, hi ? 28 : 0, sel(hi, r2, norm(r2 - small<2>(Bq))));  // lane 0: l0 = E x - 2B
      LN_SEQ();
      if (hi) ml_store_q(Li, n, 56, r1);
      LN_SEQ();
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
      Li += step;
    }
    if ((X_ABS >> b) & 1ull) {  // addition step on both lanes (T + Q, Q affine)
      QF qx, qy;
      uint32_t* w = reinterpret_cast<uint32_t*>(&qx);
      uint32_t* w2 = reinterpret_cast<uint32_t*>(&qy);
#pragma unroll
      for (int k = 0; k < 28; k++) {
        w[k] = qlds[k * 64 + threadIdx.x];
        w2[k] = qlds[(28 + k) * 64 + threadIdx.x];
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
      if (hi) {
        ml_store_q(Li, n, 28, r);
        ml_store_q(Li, n, 56, z3);
      } else {
        ml_store_q(Li, n, 0, norm(r * qx - qy * z3));
      }
      X = relax<LN_TV, LN_TD>(x3);
      Y = relax<LN_TV, LN_TD>(y3);
      Z = relax<LN_TV, LN_TD>(z3);
      Li += step;
    }
  }
}

size_t miller_lines_u32(size_t n) { return (size_t)MILLER_NLINES * ML_WORDS * n; }

hipError_t launch_miller_lines(hipStream_t st, const G2A* Q, size_t n, uint32_t* L) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_miller_lines2, dim3((unsigned)((2 * n + 63) / 64)), dim3(64), 0, st, Q, n, L);
  return hipGetLastError();
}

}  // namespace bls
