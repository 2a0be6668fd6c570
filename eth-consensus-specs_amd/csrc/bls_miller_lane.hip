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
#include "bls_kernels.h"
#include "bls_tower_inline.h"

namespace bls {


// The same Miller loop in two kernels: the G2 side (doubling/addition steps of
// T and the P-independent parts of the line coefficients) and the f
// accumulation.  Each kernel holds about half of the fused kernel's live state
// (T, Q and temporaries in the first; f and one line in the second), so the
// spills of k_miller_lane go away.  Lines are stored unscaled --
// (l0, E*ZZ, z3*ZZ) for a doubling, (l0, r, z3) for an addition -- and the
// accumulation multiplies the last two by -x_P and y_P, exactly the products
// ml_dbl_i / ml_add_i do, so the Miller values stay bit-identical.
// Layout: word w of line k of pair i at L[(k * ML_WORDS + w) * n + i], so the
// 64 lanes of a wave read and write 64 consecutive words.
namespace {

constexpr int ML_WORDS = 72;  // three Fp2 of 12 limbs each

__device__ __forceinline__ void ml_store(uint32_t* L, size_t n, int w0, const Fp2& a) {
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    L[(size_t)(w0 + j) * n] = a.c0.l[j];
    L[(size_t)(w0 + 12 + j) * n] = a.c1.l[j];
  }
}
__device__ __forceinline__ Fp2 ml_load(const uint32_t* L, size_t n, int w0) {
  Fp2 a;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    a.c0.l[j] = L[(size_t)(w0 + j) * n];
    a.c1.l[j] = L[(size_t)(w0 + 12 + j) * n];
  }
  return a;
}

}  // namespace

// The G2 side with TWO lanes per pair.  A doubling step of k_miller_lines is
// 7 squarings + 4 products in Fp2 in three dependency levels; lanes 2k / 2k+1
// split each level and exchange results by DPP (quad_perm [1,0,3,2]):
//   level 1   lane 0: A = x^2, ZZ = z^2          lane 1: B = y^2, YZ = (y + z)^2
//   level 2   lane 0: C = B^2, XB = (x + B)^2,   lane 1: F = E^2, z3 ZZ, E ZZ
//                     E x  (l0 = E x - 2B)       (E = 3A, z3 = YZ - B - ZZ)
//   level 3   both: y3 = E (D - x3) - 8C         (D = 2(XB - A - C), x3 = F - 2D)
// Each lane stores the line words it formed (lane 0: l0, lane 1: E ZZ and
// z3 ZZ), so only C, XB and F cross lanes in level 2.  The five addition
// steps run on both lanes (lane 0 stores l0, lane 1 the rest).  ~15 instead of
// 26 FME per doubling and lane; the same canonical values as k_miller_lines.
namespace {
__device__ __forceinline__ uint32_t ln_swap(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ Fp2 ln_swap2(const Fp2& a) {
  Fp2 r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.l[i] = ln_swap(a.c0.l[i]);
    r.c1.l[i] = ln_swap(a.c1.l[i]);
  }
  return r;
}
__device__ __forceinline__ Fp2 ln_sel2(bool c, const Fp2& a, const Fp2& b) {
  return Fp2{fp_select(c, a.c0, b.c0), fp_select(c, a.c1, b.c1)};
}
}  // namespace

__global__ void __launch_bounds__(64) k_miller_lines2(const G2A* Q, size_t n, uint32_t* L) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = t >> 1;
  const bool hi = (t & 1) != 0;
  if (i >= n) return;  // both lanes of a pair leave together
  const G2A q = Q[i];
  if (q.inf) return;
  G2J T{q.x, q.y, fp2_one()};
  uint32_t* Li = L + i;
  const size_t step = (size_t)ML_WORDS * n;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    {
      // level 1: lane 0 squares x and z, lane 1 y and y + z
      const Fp2 s0 = f2sqr(ln_sel2(hi, T.y, T.x));
      const Fp2 s1 = f2sqr(ln_sel2(hi, f2add(T.y, T.z), T.z));
      const Fp2 o0 = ln_swap2(s0), o1 = ln_swap2(s1);
      const Fp2 A = ln_sel2(hi, o0, s0), ZZ = ln_sel2(hi, o1, s1);
      const Fp2 Bq = ln_sel2(hi, s0, o0), YZ = ln_sel2(hi, s1, o1);
      const Fp2 E = f2add(fp2_dbl(A), A);
      const Fp2 z3 = f2sub(f2sub(YZ, Bq), ZZ);
      // level 2: lane 0: C = B^2, XB = (x + B)^2, E x;  lane 1: F = E^2, E ZZ, z3 ZZ
      const Fp2 r0 = f2sqr(ln_sel2(hi, E, Bq));                        // lane 0: C;   lane 1: F
      const Fp2 xb = f2add(T.x, Bq);
      const Fp2 r1 = f2mul(ln_sel2(hi, z3, xb), ln_sel2(hi, ZZ, xb));  // lane 0: XB;  lane 1: z3 ZZ
      const Fp2 r2 = f2mul(E, ln_sel2(hi, ZZ, T.x));                   // lane 0: E x; lane 1: E ZZ
      // stores: lane 0 l0 (words 0..23), lane 1 E ZZ (24..47) and z3 ZZ (48..71)
      {
        const Fp2 w0 = ln_sel2(hi, r2, f2sub(r2, fp2_dbl(Bq)));
        uint32_t* o = Li + (size_t)(hi ? 24 : 0) * n;
#pragma unroll
        for (int j = 0; j < 12; ++j) {
          o[(size_t)j * n] = w0.c0.l[j];
          o[(size_t)(12 + j) * n] = w0.c1.l[j];
        }
        if (hi) {
#pragma unroll
          for (int j = 0; j < 12; ++j) {
            Li[(size_t)(48 + j) * n] = r1.c0.l[j];
            Li[(size_t)(60 + j) * n] = r1.c1.l[j];
          }
        }
      }
      const Fp2 p0 = ln_swap2(r0), p1 = ln_swap2(r1);
      const Fp2 C = ln_sel2(hi, p0, r0), XB = ln_sel2(hi, p1, r1), F = ln_sel2(hi, r0, p0);
      // level 3 (both lanes)
      const Fp2 D = fp2_dbl(f2sub(f2sub(XB, A), C));
      const Fp2 x3 = f2sub(F, fp2_dbl(D));
      const Fp2 C8 = fp2_dbl(fp2_dbl(fp2_dbl(C)));
      T.y = f2sub(f2mul(E, f2sub(D, x3)), C8);
      T.x = x3;
      T.z = z3;
      Li += step;
    }
    if ((X_ABS >> b) & 1ull) {  // addition step on both lanes (as k_miller_lines)
      const Fp2 z1z1 = f2sqr(T.z);
      const Fp2 u2 = f2mul(q.x, z1z1);
      const Fp2 s2 = f2mul(f2mul(q.y, T.z), z1z1);
      const Fp2 h = f2sub(u2, T.x);
      const Fp2 hh = f2sqr(h);
      const Fp2 i4 = fp2_dbl(fp2_dbl(hh));
      const Fp2 j = f2mul(h, i4);
      const Fp2 r = fp2_dbl(f2sub(s2, T.y));
      const Fp2 v = f2mul(T.x, i4);
      const Fp2 x3 = f2sub(f2sub(f2sqr(r), j), fp2_dbl(v));
      const Fp2 y3 = f2sub(f2mul(r, f2sub(v, x3)), fp2_dbl(f2mul(T.y, j)));
      const Fp2 z3 = f2sub(f2sub(f2sqr(f2add(T.z, h)), z1z1), hh);
      if (hi) {
        ml_store(Li, n, 24, r);
        ml_store(Li, n, 48, z3);
      } else {
        ml_store(Li, n, 0, f2sub(f2mul(r, q.x), f2mul(q.y, z3)));
      }
      T.x = x3;
      T.y = y3;
      T.z = z3;
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
