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

// f_{|x|,Q}(P) conjugated (x < 0); bit-identical to miller_loop().  Skipped
// pairs (ok[i] == 0 or an identity point) give 1.
__global__ void __launch_bounds__(64) k_miller_lane(const G1A* P, const G2A* Q, const int* ok, size_t n, Fp12* out) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const G1A p = P[i];
  const G2A q = Q[i];
  if ((ok && !ok[i]) || p.inf || q.inf) {
    out[i] = fp12_one();
    return;
  }
  const Fp nxP = fp_neg(p.x);
  G2J T{q.x, q.y, fp2_one()};
  Fp12 f = fp12_one();
  Fp2 l0, l2, l3;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = f12sqr(f);
    ml_dbl_i(T, nxP, p.y, l0, l2, l3);
    f = f12line(f, l0, l2, l3);
    if ((X_ABS >> b) & 1ull) {
      ml_add_i(T, q.x, q.y, nxP, p.y, l0, l2, l3);
      f = f12line(f, l0, l2, l3);
    }
  }
  out[i] = fp12_conj(f);
}

hipError_t launch_miller_lane(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, Fp12* f) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_miller_lane, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, P, Q, ok, n, f);
  return hipGetLastError();
}


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

__global__ void __launch_bounds__(64) k_miller_lines(const G2A* Q, size_t n, uint32_t* L) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const G2A q = Q[i];
  if (q.inf) return;  // k_miller_acc skips the pair and never reads its lines
  G2J t{q.x, q.y, fp2_one()};
  uint32_t* Li = L + i;
  const size_t step = (size_t)ML_WORDS * n;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    {  // ml_dbl_i without the P factors
      const Fp2 A = f2sqr(t.x), Bq = f2sqr(t.y), C = f2sqr(Bq);
      const Fp2 D = fp2_dbl(f2sub(f2sub(f2sqr(f2add(t.x, Bq)), A), C));
      const Fp2 E = f2add(fp2_dbl(A), A);
      const Fp2 F = f2sqr(E);
      const Fp2 ZZ = f2sqr(t.z);
      ml_store(Li, n, 0, f2sub(f2mul(E, t.x), fp2_dbl(Bq)));
      ml_store(Li, n, 24, f2mul(E, ZZ));
      const Fp2 z3 = f2sub(f2sub(f2sqr(f2add(t.y, t.z)), Bq), ZZ);
      ml_store(Li, n, 48, f2mul(z3, ZZ));
      const Fp2 x3 = f2sub(F, fp2_dbl(D));
      const Fp2 C8 = fp2_dbl(fp2_dbl(fp2_dbl(C)));
      t.y = f2sub(f2mul(E, f2sub(D, x3)), C8);
      t.x = x3;
      t.z = z3;
      Li += step;
    }
    if ((X_ABS >> b) & 1ull) {  // ml_add_i without the P factors
      const Fp2 z1z1 = f2sqr(t.z);
      const Fp2 u2 = f2mul(q.x, z1z1);
      const Fp2 s2 = f2mul(f2mul(q.y, t.z), z1z1);
      const Fp2 h = f2sub(u2, t.x);
      const Fp2 hh = f2sqr(h);
      const Fp2 i4 = fp2_dbl(fp2_dbl(hh));
      const Fp2 j = f2mul(h, i4);
      const Fp2 r = fp2_dbl(f2sub(s2, t.y));
      const Fp2 v = f2mul(t.x, i4);
      const Fp2 x3 = f2sub(f2sub(f2sqr(r), j), fp2_dbl(v));
      const Fp2 y3 = f2sub(f2mul(r, f2sub(v, x3)), fp2_dbl(f2mul(t.y, j)));
      const Fp2 z3 = f2sub(f2sub(f2sqr(f2add(t.z, h)), z1z1), hh);
      ml_store(Li, n, 0, f2sub(f2mul(r, q.x), f2mul(q.y, z3)));
      ml_store(Li, n, 24, r);
      ml_store(Li, n, 48, z3);
      t.x = x3;
      t.y = y3;
      t.z = z3;
      Li += step;
    }
  }
}

__global__ void __launch_bounds__(64) k_miller_acc(const G1A* P, const G2A* Q, const int* ok, size_t n,
                                                   const uint32_t* L, Fp12* out) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const G1A p = P[i];
  if ((ok && !ok[i]) || p.inf || Q[i].inf) {
    out[i] = fp12_one();
    return;
  }
  const Fp nxP = fp_neg(p.x);
  const Fp yP = p.y;
  const uint32_t* Li = L + i;
  const size_t step = (size_t)ML_WORDS * n;
  Fp12 f = fp12_one();
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = f12sqr(f);
    // keep the line loads after the squaring: hoisted above it they hold 72
    // registers through the squaring's Fp6 temporaries and push f to scratch
    asm volatile("" ::: "memory");
    f = f12line(f, ml_load(Li, n, 0), f2mulfp(ml_load(Li, n, 24), nxP), f2mulfp(ml_load(Li, n, 48), yP));
    Li += step;
    if ((X_ABS >> b) & 1ull) {
      asm volatile("" ::: "memory");
      f = f12line(f, ml_load(Li, n, 0), f2mulfp(ml_load(Li, n, 24), nxP), f2mulfp(ml_load(Li, n, 48), yP));
      Li += step;
    }
  }
  out[i] = fp12_conj(f);
}

size_t miller_lines_u32(size_t n) { return (size_t)MILLER_NLINES * ML_WORDS * n; }

hipError_t launch_miller_lines(hipStream_t st, const G2A* Q, size_t n, uint32_t* L) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_miller_lines, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, Q, n, L);
  return hipGetLastError();
}

hipError_t launch_miller_acc(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, const uint32_t* L,
                             Fp12* f) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_miller_acc, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, P, Q, ok, n, L, f);
  return hipGetLastError();
}

}  // namespace bls
