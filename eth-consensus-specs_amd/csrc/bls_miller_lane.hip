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

}  // namespace bls
