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
#include "bls_miller_lines.h"

namespace bls {


// The Miller loop in two kernels: the G2 side here (doubling/addition steps of T and the P-independent parts of
// the line coefficients) and the f accumulation (k_miller_acc4q, bls_miller_pair.hip).  Lines are stored unscaled
// -- (l0, E*ZZ, z3*ZZ) for a doubling, (l0, r, z3) for an addition -- and the accumulation multiplies the last two
// by -x_P and y_P.  Layout: word w of line k of pair i at L[(k * ML_WORDS + w) * n + i] (bls_kernels.h), so the
// 64 lanes of a wave read and write consecutive words; the words are the 14 digits of bound-typed values
// FqB<ML_LV, ML_LD> (bls_fqb.h), which the accumulation multiplies without unpacking.
//
// TWO lanes per pair: the step code is mlines::Line2 (bls_miller_lines.h), shared with k_miller_fused.
__global__ void __launch_bounds__(64) k_miller_lines2(const G2A* Q, size_t n, size_t ld, uint32_t* L) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = t >> 1;
  if (i >= n) return;  // both lanes of a pair leave together
  const G2A q = Q[i];
  if (q.inf) return;
  __shared__ uint32_t qlds[56 * 64];
  mlines::Line2<> T;
  T.init(q, (t & 1) != 0, qlds, (int)threadIdx.x);
  uint32_t* Li = L + i;
  const size_t step = (size_t)ML_WORDS * ld;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    __asm__ volatile("" : "+v"(Li));  // no per-row induction pointers carried across the loop
    T.dbl(Li, ld);
    Li += step;
    if ((X_ABS >> b) & 1ull) {
      T.add(Li, ld, qlds, (int)threadIdx.x);
      Li += step;
    }
  }
}

// the leading dimension of n pairs' records: a multiple of 32 pairs, so every record row starts on a 128-B line.
// (With ld = n a row started 64 B into a line whenever n = 16 mod 32 -- a C2 batch of 10,064 pairs -- and the
// line straddling two workgroups' 32-pair spans was fetched once per XCD: FETCH 1.50x the record bytes for
// k_miller_acc4q<2>, reproduced by tools/microbench/fetchcal.hip.)
size_t miller_lines_ld(size_t n) { return (n + 31) & ~(size_t)31; }
size_t miller_lines_u32(size_t n) { return (size_t)MILLER_NLINES * ML_WORDS * miller_lines_ld(n); }

hipError_t launch_miller_lines(hipStream_t st, const G2A* Q, size_t n, uint32_t* L) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_miller_lines2, dim3((unsigned)((2 * n + 63) / 64)), dim3(64), 0, st, Q, n, miller_lines_ld(n),
                     L);
  return hipGetLastError();
}

}  // namespace bls
