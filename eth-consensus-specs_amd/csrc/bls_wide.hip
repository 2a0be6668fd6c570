// Kernels in the wavefront-cooperative form of bls_wide.h: one wave per item
// (per-call path), and the device self-test of the wide products against the
// lane form of bls_fq.h.
#include "bls_kernels.h"
#include "bls_lane.h"
#include "bls_wide.h"

namespace bls {

using namespace wide;

// Self-test: wave w takes a[4w .. 4w+4) (canonical Montgomery Fp): half h multiplies a[4w + 2h] by a[4w + 2h + 1]
// in every wide form and compares with the lane form; bad[w] = bitmask of the forms that differ.
__global__ void __launch_bounds__(64) k_wide_selftest(size_t nw, const uint8_t* be48, int* bad) {
  const size_t w = blockIdx.x;
  if (w >= nw) return;
  Fp a[4];  // test kernel: the four inputs of this wave, big-endian integers < p -> Montgomery form
#pragma unroll
  for (int k = 0; k < 4; k++) a[k] = fp_to_mont(raw_from_be48(be48 + 48 * (4 * w + k)));
  const int h = whalf();
  const WK K = wk_init();
  const Fp x = a[2 * h], y = a[2 * h + 1];
  const Fp u = a[((2 * h + 2) & 3)], v = a[((2 * h + 3) & 3)];
  const uint32_t X = w_from_fp(x), Y = w_from_fp(y), U = w_from_fp(u), V = w_from_fp(v);
  int m = 0;
  // product, square, dot2
  if (!fp_eq(w_to_fp(wmul(X, Y)), fq_pack(fq_mul(fq_unpack(x), fq_unpack(y))))) m |= 1;
  if (!fp_eq(w_to_fp(wsqr(X)), fq_pack(fq_sqr(fq_unpack(x))))) m |= 2;
  if (!fp_eq(w_to_fp(wdot2(X, Y, U, V)), fq_pack(fq_mul_dot2(fq_unpack(x), fq_unpack(y), fq_unpack(u), fq_unpack(v)))))
    m |= 4;
  // a chain: 64 products of unnormalised sums and differences (bounds of repeated use)
  uint32_t c = X;
  Fq cl = fq_unpack(x);
  for (int i = 0; i < 64; i++) {
    c = wmul(wadd(c, Y), wsub(K, c, U));
    cl = fq_mul(fq_norm(fq_add(cl, fq_unpack(y))), fq_norm(fq_sub(cl, fq_unpack(u))));
  }
  if (!fp_eq(w_to_fp(c), fq_pack(cl))) m |= 8;
  // Fp2 product and square against bls_tower_inline.h
  const W2 A{X, Y}, B{U, V};
  const Fp2 al{x, y}, bl{u, v};
  if (!fp2_eq(w2_to_fp2(w2mul(K, A, B)), f2mul(al, bl))) m |= 16;
  if (!fp2_eq(w2_to_fp2(w2sqr(K, A)), f2sqr(al))) m |= 32;
  // fixed-exponent power (the square-root exponent) against fq_pow_w3
  if (!fp_eq(w_to_fp(wpow(X, EXP_SQRT, EXP_SQRT_BITS)), fq_pack(fq_pow_w3(fq_unpack(x), EXP_SQRT, EXP_SQRT_BITS))))
    m |= 64;
  // round trip and the other half
  if (!fp_eq(w_to_fp(X), x)) m |= 128;
  if (!fp_eq(w_to_fp(wswap(X)), a[2 * (h ^ 1)])) m |= 256;
  // zero tests: x - x, and p itself in redundant digits (x + 64p - x)
  if (!w_is_zero(wsub(K, X, X))) m |= 512;
  const int mh = m;
  const int mo = __builtin_amdgcn_readlane(mh, 32);
  if (threadIdx.x == 0) bad[w] = mh | (mo << 10);
}

hipError_t launch_wide_selftest(hipStream_t st, size_t nw, const uint8_t* be48, int* bad) {
  if (!nw) return hipSuccess;
  hipLaunchKernelGGL(k_wide_selftest, dim3((unsigned)nw), dim3(64), 0, st, nw, be48, bad);
  return hipGetLastError();
}

}  // namespace bls
