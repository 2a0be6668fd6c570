// Microbenchmark: latency of ONE dependent chain of wide (wavefront-cooperative, bls_wide.h) Fp products on a
// single wave -- the per-call path's unit of latency -- against variants of the product, and the lane product
// (bls_fq.h) on one wave for scale.  Prints ns and shader-clock cycles per product.  Run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -I eth-consensus-specs_amd/csrc tools/microbench/widerate.hip -o /tmp/widerate
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "bls_fq.h"
#include "bls_wide.h"

using namespace bls;
using namespace bls::wide;
#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                         \
    }                                                                   \
  } while (0)

__device__ Fp seed_fp(uint32_t s) {
  Fp x;
  for (int j = 0; j < 12; j++) x.l[j] = 0x9e3779b9u * (j + 1 + s) ^ (s * 0x85ebca6bu);
  x.l[11] &= 0x0fffffffu;
  return x;
}

// ---- variant 1: column sums in two interleaved accumulators (even / odd i), so consecutive v_mad_u64_u32 do not
// depend on each other; the same for the two reduction walks
__device__ __forceinline__ void wmac2(uint64_t& a0, uint64_t& a1, uint32_t x, uint32_t y) {
  uint32_t s = wpos() < 14 ? y : 0u;
  for14([&](auto I) {
    constexpr int i = decltype(I)::value;
    if (i) s = shr1(s);
    if (i & 1)
      a1 += (uint64_t)rbc<i>(x) * s;
    else
      a0 += (uint64_t)rbc<i>(x) * s;
  });
}
__device__ __forceinline__ uint32_t wredc2(uint64_t acc) {
  const int k = wpos();
  const uint32_t t = wnorm64(acc);
  uint64_t am0 = 0, am1 = 0;
  uint32_t s = k < 14 ? t : 0u;
  for14([&](auto I) {
    constexpr int i = decltype(I)::value;
    if (i) s = shr1(s);
    if (i & 1)
      am1 += (uint64_t)NINV29[i] * s;
    else
      am0 += (uint64_t)NINV29[i] * s;
  });
  const uint32_t mn = wnorm64(am0 + am1);
  const uint32_t m = k < 14 ? mn : 0u;
  uint64_t au0 = t, au1 = 0;
  s = m;
  for14([&](auto I) {
    constexpr int i = decltype(I)::value;
    if (i) s = shr1(s);
    if (i & 1)
      au1 += (uint64_t)P29[i] * s;
    else
      au0 += (uint64_t)P29[i] * s;
  });
  const uint32_t u = wnorm64(au0 + au1);
  const uint64_t bal = __builtin_amdgcn_ballot_w64(k < 14 && u != 0u);
  const bool lowc = ((bal >> (threadIdx.x & 32u)) & 0x3fffull) != 0;
  const uint32_t u2 = u + ((k == 14 && lowc) ? 1u : 0u);
  const int j = wdig();
  const int src = (int)(threadIdx.x & 32u) + (j < 14 ? 14 + j : 31);
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)u2);
}
__device__ __forceinline__ uint32_t wmul_v1(uint32_t x, uint32_t y) {
  uint64_t a0 = 0, a1 = 0;
  wmac2(a0, a1, x, y);
  return wredc2(a0 + a1);
}

__global__ void __launch_bounds__(64) k_wmul(uint32_t* out, int iters) {
  uint32_t x = w_from_fp(seed_fp(1 + threadIdx.x / 32)), y = w_from_fp(seed_fp(7));
  for (int it = 0; it < iters; it++) x = wmul(x, y);
  out[threadIdx.x] = x;
}
__global__ void __launch_bounds__(64) k_wmul_v1(uint32_t* out, int iters) {
  uint32_t x = w_from_fp(seed_fp(1 + threadIdx.x / 32)), y = w_from_fp(seed_fp(7));
  for (int it = 0; it < iters; it++) x = wmul_v1(x, y);
  out[threadIdx.x] = x;
}
// two independent chains interleaved in one wave: time per iteration against one chain shows how much of a
// product's latency is dependency stalls that a second independent product fills
__global__ void __launch_bounds__(64) k_wmul_x2(uint32_t* out, int iters) {
  uint32_t x = w_from_fp(seed_fp(1 + threadIdx.x / 32)), z = w_from_fp(seed_fp(3)), y = w_from_fp(seed_fp(7));
  for (int it = 0; it < iters; it++) {
    x = wmul(x, y);
    z = wmul(z, y);
  }
  out[threadIdx.x] = x ^ z;
}
__global__ void __launch_bounds__(64) k_wdot2(uint32_t* out, int iters) {
  uint32_t x = w_from_fp(seed_fp(1 + threadIdx.x / 32)), z = w_from_fp(seed_fp(3)), y = w_from_fp(seed_fp(7));
  for (int it = 0; it < iters; it++) x = wdot2(x, y, z, y);
  out[threadIdx.x] = x;
}
// the pieces: the column-sum walk alone (14 steps), the reduction alone
__global__ void __launch_bounds__(64) k_wmac(uint32_t* out, int iters) {
  uint32_t x = w_from_fp(seed_fp(1 + threadIdx.x / 32)), y = w_from_fp(seed_fp(7));
  for (int it = 0; it < iters; it++) {
    uint64_t a = 0;
    wmac(a, x, y);
    x = (uint32_t)a ^ (uint32_t)(a >> 32);
  }
  out[threadIdx.x] = x;
}
__global__ void __launch_bounds__(64) k_wredc(uint32_t* out, int iters) {
  uint32_t x = w_from_fp(seed_fp(1 + threadIdx.x / 32));
  for (int it = 0; it < iters; it++) x = wredc((uint64_t)x * 0x12345u);
  out[threadIdx.x] = x;
}
__global__ void __launch_bounds__(64) k_fq(uint32_t* out, int iters) {
  Fq x = fq_unpack(seed_fp(threadIdx.x)), y = fq_unpack(seed_fp(7));
  for (int it = 0; it < iters; it++) x = fq_mul(x, y);
  out[threadIdx.x] = x.d[0] ^ x.d[13];
}

template <class K>
static float run(K k, uint32_t* d, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 16);
  hipEventRecord(a, 0);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, iters);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  uint32_t* d;
  CK(hipMalloc(&d, 4096));
  int clk = 0;
  CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));
  const double ghz = clk / 1e6;
  const int N = 20000;
  struct {
    const char* name;
    float ms;
  } r[] = {{"wmul (shipped)", run(k_wmul, d, N)},
           {"wmul v1 (two accumulators)", run(k_wmul_v1, d, N)},
           {"wmul x2 (two chains, per iter)", run(k_wmul_x2, d, N)},
           {"wdot2", run(k_wdot2, d, N)},
           {"wmac walk only", run(k_wmac, d, N)},
           {"wredc only", run(k_wredc, d, N)},
           {"fq_mul (lane form, one wave)", run(k_fq, d, N)}};
  printf("clock %.3f GHz (attribute), %d dependent products per chain, one wave\n", ghz, N);
  for (auto& x : r) printf("%-32s %8.1f ns/product  %7.0f cycles\n", x.name, x.ms * 1e6 / N, x.ms * 1e6 / N * ghz);
  return 0;
}
