// Microbenchmark: packed Fp (bls_fp.h, radix-2^29 products on 12-limb
// operands) against the redundant digit form Fq (bls_fq.h), one dependent
// chain per lane, for a lone product and for the Karatsuba Fp2 product with
// its subtractions.  (profiles/r02l_fqrate_microbench.txt was measured with
// the first, radix-2^28 version of Fq; the product has the same shape.)  Run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -I eth-consensus-specs_amd/csrc tools/microbench/fqrate.hip -o /tmp/fqrate
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "bls_fq.h"
#include "bls_tower_inline.h"

using namespace bls;
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

__global__ void __launch_bounds__(64) k_fp(uint32_t* out, int iters) {
  Fp x = seed_fp(blockIdx.x * 64 + threadIdx.x), y = seed_fp(7);
  for (int it = 0; it < iters; it++) x = fp_mul_i(x, y);
  out[(size_t)blockIdx.x * 64 + threadIdx.x] = x.l[0] ^ x.l[11];
}
__global__ void __launch_bounds__(64) k_fq(uint32_t* out, int iters) {
  Fq x = fq_unpack(seed_fp(blockIdx.x * 64 + threadIdx.x)), y = fq_unpack(seed_fp(7));
  for (int it = 0; it < iters; it++) x = fq_mul(x, y);
  out[(size_t)blockIdx.x * 64 + threadIdx.x] = x.d[0] ^ x.d[13];
}
__global__ void __launch_bounds__(64) k_fp2(uint32_t* out, int iters) {
  Fp2 x{seed_fp(blockIdx.x * 64 + threadIdx.x), seed_fp(3)}, y{seed_fp(7), seed_fp(9)};
  for (int it = 0; it < iters; it++) x = f2mul(x, y);
  out[(size_t)blockIdx.x * 64 + threadIdx.x] = x.c0.l[0] ^ x.c1.l[11];
}
__global__ void __launch_bounds__(64) k_fq2(uint32_t* out, int iters) {
  Fq2 x{fq_unpack(seed_fp(blockIdx.x * 64 + threadIdx.x)), fq_unpack(seed_fp(3))};
  const Fq2 y{fq_unpack(seed_fp(7)), fq_unpack(seed_fp(9))};
  for (int it = 0; it < iters; it++) {
    const Fq t0 = fq_mul(x.c0, y.c0), t1 = fq_mul(x.c1, y.c1);
    const Fq t2 = fq_mul(fq_add(x.c0, x.c1), fq_add(y.c0, y.c1));
    x = Fq2{fq_norm(fq_sub(t0, t1)), fq_norm(fq_sub2(t2, fq_add(t0, t1)))};
  }
  out[(size_t)blockIdx.x * 64 + threadIdx.x] = x.c0.d[0] ^ x.c1.d[13];
}

int main() {
  uint32_t* d;
  CK(hipMalloc(&d, sizeof(uint32_t) * 64 * 65536));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct K {
    const char* name;
    void (*k)(uint32_t*, int);
    int fme;
  } ks[] = {{"Fp  product (packed)", k_fp, 1}, {"Fq  product (digit form)", k_fq, 1},
            {"Fp2 Karatsuba (packed)", k_fp2, 3}, {"Fq2 Karatsuba + norm", k_fq2, 3}};
  int grids[] = {1024, 2048, 4096};
  for (auto& k : ks) {
    for (int g : grids) {
      int iters = 1000;
      hipLaunchKernelGGL(k.k, dim3(g), dim3(64), 0, 0, d, 4);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.k, dim3(g), dim3(64), 0, 0, d, iters);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      double fme = (double)g * 64 * iters * k.fme;
      printf("%-26s waves=%5d (%.1f/SIMD) %8.3f ms %7.2f G FME/s (%.1f%% of 39.3T / 288)\n", k.name, g, g / 1024.0,
             ms, fme / (ms * 1e-3) / 1e9, 100.0 * fme / (ms * 1e-3) / (39.32e12 / 288));
    }
  }
  return 0;
}
