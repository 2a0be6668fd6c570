// Microbenchmark: throughput of the device Montgomery multiplication (fp_mul,
// bls_fp.h) vs waves per SIMD and independent chains per lane.  Run on the
// GPU box:  hipcc --offload-arch=gfx950 -O3 -I eth-consensus-specs_amd/csrc fmerate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "bls_fp.h"

using namespace bls;
#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

template <int ILP>
__global__ void __launch_bounds__(64) k_chain(Fp* out, int iters) {
  Fp x[ILP], y;
  for (int j = 0; j < 12; j++) y.l[j] = 0x01234567u * (j + 3) ^ threadIdx.x;
  y.l[11] &= 0x0fffffffu;
#pragma unroll
  for (int c = 0; c < ILP; c++) {
    for (int j = 0; j < 12; j++) x[c].l[j] = 0x9e3779b9u * (j + 1 + c) + blockIdx.x;
    x[c].l[11] &= 0x0fffffffu;
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < ILP; c++) x[c] = fp_mul(x[c], y);
  }
  Fp s = x[0];
#pragma unroll
  for (int c = 1; c < ILP; c++) s = fp_add(s, x[c]);
  out[(size_t)blockIdx.x * 64 + threadIdx.x] = s;
}

// inlined product (digits kept in registers, no call)
template <int ILP>
__global__ void __launch_bounds__(64) k_chain_inl(Fp* out, int iters) {
  Fp x[ILP], y;
  for (int j = 0; j < 12; j++) y.l[j] = 0x01234567u * (j + 3) ^ threadIdx.x;
  y.l[11] &= 0x0fffffffu;
  uint32_t yd[14];
  fp_unpack29(yd, y);
#pragma unroll
  for (int c = 0; c < ILP; c++) {
    for (int j = 0; j < 12; j++) x[c].l[j] = 0x9e3779b9u * (j + 1 + c) + blockIdx.x;
    x[c].l[11] &= 0x0fffffffu;
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < ILP; c++) {
      uint32_t xd[14];
      fp_unpack29(xd, x[c]);
      x[c] = fp_mul_digits(xd, yd);
    }
  }
  Fp s = x[0];
#pragma unroll
  for (int c = 1; c < ILP; c++) s = fp_add(s, x[c]);
  out[(size_t)blockIdx.x * 64 + threadIdx.x] = s;
}

int main() {
  Fp* d;
  CK(hipMalloc(&d, sizeof(Fp) * 64 * 65536));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct K {
    const char* name;
    void (*k)(Fp*, int);
    int ilp;
  } ks[] = {{"fp_mul call ILP1", k_chain<1>, 1},        {"fp_mul call ILP2", k_chain<2>, 2},
            {"fp_mul inline ILP1", k_chain_inl<1>, 1},  {"fp_mul inline ILP2", k_chain_inl<2>, 2},
            {"fp_mul inline ILP4", k_chain_inl<4>, 4}};
  int grids[] = {160, 512, 1024, 2048, 4096, 8192, 16384};
  for (auto& k : ks) {
    for (int g : grids) {
      int iters = 2000;
      hipLaunchKernelGGL(k.k, dim3(g), dim3(64), 0, 0, d, 4);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.k, dim3(g), dim3(64), 0, 0, d, iters);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      double fme = (double)g * 64 * iters * k.ilp;
      printf("%-22s waves=%6d (%.2f/SIMD) %9.3f ms  %7.2f G FME/s  (%.1f%% of 31.5T mad/390)\n", k.name, g,
             g / 1024.0, ms, fme / (ms * 1e-3) / 1e9, 100.0 * fme / (ms * 1e-3) / (31.5e12 / 390));
    }
  }
  return 0;
}
