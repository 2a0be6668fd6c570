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

// by-value noinline product (register calling convention, no scratch)
__device__ __noinline__ Fp fp_mul_v(Fp a, Fp b) {
  uint32_t x[14], y[14];
  fp_unpack29(x, a);
  fp_unpack29(y, b);
  return fp_mul_digits(x, y);
}

__global__ void __launch_bounds__(64) k_chain_val(Fp* out, int iters) {
  Fp x, y;
  for (int j = 0; j < 12; j++) y.l[j] = 0x01234567u * (j + 3) ^ threadIdx.x;
  y.l[11] &= 0x0fffffffu;
  for (int j = 0; j < 12; j++) x.l[j] = 0x9e3779b9u * (j + 1) + blockIdx.x;
  x.l[11] &= 0x0fffffffu;
  for (int it = 0; it < iters; it++) x = fp_mul_v(x, y);
  out[(size_t)blockIdx.x * 64 + threadIdx.x] = x;
}

// 2-lane sliced Fp2 product: lane pair (2t, 2t+1) holds (re, im); one call =
// one Fp2 product per pair = 2 Fp products per lane + operand swaps (DPP).
__device__ __forceinline__ uint32_t swap_pair(uint32_t v) {
  return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ Fp fp_swap(const Fp& a) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = swap_pair(a.l[i]);
  return r;
}
__global__ void __launch_bounds__(64) k_fp2_sliced(Fp* out, int iters) {
  Fp x, y;
  for (int j = 0; j < 12; j++) y.l[j] = 0x01234567u * (j + 3) ^ threadIdx.x;
  y.l[11] &= 0x0fffffffu;
  for (int j = 0; j < 12; j++) x.l[j] = 0x9e3779b9u * (j + 1) + blockIdx.x;
  x.l[11] &= 0x0fffffffu;
  const bool re = (threadIdx.x & 1) == 0;
  const Fp yo = fp_swap(y);
  for (int it = 0; it < iters; it++) {
    const Fp xo = fp_swap(x);
    // re: x y - x' y' ; im: x' y + x y'
    Fp u = fp_mul_v(x, re ? y : yo);
    Fp v = fp_mul_v(xo, re ? yo : y);
    x = re ? fp_sub(u, v) : fp_add(u, v);
  }
  out[(size_t)blockIdx.x * 64 + threadIdx.x] = x;
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
  } ks[] = {{"fp_mul call(ref)", k_chain<1>, 1},
            {"fp_mul inline", k_chain_inl<1>, 1},
            {"fp_mul call(value)", k_chain_val, 1},
            {"fp2 sliced (2 FME/lane)", k_fp2_sliced, 2}};
  int grids[] = {160, 512, 1024, 2048, 4096};
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
