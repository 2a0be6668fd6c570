// One lane per pair, inlined Miller loop (launch_miller_lane, bls_miller_lane.hip)
// versus the wave-program Miller kernels of the library.  Checks bit-equality
// with bls::miller_loop (same formulas, out-of-line tower code) and times both.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I ../../eth-consensus-specs_amd/csrc miller_lane.hip
//        -o miller_lane -L ../../eth-consensus-specs_amd -lblsmi355x -Wl,-rpath,'$ORIGIN/../../eth-consensus-specs_amd' 
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bls_kernels.h"
#include "bls_pairing.h"

namespace bls {

__global__ void k_miller_ref(const G1A* P, const G2A* Q, size_t n, Fp12* out) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i < n) out[i] = miller_loop(P[i], Q[i]);
}

__global__ void k_points(size_t n, G1A* P, G2A* Q) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const size_t k = i % 256;  // 256 distinct pairs, repeated
  P[i] = jac_to_aff(jac_mul_u64(jac_from_aff(g1_generator()), 3 + 7 * k));
  Q[i] = jac_to_aff(jac_mul_u64(jac_from_aff(g2_generator()), 5 + 11 * k));
}

}  // namespace bls

using namespace bls;

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e = (x);                                                                  \
    if (e != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 10000;
  G1A* P;
  G2A* Q;
  Fp12 *f1, *f2;
  CK(hipMalloc(&P, n * sizeof(G1A)));
  CK(hipMalloc(&Q, n * sizeof(G2A)));
  CK(hipMalloc(&f1, n * sizeof(Fp12)));
  CK(hipMalloc(&f2, n * sizeof(Fp12)));
  const unsigned g = (unsigned)((n + 63) / 64);
  hipLaunchKernelGGL(k_points, dim3(g), dim3(64), 0, 0, n, P, Q);
  CK(hipDeviceSynchronize());
  const size_t nc = n < 256 ? n : 256;
  hipLaunchKernelGGL(k_miller_ref, dim3((unsigned)((nc + 63) / 64)), dim3(64), 0, 0, P, Q, nc, f2);
  CK(launch_miller_lane(0, P, Q, nullptr, n, f1));
  CK(hipDeviceSynchronize());
  Fp12* h1 = (Fp12*)malloc(nc * sizeof(Fp12));
  Fp12* h2 = (Fp12*)malloc(nc * sizeof(Fp12));
  CK(hipMemcpy(h1, f1, nc * sizeof(Fp12), hipMemcpyDeviceToHost));
  CK(hipMemcpy(h2, f2, nc * sizeof(Fp12), hipMemcpyDeviceToHost));
  printf("lane Miller == bls::miller_loop on %zu pairs: %s\n", nc, memcmp(h1, h2, nc * sizeof(Fp12)) ? "MISMATCH" : "ok");
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float ms;
  for (int rep = 0; rep < 3; rep++) {
    CK(hipEventRecord(a, 0));
    CK(launch_miller_lane(0, P, Q, nullptr, n, f1));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("k_miller_lane   n=%zu: %.3f ms\n", n, ms);
  }
  for (int rep = 0; rep < 3; rep++) {
    CK(hipEventRecord(a, 0));
    CK(launch_miller2(0, P, Q, nullptr, n, f2));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("launch_miller2  n=%zu: %.3f ms (library VM, 2 pairs per f)\n", n, ms);
  }
  for (int rep = 0; rep < 2; rep++) {
    CK(hipEventRecord(a, 0));
    CK(launch_miller_wave(0, P, Q, nullptr, n, f2));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("launch_miller_wave n=%zu: %.3f ms (library VM, 1 pair per f)\n", n, ms);
  }
  return 0;
}
