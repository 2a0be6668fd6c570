// Microbenchmark: issue rate of v_mad_u64_u32 and of a compiler-generated
// 381-bit CIOS Montgomery multiplication on gfx950.  Run on the GPU box.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// 8 independent accumulation chains of v_mad_u64_u32 per lane.
__global__ void __launch_bounds__(256) mad_chains(uint64_t* out, int iters, uint32_t a, uint32_t b) {
  uint64_t acc[8];
  for (int k = 0; k < 8; k++) acc[k] = threadIdx.x + k;
  uint32_t x = a + threadIdx.x, y = b ^ blockIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cc) : "v"(x), "v"(y)); }
    }
  }
  uint64_t s = 0;
  for (int k = 0; k < 8; k++) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// same, but a single dependent chain (latency)
__global__ void __launch_bounds__(256) mad_dep(uint64_t* out, int iters, uint32_t a, uint32_t b) {
  uint64_t acc = threadIdx.x;
  uint32_t x = a + threadIdx.x, y = b ^ blockIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 8; k++) { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(x), "v"(y)); }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
// plain 32-bit adds, 8 chains (full-rate reference)
__global__ void __launch_bounds__(256) add_chains(uint64_t* out, int iters, uint32_t a, uint32_t b) {
  uint32_t acc[8];
  for (int k = 0; k < 8; k++) acc[k] = threadIdx.x + k;
  uint32_t x = a + threadIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 8; k++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[k]) : "v"(x));
  }
  uint32_t s = 0;
  for (int k = 0; k < 8; k++) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) mul_lo_chains(uint64_t* out, int iters, uint32_t a, uint32_t b) {
  uint32_t acc[8];
  for (int k = 0; k < 8; k++) acc[k] = threadIdx.x + k;
  uint32_t x = a + threadIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 8; k++) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[k]) : "v"(x));
  }
  uint32_t s = 0;
  for (int k = 0; k < 8; k++) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 8 independent chains of v_mad_i64_i32 (signed 32x32+64)
__global__ void __launch_bounds__(256) madi_chains(uint64_t* out, int iters, uint32_t a, uint32_t b) {
  uint64_t acc[8];
  for (int k = 0; k < 8; k++) acc[k] = threadIdx.x + k;
  uint32_t x = a + threadIdx.x, y = b ^ blockIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      { uint64_t cc; asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cc) : "v"(x), "v"(y)); }
    }
  }
  uint64_t s = 0;
  for (int k = 0; k < 8; k++) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// 8 independent chains of v_add_co_u32 + v_addc_co_u32 (a 64-bit add as 2 ops)
__global__ void __launch_bounds__(256) addc_chains(uint64_t* out, int iters, uint32_t a, uint32_t b) {
  uint32_t lo[8], hi[8];
  for (int k = 0; k < 8; k++) { lo[k] = threadIdx.x + k; hi[k] = k; }
  uint32_t x = a + threadIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 8; k++)
      asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc" : "+v"(lo[k]), "+v"(hi[k]) : "v"(x) : "vcc");
  }
  uint32_t s = 0;
  for (int k = 0; k < 8; k++) s ^= lo[k] ^ hi[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// 8 independent v_lshl_add_u64 chains (64-bit add in one op)
__global__ void __launch_bounds__(256) add64_chains(uint64_t* out, int iters, uint32_t a, uint32_t b) {
  uint64_t acc[8];
  for (int k = 0; k < 8; k++) acc[k] = threadIdx.x + k;
  uint64_t x = a + threadIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 8; k++) asm volatile("v_lshl_add_u64 %0, %1, 0, %0" : "+v"(acc[k]) : "v"(x));
  }
  uint64_t s = 0;
  for (int k = 0; k < 8; k++) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

struct Fp { uint32_t v[12]; };
__constant__ uint32_t P[12] = {0xffffaaab,0xb9feffff,0xb153ffff,0x1eabfffe,0xf6b0f624,0x6730d2a0,0xf38512bf,0x64774b84,0x434bacd7,0x4b1ba7b6,0x397fe69a,0x1a0111ea};
#define NINV 0xfffcfffdu
__device__ __forceinline__ void mont_mul(Fp& r, const Fp& a, const Fp& b) {
  uint32_t t[14] = {0};
  #pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t c = 0;
    #pragma unroll
    for (int j = 0; j < 12; j++) {
      uint64_t x = (uint64_t)a.v[j] * b.v[i] + t[j] + c;
      t[j] = (uint32_t)x; c = x >> 32;
    }
    uint64_t s = (uint64_t)t[12] + c; t[12] = (uint32_t)s; t[13] = (uint32_t)(s >> 32);
    uint32_t m = t[0] * NINV;
    uint64_t x = (uint64_t)m * P[0] + t[0]; c = x >> 32;
    #pragma unroll
    for (int j = 1; j < 12; j++) {
      x = (uint64_t)m * P[j] + t[j] + c;
      t[j-1] = (uint32_t)x; c = x >> 32;
    }
    s = (uint64_t)t[12] + c; t[11] = (uint32_t)s; t[12] = t[13] + (uint32_t)(s >> 32);
  }
  // final sub
  uint32_t d[12]; int64_t br = 0;
  #pragma unroll
  for (int j = 0; j < 12; j++) { int64_t x = (int64_t)t[j] - P[j] + br; d[j] = (uint32_t)x; br = x >> 32; }
  bool ge = (t[12] != 0) || (br == 0);
  #pragma unroll
  for (int j = 0; j < 12; j++) r.v[j] = ge ? d[j] : t[j];
}

__global__ void __launch_bounds__(256) montmul_k(uint64_t* out, int iters, uint32_t a, uint32_t b) {
  Fp x, y;
  for (int j = 0; j < 12; j++) { x.v[j] = a * (j + 1) + threadIdx.x; y.v[j] = b * (j + 7) ^ blockIdx.x; }
  x.v[11] &= 0xfffffff; y.v[11] &= 0xfffffff;
  for (int it = 0; it < iters; it++) { mont_mul(x, x, y); }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x.v[0] ^ x.v[5];
}
int main() {
  uint64_t* d; CK(hipMalloc(&d, sizeof(uint64_t) * 4096 * 1024));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int iters = 4096;
  struct { const char* name; void (*k)(uint64_t*, int, uint32_t, uint32_t); } ks[] = {
    {"v_mad_u64_u32 x8 indep", mad_chains}, {"v_mad_u64_u32 dependent", mad_dep},
    {"v_mad_i64_i32 x8 indep", madi_chains}, {"v_add_co+addc x8 (2 ops)", addc_chains},
    {"v_lshl_add_u64 x8 indep", add64_chains},
    {"v_add_u32 x8 indep", add_chains}, {"v_mul_lo_u32 x8 indep", mul_lo_chains}, {"montmul (x8 = FME/8)", montmul_k}};
  int grids[] = {1024, 4096};
  for (auto& K : ks) {
    for (int g : grids) {
      hipLaunchKernelGGL(K.k, dim3(g), dim3(256), 0, 0, d, 16, 3u, 5u);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      int it2 = (K.k == montmul_k) ? iters / 8 : iters; hipLaunchKernelGGL(K.k, dim3(g), dim3(256), 0, 0, d, it2, 3u, 5u);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      double ops = (double)g * 256 * iters * 8; if (K.k == montmul_k) ops = (double)g*256*(iters/8);
      printf("%-28s grid=%5d  %8.3f ms  %8.2f T lane-ops/s\n", K.name, g, ms, ops / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
