// Wave-program kernels (bls_vm.h): Miller loop (G pairs per 64-lane
// workgroup) and chunked Fp12 products.  (The final-exponentiation check is
// k_fe_check, bls_fe.hip.)
#include "bls_kernels.h"
#include "bls_vm.h"

namespace bls {

// ---- slot <-> Fp12 (w-basis order: slot 2k = Re c_k, 2k+1 = Im c_k) ----
__device__ __forceinline__ const Fp& fp12_slot_src(const Fp12& f, int j) {
  const int k = j >> 1, part = j & 1;
  const Fp6& h = (k & 1) ? f.c1 : f.c0;
  const Fp2& c = (k >> 1) == 0 ? h.c0 : ((k >> 1) == 1 ? h.c1 : h.c2);
  return part ? c.c1 : c.c0;
}
__device__ __forceinline__ Fp& fp12_slot_dst(Fp12& f, int j) {
  const int k = j >> 1, part = j & 1;
  Fp6& h = (k & 1) ? f.c1 : f.c0;
  Fp2& c = (k >> 1) == 0 ? h.c0 : ((k >> 1) == 1 ? h.c1 : h.c2);
  return part ? c.c1 : c.c0;
}

// lanes 0..11 load/store one coefficient each
__device__ __forceinline__ void load_fp12(Fd* dst, const Fp12* src) {
  if (threadIdx.x < 12) dst[threadIdx.x] = fd_from_fp(fp12_slot_src(*src, threadIdx.x));
  __syncthreads();
}

constexpr int imax(int a, int b) { return a > b ? a : b; }

// ============================================================ Miller loop ==
// Item region (WL_ML_*): f (12) | T (6) | P (2: -xP, yP) | Q (4) | scratch
constexpr int ML_G = 2;  // pairs per workgroup

template <int G>
__global__ void __launch_bounds__(64, 3) k_miller_vm(const G1A* P, const G2A* Q, const int* ok, size_t n, Fp12* fout) {
  __shared__ Fd slots[WP_NCONST + G * WL_ML_STRIDE];
  __shared__ int skip[G];
  const int lane = threadIdx.x;
  const size_t i0 = (size_t)blockIdx.x * G;
  vm_load_consts(slots);
  if (lane < G) {
    const size_t i = i0 + lane;
    skip[lane] = i >= n || (ok && !ok[i]) || P[i].inf || Q[i].inf;
  }
  __syncthreads();
  const int item0 = WP_NCONST;
  // 12 values per pair: T (x, y, 1), P (-x, y), Q (x, y)
  for (int k = lane; k < 12 * G; k += 64) {
    const int g = k / 12, j = k % 12;
    const size_t i = i0 + g;
    Fd* r = slots + item0 + g * WL_ML_STRIDE;
    Fp v = fp_zero();
    if (!skip[g]) {
      const G2A& q = Q[i];
      if (j < 4) v = (j & 1) ? (j < 2 ? q.x.c1 : q.y.c1) : (j < 2 ? q.x.c0 : q.y.c0);
      else if (j == 4) v = FP_ONE;
      else if (j == 6) v = fp_neg(P[i].x);
      else if (j == 7) v = P[i].y;
      else if (j >= 8) v = (j & 1) ? (j < 10 ? q.x.c1 : q.y.c1) : (j < 10 ? q.x.c0 : q.y.c0);
    }
    if (j < 6) r[WL_ML_T + j] = fd_from_fp(v);
    else if (j < 8) r[WL_ML_P + j - 6] = fd_from_fp(v);
    else r[WL_ML_Q + j - 8] = fd_from_fp(v);
  }
  __syncthreads();
  vm_run<G>(VM_PROG(ML_DBL_FIRST), slots, item0, WL_ML_STRIDE, nullptr);
  if ((X_ABS >> 62) & 1ull) vm_run<G>(VM_PROG(ML_ADD), slots, item0, WL_ML_STRIDE, nullptr);
  for (int b = 61; b >= 0; --b) {
    vm_run<G>(VM_PROG(ML_DBL), slots, item0, WL_ML_STRIDE, nullptr);
    if ((X_ABS >> b) & 1ull) vm_run<G>(VM_PROG(ML_ADD), slots, item0, WL_ML_STRIDE, nullptr);
  }
  // x < 0: conjugate (negate the odd w-coefficients: slots 2,3,6,7,10,11)
  for (int k = lane; k < 12 * G; k += 64) {
    const int g = k / 12, j = k % 12;
    const size_t i = i0 + g;
    if (i >= n) continue;
    Fp v = fp_from_fd(slots[item0 + g * WL_ML_STRIDE + WL_ML_F + j]);
    if ((j >> 1) & 1) v = fp_neg(v);
    if (skip[g]) v = j == 0 ? FP_ONE : fp_zero();
    fp12_slot_dst(fout[i], j) = v;
  }
}

// Products of consecutive chunks: out[b] = prod in[b*chunk .. min(n, (b+1)*chunk))
__global__ void __launch_bounds__(64) k_fp12_chunk_prod(const Fp12* in, size_t n, int chunk, Fp12* outp) {
  __shared__ Fd s[WP_NCONST + WL_CH_STRIDE];
  const size_t lo = (size_t)blockIdx.x * chunk;
  const size_t hi = lo + chunk < n ? lo + chunk : n;
  vm_load_consts(s);
  const int base = WP_NCONST;
  load_fp12(s + base, in + lo);
  for (size_t i = lo + 1; i < hi; i++) {
    load_fp12(s + base + 12, in + i);
    vm_run<1>(VM_PROG(CH_MUL), s, base, 0, nullptr);
  }
  if (threadIdx.x < 12) fp12_slot_dst(outp[blockIdx.x], threadIdx.x) = fp_from_fd(s[base + threadIdx.x]);
}

// Products of consecutive chunks of pairwise products: out[b] = prod_{i in chunk b} a[i] b[i] (the bisection
// tree's leaves, chunk = 1: an item's two Miller values, bls_capi.hip fav_bisect)
__global__ void __launch_bounds__(64) k_fp12_chunk_prod2(const Fp12* a, const Fp12* b, size_t n, int chunk,
                                                          Fp12* outp) {
  __shared__ Fd s[WP_NCONST + WL_CH_STRIDE];
  const size_t lo = (size_t)blockIdx.x * chunk;
  const size_t hi = lo + chunk < n ? lo + chunk : n;
  vm_load_consts(s);
  const int base = WP_NCONST;
  load_fp12(s + base, a + lo);
  for (size_t i = lo; i < hi; i++) {
    if (i != lo) {
      load_fp12(s + base + 12, a + i);
      vm_run<1>(VM_PROG(CH_MUL), s, base, 0, nullptr);
    }
    load_fp12(s + base + 12, b + i);
    vm_run<1>(VM_PROG(CH_MUL), s, base, 0, nullptr);
  }
  if (threadIdx.x < 12) fp12_slot_dst(outp[blockIdx.x], threadIdx.x) = fp_from_fd(s[base + threadIdx.x]);
}

// Ragged segments: out[b] = prod in[io[b] + b .. io[b + 1] + b] (inclusive).
__global__ void __launch_bounds__(64) k_fp12_seg_prod(const Fp12* in, const uint64_t* io, size_t B, Fp12* outp) {
  __shared__ Fd s[WP_NCONST + WL_CH_STRIDE];
  const size_t b = blockIdx.x;
  const size_t lo = io[b] + b, hi = io[b + 1] + b + 1;
  vm_load_consts(s);
  const int base = WP_NCONST;
  load_fp12(s + base, in + lo);
  for (size_t i = lo + 1; i < hi; i++) {
    load_fp12(s + base + 12, in + i);
    vm_run<1>(VM_PROG(CH_MUL), s, base, 0, nullptr);
  }
  if (threadIdx.x < 12) fp12_slot_dst(outp[b], threadIdx.x) = fp_from_fd(s[base + threadIdx.x]);
}

// Every Fp12 product tree runs on the final exponentiation's lane-parallel product (bls_fe.hip *_fe kernels: three
// phases over the 64 lanes per product, where the wave program keeps most lanes idle): C3 +2.8 %
// (profiles/r06v_prod_fe_ab.txt).  Knob BLS_PROD_VM = 1: the wave-program kernels of this file.
static bool prod_fe() {
  static const bool on = !(getenv("BLS_PROD_VM") && atoi(getenv("BLS_PROD_VM")) != 0);
  return on;
}

hipError_t launch_fp12_seg_prod(hipStream_t st, const Fp12* in, const uint64_t* io, size_t B, Fp12* out) {
  if (prod_fe()) return launch_fp12_seg_prod_fe(st, in, io, B, out);
  if (!B) return hipSuccess;
  hipLaunchKernelGGL(k_fp12_seg_prod, dim3((unsigned)B), dim3(64), 0, st, in, io, B, out);
  return hipGetLastError();
}

hipError_t launch_miller_wave(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, Fp12* f) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_miller_vm<ML_G>, dim3((unsigned)((n + ML_G - 1) / ML_G)), dim3(64), 0, st, P, Q, ok, n, f);
  return hipGetLastError();
}

hipError_t launch_fp12_chunk_prod(hipStream_t st, const Fp12* in, size_t n, int chunk, Fp12* out) {
  if (prod_fe()) return launch_fp12_chunk_prod_fe(st, in, n, chunk, out);
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_fp12_chunk_prod, dim3((unsigned)((n + chunk - 1) / chunk)), dim3(64), 0, st, in, n, chunk, out);
  return hipGetLastError();
}

hipError_t launch_fp12_chunk_prod2(hipStream_t st, const Fp12* a, const Fp12* b, size_t n, int chunk, Fp12* out) {
  if (prod_fe()) return launch_fp12_chunk_prod2_fe(st, a, b, n, chunk, out);
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_fp12_chunk_prod2, dim3((unsigned)((n + chunk - 1) / chunk)), dim3(64), 0, st, a, b, n, chunk,
                     out);
  return hipGetLastError();
}

// Product of n values into out[0] via chunked passes; tmp holds >= n/8 + 16 entries.
hipError_t launch_fp12_prod_vm(hipStream_t st, const Fp12* in, size_t n, Fp12* tmp, Fp12* out) {
  const Fp12* cur = in;
  Fp12* bufs[2] = {tmp, tmp + (n + 15) / 16 + 1};
  int w = 0;
  while (n > 1) {
    const int chunk = n > 64 ? 16 : (int)n;
    const size_t blocks = (n + chunk - 1) / chunk;
    Fp12* dst = blocks == 1 ? out : bufs[w];
    const hipError_t e = launch_fp12_chunk_prod(st, cur, n, chunk, dst);
    if (e != hipSuccess) return e;
    cur = dst;
    n = blocks;
    w ^= 1;
  }
  if (cur != out) return hipMemcpyAsync(out, cur, sizeof(Fp12), hipMemcpyDeviceToDevice, st);
  return hipSuccess;
}

}  // namespace bls
