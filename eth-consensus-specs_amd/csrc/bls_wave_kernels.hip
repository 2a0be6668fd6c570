// Wave-cooperative kernels: Miller loop (one 64-lane workgroup per pair) and
// final exponentiation (one workgroup), both driven by wave programs.
#include "bls_kernels.h"
#include "bls_wave.h"

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
__device__ __forceinline__ void load_fp12(Fp* dst, const Fp12* src) {
  if (threadIdx.x < 12) dst[threadIdx.x] = fp12_slot_src(*src, threadIdx.x);
  __syncthreads();
}
__device__ __forceinline__ void store_fp12(Fp12* dst, const Fp* src) {
  if (threadIdx.x < 12) fp12_slot_dst(*dst, threadIdx.x) = src[threadIdx.x];
  __syncthreads();
}

// ============================================================ Miller loop ==
constexpr int ML_F = 0, ML_T = 12, ML_P = 18, ML_Q = 20, ML_S = 24;
constexpr int ML_SCRATCH = (WP_ML_DBL_SCRATCH > WP_ML_ADD_SCRATCH ? WP_ML_DBL_SCRATCH : WP_ML_ADD_SCRATCH) >
                                   WP_ML_DBL_FIRST_SCRATCH
                               ? (WP_ML_DBL_SCRATCH > WP_ML_ADD_SCRATCH ? WP_ML_DBL_SCRATCH : WP_ML_ADD_SCRATCH)
                               : WP_ML_DBL_FIRST_SCRATCH;

__global__ void __launch_bounds__(64) k_miller_wave(const G1A* P, const G2A* Q, const int* ok, size_t n, Fp12* fout) {
  __shared__ Fp slots[ML_S + ML_SCRATCH];
  const size_t i = blockIdx.x;
  if (i >= n) return;
  const int lane = threadIdx.x;
  const bool skip = (ok && !ok[i]) || P[i].inf || Q[i].inf;
  if (skip) {
    if (lane == 0) fout[i] = fp12_one();
    return;
  }
  if (lane < 12) {
    Fp v = fp_zero();
    if (lane < 6) {
      const G2A& q = Q[i];
      const Fp2& c = lane < 2 ? q.x : (lane < 4 ? q.y : q.y);
      v = (lane & 1) ? c.c1 : c.c0;
      if (lane == 4) v = FP_ONE;
      if (lane == 5) v = fp_zero();
      slots[ML_T + lane] = v;
    } else if (lane < 8) {
      slots[ML_P + lane - 6] = lane == 6 ? fp_neg(P[i].x) : P[i].y;
    } else {
      const G2A& q = Q[i];
      const int j = lane - 8;
      const Fp2& c = j < 2 ? q.x : q.y;
      slots[ML_Q + j] = (j & 1) ? c.c1 : c.c0;
    }
  }
  __syncthreads();
  const int fb[5] = {ML_F, ML_T, ML_P, ML_Q, ML_S};
  wave_run(WAVE_PROG(ML_DBL_FIRST), slots, fb);
  if ((X_ABS >> 62) & 1ull) wave_run(WAVE_PROG(ML_ADD), slots, fb);
  for (int b = 61; b >= 0; --b) {
    wave_run(WAVE_PROG(ML_DBL), slots, fb);
    if ((X_ABS >> b) & 1ull) wave_run(WAVE_PROG(ML_ADD), slots, fb);
  }
  // x < 0: conjugate (negate the odd w-coefficients: slots 2,3,6,7,10,11)
  if (lane < 12) {
    Fp v = slots[ML_F + lane];
    if ((lane >> 1) & 1) v = fp_neg(v);
    fp12_slot_dst(fout[i], lane) = v;
  }
}

// ===================================================== final exponentiation ==
constexpr int FE_R = 6;       // 12-slot registers
constexpr int FE_SCR = WP_FP12_MUL_SCRATCH > WP_FP12_SQR_SCRATCH ? WP_FP12_MUL_SCRATCH : WP_FP12_SQR_SCRATCH;
constexpr int FE_S = 12 * FE_R;

struct FeCtx {
  Fp* s;
};

__device__ __forceinline__ void w_mul(Fp* s, int dst, int a, int b) {
  const int fb[4] = {12 * a, 12 * b, 12 * dst, FE_S};
  wave_run(WAVE_PROG(FP12_MUL), s, fb);
}
__device__ __forceinline__ void w_sqr(Fp* s, int dst, int a) {
  const int fb[3] = {12 * a, 12 * dst, FE_S};
  wave_run(WAVE_PROG(FP12_SQR), s, fb);
}
__device__ __forceinline__ void w_copy(Fp* s, int dst, int a) {
  if (threadIdx.x < 12) s[12 * dst + threadIdx.x] = s[12 * a + threadIdx.x];
  __syncthreads();
}
__device__ __forceinline__ void w_conj(Fp* s, int dst, int a) {
  if (threadIdx.x < 12) {
    Fp v = s[12 * a + threadIdx.x];
    s[12 * dst + threadIdx.x] = ((threadIdx.x >> 1) & 1) ? fp_neg(v) : v;
  }
  __syncthreads();
}
// frob2: coefficient k times gamma_{2,k} in Fp (dst != a not required)
__device__ __forceinline__ void w_frob2(Fp* s, int dst, int a) {
  Fp v;
  const int j = threadIdx.x;
  if (j < 12) {
    const int k = j >> 1;
    const Fp g = k == 0 ? FP_ONE
                        : (k == 1 ? FROB2_1.c0 : (k == 2 ? FROB2_2.c0 : (k == 3 ? FROB2_3.c0 : (k == 4 ? FROB2_4.c0 : FROB2_5.c0))));
    v = k == 0 ? s[12 * a + j] : fp_mul(s[12 * a + j], g);
  }
  __syncthreads();
  if (j < 12) s[12 * dst + j] = v;
  __syncthreads();
}
// frob1: conj(c_k) * gamma_{1,k}
__device__ __forceinline__ void w_frob1(Fp* s, int dst, int a) {
  Fp v;
  const int j = threadIdx.x;
  if (j < 12) {
    const int k = j >> 1;
    const Fp2 g = k == 0 ? fp2_one()
                         : (k == 1 ? FROB1_1 : (k == 2 ? FROB1_2 : (k == 3 ? FROB1_3 : (k == 4 ? FROB1_4 : FROB1_5))));
    const Fp ca = s[12 * a + 2 * k], cb = s[12 * a + 2 * k + 1];
    // (ca - cb i)(ga + gb i) = ca ga + cb gb + (ca gb - cb ga) i
    if ((j & 1) == 0)
      v = fp_add(fp_mul(ca, g.c0), fp_mul(cb, g.c1));
    else
      v = fp_sub(fp_mul(ca, g.c1), fp_mul(cb, g.c0));
  }
  __syncthreads();
  if (j < 12) s[12 * dst + j] = v;
  __syncthreads();
}
// dst = a^x (x = -|x|, cyclotomic: inverse = conjugate); dst != a
__device__ void w_pow_x(Fp* s, int dst, int a) {
  w_copy(s, dst, a);
  for (int b = 62; b >= 0; --b) {
    w_sqr(s, dst, dst);
    if ((X_ABS >> b) & 1ull) w_mul(s, dst, dst, a);
  }
  w_conj(s, dst, dst);
}

__global__ void __launch_bounds__(64) k_final_check_wave(const Fp12* fin, int* out) {
  __shared__ Fp s[FE_S + FE_SCR];
  __shared__ Fp12 inv;
  __shared__ int okc;
  const int lane = threadIdx.x;
  // registers: 0 = f/t, 1 = tmp, 2 = a, 3 = b, 4 = c, 5 = t3
  load_fp12(s + 0, fin);
  if (lane == 0) inv = fp12_inv(*fin);
  __syncthreads();
  load_fp12(s + 12, &inv);
  w_conj(s, 2, 0);
  w_mul(s, 0, 2, 1);  // t = conj(f) * f^-1
  w_frob2(s, 1, 0);
  w_mul(s, 0, 1, 0);  // t = t^(p^2) * t
  // a = t^((x-1)^2)
  w_pow_x(s, 1, 0);
  w_conj(s, 2, 0);
  w_mul(s, 2, 1, 2);  // a = t^(x-1)
  w_pow_x(s, 1, 2);
  w_conj(s, 3, 2);
  w_mul(s, 2, 1, 3);  // a = a^(x-1)
  // b = a^(x+p)
  w_pow_x(s, 1, 2);
  w_frob1(s, 3, 2);
  w_mul(s, 3, 1, 3);
  // c = b^(x^2+p^2-1)
  w_pow_x(s, 1, 3);
  w_pow_x(s, 4, 1);
  w_frob2(s, 1, 3);
  w_mul(s, 4, 4, 1);
  w_conj(s, 1, 3);
  w_mul(s, 4, 4, 1);
  // t^3
  w_sqr(s, 5, 0);
  w_mul(s, 5, 5, 0);
  w_mul(s, 4, 4, 5);
  if (lane == 0) okc = 1;
  __syncthreads();
  if (lane < 12) {
    const Fp v = s[48 + lane];
    const bool good = lane == 0 ? fp_is_one(v) : fp_is_zero(v);
    if (!good) okc = 0;
  }
  __syncthreads();
  if (lane == 0) *out = okc;
}

hipError_t launch_miller_wave(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, Fp12* f) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_miller_wave, dim3((unsigned)n), dim3(64), 0, st, P, Q, ok, n, f);
  return hipGetLastError();
}

hipError_t launch_final_check_wave(hipStream_t st, const Fp12* f, int* out) {
  hipLaunchKernelGGL(k_final_check_wave, dim3(1), dim3(64), 0, st, f, out);
  return hipGetLastError();
}

}  // namespace bls
