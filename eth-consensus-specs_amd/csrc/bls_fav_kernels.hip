// FastAggregateVerify batch kernels, split by how the work parallelises:
//   - lane kernels (one or two lanes per item) for the long sequential
//     chains: SHA-256 expand, SSWU (square roots, inversions, Jacobi
//     symbols), signature decompression, RLC scalars;
//   - wave-program kernels (bls_vm.h, G items per 64-lane workgroup) for the
//     point arithmetic: 3-isogeny + cofactor clearing of hash_to_G2, and the
//     two per-item signature-side chains ([|x|] sigma for the subgroup check
//     and r * apk in G1) advanced together one scalar bit per step with
//     complete (exception-free) projective formulas.
#include "bls_kernels.h"
#include "bls_lane.h"
#include "bls_fq_g2.h"
#include "bls_pp_lane.h"
#include "bls_vm.h"

#include <stdlib.h>

namespace bls {

__device__ static const uint8_t DST_POP_FAV[43] = {
    'B', 'L', 'S', '_', 'S', 'I', 'G', '_', 'B', 'L', 'S', '1', '2', '3', '8', '1', 'G', '2', '_', 'X', 'M', 'D',
    ':', 'S', 'H', 'A', '-', '2', '5', '6', '_', 'S', 'S', 'W', 'U', '_', 'R', 'O', '_', 'P', 'O', 'P', '_'};

constexpr int FAV_G = 2;  // items per wave-program workgroup

// ------------------------------------------------------------ hash_to_G2 --
// (1) lane (item, t): expand_message_xmd + hash_to_field, then SSWU of u_t.
// U[8 i + 4 t ..] = (x.c0, x.c1, y.c0, y.c1) of the E2' point.
__global__ void __launch_bounds__(64) k_h2c_sswu(size_t B, const uint8_t* msgs32, const int* status, Fp* U) {
  const size_t k = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = k >> 1;
  const int t = (int)(k & 1);
  if (i >= B) return;
  if (status && !status[i]) return;
  Fp2 u[2];
  hash_to_field_fp2(u, msgs32 + 32 * i, 32, DST_POP_FAV, 43);
  Fp2 x, y;
  map_to_curve_sswu_lane(x, y, u[t]);
  Fp* o = U + 8 * i + 4 * t;
  o[0] = x.c0;
  o[1] = x.c1;
  o[2] = y.c0;
  o[3] = y.c1;
}

// Messages of any length (AggregateVerify): item i is msgs[offs[i] .. offs[i+1]).
__global__ void __launch_bounds__(64) k_h2c_sswu_var(size_t B, const uint8_t* msgs, const uint64_t* offs, Fp* U) {
  const size_t k = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = k >> 1;
  const int t = (int)(k & 1);
  if (i >= B) return;
  Fp2 u[2];
  hash_to_field_fp2(u, msgs + offs[i], (uint32_t)(offs[i + 1] - offs[i]), DST_POP_FAV, 43);
  Fp2 x, y;
  map_to_curve_sswu_lane(x, y, u[t]);
  Fp* o = U + 8 * i + 4 * t;
  o[0] = x.c0;
  o[1] = x.c1;
  o[2] = y.c0;
  o[3] = y.c1;
}

// (2) isogeny, sum, cofactor clearing and affine conversion on the VM, in
// phases (HBM staging in Fd form, 24 slots per item: Q | M | A | C):
//   k_h2c_iso    U -> Q = iso(U0) + iso(U1), flag
//   k_g2x_chain  M = [|x|] Q
//   k_h2c_pre    Q, M -> A, C  (h_eff Q = C - [|x|] A)
//   k_g2x_chain  M = [|x|] A
//   k_h2c_post   C, M -> H affine
// The [|x|] chains are 63 dependent doubling levels of 10-12 products per
// item; their own kernel has a compact layout (WL_XC: base | M | scratch) so
// 5 items share a workgroup instead of 2.
// flag[i] = 1 when an isogeny denominator vanished (the item is recomputed
// by k_h2c_fallback; unreachable for SHA-256 outputs in practice).
constexpr int HCF_Q = 0, HCF_M = 6, HCF_A = 12, HCF_C = 18;

template <int G>
__device__ __forceinline__ void hc_stage_in(Fd* s, const int* live, size_t i0, const Fd* hf, int src, int dst, int n) {
  for (int k = threadIdx.x; k < n * G; k += 64) {
    const int g = k / n, j = k % n;
    s[WP_NCONST + g * WL_HC_STRIDE + dst + j] = live[g] ? hf[HCF * (i0 + g) + src + j] : fd_zero();
  }
}
template <int G>
__device__ __forceinline__ void hc_stage_out(const Fd* s, size_t B, size_t i0, Fd* hf, int src, int dst, int n) {
  for (int k = threadIdx.x; k < n * G; k += 64) {
    const int g = k / n, j = k % n;
    if (i0 + g < B) hf[HCF * (i0 + g) + dst + j] = s[WP_NCONST + g * WL_HC_STRIDE + src + j];
  }
}
template <int G>
__device__ __forceinline__ void hc_live(int* live, size_t i0, size_t B, const int* status) {
  if (threadIdx.x < G) {
    const size_t i = i0 + threadIdx.x;
    live[threadIdx.x] = i < B && (!status || status[i]);
  }
}

template <int G>
__global__ void __launch_bounds__(64, 3) k_h2c_iso(size_t B, const int* status, const Fp* U, Fd* hf, int* flag) {
  __shared__ Fd s[WP_NCONST + G * WL_HC_STRIDE];
  __shared__ int live[G];
  const int lane = threadIdx.x;
  const size_t i0 = (size_t)blockIdx.x * G;
  hc_live<G>(live, i0, B, status);
  vm_load_consts(s);
  const int item0 = WP_NCONST;
  for (int k = lane; k < 8 * G; k += 64) {
    const int g = k >> 3, j = k & 7;
    s[item0 + g * WL_HC_STRIDE + WL_HC_U + j] = live[g] ? fd_from_fp(U[8 * (i0 + g) + j]) : fd_zero();
  }
  __syncthreads();
  vm_run<G>(VM_PROG(HC_ISO), s, item0, WL_HC_STRIDE, nullptr);
  hc_stage_out<G>(s, B, i0, hf, WL_HC_Q, HCF_Q, 6);
  if (lane < G && i0 + lane < B) {
    const Fd* r = s + item0 + lane * WL_HC_STRIDE;
    const bool bad = fd_is_zero(r[WL_HC_IZ]) && fd_is_zero(r[WL_HC_IZ + 1]);
    const bool bad2 = fd_is_zero(r[WL_HC_IZ + 2]) && fd_is_zero(r[WL_HC_IZ + 3]);
    flag[i0 + lane] = live[lane] && (bad || bad2);
  }
}

// M = [|x|] B for projective E2 points staged as Fd slots (item stride HCF).
template <int G>
__global__ void __launch_bounds__(64) k_g2x_chain(size_t B, Fd* hf, int src, int dst) {
  __shared__ Fd s[WP_NCONST + G * WL_XC_STRIDE];
  const int lane = threadIdx.x;
  const size_t i0 = (size_t)blockIdx.x * G;
  const int item0 = WP_NCONST;
  for (int k = lane; k < 6 * G; k += 64) {
    const int g = k / 6, j = k % 6;
    s[item0 + g * WL_XC_STRIDE + WL_XC_B + j] = i0 + g < B ? hf[HCF * (i0 + g) + src + j] : fd_zero();
  }
  vm_load_consts(s);  // ends with a barrier
  vm_run<G>(VM_PROG(XC_0), s, item0, WL_XC_STRIDE, nullptr);
  vm_run<G>(VM_PROG(XC_1), s, item0, WL_XC_STRIDE, nullptr);
  vm_run<G>(VM_PROG(XC_2), s, item0, WL_XC_STRIDE, nullptr);
  vm_run<G>(VM_PROG(XC_3), s, item0, WL_XC_STRIDE, nullptr);
  vm_run<G>(VM_PROG(XC_4), s, item0, WL_XC_STRIDE, nullptr);
  vm_run<G>(VM_PROG(XC_5), s, item0, WL_XC_STRIDE, nullptr);
  for (int k = lane; k < 6 * G; k += 64) {
    const int g = k / 6, j = k % 6;
    if (i0 + g < B) hf[HCF * (i0 + g) + dst + j] = s[item0 + g * WL_XC_STRIDE + WL_XC_M + j];
  }
}

template <int G>
__global__ void __launch_bounds__(64, 3) k_h2c_pre(size_t B, const int* status, Fd* hf) {
  __shared__ Fd s[WP_NCONST + G * WL_HC_STRIDE];
  __shared__ int live[G];
  const size_t i0 = (size_t)blockIdx.x * G;
  hc_live<G>(live, i0, B, status);
  vm_load_consts(s);
  hc_stage_in<G>(s, live, i0, hf, HCF_Q, WL_HC_Q, 6);
  hc_stage_in<G>(s, live, i0, hf, HCF_M, WL_HC_M, 6);
  __syncthreads();
  vm_run<G>(VM_PROG(HC_PRE), s, WP_NCONST, WL_HC_STRIDE, nullptr);
  hc_stage_out<G>(s, B, i0, hf, WL_HC_A, HCF_A, 6);
  hc_stage_out<G>(s, B, i0, hf, WL_HC_C, HCF_C, 6);
}

template <int G>
__global__ void __launch_bounds__(64, 3) k_h2c_post(size_t B, const int* status, Fd* hf) {
  __shared__ Fd s[WP_NCONST + G * WL_HC_STRIDE];
  __shared__ int live[G];
  const size_t i0 = (size_t)blockIdx.x * G;
  hc_live<G>(live, i0, B, status);
  vm_load_consts(s);
  hc_stage_in<G>(s, live, i0, hf, HCF_C, WL_HC_C, 6);
  hc_stage_in<G>(s, live, i0, hf, HCF_M, WL_HC_M, 6);
  __syncthreads();
  vm_run<G>(VM_PROG(HC_POST), s, WP_NCONST, WL_HC_STRIDE, nullptr);
  hc_stage_out<G>(s, B, i0, hf, WL_HC_H, HCF_A, 6);  // projective H over the dead A slots
}

// Affine conversion, one lane per item: 1/Z = conj(Z) / norm(Z) with one
// binary-GCD inversion.  Inversions are long per-item chains: here the 64
// lanes of a wave carry 64 items, where a VM workgroup would run them on
// only G of its lanes.
__global__ void __launch_bounds__(64) k_h2c_affine(size_t B, const int* status, const Fd* hf, G2A* H) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= B) return;
  G2A h{fp2_zero(), fp2_zero(), true};
  if (!status || status[i]) {
    const Fd* r = hf + HCF * i + HCF_A;
    const Fp2 X{fp_from_fd(r[0]), fp_from_fd(r[1])}, Y{fp_from_fd(r[2]), fp_from_fd(r[3])};
    const Fp2 Z{fp_from_fd(r[4]), fp_from_fd(r[5])};
    const Fp n = fp2_norm(Z);
    if (!fp_is_zero(n)) {
      const Fp ni = fp_inv(n);
      const Fp2 zi{fp_mul(Z.c0, ni), fp_neg(fp_mul(Z.c1, ni))};
      h = G2A{fp2_mul(X, zi), fp2_mul(Y, zi), false};
    }
  }
  H[i] = h;
}

// The fallback runs as ONE 64-lane workgroup striding over the flags (they
// are ~never set, so the loop is B / 64 flag loads).  Its hash_to_g2 call
// chain needs 6,000 B of private segment per lane, and the runtime sizes a
// hardware queue's scratch by the largest private segment it has run times
// the device's wave slots -- not by the grid.  Launched on every job's h2c
// stream, it gave each of those queues that reservation and six jobs in
// flight exhausted the scratch pool (HSA_STATUS_ERROR_OUT_OF_RESOURCES); the
// C ABI therefore runs it on one context-wide stream (bls_capi.hip).
__global__ void __launch_bounds__(64) k_h2c_fallback(size_t B, const uint8_t* msgs32, const int* flag, G2A* H) {
  for (size_t i = threadIdx.x; i < B; i += 64)
    if (flag[i]) H[i] = jac_to_aff(hash_to_g2(msgs32 + 32 * i, 32, DST_POP_FAV, 43));
}

__global__ void __launch_bounds__(64) k_h2c_fallback_var(size_t B, const uint8_t* msgs, const uint64_t* offs,
                                                         const int* flag, G2A* H) {
  for (size_t i = threadIdx.x; i < B; i += 64)
    if (flag[i]) H[i] = jac_to_aff(hash_to_g2(msgs + offs[i], (uint32_t)(offs[i + 1] - offs[i]), DST_POP_FAV, 43));
}

// ----------------------------------------------------------- signatures --
// RLC scalar r_i = first 8 bytes of SHA-256(seed || i || msg || sig), nonzero.
static __device__ uint64_t rlc_scalar_fav(const uint8_t* seed32, uint64_t i, const uint8_t* msg32,
                                          const uint8_t* sig96) {
  Sha256 sh;
  sha256_init(sh);
  sha256_update(sh, seed32, 32);
  for (int k = 0; k < 8; k++) sha256_byte(sh, (uint8_t)(i >> (8 * k)));
  sha256_update(sh, msg32, 32);
  sha256_update(sh, sig96, 96);
  uint8_t d[32];
  sha256_final(sh, d);
  uint64_t r = 0;
  for (int k = 0; k < 8; k++) r = (r << 8) | d[k];
  return r ? r : 1;
}

// (1) lane per item: signature decompression (no subgroup check yet) and the
// RLC scalar.  Independent of the registry gather, so it runs beside it.
// The identity signature can only verify against the identity key, which the
// gather rejects: it is marked invalid here.
__global__ void __launch_bounds__(64) k_sig_decode(size_t B, const uint8_t* msgs32, const uint8_t* sigs96,
                                                   const uint8_t* seed32, G2A* sig, uint64_t* rsc, int* dstat) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= B) return;
  G2A q{fp2_zero(), fp2_zero(), true};
  const int st = g2_decompress_lane(q, sigs96 + 96 * i) == DEC_OK ? 1 : 0;
  rsc[i] = st ? rlc_scalar_fav(seed32, i, msgs32 + 32 * i, sigs96 + 96 * i) : 0;
  sig[i] = q;
  dstat[i] = st;
}

// (2) the two per-item signature-side chains, 64 steps ([|x|] sigma for the
// subgroup check and r * apk), then the subgroup verdict and r * apk to
// affine.  sum r_i sigma_i is the batch MSM (bls_msm.hip).
template <int G>
__global__ void __launch_bounds__(64, 3) k_sig_vm(size_t B, const int* gstat, int* status, const int* dstat,
                                                 const G1P* apk, const G2A* sig, const uint64_t* rsc, G1P* rPj) {
  __shared__ Fd s[WP_NCONST + G * WL_SG_STRIDE];
  __shared__ int live[G];
  __shared__ uint32_t pred[G];
  const int lane = threadIdx.x;
  const size_t i0 = (size_t)blockIdx.x * G;
  vm_load_consts(s);
  uint64_t r = 0;
  if (lane < G) {
    const size_t i = i0 + lane;
    live[lane] = i < B && gstat[i] && dstat[i];
    r = live[lane] ? rsc[i] : 0;
  }
  __syncthreads();
  const int item0 = WP_NCONST;
  // sigma (4) | apk (3, projective) | M = (sigma, 1) (6) | R = (0:1:0) (3)
  for (int k = lane; k < 16 * G; k += 64) {
    const int g = k / 16, j = k % 16;
    const size_t i = i0 + g;
    Fp v = fp_zero();
    if (live[g]) {
      const G2A& q = sig[i];
      if (j < 4) v = j == 0 ? q.x.c0 : (j == 1 ? q.x.c1 : (j == 2 ? q.y.c0 : q.y.c1));
      else if (j < 7) v = j == 4 ? apk[i].x : (j == 5 ? apk[i].y : apk[i].z);
      else if (j < 11) v = j == 7 ? q.x.c0 : (j == 8 ? q.x.c1 : (j == 9 ? q.y.c0 : q.y.c1));
      else if (j == 11) v = FP_ONE;
    }
    if (j == 14) v = FP_ONE;  // Y of R
    s[item0 + g * WL_SG_STRIDE + j] = fd_from_fp(v);
  }
  __syncthreads();
  for (int b = 63; b >= 0; --b) {
    if (lane < G) pred[lane] = (uint32_t)(r >> b) & 1u;
    __syncthreads();
    if (b == 63)
      vm_run<G>(VM_PROG(SG_STEP0), s, item0, WL_SG_STRIDE, pred);
    else if ((X_ABS >> b) & 1ull)
      vm_run<G>(VM_PROG(SG_STEP2), s, item0, WL_SG_STRIDE, pred);
    else
      vm_run<G>(VM_PROG(SG_STEP1), s, item0, WL_SG_STRIDE, pred);
  }
  vm_run<G>(VM_PROG(SG_SUBCHK), s, item0, WL_SG_STRIDE, nullptr);
  if (lane < G) {
    const size_t i = i0 + lane;
    if (i < B) {
      const Fd* e = s + item0 + lane * WL_SG_STRIDE;
      bool ok = live[lane];
      // sigma in G2  <=>  psi(sigma) == -[|x|] sigma  (differences zero, M not the identity)
      for (int j = 0; j < 4; j++) ok = ok && fd_is_zero(e[WL_SG_D + j]);
      ok = ok && !(fd_is_zero(e[WL_SG_D + 4]) && fd_is_zero(e[WL_SG_D + 5]));
      rPj[i] = G1P{fp_from_fd(e[WL_SG_R]), fp_from_fd(e[WL_SG_R + 1]), fp_from_fd(e[WL_SG_R + 2])};
      status[i] = ok ? 1 : 0;
    }
  }
}

// r_i apk_i to affine, one lane per item (see k_h2c_affine).
__global__ void __launch_bounds__(64) k_g1_affine(size_t B, const int* status, const G1P* rPj, G1A* rP) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= B) return;
  G1A o{fp_zero(), fp_zero(), true};
  if (status[i]) {
    const G1P q = rPj[i];
    const Fp zi = fp_inv(q.z);
    o = G1A{fp_mul(q.x, zi), fp_mul(q.y, zi), false};
  }
  rP[i] = o;
}

// ------------------------------------------------ batched affine conversion --
// k_g1_affine / k_h2c_affine spend one inversion per item, and a 64-lane wave
// pays a whole inversion's time whether one lane or all need it.  Here each
// lane converts AFF_K items (item w * 64 AFF_K + lane + 64 k, so every load is
// coalesced) with Montgomery's trick: prefix products of the K denominators,
// ONE inversion, then two products per item walking back -- ~1/K of the
// inversions' SIMD time.  A zero denominator (identity, or a skipped item)
// enters the products as 1 and gets the same output as the one-item kernels.
constexpr int AFF_K = 8;

__global__ void __launch_bounds__(64) k_g1_affine_b(size_t B, const int* status, const G1P* rPj, G1A* rP) {
  const size_t base = (size_t)blockIdx.x * 64 * AFF_K + threadIdx.x;
  Fp pre[AFF_K];
  bool zero[AFF_K];
  Fp acc = FP_ONE;
#pragma unroll
  for (int k = 0; k < AFF_K; ++k) {
    const size_t i = base + 64 * k;
    const bool live = i < B && status[i];
    const Fp z = live ? rPj[i].z : FP_ONE;
    zero[k] = fp_is_zero(z);
    acc = fp_mul_i(acc, zero[k] ? FP_ONE : z);
    pre[k] = acc;
  }
  Fp inv = fp_inv(acc);  // 1 / (z_0 ... z_{K-1})
#pragma unroll
  for (int k = AFF_K - 1; k >= 0; --k) {
    const size_t i = base + 64 * k;
    if (i >= B) continue;
    const bool live = status[i] != 0;
    const Fp zk = live ? rPj[i].z : FP_ONE;
    const Fp zi = k ? fp_mul_i(inv, pre[k - 1]) : inv;
    if (k && !zero[k]) inv = fp_mul_i(inv, zk);
    G1A o{fp_zero(), fp_zero(), true};
    if (live) {
      const G1P q = rPj[i];
      const Fp zz = zero[k] ? fp_zero() : zi;  // fp_inv(0) = 0, as k_g1_affine
      o = G1A{fp_mul_i(q.x, zz), fp_mul_i(q.y, zz), false};
    }
    rP[i] = o;
  }
}

__global__ void __launch_bounds__(64) k_h2c_affine_b(size_t B, const int* status, const Fd* hf, G2A* H) {
  const size_t base = (size_t)blockIdx.x * 64 * AFF_K + threadIdx.x;
  Fp pre[AFF_K];
  bool zero[AFF_K];
  Fp acc = FP_ONE;
#pragma unroll
  for (int k = 0; k < AFF_K; ++k) {
    const size_t i = base + 64 * k;
    Fp n = FP_ONE;
    if (i < B && (!status || status[i])) {
      const Fd* r = hf + HCF * i + HCF_A;
      n = fp2_norm(Fp2{fp_from_fd(r[4]), fp_from_fd(r[5])});
    } else if (i < B) {
      n = fp_zero();  // skipped item: identity output
    }
    zero[k] = fp_is_zero(n);
    acc = fp_mul_i(acc, zero[k] ? FP_ONE : n);
    pre[k] = acc;
  }
  Fp inv = fp_inv(acc);
#pragma unroll
  for (int k = AFF_K - 1; k >= 0; --k) {
    const size_t i = base + 64 * k;
    if (i >= B) continue;
    const Fd* r = hf + HCF * i + HCF_A;
    const Fp2 Z{fp_from_fd(r[4]), fp_from_fd(r[5])};
    const Fp ni = k ? fp_mul_i(inv, pre[k - 1]) : inv;  // 1 / norm(Z)
    G2A h{fp2_zero(), fp2_zero(), true};
    if (!zero[k]) {
      inv = k ? fp_mul_i(inv, fp2_norm(Z)) : inv;
      const Fp2 X{fp_from_fd(r[0]), fp_from_fd(r[1])}, Y{fp_from_fd(r[2]), fp_from_fd(r[3])};
      const Fp2 zi{fp_mul_i(Z.c0, ni), fp_neg(fp_mul_i(Z.c1, ni))};
      h = G2A{f2mul(X, zi), f2mul(Y, zi), false};
    }
    H[i] = h;
  }
}

static bool affine_single() {  // A/B knob: BLS_AFF1=1 runs the one-item-per-lane affine kernels
  static const bool one = getenv("BLS_AFF1") != nullptr;
  return one;
}

// ---------------------------------------------- hash_to_G2 on lane pairs --
// The phases after SSWU as lane-pair kernels (bls_pp_lane.h pp2_*), fused with
// their neighbours; they replace the wave-program phases k_h2c_iso / _pre /
// _post (5,000-wave launches of ~25-60 products per item whose LDS staging
// and per-level barriers cost more than the arithmetic):
//   k_h2c_sswu_iso2  lane (item, t): hash_to_field, SSWU of u_t, 3-isogeny of
//                    its own point (homogeneous projective, tools/wavec.py
//                    prog_iso_pair), swap, Q = iso(P0) + iso(P1) on the pair
//   k_g2x_pre2       M = [|x|] Q, then A = psi(Q) - M and
//                    C = psi^2(2Q) - psi(Q) + M - Q      (prog_clear_pre)
//   k_g2x_post2      M = [|x|] A, then H = C - M          (prog_clear_post)
// The formulas are complete (Renes-Costello-Batina), so H is the same point
// as the wave programs' and its affine form (k_h2c_affine) is bit-identical.
// Staging is the same hf layout (HCF Fd slots per item).
namespace {

__device__ __forceinline__ PP<Fp2> pp2_swap(const PP<Fp2>& p) { return PP<Fp2>{cl_swap2(p.x), cl_swap2(p.y), cl_swap2(p.z)}; }
__device__ __forceinline__ PP<Fp2> pp2_sel(bool c, const PP<Fp2>& a, const PP<Fp2>& b) {
  return PP<Fp2>{cl_sel(c, a.x, b.x), cl_sel(c, a.y, b.y), cl_sel(c, a.z, b.z)};
}
__device__ __forceinline__ PP<Fp2> pp2_neg(const PP<Fp2>& p) { return PP<Fp2>{p.x, fp2_neg(p.y), p.z}; }
__device__ __forceinline__ PP<Fp2> pp2_psi(const PP<Fp2>& p) {
  return PP<Fp2>{f2mul(fp2_conj(p.x), PSI_CX), f2mul(fp2_conj(p.y), PSI_CY), fp2_conj(p.z)};
}
__device__ __forceinline__ PP<Fp2> pp2_psi2(const PP<Fp2>& p) {
  return PP<Fp2>{f2mul(p.x, PSI2_CX), f2mul(p.y, PSI2_CY), p.z};
}

// (x, y) affine on E2' -> iso(x, y) = (xnum yden : y ynum xden : xden yden) on E2 (RFC 9380 App. E.3)
__device__ __forceinline__ PP<Fp2> iso_proj_lane(const Fp2& x, const Fp2& y) {
  const Fp2 xx = f2sqr(x), xxx = f2mul(xx, x);
  const Fp2 xnum = fadd(fadd(f2mul(ISO_XNUM_3, xxx), f2mul(ISO_XNUM_2, xx)), fadd(f2mul(ISO_XNUM_1, x), ISO_XNUM_0));
  const Fp2 xden = fadd(fadd(xx, f2mul(ISO_XDEN_1, x)), ISO_XDEN_0);
  const Fp2 ynum = fadd(fadd(f2mul(ISO_YNUM_3, xxx), f2mul(ISO_YNUM_2, xx)), fadd(f2mul(ISO_YNUM_1, x), ISO_YNUM_0));
  const Fp2 yden = fadd(fadd(xxx, f2mul(ISO_YDEN_2, xx)), fadd(f2mul(ISO_YDEN_1, x), ISO_YDEN_0));
  return PP<Fp2>{f2mul(xnum, yden), f2mul(f2mul(y, ynum), xden), f2mul(xden, yden)};
}

// lane 0 writes X, Y.c0; lane 1 Y.c1, Z (six consecutive Fd slots)
__device__ __forceinline__ void pp2_store(Fd* o, const PP<Fp2>& p, bool hi) {
  if (!hi) {
    o[0] = fd_from_fp(p.x.c0);
    o[1] = fd_from_fp(p.x.c1);
    o[2] = fd_from_fp(p.y.c0);
  } else {
    o[3] = fd_from_fp(p.y.c1);
    o[4] = fd_from_fp(p.z.c0);
    o[5] = fd_from_fp(p.z.c1);
  }
}
__device__ __forceinline__ PP<Fp2> pp2_load(const Fd* in) {
  return PP<Fp2>{Fp2{fp_from_fd(in[0]), fp_from_fd(in[1])}, Fp2{fp_from_fd(in[2]), fp_from_fd(in[3])},
                 Fp2{fp_from_fd(in[4]), fp_from_fd(in[5])}};
}

// M = [|x|] Bp (two lanes per item; the leading bit of |x| is bit 63)
__device__ __forceinline__ PP<Fp2> pp2_mul_xabs(const PP<Fp2>& Bp, bool hi) {
  PP<Fp2> M = Bp;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    M = pp2_dbl(M, hi);
    if ((X_ABS >> b) & 1ull) M = pp2_add(M, Bp, hi);
  }
  return M;
}

}  // namespace

// msgs: 32-byte messages (offs == nullptr) or msgs[offs[i] .. offs[i+1]); status: items to skip (may be null)
__global__ void __launch_bounds__(64) k_h2c_sswu_iso2(size_t B, const uint8_t* msgs, const uint64_t* offs,
                                                      const int* status, Fd* hf, int* flag) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = t >> 1;
  const bool hi = (t & 1) != 0;
  if (i >= B) return;  // both lanes of an item leave together
  Fd* o = hf + HCF * i + HCF_Q;
  if (status && !status[i]) {
    pp2_store(o, PP<Fp2>{fp2_zero(), fp2_zero(), fp2_zero()}, hi);
    if (!hi) flag[i] = 0;
    return;
  }
  Fp2 u[2];
  if (offs)
    hash_to_field_fp2(u, msgs + offs[i], (uint32_t)(offs[i + 1] - offs[i]), DST_POP_FAV, 43);
  else
    hash_to_field_fp2(u, msgs + 32 * i, 32, DST_POP_FAV, 43);
  Fp2 x, y;
  map_to_curve_sswu_lane(x, y, hi ? u[1] : u[0]);
  const PP<Fp2> mine = iso_proj_lane(x, y);
  const PP<Fp2> other = pp2_swap(mine);
  const uint32_t bad = fp2_is_zero(mine.z) ? 1u : 0u;  // an isogeny denominator vanished: k_h2c_fallback
  const uint32_t any_bad = bad | cl_swap(bad);
  const PP<Fp2> Q = pp2_add(pp2_sel(hi, other, mine), pp2_sel(hi, mine, other), hi);
  pp2_store(o, Q, hi);
  if (!hi) flag[i] = any_bad ? 1 : 0;
}

__global__ void __launch_bounds__(64) k_g2x_pre2(size_t B, Fd* hf) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = t >> 1;
  const bool hi = (t & 1) != 0;
  if (i >= B) return;
  Fd* r = hf + HCF * i;
  const PP<Fp2> Q = pp2_load(r + HCF_Q);
  const PP<Fp2> M = pp2_mul_xabs(Q, hi);
  const PP<Fp2> pq = pp2_psi(Q);
  const PP<Fp2> A = pp2_add(pq, pp2_neg(M), hi);                       // t1 + t2, t1 = -M
  const PP<Fp2> t3 = pp2_psi2(pp2_dbl(Q, hi));                         // psi^2(2Q)
  const PP<Fp2> C = pp2_add(pp2_add(t3, pp2_neg(pq), hi), pp2_add(M, pp2_neg(Q), hi), hi);
  pp2_store(r + HCF_A, A, hi);
  pp2_store(r + HCF_C, C, hi);
}

__global__ void __launch_bounds__(64) k_g2x_post2(size_t B, Fd* hf) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = t >> 1;
  const bool hi = (t & 1) != 0;
  if (i >= B) return;
  Fd* r = hf + HCF * i;
  const PP<Fp2> M = pp2_mul_xabs(pp2_load(r + HCF_A), hi);
  const PP<Fp2> H = pp2_add(pp2_load(r + HCF_C), pp2_neg(M), hi);
  pp2_store(r + HCF_A, H, hi);  // projective H over the dead A slots (k_h2c_affine reads them)
}

// The cofactor-clearing chains on ONE lane per item in Jacobian coordinates
// (bls_pp_lane.h j2_*: 16 instead of 2 x 12 FME per doubling and item); the
// pre/post steps stay complete projective (pp_add).  An exceptional case of
// the incomplete chain additions raises flag[i], and k_h2c_fallback recomputes
// the item with the reference-path formulas.  Items with status 0 are skipped.
__device__ __forceinline__ PP<Fp2> pp_neg2(const PP<Fp2>& p) { return PP<Fp2>{p.x, fp2_neg(p.y), p.z}; }
__device__ __forceinline__ PP<Fp2> pp_psi2x(const PP<Fp2>& p) {
  return PP<Fp2>{f2mul(fp2_conj(p.x), PSI_CX), f2mul(fp2_conj(p.y), PSI_CY), fp2_conj(p.z)};
}
__device__ __forceinline__ void pp_store1(Fd* o, const PP<Fp2>& p) {
  o[0] = fd_from_fp(p.x.c0);
  o[1] = fd_from_fp(p.x.c1);
  o[2] = fd_from_fp(p.y.c0);
  o[3] = fd_from_fp(p.y.c1);
  o[4] = fd_from_fp(p.z.c0);
  o[5] = fd_from_fp(p.z.c1);
}

// [|x|] of a projective point through the digit-form Jacobian chain (bls_fq_g2.h): (X Z, Y Z^2, Z) in, (X Z, Y, Z^3)
// out, canonical packed
// (noinline: one copy for both kernels; a call per chain is nothing against its 68 steps, and inlined twice it
// doubled this file's device compile time)
__device__ __noinline__ PP<Fp2> pp_mul_xabs_q(const PP<Fp2>& P, bool& exc) {
  const Fq2 z = fq2_unpack(P.z);
  const J2Q J{fq2_mul(fq2_unpack(P.x), z), fq2_mul(fq2_unpack(P.y), fq2_sqr(z)), z};
  const J2Q M = j2q_mul_xabs(J, exc);
  return PP<Fp2>{fq2_pack(fq2_mul(M.x, M.z)), fq2_pack(M.y), fq2_pack(fq2_mul(fq2_sqr(M.z), M.z))};
}
static bool h2c_chain_packed() {  // A/B knob: BLS_H2C_PACKED=1 runs the cofactor chains on packed Fp (j2_*)
  static const bool packed = getenv("BLS_H2C_PACKED") != nullptr;
  return packed;
}

template <bool DIGITS>
__global__ void __launch_bounds__(64) k_g2x_pre1t(size_t B, const int* status, Fd* hf, int* flag) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= B || (status && !status[i])) return;
  Fd* r = hf + HCF * i;
  const PP<Fp2> Q = pp2_load(r + HCF_Q);
  bool exc = false;
  const PP<Fp2> M = DIGITS ? pp_mul_xabs_q(Q, exc) : j2_to_pp(j2_mul_xabs(j2_from_pp(Q), exc));
  const PP<Fp2> pq = pp_psi2x(Q);
  pp_store1(r + HCF_A, pp_add(pq, pp_neg2(M)));  // t1 + t2, t1 = -M
  const PP<Fp2> mq = pp_add(M, pp_neg2(Q));
  const PP<Fp2> t3{f2mul(Q.x, PSI2_CX), f2mul(Q.y, PSI2_CY), Q.z};  // psi^2(Q); psi^2(2Q) = 2 psi^2(Q)
  pp_store1(r + HCF_C, pp_add(pp_add(pp_dbl(t3), pp_neg2(pq)), mq));
  if (exc) flag[i] = 1;
}

template <bool DIGITS>
__global__ void __launch_bounds__(64) k_g2x_post1t(size_t B, const int* status, Fd* hf, int* flag) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= B || (status && !status[i])) return;
  Fd* r = hf + HCF * i;
  bool exc = false;
  const PP<Fp2> A = pp2_load(r + HCF_A);
  const PP<Fp2> M = DIGITS ? pp_mul_xabs_q(A, exc) : j2_to_pp(j2_mul_xabs(j2_from_pp(A), exc));
  pp_store1(r + HCF_A, pp_add(pp2_load(r + HCF_C), pp_neg2(M)));  // projective H over the dead A slots
  if (exc) flag[i] = 1;
}


// The same split into lean kernels: the one-lane Jacobian chain alone (its
// register budget is the chain's), and the pre/post steps on lane pairs.
__global__ void __launch_bounds__(64) k_g2x_j1(size_t B, const int* status, Fd* hf, int src, int dst, int* flag) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= B || (status && !status[i])) return;
  Fd* r = hf + HCF * i;
  bool exc = false;
  pp_store1(r + dst, j2_to_pp(j2_mul_xabs(j2_from_pp(pp2_load(r + src)), exc)));
  if (exc) flag[i] = 1;
}
__global__ void __launch_bounds__(64) k_h2c_pre_pair(size_t B, Fd* hf) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = t >> 1;
  const bool hi = (t & 1) != 0;
  if (i >= B) return;
  Fd* r = hf + HCF * i;
  const PP<Fp2> Q = pp2_load(r + HCF_Q), M = pp2_load(r + HCF_M);
  const PP<Fp2> pq = pp2_psi(Q);
  pp2_store(r + HCF_A, pp2_add(pq, pp2_neg(M), hi), hi);
  const PP<Fp2> t3 = pp2_psi2(pp2_dbl(Q, hi));
  pp2_store(r + HCF_C, pp2_add(pp2_add(t3, pp2_neg(pq), hi), pp2_add(M, pp2_neg(Q), hi), hi), hi);
}
__global__ void __launch_bounds__(64) k_h2c_post_pair(size_t B, Fd* hf) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = t >> 1;
  const bool hi = (t & 1) != 0;
  if (i >= B) return;
  Fd* r = hf + HCF * i;
  pp2_store(r + HCF_A, pp2_add(pp2_load(r + HCF_C), pp2_neg(pp2_load(r + HCF_M)), hi), hi);
}

static hipError_t launch_h2c_lane2(hipStream_t st, size_t B, const uint8_t* msgs, const uint64_t* offs,
                                   const int* status, Fd* hf, G2A* H, int* flag) {
  const dim3 g((unsigned)((2 * B + 63) / 64));
  hipLaunchKernelGGL(k_h2c_sswu_iso2, g, dim3(64), 0, st, B, msgs, offs, status, hf, flag);
  // default: one-lane Jacobian chains fused with pre/post (k_g2x_pre1t / _post1t, digit form).  A/B knobs (interleaved medians,
  // profiles/r02o_h2c_chains_ab.txt): BLS_H2C_SPLIT = one-lane chains alone + lane-pair pre/post kernels (1.465M
  // FAV/s against 1.482M), BLS_H2C_CHAIN2 = lane-pair complete-formula chains fused with pre/post (1.437M)
  static const bool pair_chains = getenv("BLS_H2C_CHAIN2") != nullptr, split = getenv("BLS_H2C_SPLIT") != nullptr;
  const dim3 g1((unsigned)((B + 63) / 64));
  if (split) {
    hipLaunchKernelGGL(k_g2x_j1, g1, dim3(64), 0, st, B, status, hf, HCF_Q, HCF_M, flag);
    hipLaunchKernelGGL(k_h2c_pre_pair, g, dim3(64), 0, st, B, hf);
    hipLaunchKernelGGL(k_g2x_j1, g1, dim3(64), 0, st, B, status, hf, HCF_A, HCF_M, flag);
    hipLaunchKernelGGL(k_h2c_post_pair, g, dim3(64), 0, st, B, hf);
  } else if (pair_chains) {
    hipLaunchKernelGGL(k_g2x_pre2, g, dim3(64), 0, st, B, hf);
    hipLaunchKernelGGL(k_g2x_post2, g, dim3(64), 0, st, B, hf);
  } else if (h2c_chain_packed()) {
    hipLaunchKernelGGL(k_g2x_pre1t<false>, g1, dim3(64), 0, st, B, status, hf, flag);
    hipLaunchKernelGGL(k_g2x_post1t<false>, g1, dim3(64), 0, st, B, status, hf, flag);
  } else {
    hipLaunchKernelGGL(k_g2x_pre1t<true>, g1, dim3(64), 0, st, B, status, hf, flag);
    hipLaunchKernelGGL(k_g2x_post1t<true>, g1, dim3(64), 0, st, B, status, hf, flag);
  }
  if (affine_single())
    hipLaunchKernelGGL(k_h2c_affine, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, st, B, status, hf, H);
  else
    hipLaunchKernelGGL(k_h2c_affine_b, dim3((unsigned)((B + 64 * AFF_K - 1) / (64 * AFF_K))), dim3(64), 0, st, B,
                       status, hf, H);
  return hipGetLastError();
}
// A/B knob: BLS_H2C_VM=1 runs SSWU + the wave-program phases (k_h2c_iso / _pre / _post)
static bool h2c_use_vm() {
  static const bool vm = getenv("BLS_H2C_VM") != nullptr;
  return vm;
}

static inline unsigned nblk(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }


static int env_int_or(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}
static int env_g(const char* name, int dflt) {
  const char* v = getenv(name);
  const int g = v ? atoi(v) : dflt;
  return (g == 2 || g == 4 || g == 6) ? g : dflt;
}

size_t h2c_scratch_fd(size_t B) { return (size_t)HCF * B; }

template <int G>
static hipError_t launch_h2c_phases(hipStream_t st, size_t B, const int* status, const Fp* U, Fd* hf, G2A* H,
                                    int* flag, int xg) {
  hipLaunchKernelGGL(k_h2c_iso<G>, dim3(nblk(B, G)), dim3(64), 0, st, B, status, U, hf, flag);
  for (int pass = 0; pass < 2; pass++) {  // M = [|x|] Q, then M = [|x|] A
    const int src = pass ? HCF_A : HCF_Q;
    if (xg == 1) {  // default: lane chains (bls_chain_lane.hip)
      hipError_t e = launch_g2x_lane(st, B, hf, src, HCF_M);
      if (e != hipSuccess) return e;
    } else if (xg == 4)
      hipLaunchKernelGGL(k_g2x_chain<4>, dim3(nblk(B, 4)), dim3(64), 0, st, B, hf, src, HCF_M);
    else if (xg == 6)
      hipLaunchKernelGGL(k_g2x_chain<6>, dim3(nblk(B, 6)), dim3(64), 0, st, B, hf, src, HCF_M);
    else
      hipLaunchKernelGGL(k_g2x_chain<5>, dim3(nblk(B, 5)), dim3(64), 0, st, B, hf, src, HCF_M);
    if (!pass) hipLaunchKernelGGL(k_h2c_pre<G>, dim3(nblk(B, G)), dim3(64), 0, st, B, status, hf);
  }
  hipLaunchKernelGGL(k_h2c_post<G>, dim3(nblk(B, G)), dim3(64), 0, st, B, status, hf);
  if (affine_single())
    hipLaunchKernelGGL(k_h2c_affine, dim3(nblk(B, 64)), dim3(64), 0, st, B, status, hf, H);
  else
    hipLaunchKernelGGL(k_h2c_affine_b, dim3(nblk(B, 64 * AFF_K)), dim3(64), 0, st, B, status, hf, H);
  return hipGetLastError();
}

hipError_t launch_h2c(hipStream_t st, size_t B, const uint8_t* msgs32, const int* status, Fp* U, Fd* hf, G2A* H,
                      int* flag) {
  if (!B) return hipSuccess;
  if (!h2c_use_vm()) return launch_h2c_lane2(st, B, msgs32, nullptr, status, hf, H, flag);
  hipLaunchKernelGGL(k_h2c_sswu, dim3(nblk(2 * B, 64)), dim3(64), 0, st, B, msgs32, status, U);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  static const int hg = env_g("BLS_H2C_G", 2);  // tuning knobs: items per workgroup
  // [|x|] chains of cofactor clearing: 1 (default) = two lanes per item (k_g2x_lane2: 1.35-1.37M FAV/s against
  // 1.33-1.35M for the 5-item wave program); 4/5/6 = wave programs with that many items per workgroup
  static const int xg = env_int_or("BLS_XC_G", 1);
  return hg == 4 ? launch_h2c_phases<4>(st, B, status, U, hf, H, flag, xg)
                 : launch_h2c_phases<2>(st, B, status, U, hf, H, flag, xg);
}

hipError_t launch_h2c_msgs(hipStream_t st, size_t B, const uint8_t* msgs, const uint64_t* offs, Fp* U, Fd* hf,
                           G2A* H, int* flag) {
  if (!B) return hipSuccess;
  if (!h2c_use_vm()) return launch_h2c_lane2(st, B, msgs, offs, nullptr, hf, H, flag);
  hipLaunchKernelGGL(k_h2c_sswu_var, dim3(nblk(2 * B, 64)), dim3(64), 0, st, B, msgs, offs, U);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_h2c_phases<2>(st, B, nullptr, U, hf, H, flag, env_int_or("BLS_XC_G", 1));
}

hipError_t launch_h2c_fallback(hipStream_t st, size_t B, const uint8_t* msgs, const uint64_t* offs, const int* flag,
                               G2A* H) {
  if (!B) return hipSuccess;
  if (offs)
    hipLaunchKernelGGL(k_h2c_fallback_var, dim3(1), dim3(64), 0, st, B, msgs, offs, flag, H);
  else
    hipLaunchKernelGGL(k_h2c_fallback, dim3(1), dim3(64), 0, st, B, msgs, flag, H);
  return hipGetLastError();
}

hipError_t launch_sig_decode(hipStream_t st, size_t B, const uint8_t* msgs32, const uint8_t* sigs96,
                             const uint8_t* seed32, G2A* sig, uint64_t* rsc, int* dstat) {
  if (!B) return hipSuccess;
  hipLaunchKernelGGL(k_sig_decode, dim3(nblk(B, 64)), dim3(64), 0, st, B, msgs32, sigs96, seed32, sig, rsc, dstat);
  return hipGetLastError();
}

hipError_t launch_sig_vm(hipStream_t st, size_t B, const int* gstat, int* status, const int* dstat,
                         const G1P* apk_aff, const G2A* sig, const uint64_t* rsc, G1P* rPj, G1A* rP) {
  if (!B) return hipSuccess;
  static const int sg = env_int_or("BLS_SIG_G", 1);  // 1: one lane per item; 2/4/6: wave programs
  if (sg == 1) {
    hipError_t e = launch_sig_lane(st, B, gstat, status, dstat, apk_aff, sig, rsc, rPj);
    if (e != hipSuccess) return e;
  } else if (sg == 4)
    hipLaunchKernelGGL(k_sig_vm<4>, dim3(nblk(B, 4)), dim3(64), 0, st, B, gstat, status, dstat, apk_aff, sig, rsc,
                       rPj);
  else if (sg == 6)
    hipLaunchKernelGGL(k_sig_vm<6>, dim3(nblk(B, 6)), dim3(64), 0, st, B, gstat, status, dstat, apk_aff, sig, rsc,
                       rPj);
  else
    hipLaunchKernelGGL(k_sig_vm<2>, dim3(nblk(B, 2)), dim3(64), 0, st, B, gstat, status, dstat, apk_aff, sig, rsc,
                       rPj);
  if (affine_single())
    hipLaunchKernelGGL(k_g1_affine, dim3(nblk(B, 64)), dim3(64), 0, st, B, status, rPj, rP);
  else
    hipLaunchKernelGGL(k_g1_affine_b, dim3(nblk(B, 64 * AFF_K)), dim3(64), 0, st, B, status, rPj, rP);
  return hipGetLastError();
}

}  // namespace bls
