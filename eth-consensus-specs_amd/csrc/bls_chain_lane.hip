// Per-item scalar-multiplication chains with one lane per item (inlined
// arithmetic, complete projective formulas of Renes-Costello-Batina for a = 0,
// the same ones the wave programs use -- tools/wavec.py rcb_dbl / rcb_add /
// rcb_add_aff).  Like the lane Miller loop (bls_miller_lane.hip), a launch of
// B items runs on B/64 SIMDs with the whole register file each, leaving the
// rest of the chip to the other streams; per item it needs several times less
// SIMD time than the 64-lane wave-program versions.
//   k_sig_lane   [|x|] sigma (G2 subgroup check psi(sigma) == -[|x|] sigma) and
//                r_i apk_i (G1, 64-bit RLC scalar), one scalar bit per step
//   k_g2x_lane   M = [|x|] B on the hash_to_G2 staging slots (cofactor clearing)
#include "bls_kernels.h"
#include "bls_fq_g1.h"
#include "bls_fq_g2.h"
#include "bls_lane.h"
#include "bls_pp_lane.h"
#include "bls_vm.h"

namespace bls {

// hf staging layout of bls_fav_kernels.hip: HCF Fd slots per item, a projective
// E2 point = 6 consecutive slots (X.c0, X.c1, Y.c0, Y.c1, Z.c0, Z.c1).

// blocks [0, nb) run r_i apk_i, blocks [nb, 2 nb) the G2 subgroup check of sigma_i, one lane per item each.
// The subgroup check runs [|x|] sigma through the Jacobian digit-form chain (bls_fq_g2.h, 16 FME per doubling on
// one lane instead of 2 x 12 on a lane pair with the complete formulas), the base point parked in LDS.  Its
// additions are incomplete, which is exact here: an exceptional step (an intermediate equal to +-sigma or the
// identity) means sigma has order below 2^64, so sigma is not in G2 (order r) and is rejected -- as is an
// identity result.
__global__ void __launch_bounds__(64) k_sig_lane2(size_t B, const int* gstat, int* status, const int* dstat,
                                                  const G1P* apk, const G2A* sig, const uint64_t* rsc, G1P* rPj) {
  __shared__ uint32_t lds[84 * 64];
  const unsigned nb = (unsigned)((B + 63) / 64);
  if (blockIdx.x < nb) {  // r_i apk_i in the redundant digit form (bls_fq_g1.h), canonical output
    const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= B || !(gstat[i] && dstat[i])) return;
    const G1P a = apk[i];
    const G1Q A{fq_unpack(a.x), fq_unpack(a.y), fq_unpack(a.z)};
    const uint64_t r = rsc[i];
    G1Q R{fq_zero(), fq_unpack(FP_ONE), fq_zero()};
    if ((r >> 63) & 1ull) R = A;
#pragma unroll 1
    for (int b = 62; b >= 0; --b) {
      R = g1q_dbl(R);
      if ((r >> b) & 1ull) R = g1q_add(R, A);
    }
    rPj[i] = G1P{fq_pack(R.x), fq_pack(R.y), fq_pack(R.z)};
    return;
  }
  const size_t i = (size_t)(blockIdx.x - nb) * 64 + threadIdx.x;
  if (i >= B) return;
  if (!(gstat[i] && dstat[i])) {
    status[i] = 0;
    return;
  }
  const G2A s = sig[i];
  bool exc = false;
  const J2Q M = j2q_mul_xabs_lds(J2Q{fq2_unpack(s.x), fq2_unpack(s.y), fq2_unpack(fp2_one())}, exc, lds);
  // sigma in G2  <=>  psi(sigma) == -[|x|] sigma:  conj(x) CX Z^2 == X,  conj(y) CY Z^3 == -Y,  Z != 0
  const Fp2 X = fq2_pack(M.x), Y = fq2_pack(M.y), Z = fq2_pack(M.z);
  const Fp2 zz = f2sqr(Z);
  const Fp2 px = f2mul(f2mul(fp2_conj(s.x), PSI_CX), zz);
  const Fp2 py = f2mul(f2mul(fp2_conj(s.y), PSI_CY), f2mul(zz, Z));
  const Fp2 dx = fp2_sub(px, X), dy = fp2_add(py, Y);
  status[i] = (!exc && !fp2_is_zero(Z) && fp2_is_zero(dx) && fp2_is_zero(dy)) ? 1 : 0;
}

// Signature decode + G2 subgroup check (bls_ops.h sig_validate semantics: the identity encoding is accepted), one
// lane per signature, inline and scratch-free: g2_decompress_lane_w (bls_lane.h) and the subgroup check of
// k_sig_lane2 (psi(sigma) == -[|x|] sigma through the Jacobian digit-form chain, an exceptional addition rejects).
// The packed-form kernel it replaces kept a 3,696-B private segment and took ~5 ms for one per-call signature.
// Signatures must be 4-byte aligned (every caller passes 96-B records of a device buffer).
__global__ void __launch_bounds__(64) k_sig_validate(const uint8_t* sigs96, size_t n, G2A* out, int* ok) {
  __shared__ uint32_t lds[84 * 64];
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  G2A s{fp2_zero(), fp2_zero(), true};
  const int st = g2_decompress_lane_w(s, sigs96 + 96 * i);
  int v = st == DEC_INFINITY ? 1 : 0;
  if (st == DEC_OK) {
    bool exc = false;
    const J2Q M = j2q_mul_xabs_lds(J2Q{fq2_unpack(s.x), fq2_unpack(s.y), fq2_unpack(fp2_one())}, exc, lds);
    const Fp2 X = fq2_pack(M.x), Y = fq2_pack(M.y), Z = fq2_pack(M.z);
    const Fp2 zz = f2sqr(Z);
    const Fp2 px = f2mul(f2mul(fp2_conj(s.x), PSI_CX), zz);
    const Fp2 py = f2mul(f2mul(fp2_conj(s.y), PSI_CY), f2mul(zz, Z));
    v = (!exc && !fp2_is_zero(Z) && fp2_is_zero(fp2_sub(px, X)) && fp2_is_zero(fp2_add(py, Y))) ? 1 : 0;
  }
  if (!v || st == DEC_INFINITY) s = G2A{fp2_zero(), fp2_zero(), true};
  out[i] = s;
  ok[i] = v;
}

hipError_t launch_sig_validate(hipStream_t st, const uint8_t* sigs, size_t n, G2A* out, int* ok) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_sig_validate, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, sigs, n, out, ok);
  return hipGetLastError();
}

hipError_t launch_sig_lane(hipStream_t st, size_t B, const int* gstat, int* status, const int* dstat, const G1P* apk,
                           const G2A* sig, const uint64_t* rsc, G1P* rPj) {
  if (!B) return hipSuccess;
  hipLaunchKernelGGL(k_sig_lane2, dim3((unsigned)(2 * ((B + 63) / 64))), dim3(64), 0, st, B, gstat,
                     status, dstat, apk, sig, rsc, rPj);
  return hipGetLastError();
}

}  // namespace bls
