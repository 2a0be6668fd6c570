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
#include "bls_pp_lane.h"
#include "bls_vm.h"

namespace bls {

// hf staging layout of bls_fav_kernels.hip: HCF Fd slots per item, a projective
// E2 point = 6 consecutive slots (X.c0, X.c1, Y.c0, Y.c1, Z.c0, Z.c1).

// k_sig_lane with the G2 chain on lane pairs: blocks [0, nb1) run r_i apk_i
// (one lane per item), blocks [nb1, nb1 + nb2) [|x|] sigma_i (two lanes per item).
__global__ void __launch_bounds__(64) k_sig_lane2(size_t B, const int* gstat, int* status, const int* dstat,
                                                  const G1P* apk, const G2A* sig, const uint64_t* rsc, G1P* rPj) {
  const unsigned nb1 = (unsigned)((B + 63) / 64);
  if (blockIdx.x < nb1) {  // r_i apk_i in the redundant digit form (bls_fq_g1.h), canonical output
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
  const size_t t = (size_t)(blockIdx.x - nb1) * 64 + threadIdx.x;
  const size_t i = t >> 1;
  const bool hi = (t & 1) != 0;
  if (i >= B) return;  // both lanes of an item leave together
  if (!(gstat[i] && dstat[i])) {
    if (!hi) status[i] = 0;
    return;
  }
  const G2A s = sig[i];
  PP<Fp2> M{s.x, s.y, fp2_one()};
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    M = pp2_dbl(M, hi);
    if ((X_ABS >> b) & 1ull) M = pp2_add_aff(M, s.x, s.y, hi);
  }
  // sigma in G2  <=>  psi(sigma) == -M, M not the identity: lane 0 checks x, lane 1 y
  const Fp2 pc = f2mul(fp2_conj(hi ? s.y : s.x), hi ? PSI_CY : PSI_CX);
  const Fp2 d = hi ? fp2_add(f2mul(pc, M.z), M.y) : fp2_sub(f2mul(pc, M.z), M.x);
  const uint32_t mine = fp2_is_zero(d) ? 1u : 0u;
  const bool ok = mine && cl_swap(mine) && !fp2_is_zero(M.z);
  if (!hi) status[i] = ok ? 1 : 0;
}

hipError_t launch_sig_lane(hipStream_t st, size_t B, const int* gstat, int* status, const int* dstat, const G1P* apk,
                           const G2A* sig, const uint64_t* rsc, G1P* rPj) {
  if (!B) return hipSuccess;
  hipLaunchKernelGGL(k_sig_lane2, dim3((unsigned)((B + 63) / 64 + (2 * B + 63) / 64)), dim3(64), 0, st, B, gstat,
                     status, dstat, apk, sig, rsc, rPj);
  return hipGetLastError();
}

}  // namespace bls
