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

// Two independent chains per item, run by DIFFERENT waves (a wave-uniform
// branch on blockIdx, so no lane diverges): blocks [0, nb) walk r_i apk_i in
// G1, blocks [nb, 2 nb) walk [|x|] sigma_i in G2 and write the verdict.  Each
// wave holds one chain's state instead of both, which keeps the G2 chain's
// wave free of spills, and the launch is twice the waves.
// gstat: the gather's per-item status (read-only here: the MSM on another
// stream reads it concurrently); status: this kernel's verdict.
__global__ void __launch_bounds__(64) k_sig_lane(size_t B, const int* gstat, int* status, const int* dstat,
                                                 const G1P* apk, const G2A* sig, const uint64_t* rsc, G1P* rPj) {
  const unsigned nb = (unsigned)((B + 63) / 64);
  const bool g2 = blockIdx.x >= nb;
  const size_t i = (size_t)(g2 ? blockIdx.x - nb : blockIdx.x) * 64 + threadIdx.x;
  if (i >= B) return;
  const bool live = gstat[i] && dstat[i];
  if (!g2) {  // r * apk: double-and-add from bit 63 (R = identity (0 : 1 : 0) before)
    if (!live) return;
    const G1P a = apk[i];
    const PP<Fp> A{a.x, a.y, a.z};
    const uint64_t r = rsc[i];
    PP<Fp> R{fp_zero(), FP_ONE, fp_zero()};
    if ((r >> 63) & 1ull) R = A;
#pragma unroll 1
    for (int b = 62; b >= 0; --b) {
      R = pp_dbl(R);
      if ((r >> b) & 1ull) R = pp_add(R, A);
    }
    rPj[i] = G1P{R.x, R.y, R.z};
    return;
  }
  if (!live) {
    status[i] = 0;
    return;
  }
  // [|x|] sigma: the leading bit of |x| is bit 63
  const G2A s = sig[i];
  PP<Fp2> M{s.x, s.y, fp2_one()};
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    M = pp_dbl(M);
    if ((X_ABS >> b) & 1ull) M = pp_add_aff(M, s.x, s.y);
  }
  // sigma in G2  <=>  psi(sigma) == -M with M not the identity; psi(sigma) = (conj(x) cx : conj(y) cy : 1)
  const Fp2 px = f2mul(fp2_conj(s.x), PSI_CX), py = f2mul(fp2_conj(s.y), PSI_CY);
  const Fp2 dx = fp2_sub(f2mul(px, M.z), M.x);
  const Fp2 dy = fp2_add(f2mul(py, M.z), M.y);
  const bool ok = fp2_is_zero(dx) && fp2_is_zero(dy) && !fp2_is_zero(M.z);
  status[i] = ok ? 1 : 0;
}

// hf staging layout of bls_fav_kernels.hip: HCF Fd slots per item, a projective
// E2 point = 6 consecutive slots (X.c0, X.c1, Y.c0, Y.c1, Z.c0, Z.c1).

__global__ void __launch_bounds__(64) k_g2x_lane(size_t B, Fd* hf, int src, int dst) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= B) return;
  const Fd* in = hf + HCF * i + src;
  const PP<Fp2> Bp{Fp2{fp_from_fd(in[0]), fp_from_fd(in[1])}, Fp2{fp_from_fd(in[2]), fp_from_fd(in[3])},
                   Fp2{fp_from_fd(in[4]), fp_from_fd(in[5])}};
  PP<Fp2> M = Bp;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    M = pp_dbl(M);
    if ((X_ABS >> b) & 1ull) M = pp_add(M, Bp);
  }
  Fd* o = hf + HCF * i + dst;
  o[0] = fd_from_fp(M.x.c0);
  o[1] = fd_from_fp(M.x.c1);
  o[2] = fd_from_fp(M.y.c0);
  o[3] = fd_from_fp(M.y.c1);
  o[4] = fd_from_fp(M.z.c0);
  o[5] = fd_from_fp(M.z.c1);
}

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

// M = [|x|] B on the hash_to_G2 staging slots, two lanes per item
__global__ void __launch_bounds__(64) k_g2x_lane2(size_t B, Fd* hf, int src, int dst) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = t >> 1;
  const bool hi = (t & 1) != 0;
  if (i >= B) return;
  const Fd* in = hf + HCF * i + src;
  const PP<Fp2> Bp{Fp2{fp_from_fd(in[0]), fp_from_fd(in[1])}, Fp2{fp_from_fd(in[2]), fp_from_fd(in[3])},
                   Fp2{fp_from_fd(in[4]), fp_from_fd(in[5])}};
  PP<Fp2> M = Bp;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    M = pp2_dbl(M, hi);
    if ((X_ABS >> b) & 1ull) M = pp2_add(M, Bp, hi);
  }
  Fd* o = hf + HCF * i + dst;
  if (!hi) {  // lane 0 writes X and Y.c0, lane 1 Y.c1 and Z
    o[0] = fd_from_fp(M.x.c0);
    o[1] = fd_from_fp(M.x.c1);
    o[2] = fd_from_fp(M.y.c0);
  } else {
    o[3] = fd_from_fp(M.y.c1);
    o[4] = fd_from_fp(M.z.c0);
    o[5] = fd_from_fp(M.z.c1);
  }
}

// k_sig_lane with the G2 chain on ONE lane per item in Jacobian coordinates
// (bls_pp_lane.h j2_dbl / j2_add_aff: 16 FME per doubling and item against
// 2 x 12 on a lane pair).  Sigma is attacker-chosen, so the incomplete
// addition's exceptional cases are real inputs: an item that raises one reruns
// the complete projective chain (pp_dbl / pp_add_aff), a data-dependent branch
// that only such inputs take.  Blocks [0, nb) run r_i apk_i, [nb, 2 nb) [|x|] sigma_i.
__global__ void __launch_bounds__(64) k_sig_lane1j(size_t B, const int* gstat, int* status, const int* dstat,
                                                   const G1P* apk, const G2A* sig, const uint64_t* rsc, G1P* rPj) {
  const unsigned nb = (unsigned)((B + 63) / 64);
  const bool g2 = blockIdx.x >= nb;
  const size_t i = (size_t)(g2 ? blockIdx.x - nb : blockIdx.x) * 64 + threadIdx.x;
  if (i >= B) return;
  const bool live = gstat[i] && dstat[i];
  if (!g2) {
    if (!live) return;
    const G1P a = apk[i];
    const PP<Fp> A{a.x, a.y, a.z};
    const uint64_t r = rsc[i];
    PP<Fp> R{fp_zero(), FP_ONE, fp_zero()};
    if ((r >> 63) & 1ull) R = A;
#pragma unroll 1
    for (int b = 62; b >= 0; --b) {
      R = pp_dbl(R);
      if ((r >> b) & 1ull) R = pp_add(R, A);
    }
    rPj[i] = G1P{R.x, R.y, R.z};
    return;
  }
  if (!live) {
    status[i] = 0;
    return;
  }
  const G2A s = sig[i];
  bool exc = false;
  G2J M{s.x, s.y, fp2_one()};
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    M = j2_dbl(M);
    if ((X_ABS >> b) & 1ull) M = j2_add_aff(M, s.x, s.y, exc);
  }
  // sigma in G2  <=>  psi(sigma) == -M with M not the identity; psi(sigma) = (conj(x) cx, conj(y) cy) affine
  const Fp2 px = f2mul(fp2_conj(s.x), PSI_CX), py = f2mul(fp2_conj(s.y), PSI_CY);
  bool ok;
  if (!exc) {
    const Fp2 zz = f2sqr(M.z);
    ok = fp2_is_zero(fp2_sub(f2mul(px, zz), M.x)) && fp2_is_zero(fp2_add(f2mul(py, f2mul(zz, M.z)), M.y)) &&
         !fp2_is_zero(M.z);
  } else {  // complete formulas (k_sig_lane)
    PP<Fp2> P{s.x, s.y, fp2_one()};
#pragma unroll 1
    for (int b = 62; b >= 0; --b) {
      P = pp_dbl(P);
      if ((X_ABS >> b) & 1ull) P = pp_add_aff(P, s.x, s.y);
    }
    ok = fp2_is_zero(fp2_sub(f2mul(px, P.z), P.x)) && fp2_is_zero(fp2_add(f2mul(py, P.z), P.y)) &&
         !fp2_is_zero(P.z);
  }
  status[i] = ok ? 1 : 0;
}

// k_sig_lane1j with both chains in the digit form (bls_fq_g1.h, bls_fq_g2.h): one lane per chain, the G2 chain
// Jacobian with flagged exceptional additions (those items rerun the complete projective chain).
__global__ void __launch_bounds__(64) k_sig_lane1q(size_t B, const int* gstat, int* status, const int* dstat,
                                                   const G1P* apk, const G2A* sig, const uint64_t* rsc, G1P* rPj) {
  const unsigned nb = (unsigned)((B + 63) / 64);
  const bool g2 = blockIdx.x >= nb;
  const size_t i = (size_t)(g2 ? blockIdx.x - nb : blockIdx.x) * 64 + threadIdx.x;
  if (i >= B) return;
  const bool live = gstat[i] && dstat[i];
  if (!g2) {
    if (!live) return;
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
  if (!live) {
    status[i] = 0;
    return;
  }
  const G2A s = sig[i];
  bool exc = false;
  const J2Q M = j2q_mul_xabs(J2Q{fq2_unpack(s.x), fq2_unpack(s.y), fq2_unpack(fp2_one())}, exc);
  const Fp2 px = f2mul(fp2_conj(s.x), PSI_CX), py = f2mul(fp2_conj(s.y), PSI_CY);
  bool ok;
  if (!exc) {  // psi(sigma) == -M:  px Z^2 == X, py Z^3 == -Y, Z != 0
    const Fp2 X = fq2_pack(M.x), Y = fq2_pack(M.y), Z = fq2_pack(M.z);
    const Fp2 zz = f2sqr(Z);
    ok = fp2_is_zero(fp2_sub(f2mul(px, zz), X)) && fp2_is_zero(fp2_add(f2mul(py, f2mul(zz, Z)), Y)) &&
         !fp2_is_zero(Z);
  } else {  // complete formulas (k_sig_lane)
    PP<Fp2> P{s.x, s.y, fp2_one()};
#pragma unroll 1
    for (int b = 62; b >= 0; --b) {
      P = pp_dbl(P);
      if ((X_ABS >> b) & 1ull) P = pp_add_aff(P, s.x, s.y);
    }
    ok = fp2_is_zero(fp2_sub(f2mul(px, P.z), P.x)) && fp2_is_zero(fp2_add(f2mul(py, P.z), P.y)) &&
         !fp2_is_zero(P.z);
  }
  status[i] = ok ? 1 : 0;
}

hipError_t launch_sig_lane(hipStream_t st, size_t B, const int* gstat, int* status, const int* dstat, const G1P* apk,
                           const G2A* sig, const uint64_t* rsc, G1P* rPj) {
  if (!B) return hipSuccess;
  // A/B knobs: BLS_SIG1 = k_sig_lane (one lane per G2 chain, complete formulas), BLS_SIG1J = k_sig_lane1j (one
  // lane, Jacobian; 1.41-1.43M FAV/s against 1.43-1.50M for the lane pairs: its 512 registers still spill)
  static const bool one_lane = getenv("BLS_SIG1") != nullptr, jac = getenv("BLS_SIG1J") != nullptr;
  static const bool digits = getenv("BLS_SIG1Q") != nullptr;  // A/B knob: k_sig_lane1q (digit-form chains)
  if (digits)
    hipLaunchKernelGGL(k_sig_lane1q, dim3(2 * (unsigned)((B + 63) / 64)), dim3(64), 0, st, B, gstat, status, dstat,
                       apk, sig, rsc, rPj);
  else if (jac)
    hipLaunchKernelGGL(k_sig_lane1j, dim3(2 * (unsigned)((B + 63) / 64)), dim3(64), 0, st, B, gstat, status, dstat,
                       apk, sig, rsc, rPj);
  else if (one_lane)
    hipLaunchKernelGGL(k_sig_lane, dim3(2 * (unsigned)((B + 63) / 64)), dim3(64), 0, st, B, gstat, status, dstat, apk,
                       sig, rsc, rPj);
  else
    hipLaunchKernelGGL(k_sig_lane2, dim3((unsigned)((B + 63) / 64 + (2 * B + 63) / 64)), dim3(64), 0, st, B, gstat,
                       status, dstat, apk, sig, rsc, rPj);
  return hipGetLastError();
}

hipError_t launch_g2x_lane(hipStream_t st, size_t B, Fd* hf, int src, int dst) {
  if (!B) return hipSuccess;
  static const bool one_lane = getenv("BLS_G2X1") != nullptr;  // A/B knob: k_g2x_lane (one lane per chain)
  if (one_lane)
    hipLaunchKernelGGL(k_g2x_lane, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, st, B, hf, src, dst);
  else
    hipLaunchKernelGGL(k_g2x_lane2, dim3((unsigned)((2 * B + 63) / 64)), dim3(64), 0, st, B, hf, src, dst);
  return hipGetLastError();
}

}  // namespace bls
