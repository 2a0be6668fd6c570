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
#include "bls_tower_inline.h"
#include "bls_vm.h"

namespace bls {

// multiplication by 3b: b = 4 on E1, b = 4(1 + i) on E2
BLS_HD Fp ln_b3(const Fp& a) {
  const Fp a4 = fp_dbl(fp_dbl(a));
  return fp_add(fp_dbl(a4), a4);
}
BLS_HD Fp2 ln_b3(const Fp2& t) { return Fp2{ln_b3(fp_sub(t.c0, t.c1)), ln_b3(fp_add(t.c0, t.c1))}; }
BLS_HD Fp ln_mul(const Fp& a, const Fp& b) { return fp_mul_i(a, b); }
BLS_HD Fp2 ln_mul(const Fp2& a, const Fp2& b) { return f2mul(a, b); }
BLS_HD Fp ln_sqr(const Fp& a) { return fp_sqr_i(a); }
BLS_HD Fp2 ln_sqr(const Fp2& a) { return f2sqr(a); }

template <class F>
struct PP {
  F x, y, z;
};

template <class F>
BLS_HD PP<F> pp_dbl(const PP<F>& p) {
  const F t0 = ln_sqr(p.y);
  const F t1 = ln_mul(p.y, p.z);
  const F t2 = ln_b3(ln_sqr(p.z));
  const F u = ln_mul(p.x, p.y);
  const F z8 = fdbl(fdbl(fdbl(t0)));
  const F x3a = ln_mul(t2, z8);
  PP<F> r;
  r.z = ln_mul(t1, z8);
  const F w = fsub(t0, fadd(fdbl(t2), t2));
  r.y = fadd(ln_mul(w, fadd(t0, t2)), x3a);
  r.x = fdbl(ln_mul(w, u));
  return r;
}

template <class F>
BLS_HD PP<F> pp_finish(F t0, F t1, const F& t2, const F& t3, const F& t4, F y3) {
  t0 = fadd(fdbl(t0), t0);
  const F z3 = fadd(t1, t2);
  t1 = fsub(t1, t2);
  y3 = ln_b3(y3);
  PP<F> r;
  r.x = fsub(ln_mul(t3, t1), ln_mul(t4, y3));
  r.y = fadd(ln_mul(t1, z3), ln_mul(y3, t0));
  r.z = fadd(ln_mul(z3, t4), ln_mul(t0, t3));
  return r;
}

template <class F>
BLS_HD PP<F> pp_add(const PP<F>& p, const PP<F>& q) {
  const F t0 = ln_mul(p.x, q.x), t1 = ln_mul(p.y, q.y), t2 = ln_mul(p.z, q.z);
  const F t3 = fsub(fsub(ln_mul(fadd(p.x, p.y), fadd(q.x, q.y)), t0), t1);
  const F t4 = fsub(fsub(ln_mul(fadd(p.y, p.z), fadd(q.y, q.z)), t1), t2);
  const F y3 = fsub(fsub(ln_mul(fadd(p.x, p.z), fadd(q.x, q.z)), t0), t2);
  return pp_finish(t0, t1, ln_b3(t2), t3, t4, y3);
}

// p + (x2, y2) with (x2, y2) affine, not the identity
template <class F>
BLS_HD PP<F> pp_add_aff(const PP<F>& p, const F& x2, const F& y2) {
  const F t0 = ln_mul(p.x, x2), t1 = ln_mul(p.y, y2);
  const F t3 = fsub(fsub(ln_mul(fadd(x2, y2), fadd(p.x, p.y)), t0), t1);
  const F t4 = fadd(ln_mul(y2, p.z), p.y);
  const F y3 = fadd(ln_mul(x2, p.z), p.x);
  return pp_finish(t0, t1, ln_b3(p.z), t3, t4, y3);
}

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

hipError_t launch_sig_lane(hipStream_t st, size_t B, const int* gstat, int* status, const int* dstat, const G1P* apk,
                           const G2A* sig, const uint64_t* rsc, G1P* rPj) {
  if (!B) return hipSuccess;
  hipLaunchKernelGGL(k_sig_lane, dim3(2 * (unsigned)((B + 63) / 64)), dim3(64), 0, st, B, gstat, status, dstat, apk,
                     sig, rsc, rPj);
  return hipGetLastError();
}

hipError_t launch_g2x_lane(hipStream_t st, size_t B, Fd* hf, int src, int dst) {
  if (!B) return hipSuccess;
  hipLaunchKernelGGL(k_g2x_lane, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, st, B, hf, src, dst);
  return hipGetLastError();
}

}  // namespace bls
