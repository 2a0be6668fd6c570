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

// ---------------------------------------------------------------------------
// G2 chains on TWO lanes per item.  Both lanes of a pair hold the running
// point; each dependency level of a complete formula is split between them
// and the products are exchanged by one DPP swap (quad_perm [1,0,3,2]):
//   doubling   level 1  lane 0: y^2, z^2          lane 1: y z, x y
//              level 2  lane 0: t2 z8, w (t0+t2)  lane 1: t1 z8, w u
//   addition   level 1  lane 0: x1x2, y1y2, z1z2  lane 1: the three Karatsuba cross sums
//              level 2  (pp_finish) three of its six products per lane
// 12 instead of 22 FME per doubling and lane (squarings run as products so
// the instruction stream is uniform).  Every value is the canonical residue
// pp_dbl / pp_add / pp_add_aff produce, so the chains are bit-identical.
namespace {
__device__ __forceinline__ uint32_t cl_swap(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ Fp2 cl_swap2(const Fp2& a) {
  Fp2 r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.l[i] = cl_swap(a.c0.l[i]);
    r.c1.l[i] = cl_swap(a.c1.l[i]);
  }
  return r;
}
__device__ __forceinline__ Fp2 cl_sel(bool c, const Fp2& a, const Fp2& b) {
  return Fp2{fp_select(c, a.c0, b.c0), fp_select(c, a.c1, b.c1)};
}
// (own product, partner's product) -> (lane 0's value, lane 1's value) on both lanes
__device__ __forceinline__ void cl_xchg(bool hi, const Fp2& mine, Fp2& v0, Fp2& v1) {
  const Fp2 o = cl_swap2(mine);
  v0 = cl_sel(hi, o, mine);
  v1 = cl_sel(hi, mine, o);
}

__device__ __forceinline__ PP<Fp2> pp2_dbl(const PP<Fp2>& p, bool hi) {
  Fp2 t0, t1, zz, u;
  cl_xchg(hi, f2mul(p.y, cl_sel(hi, p.z, p.y)), t0, t1);              // y^2 | y z
  cl_xchg(hi, f2mul(cl_sel(hi, p.x, p.z), cl_sel(hi, p.y, p.z)), zz, u);  // z^2 | x y
  const Fp2 t2 = ln_b3(zz);
  const Fp2 z8 = fdbl(fdbl(fdbl(t0)));
  const Fp2 w = fsub(t0, fadd(fdbl(t2), t2));
  Fp2 x3a, z3, ws, wu;
  cl_xchg(hi, f2mul(cl_sel(hi, t1, t2), z8), x3a, z3);               // t2 z8 | t1 z8
  cl_xchg(hi, f2mul(w, cl_sel(hi, u, fadd(t0, t2))), ws, wu);        // w (t0 + t2) | w u
  PP<Fp2> r;
  r.z = z3;
  r.y = fadd(ws, x3a);
  r.x = fdbl(wu);
  return r;
}

// pp_finish with its six products three per lane
__device__ __forceinline__ PP<Fp2> pp2_finish(bool hi, Fp2 t0, Fp2 t1, const Fp2& t2, const Fp2& t3, const Fp2& t4,
                                              Fp2 y3) {
  t0 = fadd(fdbl(t0), t0);
  const Fp2 z3 = fadd(t1, t2);
  t1 = fsub(t1, t2);
  y3 = ln_b3(y3);
  Fp2 a0, a1, b0, b1, c0, c1;
  cl_xchg(hi, f2mul(cl_sel(hi, t4, t3), cl_sel(hi, y3, t1)), a0, a1);  // t3 t1 | t4 y3
  cl_xchg(hi, f2mul(cl_sel(hi, y3, t1), cl_sel(hi, t0, z3)), b0, b1);  // t1 z3 | y3 t0
  cl_xchg(hi, f2mul(cl_sel(hi, t0, z3), cl_sel(hi, t3, t4)), c0, c1);  // z3 t4 | t0 t3
  PP<Fp2> r;
  r.x = fsub(a0, a1);
  r.y = fadd(b0, b1);
  r.z = fadd(c0, c1);
  return r;
}

__device__ __forceinline__ PP<Fp2> pp2_add(const PP<Fp2>& p, const PP<Fp2>& q, bool hi) {
  Fp2 t0, m3, t1, m4, t2, m5;
  cl_xchg(hi, f2mul(cl_sel(hi, fadd(p.x, p.y), p.x), cl_sel(hi, fadd(q.x, q.y), q.x)), t0, m3);
  cl_xchg(hi, f2mul(cl_sel(hi, fadd(p.y, p.z), p.y), cl_sel(hi, fadd(q.y, q.z), q.y)), t1, m4);
  cl_xchg(hi, f2mul(cl_sel(hi, fadd(p.x, p.z), p.z), cl_sel(hi, fadd(q.x, q.z), q.z)), t2, m5);
  const Fp2 t3 = fsub(fsub(m3, t0), t1);
  const Fp2 t4 = fsub(fsub(m4, t1), t2);
  const Fp2 y3 = fsub(fsub(m5, t0), t2);
  return pp2_finish(hi, t0, t1, ln_b3(t2), t3, t4, y3);
}

__device__ __forceinline__ PP<Fp2> pp2_add_aff(const PP<Fp2>& p, const Fp2& x2, const Fp2& y2, bool hi) {
  Fp2 t0, m3, t1, m5;
  cl_xchg(hi, f2mul(cl_sel(hi, fadd(x2, y2), p.x), cl_sel(hi, fadd(p.x, p.y), x2)), t0, m3);
  cl_xchg(hi, f2mul(cl_sel(hi, x2, p.y), cl_sel(hi, p.z, y2)), t1, m5);
  const Fp2 m4 = f2mul(y2, p.z);  // both lanes
  const Fp2 t3 = fsub(fsub(m3, t0), t1);
  const Fp2 t4 = fadd(m4, p.y);
  const Fp2 y3 = fadd(m5, p.x);
  return pp2_finish(hi, t0, t1, ln_b3(p.z), t3, t4, y3);
}
}  // namespace

// k_sig_lane with the G2 chain on lane pairs: blocks [0, nb1) run r_i apk_i
// (one lane per item), blocks [nb1, nb1 + nb2) [|x|] sigma_i (two lanes per item).
__global__ void __launch_bounds__(64) k_sig_lane2(size_t B, const int* gstat, int* status, const int* dstat,
                                                  const G1P* apk, const G2A* sig, const uint64_t* rsc, G1P* rPj) {
  const unsigned nb1 = (unsigned)((B + 63) / 64);
  if (blockIdx.x < nb1) {
    const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= B || !(gstat[i] && dstat[i])) return;
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

hipError_t launch_sig_lane(hipStream_t st, size_t B, const int* gstat, int* status, const int* dstat, const G1P* apk,
                           const G2A* sig, const uint64_t* rsc, G1P* rPj) {
  if (!B) return hipSuccess;
  static const bool one_lane = getenv("BLS_SIG1") != nullptr;  // A/B knob: k_sig_lane (one lane per G2 chain)
  if (one_lane)
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
