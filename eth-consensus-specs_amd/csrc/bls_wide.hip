// Kernels in the wavefront-cooperative form of bls_wide.h: one wave per item
// (per-call path), and the device self-test of the wide products against the
// lane form of bls_fq.h.
#include "bls_kernels.h"
#include "bls_lane.h"
#include "bls_wide.h"
#include "bls_wide_g2.h"
#include "bls_pp_lane.h"
#include "bls_xmd32.h"
#include "bls_h2c.h"

namespace bls {

using namespace wide;

__device__ static const uint8_t DST_POP_WIDE[43] = {
    'B', 'L', 'S', '_', 'S', 'I', 'G', '_', 'B', 'L', 'S', '1', '2', '3', '8', '1', 'G', '2', '_', 'X', 'M', 'D',
    ':', 'S', 'H', 'A', '-', '2', '5', '6', '_', 'S', 'S', 'W', 'U', '_', 'R', 'O', '_', 'P', 'O', 'P', '_'};

// Self-test: wave w takes a[4w .. 4w+4) (canonical Montgomery Fp): half h multiplies a[4w + 2h] by a[4w + 2h + 1]
// in every wide form and compares with the lane form; bad[w] = bitmask of the forms that differ.
__global__ void __launch_bounds__(64) k_wide_selftest(size_t nw, const uint8_t* be48, int* bad) {
  const size_t w = blockIdx.x;
  if (w >= nw) return;
  Fp a[4];  // test kernel: the four inputs of this wave, big-endian integers < p -> Montgomery form
#pragma unroll
  for (int k = 0; k < 4; k++) a[k] = fp_to_mont(raw_from_be48(be48 + 48 * (4 * w + k)));
  const int h = whalf();
  const WK K = wk_init();
  const Fp x = a[2 * h], y = a[2 * h + 1];
  const Fp u = a[((2 * h + 2) & 3)], v = a[((2 * h + 3) & 3)];
  const uint32_t X = w_from_fp(x), Y = w_from_fp(y), U = w_from_fp(u), V = w_from_fp(v);
  int m = 0;
  // product, square, dot2
  if (!fp_eq(w_to_fp(wmul(X, Y)), fq_pack(fq_mul(fq_unpack(x), fq_unpack(y))))) m |= 1;
  if (!fp_eq(w_to_fp(wsqr(X)), fq_pack(fq_sqr(fq_unpack(x))))) m |= 2;
  if (!fp_eq(w_to_fp(wdot2(X, Y, U, V)), fq_pack(fq_mul_dot2(fq_unpack(x), fq_unpack(y), fq_unpack(u), fq_unpack(v)))))
    m |= 4;
  // a chain: 64 products of unnormalised sums and differences (bounds of repeated use)
  uint32_t c = X;
  Fq cl = fq_unpack(x);
  for (int i = 0; i < 64; i++) {
    c = wmul(wadd(c, Y), wsub(K, c, U));
    cl = fq_mul(fq_norm(fq_add(cl, fq_unpack(y))), fq_norm(fq_sub(cl, fq_unpack(u))));
  }
  if (!fp_eq(w_to_fp(c), fq_pack(cl))) m |= 8;
  // Fp2 product and square against bls_tower_inline.h
  const W2 A{X, Y}, B{U, V};
  const Fp2 al{x, y}, bl{u, v};
  if (!fp2_eq(w2_to_fp2(w2mul(K, A, B)), f2mul(al, bl))) m |= 16;
  if (!fp2_eq(w2_to_fp2(w2sqr(K, A)), f2sqr(al))) m |= 32;
  // fixed-exponent power (the square-root exponent) against fq_pow_w3
  if (!fp_eq(w_to_fp(wpow(X, EXP_SQRT, EXP_SQRT_BITS)), fq_pack(fq_pow_w3(fq_unpack(x), EXP_SQRT, EXP_SQRT_BITS))))
    m |= 64;
  // round trip and the other half
  if (!fp_eq(w_to_fp(X), x)) m |= 128;
  if (!fp_eq(w_to_fp(wswap(X)), a[2 * (h ^ 1)])) m |= 256;
  // zero tests: x - x, and p itself in redundant digits (x + 64p - x)
  if (!w_is_zero(wsub(K, X, X))) m |= 512;
  const int mh = m;
  const int mo = __builtin_amdgcn_readlane(mh, 32);
  if (threadIdx.x == 0) bad[w] = mh | (mo << 10);
}

// hash_to_G2 of item blockIdx.x on one workgroup of four waves (per-call path), every wave doing the same work
// except the cofactor chains' doublings, whose products are spread over the four (p2f_dbl4, bls_wide_g2.h: the
// complete projective doubling in two product rounds): hash_to_field on every lane (uniform), the SSWU map
// and 3-isogeny of u_0 in half 0 and of u_1 in half 1, their sum, the cofactor clearing
//   H = [x^2 - x - 1] Q + [x - 1] psi(Q) + psi^2(2 Q)  as  M = [|x|] Q,  A' = M - psi(Q),
//   C = psi^2(2 Q) - psi(Q) + M - Q,  H = C + [|x|] A'   (A' = -A of k_g2x_pre1t / k_g2x_post1t)
// in complete projective formulas (F2 layout), and the affine H -- or, Hz != nullptr, H in Jacobian coordinates
// (X, Y in H[i], Z in Hz[i]: no inversion; the per-call Miller loop takes it as is, and a flagged item gets Z = 1
// for the fallback's affine point).  flag[i] = 1 for the cases the fallback recomputes (SSWU `rare`, a vanishing
// isogeny denominator, an exceptional P0 + P1).
// msgs: 32-byte messages msgs[32 i ..] (offs == nullptr) or msgs[offs[i] .. offs[i+1]).
__global__ void __launch_bounds__(256) k_h2c_wide(size_t B, const uint8_t* msgs, const uint64_t* offs, G2A* H,
                                                  int* flag, Fp2* Hz) {
  const size_t i = blockIdx.x;
  if (i >= B) return;  // (the whole workgroup)
  __shared__ uint32_t x4[8 * 64];
  __shared__ uint32_t pring[PW_RING * 64];  // the SSWU exponentiations' squaring ring (wpow_2w)
  __shared__ int pcnt[2];
  const int w = (int)(threadIdx.x >> 6);  // four waves: the same work up to the cofactor chains' doublings
  const WKG K = wkg_init();
  Fp2 u[2];
  if (offs)
    hash_to_field_fp2(u, msgs + offs[i], (uint32_t)(offs[i + 1] - offs[i]), DST_POP_WIDE, 43);
  else
    hash_to_field_fp2_m32<true>(u, msgs + 32 * i);
  const bool hi = whalf() != 0;
  const Fp2 uh{fp_select(hi, u[1].c0, u[0].c0), fp_select(hi, u[1].c1, u[0].c1)};
  W2 x, y;
  bool rare = false, izero = false, exc = false;
  sswu_w(K, uh, x, y, rare, pring, pcnt, w);
  const J2W P = iso_w(K, x, y, izero);
  const J2W Po{w2swap(P.x), w2swap(P.y), w2swap(P.z)};
  // Q = P0 + P1 (W2 layout, both halves), then the cofactor chains in F2 layout on half 0's Q
  const J2F Q = j2f_of_j2w(j2w_add(K, P, Po, exc));
  const uint32_t cx = wf_from_fp2(PSI_CX), cy = wf_from_fp2(PSI_CY);
  const uint32_t c2x = w_from_fp(PSI2_CX.c0), c2y = w_from_fp(PSI2_CY.c0);
  // the cofactor clearing in complete projective formulas (P2F): no exceptional case after P0 + P1
  const P2F Qp = p2f_of_j2f(K, Q);
  const P2F M = p2f_mul_xabs4(K, Qp, x4, w);
  const P2F npq = p2f_neg(K, p2f_psi(K, Qp, cx, cy));
  const P2F Ap = p2f_add(K, M, npq);
  P2F C = p2f_add(K, p2f_psi2(p2f_dbl4(K, Qp, x4, w), c2x, c2y), npq);
  C = p2f_add(K, C, M);
  C = p2f_add(K, C, p2f_neg(K, Qp));
  const P2F M2 = p2f_mul_xabs4(K, Ap, x4, w);
  if (w) return;  // waves 1 .. 3: no barrier after the chains
  const int bad = (rare | izero | exc) ? 1 : 0;
  const int bad_any = __builtin_amdgcn_readlane(bad, 0) | __builtin_amdgcn_readlane(bad, 32);
  if (Hz) {
    Fp2 z;
    const G2A h = p2f_to_jac(K, p2f_add(K, C, M2), z);
    if (threadIdx.x == 0) {
      H[i] = h;
      Hz[i] = bad_any ? fp2_one() : z;
      flag[i] = bad_any;
    }
    return;
  }
  const G2A h = p2f_to_aff(K, p2f_add(K, C, M2));
  if (threadIdx.x == 0) {
    H[i] = h;
    flag[i] = bad_any;
  }
}

// Debug view of k_h2c_wide for one 32-byte message (tests): out[] = raw (non-Montgomery) little-endian Fp limbs of,
// per half h: u_h (2), SSWU x (2), y (2), the isogeny's Jacobian point as affine x, y (4); then Q = P0 + P1 affine
// (4), M = [|x|] Q affine (4), H affine (4), and the flags (rare, izero, exc) of both halves as one Fp word.
__device__ __forceinline__ void dbg_put(Fp* out, int k, const Fp& v) {
  if (threadIdx.x == 0) out[k] = fp_from_mont(v);
}
__global__ void __launch_bounds__(64) k_h2c_wide_dbg(const uint8_t* msg32, Fp* out) {
  const WKG K = wkg_init();
  Fp2 u[2];
  hash_to_field_fp2_m32<true>(u, msg32);
  const bool hi = whalf() != 0;
  const Fp2 uh{fp_select(hi, u[1].c0, u[0].c0), fp_select(hi, u[1].c1, u[0].c1)};
  W2 x, y;
  bool rare = false, izero = false, exc = false;
  sswu_w(K, uh, x, y, rare);
  const J2W P = iso_w(K, x, y, izero);
  const G2A pa = j2w_to_aff(K, P);
  for (int h = 0; h < 2; h++) {
    // lane 0 writes; values of half h read through w_to_fp from lane 32 h: take them from the lane's own half
    const Fp2 xs = w2_to_fp2(x), ys = w2_to_fp2(y);
    const Fp v[10] = {uh.c0, uh.c1, xs.c0, xs.c1, ys.c0, ys.c1, pa.x.c0, pa.x.c1, pa.y.c0, pa.y.c1};
    for (int k = 0; k < 10; k++) {
      const Fp vk = v[k];
      Fp o;
#pragma unroll
      for (int l = 0; l < 12; l++) o.l[l] = (uint32_t)__builtin_amdgcn_readlane((int)vk.l[l], 32 * h);
      dbg_put(out, 10 * h + k, o);
    }
  }
  const J2W Po{w2swap(P.x), w2swap(P.y), w2swap(P.z)};
  const J2W Q = j2w_add(K, P, Po, exc);
  const G2A qa = j2w_to_aff(K, Q);
  {  // the lane form on the same inputs, and the first intermediates of both forms (slots 33 ..)
    const G2J pl{w2_to_fp2(P.x), w2_to_fp2(P.y), w2_to_fp2(P.z)}, ql{w2_to_fp2(Po.x), w2_to_fp2(Po.y), w2_to_fp2(Po.z)};
    bool e2 = false;
    const G2J rl = j2_add(pl, ql, e2);
    const G2A ra = jac_to_aff(rl);
    dbg_put(out, 33, ra.x.c0);
    dbg_put(out, 34, ra.x.c1);
    dbg_put(out, 35, ra.y.c0);
    dbg_put(out, 36, ra.y.c1);
    {  // every intermediate of j2w_add against j2_add's, as a bit mask in slot 32's high word
      const J2W& wp = P;
      const J2W& wq = Po;
      const WK K1 = wk_of(K);
      (void)K1;
      int bm = 0, bit = 0;
      auto chk = [&](const W2& a, const Fp2& b) { if (!fp2_eq(w2_to_fp2(a), b)) bm |= 1 << bit; bit++; };
      const W2 Z1 = w2sqrk(K, wp.z), Z2 = w2sqrk(K, wq.z);
      const Fp2 z1 = f2sqr(pl.z), z2 = f2sqr(ql.z);
      chk(Z1, z1); chk(Z2, z2);
      const W2 U1 = w2mulk(K, wp.x, Z2), U2 = w2mulk(K, wq.x, Z1);
      const Fp2 u1x = f2mul(pl.x, z2), u2x = f2mul(ql.x, z1);
      chk(U1, u1x); chk(U2, u2x);
      const W2 S1 = w2mulk(K, w2mulk(K, wp.y, wq.z), Z2), S2 = w2mulk(K, w2mulk(K, wq.y, wp.z), Z1);
      const Fp2 s1 = f2mul(f2mul(pl.y, ql.z), z2), s2 = f2mul(f2mul(ql.y, pl.z), z1);
      chk(S1, s1); chk(S2, s2);
      const W2 H = w2subk(K.k256, U2, U1);
      const Fp2 hh = fp2_sub(u2x, u1x);
      chk(H, hh);
      const W2 RR = w2muls<2>(w2subk(K.k256, S2, S1));
      const Fp2 rr = fp2_dbl(fp2_sub(s2, s1));
      chk(RR, rr);
      const W2 I = w2sqrk(K, w2muls<2>(H));
      const Fp2 ii = f2sqr(fp2_dbl(hh));
      chk(I, ii);
      const W2 J = w2mulk(K, H, I), V = w2mulk(K, U1, I);
      const Fp2 jj = f2mul(hh, ii), vv = f2mul(u1x, ii);
      chk(J, jj); chk(V, vv);
      const W2 RRS = w2sqrk(K, RR);
      chk(RRS, f2sqr(rr));
      const W2 X3 = w2subk(K.k512_2, RRS, w2add(J, w2muls<2>(V)));
      const Fp2 x3 = fp2_sub(fp2_sub(f2sqr(rr), jj), fp2_dbl(vv));
      chk(X3, x3);
      const W2 VX = w2subk(K.k1024, V, X3);
      chk(VX, fp2_sub(vv, x3));
      const W2 Y3 = w2subk(K.k512_2, w2mulk(K, RR, VX), w2muls<2>(w2mulk(K, S1, J)));
      chk(Y3, fp2_sub(f2mul(rr, fp2_sub(vv, x3)), fp2_dbl(f2mul(s1, jj))));
      const W2 ZZ = w2subk(K.k2, w2sqrk(K, w2add(wp.z, wq.z)), w2add(Z1, Z2));
      chk(ZZ, fp2_sub(fp2_sub(f2sqr(fp2_add(pl.z, ql.z)), z1), z2));
      const W2 SZ = w2add(wp.z, wq.z);
      chk(SZ, fp2_add(pl.z, ql.z));                                   // bit 16
      const W2 SQ = w2sqrk(K, SZ);
      chk(SQ, f2sqr(fp2_add(pl.z, ql.z)));                            // bit 17
      chk(w2add(Z1, Z2), fp2_add(z1, z2));                            // bit 18
      chk(w2subk(K.k2, SQ, w2add(Z1, Z2)), fp2_sub(f2sqr(fp2_add(pl.z, ql.z)), fp2_add(z1, z2)));  // bit 19
      chk(w2subk(K.k1, SQ, w2add(Z1, Z2)), fp2_sub(f2sqr(fp2_add(pl.z, ql.z)), fp2_add(z1, z2)));  // bit 20
      chk(W2{wsubk(K.k2, 0u, Z1.c0), 0u}, Fp2{fp_neg(z1.c0), fp_zero()});                          // bit 21
      chk(W2{wnorm(K.k2), 0u}, fp2_zero());                                                       // bit 22
      chk(Q.x, rl.x);                                                                             // bit 23
      chk(Q.y, rl.y);                                                                             // bit 24
      chk(Q.z, rl.z);                                                                             // bit 25
      const G2A qw = j2w_to_aff(K, Q);
      chk(w2_from_fp2(qw.x), ra.x);                                                               // bit 26
      chk(w2_from_fp2(qw.y), ra.y);                                                               // bit 27
      chk(w2mulk(K, ZZ, H), rl.z);                                                                // bit 28
      {  // raw lanes of the c1 parts after slot 72: ZZ, SQ, Z1 + Z2, Z1, Z2
        uint32_t* raw = reinterpret_cast<uint32_t*>(out + 72);
        const W2 S12 = w2add(Z1, Z2);
        raw[threadIdx.x] = ZZ.c1;
        raw[64 + threadIdx.x] = SQ.c1;
        raw[128 + threadIdx.x] = S12.c1;
        raw[192 + threadIdx.x] = Z1.c1;
        raw[256 + threadIdx.x] = Z2.c1;
      }
      {  // canonical raw values: P.z (own), Po.z, ZZ, H, Q.z, rl.z -- 12 Fp at slot 52
        const Fp2 vals[9] = {w2_to_fp2(wp.z), w2_to_fp2(wq.z), w2_to_fp2(ZZ), w2_to_fp2(H), w2_to_fp2(Q.z), rl.z,
                             w2_to_fp2(SQ), w2_to_fp2(Z1), w2_to_fp2(Z2)};
        for (int q2 = 0; q2 < 9; q2++) {
          dbg_put(out, 52 + 2 * q2, vals[q2].c0);
          dbg_put(out, 53 + 2 * q2, vals[q2].c1);
        }
      }
      const int b0 = __builtin_amdgcn_readlane(bm, 0);
      if (threadIdx.x == 0) {
        Fp o = fp_zero();
        o.l[1] = (uint32_t)b0;
        out[32] = o;
      }
    }
    const W2 z1z1 = w2sqrk(K, P.z);
    const Fp2 z1l = f2sqr(pl.z);
    const W2 u1 = w2mulk(K, P.x, w2sqrk(K, Po.z));
    const Fp2 u1l = f2mul(pl.x, f2sqr(ql.z));
    const Fp2 zw = w2_to_fp2(z1z1), uw = w2_to_fp2(u1);
    dbg_put(out, 37, zw.c0);
    dbg_put(out, 38, zw.c1);
    dbg_put(out, 39, z1l.c0);
    dbg_put(out, 40, z1l.c1);
    dbg_put(out, 41, uw.c0);
    dbg_put(out, 42, uw.c1);
    dbg_put(out, 43, u1l.c0);
    dbg_put(out, 44, u1l.c1);
  }
  dbg_put(out, 20, qa.x.c0);
  dbg_put(out, 21, qa.x.c1);
  dbg_put(out, 22, qa.y.c0);
  dbg_put(out, 23, qa.y.c1);
  const J2W M = j2w_mul_xabs(K, Q, exc);
  const G2A ma = j2w_to_aff(K, M);
  dbg_put(out, 24, ma.x.c0);
  dbg_put(out, 25, ma.x.c1);
  dbg_put(out, 26, ma.y.c0);
  dbg_put(out, 27, ma.y.c1);
  const W2 cx = w2const(PSI_CX), cy = w2const(PSI_CY);
  const uint32_t c2x = w_from_fp(PSI2_CX.c0), c2y = w_from_fp(PSI2_CY.c0);
  const J2W npq = j2w_neg(K, j2w_psi(K, Q, cx, cy));
  const J2W Ap = j2w_add(K, M, npq, exc);
  J2W C = j2w_add(K, j2w_psi2(K, j2w_dbl(K, Q), c2x, c2y), npq, exc);
  C = j2w_add(K, C, M, exc);
  C = j2w_add(K, C, j2w_neg(K, Q), exc);
  const J2W M2 = j2w_mul_xabs(K, Ap, exc);
  const G2A h = j2w_to_aff(K, j2w_add(K, C, M2, exc));
  dbg_put(out, 28, h.x.c0);
  dbg_put(out, 29, h.x.c1);
  dbg_put(out, 30, h.y.c0);
  dbg_put(out, 31, h.y.c1);
  const int fl = (rare ? 1 : 0) | (izero ? 2 : 0) | (exc ? 4 : 0);
  const int f0 = __builtin_amdgcn_readlane(fl, 0), f1 = __builtin_amdgcn_readlane(fl, 32);
  __syncthreads();
  if (threadIdx.x == 0) out[32].l[0] = (uint32_t)(f0 | (f1 << 8));
}

hipError_t launch_h2c_wide_dbg(hipStream_t st, const uint8_t* msg32, Fp* out) {
  hipLaunchKernelGGL(k_h2c_wide_dbg, dim3(1), dim3(64), 0, st, msg32, out);
  return hipGetLastError();
}

hipError_t launch_h2c_wide(hipStream_t st, size_t B, const uint8_t* msgs, const uint64_t* offs, G2A* H, int* flag,
                           Fp2* Hz) {
  if (!B) return hipSuccess;
  hipLaunchKernelGGL(k_h2c_wide, dim3((unsigned)B), dim3(256), 0, st, B, msgs, offs, H, flag, Hz);
  return hipGetLastError();
}

// Signature decode + G2 subgroup check of item blockIdx.x on one wave (per-call path; k_sig_validate semantics:
// the identity encoding is accepted, every other failure is invalid).  Decoding up to the Montgomery x on every
// lane (g2_decompress_lane_w's checks), then in wide arithmetic (both halves, the same chain): y^2 = x^3 + 4(1 + u)
// by the norm square root (bls_lane.h fp2_sqrt_lane_i; the pure-Fp case, unreachable for x of a valid point with
// probability ~2^-381, runs fp2_sqrt_lane_i on the lanes -- a wave-uniform branch), the sign, and
// psi(sigma) == -[|x|] sigma through the wide Jacobian chain (an exceptional addition means a small order: reject).
// Two waves: wave 1 only multiplies in the square roots' exponentiations (wpow_2w) and otherwise repeats wave 0.
__global__ void __launch_bounds__(128) k_sig_validate_wide(const uint8_t* sigs96, size_t n, G2A* out, int* ok) {
  const size_t i = blockIdx.x;
  if (i >= n) return;  // (the whole workgroup)
  __shared__ uint32_t pring[PW_RING * 64];
  __shared__ int pcnt[2];
  const int wv = (int)(threadIdx.x >> 6);
  const WKG K = wkg_init();
  const WK K1 = wk_of(K);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(sigs96 + 96 * i);
  Fp x1, x0;
#pragma unroll
  for (int k = 0; k < 12; k++) {
    x1.l[11 - k] = __builtin_bswap32(w[k]);
    x0.l[11 - k] = __builtin_bswap32(w[12 + k]);
  }
  const uint32_t f = x1.l[11] >> 24;
  const bool c_flag = f & 0x80, b_flag = f & 0x40, a_flag = f & 0x20;
  x1.l[11] &= 0x1fffffffu;
  const bool x_zero = fp_is_zero(x1) && fp_is_zero(x0);
  G2A s{fp2_zero(), fp2_zero(), true};
  int v = 0;
  // every condition below is wave-uniform (all lanes decode the same bytes)
  if (c_flag && b_flag == x_zero) {
    if (x_zero) {
      v = a_flag ? 0 : 1;  // the identity encoding
    } else if (raw_lt_p(x1) && raw_lt_p(x0)) {
      const W2 xm = w2_from_fp2(Fp2{fp_mul_i(x0, FP_R2), fp_mul_i(x1, FP_R2)});
      const W2 rhs = w2add(w2mul(K1, w2sqr(K1, xm), xm), w2const(FP2_B2));
      W2 y{0u, 0u};
      bool on = true;
      if (w_is_zero(rhs.c1)) {  // rhs in Fp: the lane form
        Fp2 yl;
        on = fp2_sqrt_lane_i(yl, w2_to_fp2(rhs));
        y = w2_from_fp2(yl);
      } else {
        const uint32_t nrm = wadd(wsqr(rhs.c0), wsqr(rhs.c1));
        const uint32_t nr = wpow_2w(nrm, EXP_SQRT, EXP_SQRT_BITS, pring, pcnt, wv);
        on = w_eq(K1, wsqr(nr), nrm);
        const uint32_t inv2 = w_from_fp(FP_INV2);
        const uint32_t t = wmul(wadd(rhs.c0, nr), inv2);
        const uint32_t sr = wpow_2w(t, EXP_SQRT_M3, EXP_SQRT_M3_BITS, pring, pcnt, wv);
        const uint32_t ts = wmul(t, sr), hs = wmul(wmul(rhs.c1, inv2), sr);
        const bool tsq = w_is_one(wmul(ts, sr));
        const uint32_t nts = wneg(K1, ts);
        y = w2red(K, W2{tsq ? ts : hs, tsq ? hs : nts});
      }
      if (on) {
        const Fp2 yl = w2_to_fp2(y);
        if (fp2_lex_largest(yl) != a_flag) y = w2neg(K1, y);
        y = w2red(K, y);
        bool exc = false;
        // the subgroup chain in F2 layout (bls_wide_g2.h J2F)
        const uint32_t xf = wf_of_w2(xm), yf = wf_of_w2(y), kn = K.kneg;
        const J2F M = j2f_mul_xabs(K, J2F{xf, yf, wf_from_fp2(fp2_one())}, exc);
        // psi(sigma) == -M:  conj(x) CX Z^2 == X,  conj(y) CY Z^3 == -Y,  Z != 0
        const uint32_t zz = wf_mul(kn, M.z, M.z);
        const uint32_t px = wf_mul(kn, wf_mul(kn, wf_conj(K.k1, xf), wf_from_fp2(PSI_CX)), zz);
        const uint32_t py = wf_mul(kn, wf_mul(kn, wf_conj(K.k1, yf), wf_from_fp2(PSI_CY)), wf_mul(kn, zz, M.z));
        const bool zx = wf_is_zero(wsubk(K.k2048_2, px, M.x));  // M.x < 1028p (the chain ends on a doubling)
        const bool zy = wf_is_zero(wadd(py, M.y));
        const bool zz0 = wf_is_zero(M.z);
        if (!exc && !zz0 && zx && zy) {
          v = 1;
          s = G2A{w2_to_fp2(xm), w2_to_fp2(y), false};
        }
      }
    }
  }
  if (threadIdx.x == 0) {
    out[i] = s;
    ok[i] = v;
  }
}

hipError_t launch_sig_validate_wide(hipStream_t st, const uint8_t* sigs, size_t n, G2A* out, int* ok) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_sig_validate_wide, dim3((unsigned)n), dim3(128), 0, st, sigs, n, out, ok);
  return hipGetLastError();
}

// ---- G1: KeyValidate with two keys per wave (one per half) ------------------
// bls_fq_g1.h g1q_add_aff / g1q_add / g1q_dbl (complete projective, a = 0, 3b = 12) with the same subtraction
// constants (64p, 128p) and the same value bounds (accumulator X < 66p, Y, Z < 4p; products below 2.0001p).
struct G1W {
  uint32_t x, y, z;
};
__device__ __forceinline__ G1W g1w_add_aff(const WKG& K, const G1W& p, uint32_t x2, uint32_t y2) {
  const uint32_t t0 = wmul(p.x, x2);
  const uint32_t t1 = wmul(p.y, y2);
  const uint32_t t3 = wsubk(K.k2, wmul(wadd(x2, y2), wadd(p.x, p.y)), wadd(t0, t1));
  const uint32_t t4 = wadd(wmul(y2, p.z), p.y);
  const uint32_t y3 = wmuls<12>(wadd(wmul(x2, p.z), p.x));
  const uint32_t t0p = wmuls<3>(t0);
  const uint32_t t2 = wmuls<12>(p.z);
  const uint32_t z3 = wadd(t1, t2);
  const uint32_t t1p = wsubk(K.k1, t1, t2);
  G1W r;
  r.x = wsubk(K.k1, wmul(t3, t1p), wmul(t4, y3));
  r.y = wadd(wmul(t1p, z3), wmul(y3, t0p));
  r.z = wadd(wmul(z3, t4), wmul(t0p, t3));
  return r;
}
__device__ __forceinline__ G1W g1w_add(const WKG& K, const G1W& p, const G1W& q) {
  const uint32_t t0 = wmul(p.x, q.x), t1 = wmul(p.y, q.y), t2 = wmul(p.z, q.z);
  const uint32_t t3 = wsubk(K.k2, wmul(wadd(p.x, p.y), wadd(q.x, q.y)), wadd(t0, t1));
  const uint32_t t4 = wsubk(K.k2, wmul(wadd(p.y, p.z), wadd(q.y, q.z)), wadd(t1, t2));
  const uint32_t y3 = wmuls<12>(wsubk(K.k2, wmul(wadd(p.x, p.z), wadd(q.x, q.z)), wadd(t0, t2)));
  const uint32_t t0p = wmuls<3>(t0);
  const uint32_t t2p = wmuls<12>(t2);
  const uint32_t z3 = wadd(t1, t2p);
  const uint32_t t1p = wsubk(K.k1, t1, t2p);
  G1W r;
  r.x = wsubk(K.k1, wmul(t3, t1p), wmul(t4, y3));
  r.y = wadd(wmul(t1p, z3), wmul(y3, t0p));
  r.z = wadd(wmul(z3, t4), wmul(t0p, t3));
  return r;
}
// Complete projective doubling (RCB alg. 9, a = 0, as bls_fq.h's G1 chain) on FOUR waves of one workgroup (the
// per-call key check, k_key_validate_wide): its eight products have dependency depth 2 -- {Y^2, Y Z, Z^2, X Y}, then {t2 z8, t1 z8, w (t0 + t2), w u} -- so wave w
// forms product w of each level, the waves exchange them through LDS (one barrier per level), and every wave ends
// with the whole point.  x4: 8 x 64 words of LDS; w: this wave's index (0 .. 3), uniform per wave.
__device__ __forceinline__ G1W g1w_dbl4(const WKG& K, const G1W& p, uint32_t* x4, int w) {
  const int l = wlane();
  uint32_t m1;
  if (w == 0)
    m1 = wmul(p.y, p.y);
  else if (w == 1)
    m1 = wmul(p.y, p.z);
  else if (w == 2)
    m1 = wmul(p.z, p.z);
  else
    m1 = wmul(p.x, p.y);
  x4[w * 64 + l] = m1;
  __syncthreads();
  const uint32_t t0 = x4[l], t1 = x4[64 + l], t2 = wmuls<12>(x4[128 + l]), u = x4[192 + l];
  const uint32_t z8 = wmuls<8>(t0);
  const uint32_t wv = wsubk(K.k2, t0, wmuls<3>(t2));
  uint32_t m2;
  if (w == 0)
    m2 = wmul(t2, z8);
  else if (w == 1)
    m2 = wmul(t1, z8);
  else if (w == 2)
    m2 = wmul(wv, wadd(t0, t2));
  else
    m2 = wmul(wv, u);
  x4[(4 + w) * 64 + l] = m2;
  __syncthreads();
  G1W r;
  r.z = x4[320 + l];
  r.y = wadd(x4[384 + l], x4[256 + l]);
  r.x = wmuls<2>(x4[448 + l]);
  return r;
}

// [|x|] b with the doublings on four waves (the additions on every wave)
template <bool AFF>
__device__ __forceinline__ G1W g1w_mul_xabs4(const WKG& K, const G1W& b, uint32_t* x4, int w) {
  G1W m = b;
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    m = g1w_dbl4(K, m, x4, w);
    if ((X_ABS >> i) & 1ull) m = AFF ? g1w_add_aff(K, m, b.x, b.y) : g1w_add(K, m, b);
  }
  return m;
}

// KeyValidate of keys 2 blockIdx.x + half (k_key_validate semantics; the decode on every lane of the half, the
// square root and both [|x|] chains in wide arithmetic), on a workgroup of four waves doing the same work except
// the chains' doublings, whose products are spread over the four (g1w_dbl4).  Wave-uniform control flow: the two
// halves' decode verdicts are combined into selects, not branches.  INF_OK: the checked G1 decode of the pairing APIs
// (k_pt_decode semantics: the identity encoding is a valid point) instead of KeyValidate's rejection of it.
template <bool INF_OK>
__global__ void __launch_bounds__(256) k_key_validate_wide(const uint8_t* pks48, size_t n, G1A* out, int* ok) {
  const size_t base = 2 * (size_t)blockIdx.x;
  if (base >= n) return;  // (the whole workgroup)
  __shared__ uint32_t x4[8 * 64];
  const int wv = (int)(threadIdx.x >> 6);
  const WKG K = wkg_init();
  const WK K1 = wk_of(K);
  const int h = whalf();
  const size_t i = base + (size_t)h < n ? base + (size_t)h : base;  // an odd tail: half 1 repeats key base
  const uint32_t* w = reinterpret_cast<const uint32_t*>(pks48 + 48 * i);
  Fp x;
#pragma unroll
  for (int k = 0; k < 12; k++) x.l[11 - k] = __builtin_bswap32(w[k]);
  const uint32_t flags = x.l[11] >> 24;
  const bool c_flag = flags & 0x80, b_flag = flags & 0x40, a_flag = flags & 0x20;
  x.l[11] &= 0x1fffffffu;
  const bool fmt = c_flag && !b_flag && !fp_is_zero(x) && raw_lt_p(x);
  const Fp xc = fp_mul_i(fmt ? x : FP_ONE, FP_R2);  // a malformed key runs the chain on a dummy, then fails
  const uint32_t xm = w_from_fp(xc);
  const uint32_t rhs = wadd(wmul(wsqr(xm), xm), w_from_fp(FP_B1));
  const uint32_t y0 = wpow(rhs, EXP_SQRT, EXP_SQRT_BITS);
  const bool on = w_eq(K1, wsqr(y0), rhs);
  const uint32_t yr = wmul(y0, K.one);  // below 2.0001p
  const Fp yl = w_to_fp(yr);
  const bool flip = raw_gt_half(fp_from_mont(yl)) != a_flag;
  const uint32_t ny = wmul(wneg(K1, yr), K.one);
  const uint32_t y = flip ? ny : yr;
  const G1W P{xm, y, K.one};
  const G1W Q = g1w_mul_xabs4<false>(K, g1w_mul_xabs4<true>(K, P, x4, wv), x4, wv);
  if (wv) return;  // waves 1 .. 3: no barrier after the chains
  const bool eq_x = w_eq(K1, wmul(wmul(xm, w_from_fp(FP_BETA)), Q.z), wmul(Q.x, K.one));
  const bool eq_y = w_is_zero(wadd(wmul(y, Q.z), Q.y));
  const bool v = fmt && on && eq_x && eq_y;
  const bool id = INF_OK && c_flag && b_flag && !a_flag && fp_is_zero(x);
  const G1A a = v ? G1A{w_to_fp(xm), w_to_fp(y), false} : G1A{fp_zero(), fp_zero(), true};
  if (wpos() == 0 && base + (size_t)h < n) {
    out[base + h] = a;
    ok[base + h] = v || id ? 1 : 0;
  }
}

hipError_t launch_key_validate_wide(hipStream_t st, const uint8_t* pks, size_t n, G1A* out, int* ok) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_key_validate_wide<false>, dim3((unsigned)((n + 1) / 2)), dim3(256), 0, st, pks, n, out, ok);
  return hipGetLastError();
}

hipError_t launch_g1_decode_checked_wide(hipStream_t st, const uint8_t* in48, size_t n, G1A* out, int* ok) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_key_validate_wide<true>, dim3((unsigned)((n + 1) / 2)), dim3(256), 0, st, in48, n, out, ok);
  return hipGetLastError();
}

// ---- Miller loop in F2 layout (per-call path) ------------------------------
// Split like the batch kernels: the G2 side (T and the line records) per pair, then the f accumulation shared by
// the pairs.  Line record of a step: (l0, l2, l3) with the P factors applied (l2 = (E ZZ) (-x_P) or r (-x_P),
// l3 = (z3 ZZ) y_P or z3 y_P; bls_pairing.h ml_dbl_step / ml_add_step), three Fp2 in F2 layout = 3 x 64 words.
// A pair that is not live runs with P = (0, 0) and Q = the G2 generator: its lines are constants in Fp2, which
// the final exponentiation maps to 1 (as k_miller2_vm).
constexpr int MLW_STEPS = 68;  // 63 doublings + 5 additions

// one wave per pair; every Fp2 in F2 layout, products one after another.  Value bounds (units of p; products
// < 2.0001): doubling in X < 516, Y, Z < 66 -> X3 < 516, Y3, Z3 < 66; addition -> all < 66; lines l0 < 66,
// l2 and l3 products.  Subtraction constants: 64p for products and small sums, 256p / 512p / 1024p where the
// subtrahend is a coordinate; the Fp2 products negate with 4096p (kneg), squarings with 2048p.
struct WaveBar {  // barrier of the first nw waves of the workgroup: cnt counts arrivals, gen is this wave's target
  int* cnt;
  int gen, nw;
  __device__ void sync() {
    gen += nw;
    if (wlane() == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < gen) __builtin_amdgcn_s_sleep(1);
  }
};

struct LineW {
  uint32_t X, Y, Z, xQ, yQ, nxP, yP;
  // Q in Jacobian coordinates (jac: xQ, yQ are X_Q, Y_Q): Z_Q, Z_Q^2, Z_Q^3, X_Q Z_Q for the additions
  uint32_t zq, zq2, zq3, xzq;
  bool jac;
  // P in Jacobian coordinates (pz): x_P = X / Z^2, y_P = Y / Z^3, so Z^3 l(P) = Z^3 l0 + l2 (-X Z) + l3 Y: the
  // P factors -X Z and Y and every record's l0 times zp3 = Z^3 (an Fp factor: the same final exponentiation)
  uint32_t zp3;
  bool pjac;
  __device__ void init(const WKG& K, const G1A& P, const G2A& Q, bool live, const Fp2* qz = nullptr,
                       const Fp* pz = nullptr) {
    const G2A q = live ? Q : g2_generator();
    pjac = live && pz;  // (wave-uniform)
    nxP = live ? w_from_fp(fp_neg(pjac ? fp_mul(P.x, *pz) : P.x)) : 0u;
    yP = live ? w_from_fp(P.y) : 0u;
    if (pjac) zp3 = w_from_fp(fp_mul(fp_sqr(*pz), *pz));
    xQ = wf_from_fp2(q.x);
    yQ = wf_from_fp2(q.y);
    X = xQ;
    Y = yQ;
    jac = live && qz;  // (wave-uniform)
    Z = wf_from_fp2(jac ? *qz : fp2_one());
    if (jac) {
      zq = Z;
      zq2 = wf_sqr(K.k2048_2, Z);
      zq3 = wf_mul(K.kneg, zq2, Z);
      xzq = wf_mul(K.kneg, xQ, Z);
    }
  }
  // the doubling step on the pair's three line waves (w = 0, 1, 2): dbl's thirteen products in five rounds --
  // {A = X^2, B = Y^2, ZZ = Z^2}, {(Y + Z)^2, C = B^2, F = E^2}, {(X + B)^2, E X, E ZZ}, {z3 ZZ, E (D - x3),
  // E ZZ (-x_P)}, then l3 on wave 0 alone -- exchanged through xs (12 x 64 words) with the trio's counter barrier
  // tb (the f waves never wait on it).  Every wave ends with T = 2T (dbl-2009-l); wave 0 writes the record
  // (l0, l2, l3) into o[0], o[64], o[128].
  __device__ void dbl3(const WKG& K, uint32_t* o, uint32_t* xs, int w, WaveBar& tb) {
    const uint32_t kn = K.kneg, ks = K.k2048_2;
    const int l = wlane();
    xs[w * 64 + l] = w == 0 ? wf_sqr(ks, X) : (w == 1 ? wf_sqr(ks, Y) : wf_sqr(ks, Z));
    tb.sync();
    const uint32_t A = xs[l], B = xs[64 + l], ZZ = xs[128 + l];
    const uint32_t E = wmuls<3>(A);
    xs[(3 + w) * 64 + l] = w == 0 ? wf_sqr(ks, wadd(Y, Z)) : (w == 1 ? wf_sqr(ks, B) : wf_sqr(ks, E));
    tb.sync();
    const uint32_t YZ2 = xs[192 + l], C = xs[256 + l], F = xs[320 + l];
    xs[(6 + w) * 64 + l] = w == 0 ? wf_sqr(ks, wadd(X, B)) : (w == 1 ? wf_mul(kn, E, X) : wf_mul(kn, E, ZZ));
    tb.sync();
    const uint32_t XB = xs[384 + l], EX = xs[448 + l], EZZ = xs[512 + l];
    const uint32_t D = wmuls<2>(wsubk(K.k1, XB, wadd(A, C)));
    const uint32_t x3 = wsubk(K.k512_2, F, wmuls<2>(D));
    const uint32_t z3 = wsubk(K.k1, YZ2, wadd(B, ZZ));
    xs[(9 + w) * 64 + l] =
        w == 0 ? wf_mul(kn, z3, ZZ) : (w == 1 ? wf_mul(kn, E, wsubk(K.k1024, D, x3)) : wmul(EZZ, nxP));
    tb.sync();
    const uint32_t y3 = wsubk(K.k1, xs[640 + l], wmuls<8>(C));
    if (w == 0) {
      const uint32_t l0 = wsubk(K.k1, EX, wmuls<2>(B));
      o[0] = pjac ? wmul(l0, zp3) : l0;
      o[64] = xs[704 + l];
      o[128] = wmul(xs[576 + l], yP);
    }
    X = x3;
    Y = y3;
    Z = z3;
  }
  // addition of Q (affine): T = T + Q, the record into o (by the writing wave only, when write)
  __device__ void add(const WKG& K, uint32_t* o, bool write = true) {
    if (jac) return add_jac(K, o, write);
    const uint32_t kn = K.kneg, ks = K.k2048_2;
    const uint32_t z1z1 = wf_sqr(ks, Z);
    const uint32_t u2 = wf_mul(kn, xQ, z1z1);
    const uint32_t s2 = wf_mul(kn, wf_mul(kn, yQ, Z), z1z1);
    const uint32_t h = wsubk(K.k1024, u2, X);
    const uint32_t hh = wf_sqr(ks, h);
    const uint32_t i4 = wmuls<4>(hh);
    const uint32_t j = wf_mul(kn, h, i4);
    const uint32_t r = wmuls<2>(wsubk(K.k256, s2, Y));
    const uint32_t v = wf_mul(kn, X, i4);
    const uint32_t x3 = wsubk(K.k1, wf_sqr(ks, r), wadd(j, wmuls<2>(v)));
    const uint32_t y3 = wsubk(K.k1, wf_mul(kn, r, wsubk(K.k256, v, x3)), wmuls<2>(wf_mul(kn, Y, j)));
    const uint32_t z3 = wsubk(K.k1, wf_sqr(ks, wadd(Z, h)), wadd(z1z1, hh));
    if (write) {
      const uint32_t l0 = wsubk(K.k1, wf_mul(kn, r, xQ), wf_mul(kn, yQ, z3));
      o[0] = pjac ? wmul(l0, zp3) : l0;
      o[64] = wmul(r, nxP);
      o[128] = wmul(z3, yP);
    }
    X = x3;
    Y = y3;
    Z = z3;
  }
  // addition of a Jacobian Q (add-2007-bl: U1 = X Z_Q^2, S1 = Y Z_Q^3, H = U2 - U1, r = 2 (S2 - S1), Z3 = 2 Z Z_Q H).
  // The slope is r / Z3, so Z3 Z_Q^3 l(P) = Z3 Z_Q^3 y_P - r Z_Q^3 x_P + (r X_Q Z_Q - Y_Q Z3): the record
  // (l0, l2, l3) = (r X_Q Z_Q - Y_Q Z3, r Z_Q^3 (-x_P), Z3 Z_Q^3 y_P), the affine record times Z_Q^3 (an Fp2 factor,
  // which the final exponentiation maps to 1).  Bounds as the affine addition: every subtrahend a product or X < 516p.
  __device__ void add_jac(const WKG& K, uint32_t* o, bool write) {
    const uint32_t kn = K.kneg, ks = K.k2048_2;
    const uint32_t z1z1 = wf_sqr(ks, Z);
    const uint32_t u1 = wf_mul(kn, X, zq2);
    const uint32_t u2 = wf_mul(kn, xQ, z1z1);
    const uint32_t s1 = wf_mul(kn, Y, zq3);
    const uint32_t s2 = wf_mul(kn, wf_mul(kn, yQ, Z), z1z1);
    const uint32_t h = wsubk(K.k1, u2, u1);
    const uint32_t hh = wf_sqr(ks, h);
    const uint32_t i4 = wmuls<4>(hh);
    const uint32_t j = wf_mul(kn, h, i4);
    const uint32_t r = wmuls<2>(wsubk(K.k1, s2, s1));
    const uint32_t v = wf_mul(kn, u1, i4);
    const uint32_t x3 = wsubk(K.k1, wf_sqr(ks, r), wadd(j, wmuls<2>(v)));
    const uint32_t y3 = wsubk(K.k1, wf_mul(kn, r, wsubk(K.k256, v, x3)), wmuls<2>(wf_mul(kn, s1, j)));
    const uint32_t z3 = wf_mul(kn, wmuls<2>(wf_mul(kn, Z, zq)), h);
    if (write) {
      const uint32_t l0 = wsubk(K.k1, wf_mul(kn, r, xzq), wf_mul(kn, yQ, z3));
      o[0] = pjac ? wmul(l0, zp3) : l0;
      o[64] = wmul(wf_mul(kn, r, zq3), nxP);
      o[128] = wmul(wf_mul(kn, z3, zq3), yP);
    }
    X = x3;
    Y = y3;
    Z = z3;
  }
};

// f accumulation (k_miller_wide below): six waves, wave k owns the w^k coefficient of f (w-basis: w^6 = xi; w^2k is c0.c_k, w^(2k+1)
// is c1.c_k of the tower).  f lives in LDS in F2 layout; a squaring or line product reads the operands of each of
// the wave's products from LDS, so the per-wave term tables need no register indexing.
//   f^2:  c_k = sum_{i+j=k} a_i a_j + xi sum_{i+j=k+6} a_i a_j   (3-4 products per wave)
//   f l:  c_k = a_k l0 + a_{k-2} l2 + a_{k-3} l3  (indices mod 6, xi on wrap-around)   (3 products)
// Values: f below ~100p (sums of <= 4 products and one xi), lines below 66p: every product operand pair is far
// below p R, every xi argument (a sum of products, < 10.001p) below the 64p it is negated against.
__constant__ uint8_t FSQ_TERMS[6][4][4] = {  // (i, j, multiplier, xi) ; multiplier 0 pads
    {{0, 0, 1, 0}, {1, 5, 2, 1}, {2, 4, 2, 1}, {3, 3, 1, 1}},
    {{0, 1, 2, 0}, {2, 5, 2, 1}, {3, 4, 2, 1}, {0, 0, 0, 0}},
    {{0, 2, 2, 0}, {1, 1, 1, 0}, {3, 5, 2, 1}, {4, 4, 1, 1}},
    {{0, 3, 2, 0}, {1, 2, 2, 0}, {4, 5, 2, 1}, {0, 0, 0, 0}},
    {{0, 4, 2, 0}, {1, 3, 2, 0}, {2, 2, 1, 0}, {5, 5, 1, 1}},
    {{0, 5, 2, 0}, {1, 4, 2, 0}, {2, 3, 2, 0}, {0, 0, 0, 0}}};

// Fused per-call Miller loop: waves 0..5 accumulate f (each f^2 and f l as ONE reduction of
// lazily summed products, f ping-ponging between two LDS banks), waves 6 + 3 p .. 8 + 3 p run pair p's G2 side
// (LineW, each doubling's products over the three: dbl3) and the first of them writes its line records into LDS.  The two sides meet through per-pair progress counters (release / acquire at
// workgroup scope); the six f waves synchronise among themselves through a counter barrier, since the line waves
// never join an s_barrier after the start.  The line records of all steps fit in LDS (2 x 68 x 768 B).
constexpr int MLF_PAIRS = 2;

constexpr int MLF_LW = 3;  // line waves per pair
// okv != nullptr (launch_miller_wide_n): workgroup b runs pairs 2b, 2b + 1 of npairs (okv per pair, or none)
// into out[b]; otherwise one workgroup, npairs <= 2, ok0 / ok1 per pair
__global__ void __launch_bounds__(64 * (6 + MLF_LW * MLF_PAIRS)) k_miller_wide(const G1A* P, const G2A* Q,
                                                                               const int* ok0, const int* ok1,
                                                                               int npairs, Fp12* out,
                                                                               const int* okv, int per_block,
                                                                               const Fp2* qz, const Fp* pz) {
  if (per_block) {
    const int b = (int)blockIdx.x;
    P += MLF_PAIRS * b;
    Q += MLF_PAIRS * b;
    if (qz) qz += MLF_PAIRS * b;
    if (pz) pz += MLF_PAIRS * b;
    out += b;
    ok0 = okv ? okv + MLF_PAIRS * b : nullptr;
    ok1 = okv ? okv + MLF_PAIRS * b + 1 : nullptr;
    npairs = npairs - MLF_PAIRS * b < MLF_PAIRS ? npairs - MLF_PAIRS * b : MLF_PAIRS;
  }
  __shared__ uint32_t lr[MLF_PAIRS][MLW_STEPS][3 * 64];
  __shared__ uint32_t fs[2][6 * 64];
  __shared__ uint32_t xs[MLF_PAIRS][12 * 64];
  __shared__ int prog[MLF_PAIRS];
  __shared__ int tbc[MLF_PAIRS];
  __shared__ int barc;
  const WKG K = wkg_init();
  const int lane = wlane(), k = (int)(threadIdx.x >> 6);
  if (threadIdx.x < MLF_PAIRS) {
    prog[threadIdx.x] = 0;
    tbc[threadIdx.x] = 0;
  }
  if (threadIdx.x == 0) barc = 0;
  if (k < 6) fs[0][k * 64 + lane] = k == 0 ? wf_from_fp2(fp2_one()) : 0u;
  __syncthreads();
  if (k >= 6) {  // G2 side of pair (k - 6) / 3, wave (k - 6) % 3 of its trio
    const int pi = (k - 6) / MLF_LW, w3 = (k - 6) % MLF_LW;
    if (pi >= npairs) return;  // (the whole trio)
    LineW T;
    const int* okp = pi ? ok1 : ok0;
    T.init(K, P[pi], Q[pi], (!okp || *okp) && !P[pi].inf && !Q[pi].inf, qz ? qz + pi : nullptr,
           pz ? pz + pi : nullptr);
    WaveBar tb{&tbc[pi], 0, MLF_LW};
    int step = 0;
#pragma unroll 1
    for (int b = 62; b >= 0; --b) {
      T.dbl3(K, &lr[pi][step][lane], xs[pi], w3, tb);
      ++step;
      if (w3 == 0 && lane == 0) __hip_atomic_store(&prog[pi], step, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      if ((X_ABS >> b) & 1ull) {
        T.add(K, &lr[pi][step][lane], w3 == 0);
        ++step;
        if (w3 == 0 && lane == 0)
          __hip_atomic_store(&prog[pi], step, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    return;
  }
  WaveBar bar{&barc, 0, 6};
  const uint32_t kn = K.kneg;
  int c = 0, step = 0;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) {  // f = f^2: sum over FSQ_TERMS of (m a_i, xi on wrap) a_j
      const uint32_t* f = fs[c];
      uint64_t acc = 0;
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const uint32_t ii = FSQ_TERMS[k][t][0], jj = FSQ_TERMS[k][t][1], m = FSQ_TERMS[k][t][2];
        if (!m) continue;
        uint32_t x = f[ii * 64 + lane];
        x = m == 2 ? wmuls<2>(x) : x;
        x = FSQ_TERMS[k][t][3] ? wf_xi(K.k256, x) : x;
        wf_mac(acc, kn, x, f[jj * 64 + lane]);
      }
      fs[c ^ 1][k * 64 + lane] = wredc(acc);
      c ^= 1;
      bar.sync();
    }
    const int nl = ((X_ABS >> b) & 1ull) ? 2 : 1;
#pragma unroll 1
    for (int sl = 0; sl < nl; ++sl, ++step) {
#pragma unroll 1
      for (int pi = 0; pi < npairs; ++pi) {
        while (__hip_atomic_load(&prog[pi], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= step)
          __builtin_amdgcn_s_sleep(1);
        const uint32_t* l = &lr[pi][step][lane];
        const uint32_t* f = fs[c];
        const int i2 = k < 2 ? k + 4 : k - 2, i3 = k < 3 ? k + 3 : k - 3;
        uint64_t acc = 0;
        wf_mac(acc, kn, f[k * 64 + lane], l[0]);
        const uint32_t f2 = f[i2 * 64 + lane], f3 = f[i3 * 64 + lane];
        wf_mac(acc, kn, k < 2 ? wf_xi(K.k256, f2) : f2, l[64]);
        wf_mac(acc, kn, k < 3 ? wf_xi(K.k256, f3) : f3, l[128]);
        fs[c ^ 1][k * 64 + lane] = wredc(acc);
        c ^= 1;
        bar.sync();
      }
    }
  }
  // x < 0: conjugate (negate the odd w-coefficients); canonical Fp2 into the tower slot of w^k
  const uint32_t v0 = fs[c][k * 64 + lane];
  const Fp2 v = wf_to_fp2((k & 1) ? wnorm(K.k1 - v0) : v0);  // f values below 1.1 p
  if (lane == 0) {
    Fp6& h6 = (k & 1) ? out->c1 : out->c0;
    Fp2& dst = (k >> 1) == 0 ? h6.c0 : ((k >> 1) == 1 ? h6.c1 : h6.c2);
    dst = v;
  }
}

hipError_t launch_miller_wide(hipStream_t st, const G1A* P, const G2A* Q, const int* ok0, const int* ok1, int npairs,
                              Fp12* out, const Fp2* qz, const Fp* pz) {
  if (npairs < 1 || npairs > MLF_PAIRS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_miller_wide, dim3(1), dim3(64 * (6 + MLF_LW * MLF_PAIRS)), 0, st, P, Q, ok0, ok1, npairs, out,
                     nullptr, 0, qz, pz);
  return hipGetLastError();
}

// n pairs on ceil(n / 2) workgroups of k_miller_wide (one f per workgroup, out[0 .. (n + 1) / 2)): the latency of
// one wide Miller loop for a few hundred pairs, where the lane kernels' chains take ~2 ms whatever n
size_t miller_wide_nf(size_t n) { return (n + MLF_PAIRS - 1) / MLF_PAIRS; }

hipError_t launch_miller_wide_n(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, Fp12* out,
                                const Fp2* qz) {
  if (!n) return hipSuccess;
  if (n > (size_t)1 << 20) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_miller_wide, dim3((unsigned)((n + MLF_PAIRS - 1) / MLF_PAIRS)),
                     dim3(64 * (6 + MLF_LW * MLF_PAIRS)), 0, st, P, Q, nullptr, nullptr, (int)n, out, ok, 1,
                     qz, (const Fp*)nullptr);
  return hipGetLastError();
}

hipError_t launch_wide_selftest(hipStream_t st, size_t nw, const uint8_t* be48, int* bad) {
  if (!nw) return hipSuccess;
  hipLaunchKernelGGL(k_wide_selftest, dim3((unsigned)nw), dim3(64), 0, st, nw, be48, bad);
  return hipGetLastError();
}

}  // namespace bls
