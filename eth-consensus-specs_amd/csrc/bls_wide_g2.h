// G2 arithmetic in the wavefront-cooperative form of bls_wide.h (Fp2 as a pair
// of D-layout values per half-wave, two independent points per wave): the
// Jacobian chain formulas of bls_fq_g2.h with the SAME subtraction constants,
// so their value bounds (X < 1030p, Y < 650p, Z < 270p in the chain) carry
// over -- a wide product leaves a value below 2.0001p where the lane form's
// leaves one below 2p, well inside the slack of every bound there -- and the
// simplified SWU map and 3-isogeny of bls_lane.h / bls_fav_kernels.hip with
// canonical subtrahends (products, < 2.0001p) against 64p.  Zero and sign tests
// read a half's digits into every lane (w_to_fp) and decide there; they are the
// only lane-local work and run a handful of times per chain.
#pragma once
#include "bls_constants.h"
#include "bls_fp_inv.h"
#include "bls_fq_g2.h"
#include "bls_lane.h"
#include "bls_wide.h"

namespace bls {
namespace wide {

// per-lane digit vectors of the subtraction constants of bls_fq_g2.h (and R mod p), built once per kernel
struct WKG {
  uint32_t k1, k2, k256, k512_2, k1024, k2048_2, kneg, one;
};
__device__ __forceinline__ WKG wkg_init() {
  const int j = wdig();
  const Fq o = fq_unpack(FP_ONE);
  WKG r{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const bool s = j == i;
    r.k1 = s ? Q29_K1[i] : r.k1;
    r.k2 = s ? Q29_K2[i] : r.k2;
    r.k256 = s ? Q29_K256[i] : r.k256;
    r.k512_2 = s ? Q29_K512_2[i] : r.k512_2;
    r.k1024 = s ? Q29_K1024[i] : r.k1024;
    r.k2048_2 = s ? Q29_K2048_2[i] : r.k2048_2;
    r.kneg = s ? Q29_KNEG.d[i] : r.kneg;
    r.one = s ? o.d[i] : r.one;
  }
  return r;
}
__device__ __forceinline__ WK wk_of(const WKG& K) { return WK{K.k1, K.one, 0u}; }

// a + K - b per coefficient (K covering b's digits and value)
__device__ __forceinline__ uint32_t wsubk(uint32_t k, uint32_t a, uint32_t b) { return wnorm(a + (k - b)); }
__device__ __forceinline__ W2 w2subk(uint32_t k, W2 a, W2 b) { return W2{wsubk(k, a.c0, b.c0), wsubk(k, a.c1, b.c1)}; }
// fq2_mul: c0 = a0 b0 + a1 (4096p - b1), c1 = a0 b1 + a1 b0 (operands below 4096p)
__device__ __forceinline__ W2 w2mulk(const WKG& K, W2 a, W2 b) {
  return W2{wdot2(a.c0, b.c0, a.c1, wnorm(K.kneg - b.c1)), wdot2(a.c0, b.c1, a.c1, b.c0)};
}
// fq2_sqr: (a0 + a1)(a0 - a1 + 2048p), 2 a0 a1 (a1 < 2046p)
__device__ __forceinline__ W2 w2sqrk(const WKG& K, W2 a) {
  return W2{wmul(wadd(a.c0, a.c1), wsubk(K.k2048_2, a.c0, a.c1)), wmuls<2>(wmul(a.c0, a.c1))};
}
// value -> below 2.0001p (a product by R mod p)
__device__ __forceinline__ W2 w2red(const WKG& K, W2 a) { return W2{wmul(a.c0, K.one), wmul(a.c1, K.one)}; }
__device__ __forceinline__ W2 w2const(const Fp2& c) { return w2_from_fp2(c); }

struct J2W {
  W2 x, y, z;
};

// dbl-2009-l (bls_fq_g2.h j2q_dbl): X < 1030p, Y < 650p, Z < 270p in -> X3 < 1028p, Y3 < 194p, Z3 < 260p
__device__ __forceinline__ J2W j2w_dbl(const WKG& K, const J2W& p) {
  const W2 A = w2sqrk(K, p.x);
  const W2 Bq = w2sqrk(K, p.y);
  const W2 C = w2sqrk(K, Bq);
  const W2 XB2 = w2sqrk(K, w2add(p.x, Bq));
  const W2 D = w2muls<2>(w2subk(K.k2, XB2, w2add(A, C)));
  const W2 E = w2muls<3>(A);
  J2W r;
  r.x = w2subk(K.k1024, w2sqrk(K, E), w2muls<2>(D));
  const W2 DX = w2subk(K.k2048_2, D, r.x);
  r.y = w2subk(K.k1, w2mulk(K, E, DX), w2muls<8>(C));
  r.z = w2muls<2>(w2mulk(K, p.y, p.z));
  return r;
}

// add-2007-bl (bls_fq_g2.h j2q_add, incomplete): exc |= h = 0 or an identity operand
__device__ __forceinline__ J2W j2w_add(const WKG& K, const J2W& p, const J2W& q, bool& exc) {
  const W2 z1z1 = w2sqrk(K, p.z);
  const W2 z2z2 = w2sqrk(K, q.z);
  const W2 u1 = w2mulk(K, p.x, z2z2);
  const W2 u2 = w2mulk(K, q.x, z1z1);
  const W2 s1 = w2mulk(K, w2mulk(K, p.y, q.z), z2z2);
  const W2 s2 = w2mulk(K, w2mulk(K, q.y, p.z), z1z1);
  const W2 h = w2subk(K.k256, u2, u1);
  exc = exc | w2_is_zero(h) | w2_is_zero(p.z) | w2_is_zero(q.z);  // no short circuit: no per-half branch
  const W2 rr = w2muls<2>(w2subk(K.k256, s2, s1));
  const W2 i = w2sqrk(K, w2muls<2>(h));
  const W2 j = w2mulk(K, h, i);
  const W2 v = w2mulk(K, u1, i);
  J2W r;
  r.x = w2subk(K.k512_2, w2sqrk(K, rr), w2add(j, w2muls<2>(v)));
  const W2 vx = w2subk(K.k1024, v, r.x);
  r.y = w2subk(K.k512_2, w2mulk(K, rr, vx), w2muls<2>(w2mulk(K, s1, j)));
  const W2 zz = w2subk(K.k2, w2sqrk(K, w2add(p.z, q.z)), w2add(z1z1, z2z2));
  r.z = w2mulk(K, zz, h);
  return r;
}

// [|x|] p (the leading bit of |x| is bit 63)
__device__ __forceinline__ J2W j2w_mul_xabs(const WKG& K, const J2W& p, bool& exc) {
  J2W m = p;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    m = j2w_dbl(K, m);
    if ((X_ABS >> b) & 1ull) m = j2w_add(K, m, p, exc);
  }
  return m;
}

// -P: Y reduced below 2.0001p first, then 64p - Y (< 66p, inside the chain's Y bound)
__device__ __forceinline__ J2W j2w_neg(const WKG& K, const J2W& p) {
  const W2 y = w2red(K, p.y);
  return J2W{p.x, W2{wsubk(K.k1, 0u, y.c0), wsubk(K.k1, 0u, y.c1)}, p.z};
}
// psi(P) = (conj(X) cx, conj(Y) cy, conj(Z)) on Jacobian coordinates (products: every coordinate < 2.0001p)
__device__ __forceinline__ J2W j2w_psi(const WKG& K, const J2W& p, W2 cx, W2 cy) {
  const W2 xc{p.x.c0, wsubk(K.k2048_2, 0u, p.x.c1)}, yc{p.y.c0, wsubk(K.k2048_2, 0u, p.y.c1)};
  const W2 zc = w2red(K, W2{p.z.c0, wsubk(K.k2048_2, 0u, p.z.c1)});
  return J2W{w2mulk(K, xc, cx), w2mulk(K, yc, cy), zc};
}
// psi^2(P) = (X c2x, Y c2y, Z) (c2x, c2y in Fp)
__device__ __forceinline__ J2W j2w_psi2(const WKG& K, const J2W& p, uint32_t c2x, uint32_t c2y) {
  return J2W{w2mulfp(p.x, c2x), w2mulfp(p.y, c2y), p.z};
}

// ---- hash_to_G2 pieces (each half maps its own field element) -------------
__device__ __forceinline__ bool w_is_one(uint32_t v) { return fp_is_one(w_to_fp(v)); }
__device__ __forceinline__ int w2_sgn0(W2 a) { return fp2_sgn0_lane(w2_to_fp2(a)); }

// RFC 9380 simplified SWU on E2' (bls_lane.h map_to_curve_sswu_lane_i, step for step): one exponentiation before
// the final square root; `rare` marks g(x1) = 0 and g(x) in Fp (the caller's item goes to k_h2c_fallback).
// Subtrahends are products or sums of two (< 4.0002p) against 64p; every product operand stays below ~70p.
// ring / cnt / wv (all or none): the two exponentiations on two waves (wpow_2w; every wave of the workgroup calls)
__device__ __forceinline__ void sswu_w(const WKG& K, const Fp2& u_lane, W2& x, W2& y, bool& rare,
                                       uint32_t* ring = nullptr, int* cnt = nullptr, int wv = 0) {
  const WK K1 = wk_of(K);
  const int sgn_u = fp2_sgn0_lane(u_lane);
  const W2 u = w2_from_fp2(u_lane);
  const W2 zu2 = w2mul(K1, w2const(SSWU_Z), w2sqr(K1, u));
  const uint32_t nu = wadd(wsqr(u.c0), wsqr(u.c1));
  const uint32_t knu3 = wmul(w_from_fp(SSWU_K_NORM), wmul(wsqr(nu), nu));
  const W2 den = w2add(w2sqr(K1, zu2), zu2);
  const bool exc = w2_is_zero(den);
  const W2 one2{K.one, 0u};
  const W2 xn0 = w2mul(K1, w2const(SSWU_MINUS_B_OVER_A), w2add(one2, den));
  const W2 xn = w2sel(exc, w2const(SSWU_B_OVER_ZA), xn0);
  const W2 xd = w2sel(exc, one2, den);
  const W2 xd2 = w2sqr(K1, xd);
  // gxn = xn^3 + A xn xd^2 + B xd^3
  const W2 gxn = w2add(w2mul(K1, w2add(w2sqr(K1, xn), w2mul(K1, w2const(SSWU_A), xd2)), xn),
                       w2mul(K1, w2const(SSWU_B), w2mul(K1, xd2, xd)));
  const uint32_t ag = wadd(wsqr(gxn.c0), wsqr(gxn.c1));
  const uint32_t d = wadd(wsqr(xd.c0), wsqr(xd.c1));
  const uint32_t d4 = wsqr(wsqr(d));
  const uint32_t w = wmul(ag, wmul(d4, d));
  const W2 xnc = w2mul(K1, w2conj(K1, xd), xn);  // the conjugate (< 66p) as the first factor: 64p - b1 needs b1 < 62p
  const uint32_t agd4 = wmul(ag, d4), agd = wmul(ag, d);
  const bool ag0 = w_is_zero(ag);
  const uint32_t z = ring ? wpow_2w(w, EXP_SQRT_M3, EXP_SQRT_M3_BITS, ring, cnt, wv)
                          : wpow(w, EXP_SQRT_M3, EXP_SQRT_M3_BITS);
  const uint32_t z2 = wsqr(z);
  const bool square = ag0 | w_is_one(wmul(z2, w));
  const uint32_t dinv0 = wmul(z2, agd4), dinvn = wneg(K1, dinv0);
  const uint32_t dinv = square ? dinv0 : dinvn;
  const W2 x1{wmul(xnc.c0, dinv), wmul(xnc.c1, dinv)};
  const uint32_t c = wmul(agd, z);
  const W2 x2 = w2mul(K1, zu2, x1);
  x = w2sel(square, x1, x2);
  const W2 gx = w2add(w2mul(K1, w2add(w2sqr(K1, x), w2const(SSWU_A)), x), w2const(SSWU_B));
  const uint32_t cn = wmul(knu3, c);
  const uint32_t n = square ? c : cn;
  rare = ag0 | w_is_zero(gx.c1);
  // square root of gx from the root n of its norm (bls_lane.h fp2_sqrt_from_norm_root)
  const uint32_t inv2 = w_from_fp(FP_INV2);
  const uint32_t t = wmul(wadd(gx.c0, n), inv2);
  const uint32_t sr = ring ? wpow_2w(t, EXP_SQRT_M3, EXP_SQRT_M3_BITS, ring, cnt, wv)
                           : wpow(t, EXP_SQRT_M3, EXP_SQRT_M3_BITS);
  const uint32_t ts = wmul(t, sr);
  const uint32_t hs = wmul(wmul(gx.c1, inv2), sr);
  const bool tsq = w_is_one(wmul(ts, sr));
  // every choice below is a select on values computed in both halves: a branch on a per-half condition would run
  // the cross-lane moves (DPP, ds_bpermute) of the products with half of the wave disabled
  const uint32_t nts = wneg(K1, ts);
  const W2 yy = w2red(K, W2{tsq ? ts : hs, tsq ? hs : nts});  // below 2.0001p again before the sign flip
  const W2 ny = w2neg(K1, yy);
  y = w2red(K, w2sel(sgn_u != w2_sgn0(yy), ny, yy));
}

// 3-isogeny E2' -> E2 (RFC 9380 App. E.3) as Jacobian (X Z, Y Z^2, Z) of iso's projective (xnum yden : y ynum xden :
// xden yden) (bls_fav_kernels.hip iso_proj_lane); Z = 0 (a vanishing denominator) is reported through zero
__device__ __forceinline__ J2W iso_w(const WKG& K, W2 x, W2 y, bool& zero) {
  const WK K1 = wk_of(K);
  const W2 xx = w2sqr(K1, x);
  const W2 xxx = w2mul(K1, xx, x);
  const W2 xnum = w2add(w2add(w2mul(K1, w2const(ISO_XNUM_3), xxx), w2mul(K1, w2const(ISO_XNUM_2), xx)),
                        w2add(w2mul(K1, w2const(ISO_XNUM_1), x), w2const(ISO_XNUM_0)));
  const W2 xden = w2add(w2add(xx, w2mul(K1, w2const(ISO_XDEN_1), x)), w2const(ISO_XDEN_0));
  const W2 ynum = w2add(w2add(w2mul(K1, w2const(ISO_YNUM_3), xxx), w2mul(K1, w2const(ISO_YNUM_2), xx)),
                        w2add(w2mul(K1, w2const(ISO_YNUM_1), x), w2const(ISO_YNUM_0)));
  const W2 yden = w2add(w2add(xxx, w2mul(K1, w2const(ISO_YDEN_2), xx)),
                        w2add(w2mul(K1, w2const(ISO_YDEN_1), x), w2const(ISO_YDEN_0)));
  const W2 X = w2mul(K1, xnum, yden), Y = w2mul(K1, w2mul(K1, y, ynum), xden), Z = w2mul(K1, xden, yden);
  zero = w2_is_zero(Z);
  return J2W{w2mulk(K, X, Z), w2mulk(K, Y, w2sqrk(K, Z)), Z};
}

// Jacobian -> affine (x, y) canonical packed; the identity (Z = 0) -> inf
__device__ __forceinline__ G2A j2w_to_aff(const WKG& K, const J2W& p) {
  const uint32_t nz = wadd(wsqr(p.z.c0), wsqr(p.z.c1));  // norm(Z)
  const Fp nl = w_to_fp(nz);
  G2A r{fp2_zero(), fp2_zero(), true};
  const uint32_t ni = w_from_fp(fp_inv_sg_i(nl));
  const W2 zi{wmul(p.z.c0, ni), wneg(wk_of(K), wmul(p.z.c1, ni))};
  const W2 zi2 = w2mulk(K, zi, zi);
  const W2 zi3 = w2mulk(K, zi2, zi);
  const Fp2 x = w2_to_fp2(w2mulk(K, p.x, zi2)), y = w2_to_fp2(w2mulk(K, p.y, zi3));
  if (!fp_is_zero(nl)) r = G2A{x, y, false};
  return r;
}

// ---- G2 Jacobian in F2 layout: one VGPR per coordinate (c0 in half 0, c1 in half 1) --------------------------
// The same formulas, bounds and subtraction constants as J2W; an Fp2 product is one wdot2 per half instead of two
// one after another, so the cofactor chains of hash_to_G2 (after the two halves' SSWU results are added) stop
// computing everything twice.
struct J2F {
  uint32_t x, y, z;
};
// half 0's W2 value in F2 layout (c0 from half 0's c0 register, c1 from half 0's c1 register)
__device__ __forceinline__ uint32_t wf_of_w2(W2 a) {
  const uint32_t s1 = wswap(a.c1);
  return whalf() ? s1 : a.c0;
}
__device__ __forceinline__ J2F j2f_of_j2w(const J2W& p) { return J2F{wf_of_w2(p.x), wf_of_w2(p.y), wf_of_w2(p.z)}; }
// both coefficients zero (the same answer in both halves)
__device__ __forceinline__ bool wf_is_zero(uint32_t v) { return w_is_zero(v) & w_is_zero(wswap(v)); }

__device__ __forceinline__ J2F j2f_dbl(const WKG& K, const J2F& p) {
  const uint32_t ks = K.k2048_2, kn = K.kneg;
  const uint32_t A = wf_sqr(ks, p.x);
  const uint32_t Bq = wf_sqr(ks, p.y);
  const uint32_t C = wf_sqr(ks, Bq);
  const uint32_t XB2 = wf_sqr(ks, wadd(p.x, Bq));
  const uint32_t D = wmuls<2>(wsubk(K.k2, XB2, wadd(A, C)));
  const uint32_t E = wmuls<3>(A);
  J2F r;
  r.x = wsubk(K.k1024, wf_sqr(ks, E), wmuls<2>(D));
  const uint32_t DX = wsubk(K.k2048_2, D, r.x);
  r.y = wsubk(K.k1, wf_mul(kn, E, DX), wmuls<8>(C));
  r.z = wmuls<2>(wf_mul(kn, p.y, p.z));
  return r;
}

__device__ __forceinline__ J2F j2f_add(const WKG& K, const J2F& p, const J2F& q, bool& exc) {
  const uint32_t ks = K.k2048_2, kn = K.kneg;
  const uint32_t z1z1 = wf_sqr(ks, p.z);
  const uint32_t z2z2 = wf_sqr(ks, q.z);
  const uint32_t u1 = wf_mul(kn, p.x, z2z2);
  const uint32_t u2 = wf_mul(kn, q.x, z1z1);
  const uint32_t s1 = wf_mul(kn, wf_mul(kn, p.y, q.z), z2z2);
  const uint32_t s2 = wf_mul(kn, wf_mul(kn, q.y, p.z), z1z1);
  const uint32_t h = wsubk(K.k256, u2, u1);
  exc = exc | wf_is_zero(h) | wf_is_zero(p.z) | wf_is_zero(q.z);
  const uint32_t rr = wmuls<2>(wsubk(K.k256, s2, s1));
  const uint32_t i = wf_sqr(ks, wmuls<2>(h));
  const uint32_t j = wf_mul(kn, h, i);
  const uint32_t v = wf_mul(kn, u1, i);
  J2F r;
  r.x = wsubk(K.k512_2, wf_sqr(ks, rr), wadd(j, wmuls<2>(v)));
  const uint32_t vx = wsubk(K.k1024, v, r.x);
  r.y = wsubk(K.k512_2, wf_mul(kn, rr, vx), wmuls<2>(wf_mul(kn, s1, j)));
  const uint32_t zz = wsubk(K.k2, wf_sqr(ks, wadd(p.z, q.z)), wadd(z1z1, z2z2));
  r.z = wf_mul(kn, zz, h);
  return r;
}

__device__ __forceinline__ J2F j2f_mul_xabs(const WKG& K, const J2F& p, bool& exc) {
  J2F m = p;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    m = j2f_dbl(K, m);
    if ((X_ABS >> b) & 1ull) m = j2f_add(K, m, p, exc);
  }
  return m;
}
// ---- G2 homogeneous projective in F2 layout: the complete formulas of bls_pp_lane.h (Renes-Costello-Batina,
// a = 0, 3b = 12 (1 + i)) as the round-4 wide MSM kernel ran them -- no exceptional cases, so the per-call
// hash's cofactor chains need no fallback flag, and a doubling's eight products have dependency depth 2.
struct P2F {  // (X : Y : Z), every coordinate a product output (< 2.0001 p) on entry to the formulas
  uint32_t x, y, z;
};
// 3 b t = 12 xi t (t below 62 p: the xi subtraction against 64 p)
__device__ __forceinline__ uint32_t wf_b3(const WKG& K, uint32_t t) { return wmuls<12>(wf_xi(K.k1, t)); }

// pp_dbl on FOUR waves of one workgroup (w = 0 .. 3, uniform per wave): t0 = Y^2, t1 = Y Z, Z^2, u = X Y (one per
// wave), then t2 = 3b Z^2, z8 = 8 t0, w = t0 - 3 t2 and X3 = 2 w u, Y3 = w (t0 + t2) + t2 z8 (one reduction of two
// products), Z3 = t1 z8 (waves 1, 0, 2), exchanged through x4 (8 x 64 words) with one barrier per level.
// Bounds (units of p): t0, t1, Z^2, u < 2.0001; t2 < 1500; w < 4100 (against 4096 p covering 3 t2 < 4096 p)
__device__ __forceinline__ P2F p2f_dbl4(const WKG& K, const P2F& p, uint32_t* x4, int w) {
  const uint32_t kn = K.kneg;
  const int l = wlane();
  uint32_t m1;
  if (w == 0)
    m1 = wf_sqr(K.k1, p.y);
  else if (w == 1)
    m1 = wf_mul(kn, p.y, p.z);
  else if (w == 2)
    m1 = wf_sqr(K.k1, p.z);
  else
    m1 = wf_mul(kn, p.x, p.y);
  x4[w * 64 + l] = m1;
  __syncthreads();
  const uint32_t t0 = x4[l], t1 = x4[64 + l], t2 = wf_b3(K, x4[128 + l]), u = x4[192 + l];
  const uint32_t z8 = wmuls<8>(t0);
  const uint32_t wv = wsubk(kn, t0, wmuls<3>(t2));
  if (w == 0) {
    uint64_t acc = 0;
    wf_mac(acc, kn, wv, wadd(t0, t2));
    wf_mac(acc, kn, t2, z8);
    x4[256 + l] = wredc(acc);
  } else if (w == 1) {
    x4[320 + l] = wf_mul(kn, wv, wmuls<2>(u));
  } else if (w == 2) {
    x4[384 + l] = wf_mul(kn, t1, z8);
  }
  __syncthreads();
  return P2F{x4[320 + l], x4[256 + l], x4[384 + l]};
}

// pp_add / pp_finish with the cross terms as sums of products (t3 = X1 Y2 + Y1 X2, ...):
//   X3 = t3 t1' - t4 y3',  Y3 = t1' z3 + y3' 3 t0,  Z3 = z3 t4 + 3 t0 t3   (t1' = t1 - 3b t2, z3 = t1 + 3b t2,
//   y3' = 3b y3), each output one reduction; the big operands (y3' < 790 p) go first, the negated t4 (< 256 p)
//   second, inside kneg's 4096 p.  Every wave computes it (the chains' additions are few).
__device__ __forceinline__ P2F p2f_add(const WKG& K, const P2F& p, const P2F& q) {
  const uint32_t kn = K.kneg;
  const uint32_t t0 = wf_mul(kn, p.x, q.x);
  const uint32_t t1 = wf_mul(kn, p.y, q.y);
  const uint32_t t2 = wf_mul(kn, p.z, q.z);
  uint64_t a3 = 0, a4 = 0, ay = 0;
  wf_mac(a3, kn, p.x, q.y);
  wf_mac(a3, kn, p.y, q.x);
  wf_mac(a4, kn, p.y, q.z);
  wf_mac(a4, kn, p.z, q.y);
  wf_mac(ay, kn, p.x, q.z);
  wf_mac(ay, kn, p.z, q.x);
  const uint32_t t3 = wredc(a3), t4 = wredc(a4), y3 = wf_b3(K, wredc(ay));
  const uint32_t bt2 = wf_b3(K, t2);
  const uint32_t t0x3 = wmuls<3>(t0);
  const uint32_t z3 = wadd(t1, bt2);
  const uint32_t t1m = wsubk(K.k1024, t1, bt2);
  P2F r;
  uint64_t ax = 0, ayy = 0, az = 0;
  wf_mac(ax, kn, t3, t1m);
  wf_mac(ax, kn, y3, wsubk(K.k256, 0u, t4));
  wf_mac(ayy, kn, t1m, z3);
  wf_mac(ayy, kn, y3, t0x3);
  wf_mac(az, kn, z3, t4);
  wf_mac(az, kn, t0x3, t3);
  r.x = wredc(ax);
  r.y = wredc(ayy);
  r.z = wredc(az);
  return r;
}
// [|x|] p with the doublings on four waves (the additions on every wave)
__device__ __forceinline__ P2F p2f_mul_xabs4(const WKG& K, const P2F& p, uint32_t* x4, int w) {
  P2F m = p;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    m = p2f_dbl4(K, m, x4, w);
    if ((X_ABS >> b) & 1ull) m = p2f_add(K, m, p);
  }
  return m;
}
// Jacobian (X, Y, Z) (F2 layout, the chain bounds of J2F) -> projective (X Z, Y, Z^3), every coordinate a product
__device__ __forceinline__ P2F p2f_of_j2f(const WKG& K, const J2F& p) {
  const uint32_t zz = wf_sqr(K.k2048_2, p.z);
  return P2F{wf_mul(K.kneg, p.x, p.z), wmul(p.y, K.one), wf_mul(K.kneg, zz, p.z)};
}
// -P (the negated Y brought back to a product output)
__device__ __forceinline__ P2F p2f_neg(const WKG& K, const P2F& p) {
  return P2F{p.x, wmul(wsubk(K.k1, 0u, p.y), K.one), p.z};
}
// psi(P) = (conj(X) cx : conj(Y) cy : conj(Z)) (cx, cy in F2 layout; as on Jacobian coordinates)
__device__ __forceinline__ P2F p2f_psi(const WKG& K, const P2F& p, uint32_t cx, uint32_t cy) {
  const uint32_t zc = wmul(wf_conj(K.k2048_2, p.z), K.one);
  return P2F{wf_mul(K.kneg, wf_conj(K.k2048_2, p.x), cx), wf_mul(K.kneg, wf_conj(K.k2048_2, p.y), cy), zc};
}
// psi^2(P) = (X c2x : Y c2y : Z) (c2x, c2y in Fp, both halves)
__device__ __forceinline__ P2F p2f_psi2(const P2F& p, uint32_t c2x, uint32_t c2y) {
  return P2F{wmul(p.x, c2x), wmul(p.y, c2y), p.z};
}
// (X : Y : Z) -> (X / Z, Y / Z) canonical packed; Z = 0 (the identity) -> inf
__device__ __forceinline__ G2A p2f_to_aff(const WKG& K, const P2F& p) {
  const uint32_t sq = wsqr(p.z);
  const Fp nl = w_to_fp(wadd(sq, wswap(sq)));  // norm(Z) in both halves
  G2A r{fp2_zero(), fp2_zero(), true};
  const uint32_t ni = w_from_fp(fp_inv_sg_i(nl));
  const uint32_t zi = wmul(wf_conj(K.k2048_2, p.z), ni);
  const Fp2 x = wf_to_fp2(wf_mul(K.kneg, p.x, zi)), y = wf_to_fp2(wf_mul(K.kneg, p.y, zi));
  if (!fp_is_zero(nl)) r = G2A{x, y, false};
  return r;
}

// Jacobian (X Z, Y Z^2, Z) of a projective (X : Y : Z), canonical Fp2 words; z = 0 is the identity (inf set)
__device__ __forceinline__ G2A p2f_to_jac(const WKG& K, const P2F& p, Fp2& z) {
  const uint32_t zz = wf_sqr(K.k2048_2, p.z);
  const Fp2 x = wf_to_fp2(wf_mul(K.kneg, p.x, p.z)), y = wf_to_fp2(wf_mul(K.kneg, p.y, zz));
  z = wf_to_fp2(p.z);
  return G2A{x, y, fp2_is_zero(z)};
}

}  // namespace wide
}  // namespace bls
