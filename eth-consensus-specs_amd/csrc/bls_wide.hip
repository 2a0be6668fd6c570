// Kernels in the wavefront-cooperative form of bls_wide.h: one wave per item
// (per-call path), and the device self-test of the wide products against the
// lane form of bls_fq.h.
#include "bls_kernels.h"
#include "bls_lane.h"
#include "bls_wide.h"
#include "bls_wide_g2.h"
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

// hash_to_G2 of item blockIdx.x on one wave (per-call path): hash_to_field on every lane (uniform), the SSWU map
// and 3-isogeny of u_0 in half 0 and of u_1 in half 1, their sum, the cofactor clearing
//   H = [x^2 - x - 1] Q + [x - 1] psi(Q) + psi^2(2 Q)  as  M = [|x|] Q,  A' = M - psi(Q),
//   C = psi^2(2 Q) - psi(Q) + M - Q,  H = C + [|x|] A'   (A' = -A of k_g2x_pre1t / k_g2x_post1t)
// in both halves (two Jacobian representations of the same points), and the affine H from half 0.  flag[i] = 1
// for the cases the fallback recomputes (SSWU `rare`, a vanishing isogeny denominator, an exceptional addition).
// msgs: 32-byte messages msgs[32 i ..] (offs == nullptr) or msgs[offs[i] .. offs[i+1]).
__global__ void __launch_bounds__(64) k_h2c_wide(size_t B, const uint8_t* msgs, const uint64_t* offs, G2A* H,
                                                 int* flag) {
  const size_t i = blockIdx.x;
  if (i >= B) return;
  const WKG K = wkg_init();
  Fp2 u[2];
  if (offs)
    hash_to_field_fp2(u, msgs + offs[i], (uint32_t)(offs[i + 1] - offs[i]), DST_POP_WIDE, 43);
  else
    hash_to_field_fp2_m32(u, msgs + 32 * i);
  const bool hi = whalf() != 0;
  const Fp2 uh{fp_select(hi, u[1].c0, u[0].c0), fp_select(hi, u[1].c1, u[0].c1)};
  W2 x, y;
  bool rare = false, izero = false, exc = false;
  sswu_w(K, uh, x, y, rare);
  const J2W P = iso_w(K, x, y, izero);
  const J2W Po{w2swap(P.x), w2swap(P.y), w2swap(P.z)};
  const J2W Q = j2w_add(K, P, Po, exc);
  const W2 cx = w2const(PSI_CX), cy = w2const(PSI_CY);
  const uint32_t c2x = w_from_fp(PSI2_CX.c0), c2y = w_from_fp(PSI2_CY.c0);
  const J2W M = j2w_mul_xabs(K, Q, exc);
  const J2W npq = j2w_neg(K, j2w_psi(K, Q, cx, cy));
  const J2W Ap = j2w_add(K, M, npq, exc);
  J2W C = j2w_add(K, j2w_psi2(K, j2w_dbl(K, Q), c2x, c2y), npq, exc);
  C = j2w_add(K, C, M, exc);
  C = j2w_add(K, C, j2w_neg(K, Q), exc);
  const J2W M2 = j2w_mul_xabs(K, Ap, exc);
  const J2W Hj = j2w_add(K, C, M2, exc);
  const G2A h = j2w_to_aff(K, Hj);
  const int bad = (rare | izero | exc) ? 1 : 0;
  const int bad_any = __builtin_amdgcn_readlane(bad, 0) | __builtin_amdgcn_readlane(bad, 32);
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
  hash_to_field_fp2_m32(u, msg32);
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
  if (threadIdx.x == 0) {
    Fp o = fp_zero();
    o.l[0] = (uint32_t)(f0 | (f1 << 8));
    out[32] = o;
  }
}

hipError_t launch_h2c_wide_dbg(hipStream_t st, const uint8_t* msg32, Fp* out) {
  hipLaunchKernelGGL(k_h2c_wide_dbg, dim3(1), dim3(64), 0, st, msg32, out);
  return hipGetLastError();
}

hipError_t launch_h2c_wide(hipStream_t st, size_t B, const uint8_t* msgs, const uint64_t* offs, G2A* H, int* flag) {
  if (!B) return hipSuccess;
  hipLaunchKernelGGL(k_h2c_wide, dim3((unsigned)B), dim3(64), 0, st, B, msgs, offs, H, flag);
  return hipGetLastError();
}

// Signature decode + G2 subgroup check of item blockIdx.x on one wave (per-call path; k_sig_validate semantics:
// the identity encoding is accepted, every other failure is invalid).  Decoding up to the Montgomery x on every
// lane (g2_decompress_lane_w's checks), then in wide arithmetic (both halves, the same chain): y^2 = x^3 + 4(1 + u)
// by the norm square root (bls_lane.h fp2_sqrt_lane_i; the pure-Fp case, unreachable for x of a valid point with
// probability ~2^-381, runs fp2_sqrt_lane_i on the lanes -- a wave-uniform branch), the sign, and
// psi(sigma) == -[|x|] sigma through the wide Jacobian chain (an exceptional addition means a small order: reject).
__global__ void __launch_bounds__(64) k_sig_validate_wide(const uint8_t* sigs96, size_t n, G2A* out, int* ok) {
  const size_t i = blockIdx.x;
  if (i >= n) return;
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
        const uint32_t nr = wpow(nrm, EXP_SQRT, EXP_SQRT_BITS);
        on = w_eq(K1, wsqr(nr), nrm);
        const uint32_t inv2 = w_from_fp(FP_INV2);
        const uint32_t t = wmul(wadd(rhs.c0, nr), inv2);
        const uint32_t sr = wpow(t, EXP_SQRT_M3, EXP_SQRT_M3_BITS);
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
        const J2W M = j2w_mul_xabs(K, J2W{xm, y, W2{K.one, 0u}}, exc);
        // psi(sigma) == -M:  conj(x) CX Z^2 == X,  conj(y) CY Z^3 == -Y,  Z != 0
        const W2 zz = w2mulk(K, M.z, M.z);
        const W2 px = w2mulk(K, w2mulk(K, w2conj(K1, xm), w2const(PSI_CX)), zz);
        const W2 py = w2mulk(K, w2mulk(K, w2conj(K1, y), w2const(PSI_CY)), w2mulk(K, zz, M.z));
        const bool zx = w2_is_zero(w2subk(K.k2048_2, px, M.x));  // M.x < 1028p (the chain ends on a doubling)
        const bool zy = w2_is_zero(w2add(py, M.y));
        const bool zz0 = w2_is_zero(M.z);
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
  hipLaunchKernelGGL(k_sig_validate_wide, dim3((unsigned)n), dim3(64), 0, st, sigs, n, out, ok);
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
__device__ __forceinline__ G1W g1w_dbl(const WKG& K, const G1W& p) {
  const uint32_t t0 = wmul(p.y, p.y);
  const uint32_t t1 = wmul(p.y, p.z);
  const uint32_t t2 = wmuls<12>(wmul(p.z, p.z));  // 3b Z^2, < 24p
  const uint32_t u = wmul(p.x, p.y);
  const uint32_t z8 = wmuls<8>(t0);
  const uint32_t x3a = wmul(t2, z8);
  G1W r;
  r.z = wmul(t1, z8);
  const uint32_t w = wsubk(K.k2, t0, wmuls<3>(t2));  // t0 - 3 t2 + 128p
  r.y = wadd(wmul(w, wadd(t0, t2)), x3a);
  r.x = wmuls<2>(wmul(w, u));
  return r;
}
template <bool AFF>
__device__ __forceinline__ G1W g1w_mul_xabs(const WKG& K, const G1W& b) {
  G1W m = b;
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    m = g1w_dbl(K, m);
    if ((X_ABS >> i) & 1ull) m = AFF ? g1w_add_aff(K, m, b.x, b.y) : g1w_add(K, m, b);
  }
  return m;
}

// KeyValidate of keys 2 blockIdx.x + half (k_key_validate semantics; the decode on every lane of the half, the
// square root and both [|x|] chains in wide arithmetic).  Wave-uniform control flow: the two halves' decode
// verdicts are combined into selects, not branches.
__global__ void __launch_bounds__(64) k_key_validate_wide(const uint8_t* pks48, size_t n, G1A* out, int* ok) {
  const size_t base = 2 * (size_t)blockIdx.x;
  if (base >= n) return;
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
  const G1W Q = g1w_mul_xabs<false>(K, g1w_mul_xabs<true>(K, P));
  const bool eq_x = w_eq(K1, wmul(wmul(xm, w_from_fp(FP_BETA)), Q.z), wmul(Q.x, K.one));
  const bool eq_y = w_is_zero(wadd(wmul(y, Q.z), Q.y));
  const bool v = fmt && on && eq_x && eq_y;
  const G1A a = v ? G1A{w_to_fp(xm), w_to_fp(y), false} : G1A{fp_zero(), fp_zero(), true};
  if (wpos() == 0 && base + (size_t)h < n) {
    out[base + h] = a;
    ok[base + h] = v ? 1 : 0;
  }
}

hipError_t launch_key_validate_wide(hipStream_t st, const uint8_t* pks, size_t n, G1A* out, int* ok) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_key_validate_wide, dim3((unsigned)((n + 1) / 2)), dim3(64), 0, st, pks, n, out, ok);
  return hipGetLastError();
}

hipError_t launch_wide_selftest(hipStream_t st, size_t nw, const uint8_t* be48, int* bad) {
  if (!nw) return hipSuccess;
  hipLaunchKernelGGL(k_wide_selftest, dim3((unsigned)nw), dim3(64), 0, st, nw, be48, bad);
  return hipGetLastError();
}

}  // namespace bls
