// Fp inversion by Bernstein-Yang "safegcd" divsteps (Bernstein, Yang: "Fast
// constant-time gcd computation and modular inversion", TCHES 2019), in the
// half-delta ("hddivstep") form with batches of 30 steps on the low 32 bits
// and a 2x2 transition matrix applied to the full values after each batch --
// the structure of libsecp256k1's modinv32, restated for the 381-bit modulus.
//
// Why 32-bit limbs: the GPU's native products are 32 x 32 -> 64 (v_mad_i64_i32,
// v_mad_u64_u32; s_mul_i32 + s_mul_hi_i32 on the scalar unit).  The round-3
// form (radix 2^62, 15 batches of 59 steps) needed 64 x 64 -> 128 products
// in every matrix update, emulated in ~15 instructions each: 303k cycles per
// inversion on one wave (tools/microbench/widerate.hip), most of them there.
// Here 30 batches of 30 divsteps (900 >= 878 = floor((45907 * 381 + 26313) /
// 19929), the hddivstep bound for 381-bit inputs), each step a handful of
// 32-bit operations, and matrix updates of 13-limb values with native
// products.  Constant time: no data-dependent branch.
//
// Values are signed radix-2^30 limbs (13 x int32, 390 bits): limbs 0..11 in
// [0, 2^30), limb 12 signed.
#pragma once
#include "bls_fp.h"

namespace bls {

constexpr int SG_N = 13;
constexpr int32_t SG_M30 = (int32_t)((1u << 30) - 1u);

struct S30 {
  int32_t v[SG_N];
};

// p in radix 2^30 and p^-1 mod 2^30
struct SgConst {
  int32_t p[SG_N];
  uint32_t pinv30;
};
constexpr SgConst sg_const() {
  SgConst c{};
  uint64_t acc = 0;
  int bits = 0, k = 0;
  for (int i = 0; i < 12; i++) {
    acc |= (uint64_t)P_LIMBS[i] << bits;
    bits += 32;
    while (bits >= 30) {
      c.p[k++] = (int32_t)(acc & (uint64_t)SG_M30);
      acc >>= 30;
      bits -= 30;
    }
  }
  while (k < SG_N) {
    c.p[k++] = (int32_t)(acc & (uint64_t)SG_M30);
    acc >>= 30;
  }
  // p^-1 mod 2^32 by Newton iteration (p odd), then mod 2^30
  const uint32_t p0 = (uint32_t)c.p[0] | ((uint32_t)c.p[1] << 30);
  uint32_t x = p0;  // correct to 3 bits
  for (int i = 0; i < 5; i++) x *= 2u - p0 * x;
  c.pinv30 = x & (uint32_t)SG_M30;
  return c;
}
constexpr SgConst SG = sg_const();

struct SgTrans {
  int32_t u, v, q, r;
};

// 30 hddivsteps on the low 32 bits of f (odd) and g; t scaled by 2^30.  (For the wave-uniform operands of the
// per-call kernels, steps forced onto the scalar unit through readfirstlane measured slower than this VALU form:
// 98 against 83 us per inversion.)
BLS_HD int32_t sg_divsteps_30(int32_t zeta, uint32_t f0, uint32_t g0, SgTrans& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1, f = f0, g = g0;
#pragma unroll 1
  for (int i = 0; i < 30; ++i) {
    const uint32_t c1 = (uint32_t)(zeta >> 31);  // all ones if zeta < 0
    const uint32_t c2 = 0u - (g & 1u);            // all ones if g odd
    const uint32_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2;
    q += y & c2;
    r += z & c2;
    const uint32_t c3 = c1 & c2;
    zeta = (int32_t)(((uint32_t)zeta ^ c3) - 1u);
    f += g & c3;
    u += q & c3;
    v += r & c3;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return zeta;
}

// (f, g) = t (f, g) / 2^30 (exact); |u f_i + v g_i| <= 2^61 per column
BLS_HD void sg_update_fg(S30& f, S30& g, const SgTrans& t) {
  const int64_t u = t.u, v = t.v, q = t.q, r = t.r;
  int64_t cf = u * f.v[0] + v * g.v[0];
  int64_t cg = q * f.v[0] + r * g.v[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < SG_N; i++) {
    cf += u * f.v[i] + v * g.v[i];
    cg += q * f.v[i] + r * g.v[i];
    f.v[i - 1] = (int32_t)(cf & SG_M30);
    g.v[i - 1] = (int32_t)(cg & SG_M30);
    cf >>= 30;
    cg >>= 30;
  }
  f.v[SG_N - 1] = (int32_t)cf;
  g.v[SG_N - 1] = (int32_t)cg;
}

// (d, e) = t (d, e) / 2^30 mod p, d and e kept in (-2p, p); columns below 2^62
BLS_HD void sg_update_de(S30& d, S30& e, const SgTrans& t) {
  const int32_t sd = d.v[SG_N - 1] >> 31, se = e.v[SG_N - 1] >> 31;  // -1 if negative
  int32_t md = (t.u & sd) + (t.v & se), me = (t.q & sd) + (t.r & se);
  const int64_t u = t.u, v = t.v, q = t.q, r = t.r;
  int64_t cd = u * d.v[0] + v * e.v[0];
  int64_t ce = q * d.v[0] + r * e.v[0];
  // md, me: the multiples of p that make the low 30 bits vanish
  md -= (int32_t)((SG.pinv30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)SG_M30);
  me -= (int32_t)((SG.pinv30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)SG_M30);
  cd += (int64_t)SG.p[0] * md;
  ce += (int64_t)SG.p[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < SG_N; i++) {
    cd += u * d.v[i] + v * e.v[i] + (int64_t)SG.p[i] * md;
    ce += q * d.v[i] + r * e.v[i] + (int64_t)SG.p[i] * me;
    d.v[i - 1] = (int32_t)(cd & SG_M30);
    e.v[i - 1] = (int32_t)(ce & SG_M30);
    cd >>= 30;
    ce >>= 30;
  }
  d.v[SG_N - 1] = (int32_t)cd;
  e.v[SG_N - 1] = (int32_t)ce;
}

// x in (-2p, p) -> [0, p); negated first when sign < 0
BLS_HD void sg_normalize(S30& x, int32_t sign) {
  // x = sign < 0 ? -x : x, then + p while negative, - p while >= p (each twice at most, branch-free selects)
  const int32_t neg = sign >> 31;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < SG_N; i++) {
    const int32_t v = (x.v[i] ^ neg) - neg + c;  // two's complement limb negation with the borrow carried
    c = v >> 30;
    x.v[i] = i < SG_N - 1 ? (v & SG_M30) : v;
  }
#pragma unroll
  for (int round = 0; round < 2; round++) {  // add p if negative
    const int32_t m = x.v[SG_N - 1] >> 31;
    int32_t cy = 0;
#pragma unroll
    for (int i = 0; i < SG_N; i++) {
      const int32_t v = x.v[i] + (SG.p[i] & m) + cy;
      cy = v >> 30;
      x.v[i] = i < SG_N - 1 ? (v & SG_M30) : v;
    }
  }
#pragma unroll
  for (int round = 0; round < 2; round++) {  // subtract p if >= p
    S30 y;
    int32_t cy = 0;
#pragma unroll
    for (int i = 0; i < SG_N; i++) {
      const int32_t v = x.v[i] - SG.p[i] + cy;
      cy = v >> 30;
      y.v[i] = i < SG_N - 1 ? (v & SG_M30) : v;
    }
    const int32_t keep = y.v[SG_N - 1] >> 31;  // y negative: keep x
#pragma unroll
    for (int i = 0; i < SG_N; i++) x.v[i] = (x.v[i] & keep) | (y.v[i] & ~keep);
  }
}

BLS_HD S30 sg_from_fp(const Fp& a) {
  S30 r;
  uint64_t acc = 0;
  int bits = 0, k = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    acc |= (uint64_t)a.l[i] << bits;
    bits += 32;
    while (bits >= 30) {
      r.v[k++] = (int32_t)(acc & (uint64_t)SG_M30);
      acc >>= 30;
      bits -= 30;
    }
  }
  r.v[SG_N - 1] = (int32_t)acc;  // 384 - 12 * 30 = 24 bits left
  return r;
}

BLS_HD Fp sg_to_fp(const S30& x) {  // x in [0, p)
  Fp r;
  uint64_t acc = 0;
  int bits = 0, k = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    while (bits < 32 && k < SG_N) {
      acc |= (uint64_t)(uint32_t)x.v[k++] << bits;
      bits += 30;
    }
    r.l[i] = (uint32_t)acc;
    acc >>= 32;
    bits -= 32;
  }
  return r;
}

// Plain modular inverse of the integer a (canonical, < p); 0 -> 0.  Inline form for the lane kernels (an
// out-of-line call gives the kernel a private segment); fp_inv_plain_sg is the out-of-line one.
BLS_HD Fp fp_inv_plain_sg_i(const Fp& a) {
  S30 f{}, g = sg_from_fp(a), d{}, e{};
#pragma unroll
  for (int i = 0; i < SG_N; i++) f.v[i] = SG.p[i];
  e.v[0] = 1;
  int32_t zeta = -1;
#pragma unroll 1
  for (int it = 0; it < 30; it++) {
    SgTrans t;
    zeta = sg_divsteps_30(zeta, (uint32_t)f.v[0] | ((uint32_t)f.v[1] << 30),
                          (uint32_t)g.v[0] | ((uint32_t)g.v[1] << 30), t);
    sg_update_de(d, e, t);
    sg_update_fg(f, g, t);
  }
  // g = 0 and f = +-1 (gcd); the inverse is d times f's sign
  sg_normalize(d, f.v[SG_N - 1]);
  return sg_to_fp(d);
}

BLS_HDNI Fp fp_inv_plain_sg(const Fp& a) { return fp_inv_plain_sg_i(a); }

// Montgomery-form inverse, as fp_inv: (a R)^-1 R^3 / R = a^-1 R
BLS_HD Fp fp_inv_sg(const Fp& a) { return fp_mul(fp_inv_plain_sg(a), FP_R3); }
BLS_HD Fp fp_inv_sg_i(const Fp& a) { return fp_mul_i(fp_inv_plain_sg_i(a), FP_R3); }
// the general Montgomery-form inverse (0 -> 0).  It replaced a bit-serial binary extended Euclid whose
// data-dependent branches diverged across the lanes of the batch kernels (~170k VALU instructions per inverse).
BLS_HDNI Fp fp_inv(const Fp& a) { return fp_mul(fp_inv_plain_sg_i(a), FP_R3); }

}  // namespace bls
