// Fp inversion by Bernstein-Yang "safegcd" divsteps (Bernstein, Yang: "Fast
// constant-time gcd computation and modular inversion", TCHES 2019), in the
// half-delta ("hddivstep") form with batches of 59 steps on the low 64 bits
// and a 2x2 transition matrix applied to the full values after each batch --
// the structure of libsecp256k1's modinv64, restated for the 381-bit modulus.
//
// Why: fp_inv (bls_fp.h) is a bit-serial binary extended Euclid, ~760
// iterations of 12-limb shifts, compares and modular subtractions -- about
// 170k VALU instructions on one lane, a third of the lane-parallel final
// exponentiation (bls_fe.h) at one inversion per check.  Here 15 batches of 59
// divsteps (885 >= 878 = floor((45907 * 381 + 26313) / 19929), the hddivstep
// bound for 381-bit inputs) cost 59 branch-free 64-bit step bodies and two
// 7-limb matrix products each.  Constant time: no data-dependent branch.
//
// Values are signed radix-2^62 limbs (7 x int64, 434 bits): limbs 0..5 in
// [0, 2^62), limb 6 signed.
#pragma once
#include "bls_fp.h"

namespace bls {

struct S62 {
  int64_t v[7];
};

constexpr int64_t SG_M62 = (int64_t)((1ull << 62) - 1);

// p in radix 2^62 and p^-1 mod 2^62
struct SgConst {
  int64_t p[7];
  uint64_t pinv62;
};
constexpr SgConst sg_const() {
  SgConst c{};
  // p from its 12 x u32 limbs
  unsigned __int128 acc = 0;
  int bits = 0, k = 0;
  for (int i = 0; i < 12; i++) {
    acc |= (unsigned __int128)P_LIMBS[i] << bits;
    bits += 32;
    while (bits >= 62) {
      c.p[k++] = (int64_t)((uint64_t)acc & (uint64_t)SG_M62);
      acc >>= 62;
      bits -= 62;
    }
  }
  while (k < 7) {
    c.p[k++] = (int64_t)((uint64_t)acc & (uint64_t)SG_M62);
    acc >>= 62;
  }
  // p^-1 mod 2^64 by Newton iteration (p odd), then mod 2^62
  uint64_t p0 = (uint64_t)c.p[0] | ((uint64_t)c.p[1] << 62);
  uint64_t x = p0;  // correct to 3 bits
  for (int i = 0; i < 6; i++) x *= 2 - p0 * x;
  c.pinv62 = x & (uint64_t)SG_M62;
  return c;
}
constexpr SgConst SG = sg_const();

struct SgTrans {
  int64_t u, v, q, r;
};

// a wave-uniform 64-bit value as a scalar (two readfirstlane into SGPRs) on the device
BLS_HD uint64_t sg_uniform(uint64_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
#else
  return v;
#endif
}

// 59 hddivsteps on the low 64 bits of f (odd) and g; t scaled by 2^62 (starts at 8 = 2^3, 59 doublings).
// UNIFORM: the value being inverted is the same on every lane (the per-call kernels invert one norm per wave):
// the step inputs go through SGPRs, so the 59 steps -- 64-bit adds, masks and shifts only, no products -- compile
// to SALU code, one operation per cycle, instead of VALU code at 4-8 cycles per instruction for one 64-lane wave
// (tools/microbench/widerate.hip: 126 us per inversion in VALU form).
template <bool UNIFORM = false>
BLS_HD int64_t sg_divsteps_59(int64_t zeta, uint64_t f0, uint64_t g0, SgTrans& t) {
  if (UNIFORM) {
    zeta = (int64_t)sg_uniform((uint64_t)zeta);
    f0 = sg_uniform(f0);
    g0 = sg_uniform(g0);
  }
  uint64_t u = 8, v = 0, q = 0, r = 8, f = f0, g = g0;
#pragma unroll 1
  for (int i = 3; i < 62; ++i) {
    const uint64_t c1 = (uint64_t)(zeta >> 63);  // all ones if zeta < 0
    const uint64_t c2 = 0 - (g & 1u);           // all ones if g odd
    const uint64_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2;
    q += y & c2;
    r += z & c2;
    const uint64_t c3 = c1 & c2;
    zeta = (int64_t)(((uint64_t)zeta ^ c3) - 1u);
    f += g & c3;
    u += q & c3;
    v += r & c3;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  t.u = (int64_t)u;
  t.v = (int64_t)v;
  t.q = (int64_t)q;
  t.r = (int64_t)r;
  return zeta;
}

// (f, g) = t (f, g) / 2^62 (exact)
BLS_HD void sg_update_fg(S62& f, S62& g, const SgTrans& t) {
  __int128 cf = (__int128)t.u * f.v[0] + (__int128)t.v * g.v[0];
  __int128 cg = (__int128)t.q * f.v[0] + (__int128)t.r * g.v[0];
  cf >>= 62;
  cg >>= 62;
#pragma unroll
  for (int i = 1; i < 7; i++) {
    cf += (__int128)t.u * f.v[i] + (__int128)t.v * g.v[i];
    cg += (__int128)t.q * f.v[i] + (__int128)t.r * g.v[i];
    f.v[i - 1] = (int64_t)cf & SG_M62;
    g.v[i - 1] = (int64_t)cg & SG_M62;
    cf >>= 62;
    cg >>= 62;
  }
  f.v[6] = (int64_t)cf;
  g.v[6] = (int64_t)cg;
}

// (d, e) = t (d, e) / 2^62 mod p, d and e kept in (-2p, p)
BLS_HD void sg_update_de(S62& d, S62& e, const SgTrans& t) {
  const int64_t sd = d.v[6] >> 63, se = e.v[6] >> 63;  // -1 if negative
  int64_t md = (t.u & sd) + (t.v & se), me = (t.q & sd) + (t.r & se);
  __int128 cd = (__int128)t.u * d.v[0] + (__int128)t.v * e.v[0];
  __int128 ce = (__int128)t.q * d.v[0] + (__int128)t.r * e.v[0];
  // md, me: the multiples of p that make the low 62 bits vanish
  md -= (int64_t)((SG.pinv62 * (uint64_t)(int64_t)cd + (uint64_t)md) & (uint64_t)SG_M62);
  me -= (int64_t)((SG.pinv62 * (uint64_t)(int64_t)ce + (uint64_t)me) & (uint64_t)SG_M62);
  cd += (__int128)SG.p[0] * md;
  ce += (__int128)SG.p[0] * me;
  cd >>= 62;
  ce >>= 62;
#pragma unroll
  for (int i = 1; i < 7; i++) {
    cd += (__int128)t.u * d.v[i] + (__int128)t.v * e.v[i] + (__int128)SG.p[i] * md;
    ce += (__int128)t.q * d.v[i] + (__int128)t.r * e.v[i] + (__int128)SG.p[i] * me;
    d.v[i - 1] = (int64_t)cd & SG_M62;
    e.v[i - 1] = (int64_t)ce & SG_M62;
    cd >>= 62;
    ce >>= 62;
  }
  d.v[6] = (int64_t)cd;
  e.v[6] = (int64_t)ce;
}

// x in (-2p, p) -> [0, p); negated first when sign < 0
BLS_HD void sg_normalize(S62& x, int64_t sign) {
  // x = sign < 0 ? -x : x, then + p while negative, - p while >= p (each twice at most, branch-free selects)
  const int64_t neg = sign >> 63;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 7; i++) {
    int64_t v = (x.v[i] ^ neg) - neg + c;  // two's complement limb negation with the borrow carried
    c = v >> 62;
    x.v[i] = i < 6 ? (v & SG_M62) : v;
  }
#pragma unroll
  for (int round = 0; round < 2; round++) {  // add p if negative
    const int64_t m = x.v[6] >> 63;
    int64_t cy = 0;
#pragma unroll
    for (int i = 0; i < 7; i++) {
      const int64_t v = x.v[i] + (SG.p[i] & m) + cy;
      cy = v >> 62;
      x.v[i] = i < 6 ? (v & SG_M62) : v;
    }
  }
#pragma unroll
  for (int round = 0; round < 2; round++) {  // subtract p if >= p
    S62 y;
    int64_t cy = 0;
#pragma unroll
    for (int i = 0; i < 7; i++) {
      const int64_t v = x.v[i] - SG.p[i] + cy;
      cy = v >> 62;
      y.v[i] = i < 6 ? (v & SG_M62) : v;
    }
    const int64_t keep = y.v[6] >> 63;  // y negative: keep x
#pragma unroll
    for (int i = 0; i < 7; i++) x.v[i] = (x.v[i] & keep) | (y.v[i] & ~keep);
  }
}

BLS_HD S62 sg_from_fp(const Fp& a) {
  S62 r;
  unsigned __int128 acc = 0;
  int bits = 0, k = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    acc |= (unsigned __int128)a.l[i] << bits;
    bits += 32;
    if (bits >= 62) {
      r.v[k++] = (int64_t)((uint64_t)acc & (uint64_t)SG_M62);
      acc >>= 62;
      bits -= 62;
    }
  }
  r.v[6] = (int64_t)(uint64_t)acc;  // 384 - 6 * 62 = 12 bits left
  return r;
}

BLS_HD Fp sg_to_fp(const S62& x) {  // x in [0, p)
  Fp r;
  unsigned __int128 acc = 0;
  int bits = 0, k = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    while (bits < 32) {
      acc |= (unsigned __int128)(uint64_t)x.v[k++] << bits;
      bits += 62;
    }
    r.l[i] = (uint32_t)acc;
    acc >>= 32;
    bits -= 32;
  }
  return r;
}

// Plain modular inverse of the integer a (canonical, < p); 0 -> 0.  Inline form for the lane kernels (an
// out-of-line call gives the kernel a private segment); fp_inv_plain_sg is the out-of-line one.
template <bool UNIFORM = false>
BLS_HD Fp fp_inv_plain_sg_i(const Fp& a) {
  S62 f{}, g = sg_from_fp(a), d{}, e{};
#pragma unroll
  for (int i = 0; i < 7; i++) f.v[i] = SG.p[i];
  e.v[0] = 1;
  int64_t zeta = -1;
#pragma unroll 1
  for (int it = 0; it < 15; it++) {
    SgTrans t;
    zeta = sg_divsteps_59<UNIFORM>(zeta, (uint64_t)f.v[0] | ((uint64_t)f.v[1] << 62),
                                   (uint64_t)g.v[0] | ((uint64_t)g.v[1] << 62), t);
    sg_update_de(d, e, t);
    sg_update_fg(f, g, t);
  }
  // g = 0 and f = +-1 (gcd); the inverse is d times f's sign
  sg_normalize(d, f.v[6]);
  return sg_to_fp(d);
}

BLS_HDNI Fp fp_inv_plain_sg(const Fp& a) { return fp_inv_plain_sg_i(a); }

// Montgomery-form inverse, as fp_inv: (a R)^-1 R^3 / R = a^-1 R
BLS_HD Fp fp_inv_sg(const Fp& a) { return fp_mul(fp_inv_plain_sg(a), FP_R3); }
template <bool UNIFORM = false>
BLS_HD Fp fp_inv_sg_i(const Fp& a) { return fp_mul_i(fp_inv_plain_sg_i<UNIFORM>(a), FP_R3); }
// the general Montgomery-form inverse (0 -> 0).  It replaced a bit-serial binary extended Euclid whose
// data-dependent branches diverged across the lanes of the batch kernels (~170k VALU instructions per inverse).
BLS_HDNI Fp fp_inv(const Fp& a) { return fp_mul(fp_inv_plain_sg_i(a), FP_R3); }

}  // namespace bls
