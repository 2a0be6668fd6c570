// 381-bit prime-field arithmetic (Montgomery, R = 2^384, 12 x u32 limbs).
//
// Multiplication is CIOS: each limb product a_j * b_i + t_j + carry is one
// 64-bit multiply-add, which hipcc lowers to v_mad_u64_u32 on gfx950
// (288 per multiplication = one "FME" of the roofline model).
// All results are fully reduced to [0, p).
#pragma once
#include "bls_constants.h"
#include "bls_field_types.h"

namespace bls {

BLS_HD Fp fp_zero() {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = 0;
  return r;
}

BLS_HD bool fp_is_zero(const Fp& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) o |= a.l[i];
  return o == 0;
}

BLS_HD bool fp_eq(const Fp& a, const Fp& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) o |= a.l[i] ^ b.l[i];
  return o == 0;
}

BLS_HD Fp fp_select(bool c, const Fp& a, const Fp& b) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}

// s - p if s >= p else s   (s < 2p)
BLS_HD Fp fp_reduce_once(const Fp& s) {
  Fp d;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t t = (uint64_t)s.l[i] - P_LIMBS[i] - br;
    d.l[i] = (uint32_t)t;
    br = (uint32_t)(t >> 63);
  }
  return fp_select(br != 0, s, d);
}

BLS_HD Fp fp_add(const Fp& a, const Fp& b) {
  Fp s;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t t = (uint64_t)a.l[i] + b.l[i] + c;
    s.l[i] = (uint32_t)t;
    c = (uint32_t)(t >> 32);
  }
  return fp_reduce_once(s);  // a + b < 2p < 2^382: no carry out of limb 11
}

BLS_HD Fp fp_dbl(const Fp& a) { return fp_add(a, a); }

BLS_HD Fp fp_sub(const Fp& a, const Fp& b) {
  Fp d;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t t = (uint64_t)a.l[i] - b.l[i] - br;
    d.l[i] = (uint32_t)t;
    br = (uint32_t)(t >> 63);
  }
  // add p back if we borrowed
  Fp e;
  uint32_t c = 0;
  const uint32_t m = br ? 0xffffffffu : 0u;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t t = (uint64_t)d.l[i] + (P_LIMBS[i] & m) + c;
    e.l[i] = (uint32_t)t;
    c = (uint32_t)(t >> 32);
  }
  return e;
}

BLS_HD Fp fp_neg(const Fp& a) {
  Fp p;
#pragma unroll
  for (int i = 0; i < 12; i++) p.l[i] = P_LIMBS[i];
  Fp d = fp_sub(p, a);
  return fp_select(fp_is_zero(a), a, d);
}

// Montgomery product a*b/R mod p; valid for a < R, b < p (result < p).
BLS_HDNI Fp fp_mul(const Fp& a, const Fp& b) {
  uint32_t t[13];
#pragma unroll
  for (int j = 0; j < 13; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
      uint64_t x = (uint64_t)a.l[j] * b.l[i] + t[j] + c;
      t[j] = (uint32_t)x;
      c = x >> 32;
    }
    uint64_t s = (uint64_t)t[12] + c;
    uint32_t top = (uint32_t)(s >> 32);
    t[12] = (uint32_t)s;
    const uint32_t m = t[0] * P_NINV;
    uint64_t x = (uint64_t)m * P_LIMBS[0] + t[0];
    c = x >> 32;
#pragma unroll
    for (int j = 1; j < 12; j++) {
      x = (uint64_t)m * P_LIMBS[j] + t[j] + c;
      t[j - 1] = (uint32_t)x;
      c = x >> 32;
    }
    s = (uint64_t)t[12] + c;
    t[11] = (uint32_t)s;
    t[12] = top + (uint32_t)(s >> 32);
  }
  Fp r;
#pragma unroll
  for (int j = 0; j < 12; j++) r.l[j] = t[j];
  // t < 2p and t[12] == 0 because p < R/4
  return fp_reduce_once(r);
}

BLS_HDNI Fp fp_sqr(const Fp& a) { return fp_mul(a, a); }

// a^e for a fixed exponent given as 12 limbs with known bit length.
BLS_HDNI Fp fp_pow(const Fp& a, const uint32_t* e, int nbits) {
  Fp r = a;
  for (int i = nbits - 2; i >= 0; --i) {
    r = fp_sqr(r);
    if ((e[i >> 5] >> (i & 31)) & 1u) r = fp_mul(r, a);
  }
  return r;
}

BLS_HDNI Fp fp_inv(const Fp& a) { return fp_pow(a, EXP_P_MINUS_2, EXP_P_MINUS_2_BITS); }

BLS_HD bool fp_is_one(const Fp& a) { return fp_eq(a, FP_ONE); }

// Square root candidate a^((p+1)/4); returns whether it is a root.
BLS_HDNI bool fp_sqrt(Fp& out, const Fp& a) {
  out = fp_pow(a, EXP_SQRT, EXP_SQRT_BITS);
  return fp_eq(fp_sqr(out), a);
}

BLS_HDNI bool fp_is_square(const Fp& a) {
  if (fp_is_zero(a)) return true;
  return fp_is_one(fp_pow(a, EXP_LEGENDRE, EXP_LEGENDRE_BITS));
}

BLS_HD Fp fp_mul_small(const Fp& a, int k) {  // small positive k
  Fp r = a;
  for (int i = 1; i < k; i++) r = fp_add(r, a);
  return r;
}

// ---- conversion ---------------------------------------------------------
// raw integer limbs (< R) -> Montgomery form
BLS_HDNI Fp fp_to_mont(const Fp& raw) { return fp_mul(raw, FP_R2); }

BLS_HD Fp fp_from_mont(const Fp& a) {
  Fp one = fp_zero();
  one.l[0] = 1;
  return fp_mul(a, one);
}

// raw compare: a < b
BLS_HD bool raw_lt(const uint32_t* a, const uint32_t* b) {
  for (int i = 11; i >= 0; --i) {
    if (a[i] != b[i]) return a[i] < b[i];
  }
  return false;
}

// canonical (non-Montgomery) integer limbs > (p-1)/2
BLS_HD bool raw_gt_half(const Fp& canon) { return raw_lt(P_HALF, canon.l); }

BLS_HD bool raw_lt_p(const Fp& raw) { return raw_lt(raw.l, P_LIMBS); }

// 48 big-endian bytes -> raw limbs
BLS_HD Fp raw_from_be48(const uint8_t* b) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint8_t* q = b + 44 - 4 * i;
    r.l[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
  return r;
}

BLS_HD void raw_to_be48(const Fp& r, uint8_t* b) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint8_t* q = b + 44 - 4 * i;
    q[0] = (uint8_t)(r.l[i] >> 24);
    q[1] = (uint8_t)(r.l[i] >> 16);
    q[2] = (uint8_t)(r.l[i] >> 8);
    q[3] = (uint8_t)r.l[i];
  }
}

}  // namespace bls
