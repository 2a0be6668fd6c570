// 381-bit prime-field arithmetic: Montgomery form with R = 2^406, stored as
// 12 x u32 limbs, multiplied as 14 radix-2^29 digits (see fp_mul).  One
// multiplication is the "FME" unit of the roofline model.
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

// s - p if s >= p else s   (s < 2p).  __builtin_addc/subc lower to
// v_add_co/v_addc_co (v_sub_co/v_subb_co) carry chains on gfx950.
BLS_HD Fp fp_reduce_once(const Fp& s) {
  Fp d;
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d.l[i] = __builtin_subc(s.l[i], P_LIMBS[i], br, &br);
  return fp_select(br != 0, s, d);
}

BLS_HD Fp fp_add(const Fp& a, const Fp& b) {
  Fp s;
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) s.l[i] = __builtin_addc(a.l[i], b.l[i], c, &c);
  return fp_reduce_once(s);  // a + b < 2p < 2^382: no carry out of limb 11
}

BLS_HD Fp fp_dbl(const Fp& a) { return fp_add(a, a); }

BLS_HD Fp fp_sub(const Fp& a, const Fp& b) {
  Fp d;
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d.l[i] = __builtin_subc(a.l[i], b.l[i], br, &br);
  // add p back if we borrowed
  const uint32_t m = br ? 0xffffffffu : 0u;
  Fp e;
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) e.l[i] = __builtin_addc(d.l[i], P_LIMBS[i] & m, c, &c);
  return e;
}

BLS_HD Fp fp_neg(const Fp& a) {
  Fp p;
#pragma unroll
  for (int i = 0; i < 12; i++) p.l[i] = P_LIMBS[i];
  Fp d = fp_sub(p, a);
  return fp_select(fp_is_zero(a), a, d);
}

// ---- Montgomery multiplication ------------------------------------------
// Operands are stored packed (12 x u32) but multiplied as 14 digits of
// radix 2^29 with R = 2^(14*29) = 2^406, product-scanning (FIPS) order: a
// column of up to 28 digit products (< 2^58 each) plus the incoming carry
// fits one 64-bit accumulator, so every digit product is exactly one
// v_mad_u64_u32 with the running accumulator as its 64-bit addend -- no
// carry propagation or register moves inside a column.  ~390 mads + ~160
// other VALU ops per product (the 32-bit CIOS form compiled to ~1,280).
BLS_HD void fp_unpack29(uint32_t d[14], const Fp& a) {
#pragma unroll
  for (int k = 0; k < 14; k++) {
    const int bit = 29 * k, w = bit >> 5, sh = bit & 31;
    uint32_t v = a.l[w] >> sh;
    if (sh > 3 && w + 1 < 12) v |= a.l[w + 1] << (32 - sh);
    d[k] = v & 0x1fffffffu;
  }
}

BLS_HD Fp fp_pack29(const uint32_t r[14]) {
  Fp o;
#pragma unroll
  for (int i = 0; i < 12; i++) o.l[i] = 0;
#pragma unroll
  for (int k = 0; k < 14; k++) {
    const int bit = 29 * k, w = bit >> 5, sh = bit & 31;
    if (w < 12) o.l[w] |= r[k] << sh;
    if (sh > 3 && w + 1 < 12) o.l[w + 1] |= r[k] >> (32 - sh);
  }
  return o;
}

// 13-limb (416-bit) value -> 14 radix-2^29 digits (top digit keeps bits 377..405)
BLS_HD void fp_unpack29_wide(uint32_t d[14], const uint32_t* a) {
#pragma unroll
  for (int k = 0; k < 14; k++) {
    const int bit = 29 * k, w = bit >> 5, sh = bit & 31;
    uint32_t v = a[w] >> sh;
    if (sh > 3 && w + 1 < 13) v |= a[w + 1] << (32 - sh);
    d[k] = k == 13 ? (v & 0x1fffffffu) : (v & 0x1fffffffu);
  }
}

// Montgomery product of digit vectors; with x*y < p * 2^406 the result is < 2p
// and one conditional subtraction makes it canonical.  Any operands below
// 2^390 qualify (x*y/R < 2^374 < p), which lets wave programs feed unreduced
// linear combinations straight in (bls_wave.h).
// Raw form: r = x*y/R as 14 digits with r < 2p (not reduced).
BLS_HD void fp_mul_digits_raw(uint32_t r[14], const uint32_t x[14], const uint32_t y[14]) {
  uint32_t m[14];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j >= 0 && j < 14) acc += (uint64_t)x[i] * y[j];
    }
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j >= 1 && j < 14 && i < k) acc += (uint64_t)m[i] * P29[j];
    }
    if (k < 14) {
      m[k] = ((uint32_t)acc * P29_NINV) & 0x1fffffffu;
      acc += (uint64_t)m[k] * P29[0];
    } else {
      r[k - 14] = (uint32_t)acc & 0x1fffffffu;
    }
    acc >>= 29;
  }
  r[13] = (uint32_t)acc;  // result < 2p < 2^382
}

BLS_HD Fp fp_mul_digits(const uint32_t x[14], const uint32_t y[14]) {
  uint32_t r[14];
  fp_mul_digits_raw(r, x, y);
  return fp_reduce_once(fp_pack29(r));
}

// Montgomery product a*b/R mod p (R = 2^406); valid for a < 2^406, b < p.
BLS_HDNI Fp fp_mul(const Fp& a, const Fp& b) {
  uint32_t x[14], y[14];
  fp_unpack29(x, a);
  fp_unpack29(y, b);
  return fp_mul_digits(x, y);
}

// Inline product (hot loops that keep operands in registers).
BLS_HD Fp fp_mul_i(const Fp& a, const Fp& b) {
  uint32_t x[14], y[14];
  fp_unpack29(x, a);
  fp_unpack29(y, b);
  return fp_mul_digits(x, y);
}

// Out-of-line product with by-value operands (register calling convention,
// no scratch round trip): for per-lane code with many product sites.
BLS_HDNI Fp fp_mul_v(Fp a, Fp b) { return fp_mul_i(a, b); }

// Squaring: off-diagonal digit products once, doubled (105 + 14 instead of
// 196 products for the a*a half).
BLS_HD Fp fp_sqr_i(const Fp& a) {
  uint32_t x[14], m[14], r[14];
  fp_unpack29(x, a);
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    uint64_t od = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j > i && j < 14) od += (uint64_t)x[i] * x[j];
    }
    acc += od << 1;
    if ((k & 1) == 0 && (k >> 1) < 14) acc += (uint64_t)x[k >> 1] * x[k >> 1];
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j >= 1 && j < 14 && i < k) acc += (uint64_t)m[i] * P29[j];
    }
    if (k < 14) {
      m[k] = ((uint32_t)acc * P29_NINV) & 0x1fffffffu;
      acc += (uint64_t)m[k] * P29[0];
    } else {
      r[k - 14] = (uint32_t)acc & 0x1fffffffu;
    }
    acc >>= 29;
  }
  r[13] = (uint32_t)acc;
  return fp_reduce_once(fp_pack29(r));
}

BLS_HDNI Fp fp_sqr(const Fp& a) { return fp_sqr_i(a); }

// a^e for a fixed exponent given as 12 limbs with known bit length.
BLS_HDNI Fp fp_pow(const Fp& a, const uint32_t* e, int nbits) {
  Fp r = a;
  for (int i = nbits - 2; i >= 0; --i) {
    r = fp_sqr(r);
    if ((e[i >> 5] >> (i & 31)) & 1u) r = fp_mul(r, a);
  }
  return r;
}

// raw compare: a < b
BLS_HD bool raw_lt(const uint32_t* a, const uint32_t* b) {
  for (int i = 11; i >= 0; --i) {
    if (a[i] != b[i]) return a[i] < b[i];
  }
  return false;
}

// ---- binary extended Euclid (variable time; inputs are public data) ----
BLS_HD bool raw_is_even(const Fp& a) { return (a.l[0] & 1u) == 0; }
BLS_HD bool raw_is_one(const Fp& a) {
  uint32_t o = a.l[0] ^ 1u;
#pragma unroll
  for (int i = 1; i < 12; i++) o |= a.l[i];
  return o == 0;
}
BLS_HD void raw_shr1(Fp& a, uint32_t top) {
#pragma unroll
  for (int i = 0; i < 11; i++) a.l[i] = (a.l[i] >> 1) | (a.l[i + 1] << 31);
  a.l[11] = (a.l[11] >> 1) | (top << 31);
}
// a = a - b (raw, a >= b)
BLS_HD void raw_sub(Fp& a, const Fp& b) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t t = (uint64_t)a.l[i] - b.l[i] - br;
    a.l[i] = (uint32_t)t;
    br = (uint32_t)(t >> 63);
  }
}
BLS_HD bool raw_geq(const Fp& a, const Fp& b) { return !raw_lt(a.l, b.l); }
BLS_HDNI Fp fp_inv_fermat(const Fp& a) { return fp_pow(a, EXP_P_MINUS_2, EXP_P_MINUS_2_BITS); }

BLS_HD bool fp_is_one(const Fp& a) { return fp_eq(a, FP_ONE); }

// Square root candidate a^((p+1)/4); returns whether it is a root.
BLS_HDNI bool fp_sqrt(Fp& out, const Fp& a) {
  out = fp_pow(a, EXP_SQRT, EXP_SQRT_BITS);
  return fp_eq(fp_sqr(out), a);
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

// Quadratic residuosity by the binary Jacobi-symbol algorithm (variable
// time, public inputs), ~2*381 shift/subtract steps instead of a 380-bit
// exponentiation.  Montgomery form does not change the answer:
// (aR/p) = (a/p)(2/p)^406 = (a/p).
BLS_HDNI bool fp_is_square(const Fp& a_mont) {
  if (fp_is_zero(a_mont)) return true;
  Fp a = a_mont, n;
#pragma unroll
  for (int i = 0; i < 12; i++) n.l[i] = P_LIMBS[i];
  int t = 1;
  while (!fp_is_zero(a)) {
    while (raw_is_even(a)) {
      raw_shr1(a, 0);
      const uint32_t r = n.l[0] & 7u;
      if (r == 3u || r == 5u) t = -t;
    }
    if (raw_lt(a.l, n.l)) {
      Fp tmp = a;
      a = n;
      n = tmp;
      if ((a.l[0] & 3u) == 3u && (n.l[0] & 3u) == 3u) t = -t;
    }
    raw_sub(a, n);
  }
  return raw_is_one(n) && t == 1;
}

BLS_HDNI bool fp_is_square_euler(const Fp& a) {
  if (fp_is_zero(a)) return true;
  return fp_is_one(fp_pow(a, EXP_LEGENDRE, EXP_LEGENDRE_BITS));
}

}  // namespace bls

// fp_inv (Bernstein-Yang divsteps) needs the definitions above
#include "bls_fp_inv.h"
