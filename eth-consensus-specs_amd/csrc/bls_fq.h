// Radix-2^28 digit form of Fp for the lane kernels.
//
// The packed form (bls_fp.h: 12 x u32 limbs, R = 2^406) unpacks both operands
// of every product into radix-2^29 digits, repacks the result and subtracts p
// once; additions and subtractions are 12-limb carry chains whose VALU-to-VALU
// carry dependencies need a wait state each (s_nop in the gfx950 code).  In the
// Miller accumulation that bookkeeping was ~40 % of the VALU instructions.
//
// Fq keeps a value as 14 digits of 28 bits with Montgomery radix R' = 2^392,
// and lets both the digits and the value run redundant:
//   * fq_mul / fq_sqr: product-scanning Montgomery product.  A column holds at
//     most 14 digit products x_i y_j plus 14 reduction products m_i p_j and the
//     incoming carry in one 64-bit accumulator, so every digit product is one
//     v_mad_u64_u32 and no carry chain exists.  Operand digits may be up to
//     2^30 (x_i y_j <= 2^60; column sum < 14 * 2^60 + 14 * 2^56 < 2^64) and the
//     operand values up to x y < p R' (then the result is < 2p).  The result
//     digits 0..12 are exact 28-bit digits ("N" form: canonical digits, value
//     below 2p, not necessarily below p).
//   * fq_add: digit-wise sum, no carries.
//   * fq_sub(a, b) = a + K - b digit-wise, K a multiple of p whose digits are
//     each at least b's (Q28_KN: 4p with digits in [2^28, 2^29) for b in N form
//     or carry-save form; Q28_K2: 8p with digits in [2^29, 3 * 2^28] for b a sum
//     of two such).  No digit goes negative, no borrow chain.
//   * fq_norm: carry-save normalisation, d_i = (d_i mod 2^28) + (d_{i-1} >> 28)
//     for all digits at once (no chain); the value is unchanged and the digits
//     return to <= 2^28 + 2^4 ("L" form).
// Values are made canonical (packed Fp, R = 2^406, fully reduced) only at the
// edges of a kernel: fq_from_fp / fq_to_fp cost one product each.
//
// Host builds of the test harness (tests/hostcheck, BLS_FQ_CHECK) check every
// product's operand digits, operand values and column sums, and every
// subtraction's digit-wise precondition, so the bounds above are exercised by
// the host tests of every formula built on these primitives.
#pragma once
#include "bls_fp.h"
#include "bls_fq_constants.h"

#ifdef BLS_FQ_CHECK
#include <assert.h>
#endif

namespace bls {

constexpr uint32_t Q28_MASK = 0x0fffffffu;

#ifdef BLS_FQ_CHECK
// value of a digit vector in units of 2^364 (the top digit's weight)
inline double fq_check_top(const Fq& a) {
  double v = 0;
  for (int i = 0; i < 14; ++i) v += (double)a.d[i] * __builtin_ldexp(1.0, 28 * i - 364);
  return v;
}
inline void fq_check_mul(const Fq& x, const Fq& y) {
  for (int i = 0; i < 14; ++i) {
    assert(x.d[i] <= 0x44000000u && y.d[i] <= 0x44000000u);  // <= 2^30 * 1.0625
  }
  // x y < p R'  <=>  (x / 2^364)(y / 2^364) < p / 2^336
  const double pt = 1.6255 * __builtin_ldexp(1.0, 44);  // p / 2^336 = 1.62558... * 2^44
  assert(fq_check_top(x) * fq_check_top(y) < pt);
}
#define FQ_CHECK_MUL(x, y) fq_check_mul(x, y)
#define FQ_CHECK_COL(acc128) assert((acc128) < ((unsigned __int128)1 << 64))
#define FQ_CHECK_SUB(b, K)                                    \
  do {                                                        \
    for (int i_ = 0; i_ < 14; ++i_) assert((b).d[i_] <= (K)[i_]); \
  } while (0)
#else
#define FQ_CHECK_MUL(x, y) ((void)0)
#define FQ_CHECK_COL(acc128) ((void)0)
#define FQ_CHECK_SUB(b, K) ((void)0)
#endif

BLS_HD Fq fq_zero() {
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = 0;
  return r;
}

BLS_HD Fq fq_select(bool c, const Fq& a, const Fq& b) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = c ? a.d[i] : b.d[i];
  return r;
}

BLS_HD Fq fq_add(const Fq& a, const Fq& b) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = a.d[i] + b.d[i];
  return r;
}

BLS_HD Fq fq_dbl(const Fq& a) { return fq_add(a, a); }

// a - b for b in N or L form with value below ~4p (Q28_KN digit-wise >= b)
BLS_HD Fq fq_sub(const Fq& a, const Fq& b) {
  FQ_CHECK_SUB(b, Q28_KN);
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = a.d[i] + (Q28_KN[i] - b.d[i]);
  return r;
}

// a - b for b a sum of two N/L values (digits <= 2^29 + 2^23, value < ~8p)
BLS_HD Fq fq_sub2(const Fq& a, const Fq& b) {
  FQ_CHECK_SUB(b, Q28_K2);
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = a.d[i] + (Q28_K2[i] - b.d[i]);
  return r;
}

BLS_HD Fq fq_neg(const Fq& b) {
  FQ_CHECK_SUB(b, Q28_KN);
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = Q28_KN[i] - b.d[i];
  return r;
}

// carry-save normalisation: same value, digits 0..12 <= 2^28 - 1 + (max digit >> 28)
BLS_HD Fq fq_norm(const Fq& a) {
  Fq r;
  r.d[0] = a.d[0] & Q28_MASK;
#pragma unroll
  for (int i = 1; i < 13; i++) r.d[i] = (a.d[i] & Q28_MASK) + (a.d[i - 1] >> 28);
  r.d[13] = a.d[13] + (a.d[12] >> 28);
  return r;
}

// Montgomery product x y / 2^392; result in N form (exact 28-bit digits 0..12), value < 2p when x y < p R'.
BLS_HD Fq fq_mul(const Fq& x, const Fq& y) {
  FQ_CHECK_MUL(x, y);
  uint32_t m[14];
  Fq r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
#ifdef BLS_FQ_CHECK
    unsigned __int128 chk = acc;
#endif
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j >= 0 && j < 14) {
        acc += (uint64_t)x.d[i] * y.d[j];
#ifdef BLS_FQ_CHECK
        chk += (unsigned __int128)x.d[i] * y.d[j];
#endif
      }
    }
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j >= 1 && j < 14 && i < k) {
        acc += (uint64_t)m[i] * Q28_P[j];
#ifdef BLS_FQ_CHECK
        chk += (unsigned __int128)m[i] * Q28_P[j];
#endif
      }
    }
    if (k < 14) {
      m[k] = ((uint32_t)acc * Q28_NINV) & Q28_MASK;
      acc += (uint64_t)m[k] * Q28_P[0];
#ifdef BLS_FQ_CHECK
      chk += (unsigned __int128)m[k] * Q28_P[0];
#endif
    } else {
      r.d[k - 14] = (uint32_t)acc & Q28_MASK;
    }
    FQ_CHECK_COL(chk);
    acc >>= 28;
  }
  r.d[13] = (uint32_t)acc;
  return r;
}

// squaring: off-diagonal digit products once, doubled with the column (v_lshl_add_u64)
BLS_HD Fq fq_sqr(const Fq& x) {
  FQ_CHECK_MUL(x, x);
  uint32_t m[14];
  Fq r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    uint64_t od = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j > i && j < 14) od += (uint64_t)x.d[i] * x.d[j];
    }
#ifdef BLS_FQ_CHECK
    unsigned __int128 chk = (unsigned __int128)acc + 2 * (unsigned __int128)od;
#endif
    acc += od << 1;
    if ((k & 1) == 0 && (k >> 1) < 14) {
      acc += (uint64_t)x.d[k >> 1] * x.d[k >> 1];
#ifdef BLS_FQ_CHECK
      chk += (unsigned __int128)x.d[k >> 1] * x.d[k >> 1];
#endif
    }
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j >= 1 && j < 14 && i < k) {
        acc += (uint64_t)m[i] * Q28_P[j];
#ifdef BLS_FQ_CHECK
        chk += (unsigned __int128)m[i] * Q28_P[j];
#endif
      }
    }
    if (k < 14) {
      m[k] = ((uint32_t)acc * Q28_NINV) & Q28_MASK;
      acc += (uint64_t)m[k] * Q28_P[0];
#ifdef BLS_FQ_CHECK
      chk += (unsigned __int128)m[k] * Q28_P[0];
#endif
    } else {
      r.d[k - 14] = (uint32_t)acc & Q28_MASK;
    }
    FQ_CHECK_COL(chk);
    acc >>= 28;
  }
  r.d[13] = (uint32_t)acc;
  return r;
}

// ---- conversions (kernel edges) -------------------------------------------
// packed limbs (any value < 2^384) -> 14 plain 28-bit digits
BLS_HD Fq fq_unpack(const Fp& a) {
  Fq r;
#pragma unroll
  for (int k = 0; k < 14; k++) {
    const int bit = 28 * k, w = bit >> 5, sh = bit & 31;
    uint32_t v = a.l[w] >> sh;
    if (sh > 4 && w + 1 < 12) v |= a.l[w + 1] << (32 - sh);
    r.d[k] = v & Q28_MASK;
  }
  return r;
}

// Montgomery Fp (a 2^406, canonical) -> Fq (a R', N form)
BLS_HD Fq fq_from_fp(const Fp& a) { return fq_mul(fq_unpack(a), FQ_FROM_FP); }

// Fq (any redundant form) -> canonical Montgomery Fp (a 2^406 mod p, fully reduced)
BLS_HD Fp fq_to_fp(const Fq& a) {
  const Fq t = fq_mul(a, FQ_TO_FP);  // N form, value < 2p < 2^382
  Fp o;
#pragma unroll
  for (int i = 0; i < 12; i++) o.l[i] = 0;
#pragma unroll
  for (int k = 0; k < 14; k++) {
    const int bit = 28 * k, w = bit >> 5, sh = bit & 31;
    if (w < 12) o.l[w] |= t.d[k] << sh;
    if (sh > 4 && w + 1 < 12) o.l[w + 1] |= t.d[k] >> (32 - sh);
  }
  return fp_reduce_once(o);
}

// ---- Fq2 = Fq[u] / (u^2 + 1) ------------------------------------------------
BLS_HD Fq2 fq2_add(const Fq2& a, const Fq2& b) { return Fq2{fq_add(a.c0, b.c0), fq_add(a.c1, b.c1)}; }
BLS_HD Fq2 fq2_sub(const Fq2& a, const Fq2& b) { return Fq2{fq_sub(a.c0, b.c0), fq_sub(a.c1, b.c1)}; }
BLS_HD Fq2 fq2_sub2(const Fq2& a, const Fq2& b) { return Fq2{fq_sub2(a.c0, b.c0), fq_sub2(a.c1, b.c1)}; }
BLS_HD Fq2 fq2_dbl(const Fq2& a) { return Fq2{fq_dbl(a.c0), fq_dbl(a.c1)}; }
BLS_HD Fq2 fq2_neg(const Fq2& a) { return Fq2{fq_neg(a.c0), fq_neg(a.c1)}; }
BLS_HD Fq2 fq2_norm(const Fq2& a) { return Fq2{fq_norm(a.c0), fq_norm(a.c1)}; }
BLS_HD Fq2 fq2_select(bool c, const Fq2& a, const Fq2& b) {
  return Fq2{fq_select(c, a.c0, b.c0), fq_select(c, a.c1, b.c1)};
}
BLS_HD Fq2 fq2_zero() { return Fq2{fq_zero(), fq_zero()}; }
BLS_HD Fq2 fq2_one() { return Fq2{FQ_ONE, fq_zero()}; }

// Karatsuba: operands with digits <= 2^29 (sums of two N/L values); c0 = t0 - t1 (digits < 2^29.6), c1 = t2 - (t0 + t1)
// (digits < 2^30), both values < 10p
BLS_HD Fq2 fq2_mul(const Fq2& a, const Fq2& b) {
  const Fq t0 = fq_mul(a.c0, b.c0), t1 = fq_mul(a.c1, b.c1);
  const Fq t2 = fq_mul(fq_add(a.c0, a.c1), fq_add(b.c0, b.c1));
  return Fq2{fq_sub(t0, t1), fq_sub2(t2, fq_add(t0, t1))};
}
// (a0 + a1)(a0 - a1), 2 a0 a1: operands in N/L form
BLS_HD Fq2 fq2_sqr(const Fq2& a) {
  const Fq t0 = fq_mul(fq_add(a.c0, a.c1), fq_sub(a.c0, a.c1));
  const Fq t1 = fq_mul(a.c0, a.c1);
  return Fq2{t0, fq_dbl(t1)};
}
BLS_HD Fq2 fq2_mulfq(const Fq2& a, const Fq& b) { return Fq2{fq_mul(a.c0, b), fq_mul(a.c1, b)}; }
// times xi = 1 + u: (a0 - a1) + (a0 + a1) u, a in N/L form
BLS_HD Fq2 fq2_mul_xi(const Fq2& a) { return Fq2{fq_sub(a.c0, a.c1), fq_add(a.c0, a.c1)}; }

BLS_HD Fq2 fq2_from_fp2(const Fp2& a) { return Fq2{fq_from_fp(a.c0), fq_from_fp(a.c1)}; }
BLS_HD Fp2 fq2_to_fp2(const Fq2& a) { return Fp2{fq_to_fp(a.c0), fq_to_fp(a.c1)}; }

}  // namespace bls
