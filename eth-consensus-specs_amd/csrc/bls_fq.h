// Redundant radix-2^29 digit form of Fp for the lane kernels.
//
// The packed form (bls_fp.h: 12 x u32 limbs) unpacks both operands of every
// product into radix-2^29 digits, repacks the result and subtracts p once, and
// its additions and subtractions are 12-limb carry chains whose VALU-to-VALU
// carry dependencies need a wait state each (s_nop in the gfx950 code).
// Measured on MI355X at one wave per SIMD: 48 G products/s packed against 67
// G/s for a product whose operands and result stay in digit form
// (profiles/r02l_fqrate_microbench.txt, tools/microbench/fqrate.hip).
//
// Fq keeps the 14 digits of the same Montgomery representation (R = 2^406, so
// fq_unpack / fq_pack are repacking, no products), and lets both the digits
// and the value run redundant:
//   * fq_mul / fq_sqr: product-scanning Montgomery product (as fp_mul_digits).
//     A column holds at most 14 digit products x_i y_j plus 14 reduction
//     products m_i p_j and the carry in one 64-bit accumulator; the top digits
//     of operands and of p are small, so ~12 terms of each kind are full-size
//     and x_i y_j <= 2^60 keeps the column below 2^64 (operand digits up to
//     ~2^30 on both sides, or 2^29 against 2^31).  The value may be anything
//     with x y < p R (R / p ~ 2^25.3), and then the result is < 2p with exact
//     29-bit digits 0..12 ("N" form).
//   * fq_add: digit-wise sum, no carries.
//   * fq_sub(a, b) = a + K - b digit-wise with K a multiple of p whose digits
//     are each at least b's (Q29_K1 = 64p for b in N or L form, Q29_K2 =
//     128p for b a sum of two such): no digit goes negative, no borrow chain.
//   * fq_norm: carry-save normalisation d_i = (d_i mod 2^29) + (d_{i-1} >> 29)
//     of all digits at once (no chain): same value, digits back to
//     <= 2^29 + (max digit >> 29) ("L" form).
// Host builds of the test harness (tests/hostcheck, BLS_FQ_CHECK) check every
// product's column sums in 128-bit arithmetic and its operand values, and every
// subtraction's digit-wise precondition, so the bounds each formula relies on
// are exercised by the host tests of that formula.
#pragma once
#include "bls_fp.h"
#include "bls_fq_constants.h"

#ifdef BLS_FQ_CHECK
#include <assert.h>
#endif

namespace bls {

constexpr uint32_t Q29_MASK = 0x1fffffffu;

#ifdef BLS_FQ_CHECK
// value of a digit vector in units of 2^377 (the top digit's weight)
inline double fq_check_top(const Fq& a) {
  double v = 0;
  for (int i = 0; i < 14; ++i) v += (double)a.d[i] * __builtin_ldexp(1.0, 29 * i - 377);
  return v;
}
// x y < p R  <=>  (x / 2^377)(y / 2^377) < p / 2^348 = 13.0021... * 2^29
inline void fq_check_mul(const Fq& x, const Fq& y) {
  assert(fq_check_top(x) * fq_check_top(y) < 13.0 * __builtin_ldexp(1.0, 29));
}
#define FQ_CHECK_MUL(x, y) fq_check_mul(x, y)
inline void fq_check_dot2(const Fq& x, const Fq& y, const Fq& u, const Fq& v) {
  assert(fq_check_top(x) * fq_check_top(y) + fq_check_top(u) * fq_check_top(v) < 13.0 * __builtin_ldexp(1.0, 29));
}
#define FQ_CHECK_DOT2(x, y, u, v) fq_check_dot2(x, y, u, v)
#define FQ_CHECK_COL(acc128) assert((acc128) < ((unsigned __int128)1 << 64))
#define FQ_CHECK_SUB(b, K)                                        \
  do {                                                            \
    for (int i_ = 0; i_ < 14; ++i_) assert((b).d[i_] <= (K)[i_]); \
  } while (0)
#else
#define FQ_CHECK_MUL(x, y) ((void)0)
#define FQ_CHECK_DOT2(x, y, u, v) ((void)0)
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

// a - b, b in N or L form (digits <= 2^29 + 2^25) with value below ~62p
BLS_HD Fq fq_sub(const Fq& a, const Fq& b) {
  FQ_CHECK_SUB(b, Q29_K1);
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = a.d[i] + (Q29_K1[i] - b.d[i]);
  return r;
}

// a - b, b a sum of two N/L values (digits <= 2^30 + 2^25) with value below ~126p
BLS_HD Fq fq_sub2(const Fq& a, const Fq& b) {
  FQ_CHECK_SUB(b, Q29_K2);
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = a.d[i] + (Q29_K2[i] - b.d[i]);
  return r;
}

// carry-save normalisation: same value, digits 0..12 <= 2^29 - 1 + (max digit >> 29)
BLS_HD Fq fq_norm(const Fq& a) {
  Fq r;
  r.d[0] = a.d[0] & Q29_MASK;
#pragma unroll
  for (int i = 1; i < 13; i++) r.d[i] = (a.d[i] & Q29_MASK) + (a.d[i - 1] >> 29);
  r.d[13] = a.d[13] + (a.d[12] >> 29);
  return r;
}

// k a (small k, any digits): the 64-bit digit products split into a carry-save
// sum in the same pass, so the result is in L form
BLS_HD Fq fq_mul_small(const Fq& a, uint32_t k) {
  uint64_t t[14];
#pragma unroll
  for (int i = 0; i < 14; i++) t[i] = (uint64_t)a.d[i] * k;
  Fq r;
  r.d[0] = (uint32_t)t[0] & Q29_MASK;
#pragma unroll
  for (int i = 1; i < 13; i++) r.d[i] = ((uint32_t)t[i] & Q29_MASK) + (uint32_t)(t[i - 1] >> 29);
  r.d[13] = (uint32_t)t[13] + (uint32_t)(t[12] >> 29);
  return r;
}

// Montgomery product x y / 2^406; result in N form (exact 29-bit digits 0..12), value < 2p when x y < p R.
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
        acc += (uint64_t)m[i] * P29[j];
#ifdef BLS_FQ_CHECK
        chk += (unsigned __int128)m[i] * P29[j];
#endif
      }
    }
    if (k < 14) {
      m[k] = ((uint32_t)acc * P29_NINV) & Q29_MASK;
      acc += (uint64_t)m[k] * P29[0];
#ifdef BLS_FQ_CHECK
      chk += (unsigned __int128)m[k] * P29[0];
#endif
    } else {
      r.d[k - 14] = (uint32_t)acc & Q29_MASK;
    }
    FQ_CHECK_COL(chk);
    acc >>= 29;
  }
  r.d[13] = (uint32_t)acc;
  return r;
}

// Montgomery (x y + u v) / 2^406 with ONE reduction: both digit products of a column go into the same accumulator
// ahead of the reduction products (28 + 14 terms).  N form, value < 2p when x y + u v < p R.  Karatsuba's
// three products, two subtractions and two normalisations for an Fp2 product become two of these
// (a0 b0 + a1 (-b1), a0 b1 + a1 b0) on a negation K - b1 (bls_fqb.h).
BLS_HD Fq fq_mul_dot2(const Fq& x, const Fq& y, const Fq& u, const Fq& v) {
  FQ_CHECK_DOT2(x, y, u, v);
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
        acc += (uint64_t)u.d[i] * v.d[j];
#ifdef BLS_FQ_CHECK
        chk += (unsigned __int128)x.d[i] * y.d[j] + (unsigned __int128)u.d[i] * v.d[j];
#endif
      }
    }
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j >= 1 && j < 14 && i < k) {
        acc += (uint64_t)m[i] * P29[j];
#ifdef BLS_FQ_CHECK
        chk += (unsigned __int128)m[i] * P29[j];
#endif
      }
    }
    if (k < 14) {
      m[k] = ((uint32_t)acc * P29_NINV) & Q29_MASK;
      acc += (uint64_t)m[k] * P29[0];
#ifdef BLS_FQ_CHECK
      chk += (unsigned __int128)m[k] * P29[0];
#endif
    } else {
      r.d[k - 14] = (uint32_t)acc & Q29_MASK;
    }
    FQ_CHECK_COL(chk);
    acc >>= 29;
  }
  r.d[13] = (uint32_t)acc;
  return r;
}

// squaring: off-diagonal digit products once, doubled with the column (v_lshl_add_u64): 105 + 14 + 196 mads
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
        acc += (uint64_t)m[i] * P29[j];
#ifdef BLS_FQ_CHECK
        chk += (unsigned __int128)m[i] * P29[j];
#endif
      }
    }
    if (k < 14) {
      m[k] = ((uint32_t)acc * P29_NINV) & Q29_MASK;
      acc += (uint64_t)m[k] * P29[0];
#ifdef BLS_FQ_CHECK
      chk += (unsigned __int128)m[k] * P29[0];
#endif
    } else {
      r.d[k - 14] = (uint32_t)acc & Q29_MASK;
    }
    FQ_CHECK_COL(chk);
    acc >>= 29;
  }
  r.d[13] = (uint32_t)acc;
  return r;
}

// ---- conversions (kernel edges) -------------------------------------------
// packed Montgomery Fp -> digits (same value, N form when the input is canonical)
BLS_HD Fq fq_unpack(const Fp& a) {
  Fq r;
  fp_unpack29(r.d, a);
  return r;
}
// any redundant Fq -> canonical packed Montgomery Fp: one product by R mod p (FP_ONE's digits) brings the value
// below 2p with exact digits, then pack and one conditional subtraction
BLS_HD Fp fq_pack(const Fq& a) {
  const Fq t = fq_mul(a, fq_unpack(FP_ONE));
  return fp_reduce_once(fp_pack29(t.d));
}
// an N-form value (a product output, < 2p) -> canonical packed Fp without the product
BLS_HD Fp fq_pack_n(const Fq& a) { return fp_reduce_once(fp_pack29(a.d)); }

// a^e for a fixed exponent (little-endian u32 limbs, bit nbits-1 set), sliding window w = 3, every operand in N
// form (products of products); control flow depends only on e.  Result in N form.
BLS_HD Fq fq_pow_w3(const Fq& a, const uint32_t* e, int nbits) {
  const Fq a2 = fq_sqr(a);
  const Fq t1 = a;
  const Fq t3 = fq_mul(t1, a2);
  const Fq t5 = fq_mul(t3, a2);
  const Fq t7 = fq_mul(t5, a2);
  Fq r = t1;
  bool started = false;
  int i = nbits - 1;
  while (i >= 0) {
    if (!((e[i >> 5] >> (i & 31)) & 1u)) {
      r = fq_sqr(r);
      --i;
      continue;
    }
    int j = i - 2 < 0 ? 0 : i - 2;  // window [i .. j], ending on a set bit
    while (!((e[j >> 5] >> (j & 31)) & 1u)) ++j;
    uint32_t w = 0;
    for (int k = i; k >= j; --k) w = (w << 1) | ((e[k >> 5] >> (k & 31)) & 1u);
    // a value select, not a reference to one of the four: a reference chosen at run time made them addressable
    // (a private-memory copy of t1..t7 in every kernel that inlines this)
    const Fq m = fq_select(w == 1u, t1, fq_select(w == 3u, t3, fq_select(w == 5u, t5, t7)));
    if (!started) {
      r = m;
      started = true;
    } else {
      for (int k = i; k >= j; --k) r = fq_sqr(r);
      r = fq_mul(r, m);
    }
    i = j - 1;
  }
  return r;
}

}  // namespace bls
