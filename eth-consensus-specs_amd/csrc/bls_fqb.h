// Bound-typed redundant digit form: the Fq arithmetic of bls_fq.h with its
// preconditions proved at compile time.
//
// FqB<V, D> is an Fq whose value is below V p and whose digits 0..12 are at
// most D (digit 13 is then at most top(V) = floor(V p / 2^377), since every
// digit is non-negative).  Every operation returns the bound of its result:
//   add            FqB<V1 + V2, D1 + D2>
//   sub(a, b)      a + K - b digit-wise with K = c p in borrowed digits, each
//                  of K's digits >= b's bound (k_for<V2, D2>: the smallest c
//                  whose top digit also covers b's): FqB<V1 + c, D1 + max K>
//   norm           carry-save normalisation: FqB<V, 2^29 - 1 + (D >> 29)>
//   mul / sqr      static_assert V1 V2 <= floor(R / p) (x y < p R, so the
//                  Montgomery output is < 2p) and that every product-scanning
//                  column -- digit products, reduction products m_i p_j and
//                  the 2^35 carry -- stays below 2^64 for these digit bounds;
//                  result FqB<2, 2^29 - 1> (N form)
//   relax<V, D>    widening to a declared bound (static_assert)
// Loop-carried state is declared at a fixed bound and every step's result is
// relaxed to it, so a loop compiles only if its bounds close (an induction
// the compiler checks).  No bound exists at run time: FqB is an Fq.
#pragma once
#include "bls_fq.h"

namespace bls {

namespace fqb_detail {
constexpr uint64_t MASK = Q29_MASK;
constexpr uint64_t R_OVER_P = 41291124;  // floor(2^406 / p)
// floor(V p / 2^377) <= ceil(V * 13.00209)   (p / 2^377 = 13.0020898...)
constexpr uint64_t top(uint64_t V) { return (V * 13002090ull + 999999ull) / 1000000ull; }

// every column of a product-scanning Montgomery product of x (digits 0..12 <= dx, digit 13 <= tx) and y, plus its
// reduction products m_i p_j (m_i < 2^29) and the incoming carry (< 2^35), stays below 2^64
constexpr bool columns_fit(uint64_t dx, uint64_t tx, uint64_t dy, uint64_t ty) {
  for (int k = 0; k < 27; ++k) {
    unsigned __int128 s = (unsigned __int128)1 << 35;
    for (int i = 0; i < 14; ++i) {
      const int j = k - i;
      if (j < 0 || j > 13) continue;
      s += (unsigned __int128)(i == 13 ? tx : dx) * (j == 13 ? ty : dy);  // x_i y_j
      s += (unsigned __int128)MASK * P29[j];                                // m_i p_j (m_i < 2^29)
    }
    if (s >= ((unsigned __int128)1 << 64)) return false;
  }
  return true;
}

// the same for x y + u v accumulated in one column sum (fq_mul_dot2)
constexpr bool columns_fit2(uint64_t dx, uint64_t tx, uint64_t dy, uint64_t ty, uint64_t du, uint64_t tu, uint64_t dv,
                            uint64_t tv) {
  for (int k = 0; k < 27; ++k) {
    unsigned __int128 s = (unsigned __int128)1 << 35;
    for (int i = 0; i < 14; ++i) {
      const int j = k - i;
      if (j < 0 || j > 13) continue;
      s += (unsigned __int128)(i == 13 ? tx : dx) * (j == 13 ? ty : dy);
      s += (unsigned __int128)(i == 13 ? tu : du) * (j == 13 ? tv : dv);
      s += (unsigned __int128)MASK * P29[j];
    }
    if (s >= ((unsigned __int128)1 << 64)) return false;
  }
  return true;
}

// c p in 14 borrowed digits with digits 0..12 >= lo; ok = false if c p does not fit or the top digit goes negative
struct KConst {
  uint32_t d[14];
  uint64_t c, max;
  bool ok;
};
constexpr KConst make_k(uint64_t c, uint64_t lo) {
  KConst k{};
  uint64_t w[14] = {};
  uint64_t carry = 0;
  for (int i = 0; i < 14; ++i) {
    const uint64_t t = (uint64_t)P29[i] * c + carry;
    w[i] = i < 13 ? (t & MASK) : t;
    carry = i < 13 ? (t >> 29) : 0;
  }
  uint64_t e_prev = 0, mx = 0;
  k.ok = true;
  for (int i = 0; i < 13; ++i) {
    uint64_t e = 0;
    while (w[i] + (e << 29) < lo + e_prev) ++e;
    const uint64_t v = w[i] + (e << 29) - e_prev;
    if (v > 0xffffffffull) k.ok = false;
    k.d[i] = (uint32_t)v;
    mx = v > mx ? v : mx;
    e_prev = e;
  }
  if (w[13] < e_prev || w[13] - e_prev > 0xffffffffull) k.ok = false;
  k.d[13] = (uint32_t)(w[13] - e_prev);
  k.max = mx > k.d[13] ? mx : k.d[13];
  k.c = c;
  return k;
}
// the smallest multiple of p whose borrowed digits cover a subtrahend with value < V p and digits <= D
constexpr KConst k_for(uint64_t V, uint64_t D) {
  for (uint64_t c = 1; c < (1ull << 24); ++c) {
    const KConst k = make_k(c, D);
    if (k.ok && k.d[13] >= top(V)) return k;
  }
  return KConst{};
}
template <uint64_t V, uint64_t D>
struct KFor {
  static constexpr KConst k = k_for(V, D);
  static_assert(k.ok, "no subtraction constant covers this subtrahend");
};
}  // namespace fqb_detail

template <uint64_t V, uint64_t D>
struct FqB {
  static_assert(V >= 1 && V <= (1ull << 24), "value bound out of range");
  static_assert(D <= 0xffffffffull, "digit bound exceeds 32 bits");
  static_assert(fqb_detail::top(V) <= 0xffffffffull, "top digit exceeds 32 bits");
  static constexpr uint64_t val = V, dig = D;
  Fq x;
};
using FqN = FqB<2, fqb_detail::MASK>;  // product output
using FqC = FqB<1, fqb_detail::MASK>;  // canonical (an unpacked packed Fp)

template <uint64_t V, uint64_t D>
BLS_HD FqB<V, D> fqb(const Fq& x) {
  return FqB<V, D>{x};
}
BLS_HD FqC fqb_canon(const Fp& a) { return FqC{fq_unpack(a)}; }

template <uint64_t V1, uint64_t D1, uint64_t V2, uint64_t D2>
BLS_HD FqB<V1 + V2, D1 + D2> operator+(const FqB<V1, D1>& a, const FqB<V2, D2>& b) {
  return {fq_add(a.x, b.x)};
}

template <uint64_t V1, uint64_t D1, uint64_t V2, uint64_t D2>
BLS_HD FqB<V1 + fqb_detail::KFor<V2, D2>::k.c, D1 + fqb_detail::KFor<V2, D2>::k.max> operator-(const FqB<V1, D1>& a,
                                                                                                const FqB<V2, D2>& b) {
  constexpr fqb_detail::KConst K = fqb_detail::KFor<V2, D2>::k;
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = a.x.d[i] + (K.d[i] - b.x.d[i]);
  return {r};
}

template <uint64_t V, uint64_t D>
BLS_HD FqB<V, fqb_detail::MASK + (D >> 29)> norm(const FqB<V, D>& a) {
  return {fq_norm(a.x)};
}

template <uint64_t K, uint64_t V, uint64_t D>
BLS_HD FqB<K * V, fqb_detail::MASK + ((K * D) >> 29)> small(const FqB<V, D>& a) {
  static_assert(K * D < (1ull << 61), "small multiple overflows");
  return {fq_mul_small(a.x, (uint32_t)K)};
}

template <uint64_t V1, uint64_t D1, uint64_t V2, uint64_t D2>
BLS_HD FqN operator*(const FqB<V1, D1>& a, const FqB<V2, D2>& b) {
  static_assert(V1 * V2 <= fqb_detail::R_OVER_P, "product operand values exceed p R");
  static_assert(fqb_detail::columns_fit(D1, fqb_detail::top(V1), D2, fqb_detail::top(V2)),
                "product column exceeds 64 bits");
  return {fq_mul(a.x, b.x)};
}
// Montgomery (a b + c d): one reduction for two products (fq_mul_dot2)
template <uint64_t V1, uint64_t D1, uint64_t V2, uint64_t D2, uint64_t V3, uint64_t D3, uint64_t V4, uint64_t D4>
BLS_HD FqN dot2(const FqB<V1, D1>& a, const FqB<V2, D2>& b, const FqB<V3, D3>& c, const FqB<V4, D4>& d) {
  static_assert(V1 * V2 + V3 * V4 <= fqb_detail::R_OVER_P, "dot product operand values exceed p R");
  static_assert(fqb_detail::columns_fit2(D1, fqb_detail::top(V1), D2, fqb_detail::top(V2), D3, fqb_detail::top(V3), D4,
                                         fqb_detail::top(V4)),
                "dot product column exceeds 64 bits");
  return {fq_mul_dot2(a.x, b.x, c.x, d.x)};
}
// -b as K - b digit-wise (K = c p covering b's digits, as in a - b)
template <uint64_t V, uint64_t D>
BLS_HD FqB<fqb_detail::KFor<V, D>::k.c, fqb_detail::KFor<V, D>::k.max> neg(const FqB<V, D>& b) {
  constexpr fqb_detail::KConst K = fqb_detail::KFor<V, D>::k;
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = K.d[i] - b.x.d[i];
  return {r};
}
// whether dot2(a, b, c, d) fits its columns with these bounds
template <class A, class B, class C, class D>
constexpr bool dot2_fits() {
  return fqb_detail::columns_fit2(A::dig, fqb_detail::top(A::val), B::dig, fqb_detail::top(B::val), C::dig,
                                  fqb_detail::top(C::val), D::dig, fqb_detail::top(D::val));
}

template <uint64_t V, uint64_t D>
BLS_HD FqN sqr(const FqB<V, D>& a) {
  static_assert(V * V <= fqb_detail::R_OVER_P, "square operand value exceeds sqrt(p R)");
  static_assert(fqb_detail::columns_fit(D, fqb_detail::top(V), D, fqb_detail::top(V)), "square column exceeds 64 bits");
  return {fq_sqr(a.x)};
}

template <uint64_t V, uint64_t D, uint64_t V1, uint64_t D1>
BLS_HD FqB<V, D> relax(const FqB<V1, D1>& a) {
  static_assert(V1 <= V && D1 <= D, "value does not fit the declared bound");
  return {a.x};
}
template <uint64_t V1, uint64_t D1, uint64_t V2, uint64_t D2>
BLS_HD FqB<(V1 > V2 ? V1 : V2), (D1 > D2 ? D1 : D2)> sel(bool c, const FqB<V1, D1>& a, const FqB<V2, D2>& b) {
  return {fq_select(c, a.x, b.x)};
}

// ---- Fp2 = Fp[i]/(i^2 + 1), one bound for both coefficients ----------------
template <uint64_t V, uint64_t D>
struct Fq2B {
  FqB<V, D> c0, c1;
};
template <uint64_t V, uint64_t D>
BLS_HD Fq2B<V, D> fq2b(const FqB<V, D>& c0, const FqB<V, D>& c1) {
  return {c0, c1};
}
template <uint64_t V, uint64_t D>
BLS_HD Fq2B<V, D> fq2b_zero() {
  return {{fq_zero()}, {fq_zero()}};
}

template <uint64_t V1, uint64_t D1, uint64_t V2, uint64_t D2>
BLS_HD auto operator+(const Fq2B<V1, D1>& a, const Fq2B<V2, D2>& b) {
  return Fq2B<V1 + V2, D1 + D2>{a.c0 + b.c0, a.c1 + b.c1};
}
template <uint64_t V1, uint64_t D1, uint64_t V2, uint64_t D2>
BLS_HD auto operator-(const Fq2B<V1, D1>& a, const Fq2B<V2, D2>& b) {
  using R = decltype(a.c0 - b.c0);
  return Fq2B<R::val, R::dig>{a.c0 - b.c0, a.c1 - b.c1};
}
template <uint64_t V, uint64_t D>
BLS_HD auto norm(const Fq2B<V, D>& a) {
  using R = decltype(norm(a.c0));
  return Fq2B<R::val, R::dig>{norm(a.c0), norm(a.c1)};
}
template <uint64_t K, uint64_t V, uint64_t D>
BLS_HD auto small(const Fq2B<V, D>& a) {
  using R = decltype(small<K>(a.c0));
  return Fq2B<R::val, R::dig>{small<K>(a.c0), small<K>(a.c1)};
}
template <uint64_t V, uint64_t D, uint64_t V1, uint64_t D1>
BLS_HD Fq2B<V, D> relax(const Fq2B<V1, D1>& a) {
  return {relax<V, D>(a.c0), relax<V, D>(a.c1)};
}
template <uint64_t V1, uint64_t D1, uint64_t V2, uint64_t D2>
BLS_HD auto sel(bool c, const Fq2B<V1, D1>& a, const Fq2B<V2, D2>& b) {
  using R = decltype(sel(c, a.c0, b.c0));
  return Fq2B<R::val, R::dig>{sel(c, a.c0, b.c0), sel(c, a.c1, b.c1)};
}
// xi a = (1 + i) a = (a0 - a1) + (a0 + a1) i
template <uint64_t V, uint64_t D>
BLS_HD auto xi(const Fq2B<V, D>& a) {
  using R0 = decltype(a.c0 - a.c1);
  using R = FqB<(R0::val > 2 * V ? R0::val : 2 * V), (R0::dig > 2 * D ? R0::dig : 2 * D)>;
  return Fq2B<R::val, R::dig>{relax<R::val, R::dig>(a.c0 - a.c1), relax<R::val, R::dig>(a.c0 + a.c1)};
}
// c0 = a0 b0 - a1 b1 = a0 b0 + a1 (K - b1), c1 = a0 b1 + a1 b0: two dot products with one reduction each (4 digit
// products + 2 reductions, ~16 % fewer instructions than Karatsuba's 3 products + 3 reductions and its
// additions, subtractions and normalisations); K - b1 is normalised only when its borrowed digits would overflow
// a column.  Both coefficients come out in N form.
template <uint64_t V1, uint64_t D1, uint64_t V2, uint64_t D2>
BLS_HD Fq2B<2, fqb_detail::MASK> operator*(const Fq2B<V1, D1>& a, const Fq2B<V2, D2>& b) {
  const auto nb = neg(b.c1);
  using A = FqB<V1, D1>;
  using B = FqB<V2, D2>;
  FqN c0;
  if constexpr (dot2_fits<A, B, A, decltype(nb)>()) {
    c0 = dot2(a.c0, b.c0, a.c1, nb);
  } else {
    c0 = dot2(a.c0, b.c0, a.c1, norm(nb));
  }
  return {c0, dot2(a.c0, b.c1, a.c1, b.c0)};
}

// complex squaring: (a0 + a1)(a0 - a1), 2 a0 a1
template <uint64_t V, uint64_t D>
BLS_HD auto sqr(const Fq2B<V, D>& a) {
  const FqN t0 = (a.c0 + a.c1) * norm(a.c0 - a.c1);
  const auto t1 = small<2>(FqN(a.c0 * a.c1));
  using R = FqB<(decltype(t1)::val > 2 ? decltype(t1)::val : 2), decltype(t1)::dig>;
  return Fq2B<R::val, R::dig>{relax<R::val, R::dig>(t0), relax<R::val, R::dig>(t1)};
}

// ---- Fp6 = Fp2[v]/(v^3 - xi) -----------------------------------------------
template <uint64_t V, uint64_t D>
struct Fq6B {
  Fq2B<V, D> c0, c1, c2;
};
template <uint64_t V1, uint64_t D1, uint64_t V2, uint64_t D2>
BLS_HD auto operator+(const Fq6B<V1, D1>& a, const Fq6B<V2, D2>& b) {
  return Fq6B<V1 + V2, D1 + D2>{a.c0 + b.c0, a.c1 + b.c1, a.c2 + b.c2};
}
template <uint64_t V, uint64_t D>
BLS_HD auto norm(const Fq6B<V, D>& a) {
  using R = decltype(norm(a.c0.c0));
  return Fq6B<R::val, R::dig>{norm(a.c0), norm(a.c1), norm(a.c2)};
}
template <uint64_t V, uint64_t D, uint64_t V1, uint64_t D1>
BLS_HD Fq6B<V, D> relax(const Fq6B<V1, D1>& a) {
  return {relax<V, D>(a.c0), relax<V, D>(a.c1), relax<V, D>(a.c2)};
}
template <uint64_t V1, uint64_t D1, uint64_t V2, uint64_t D2>
BLS_HD auto sel(bool c, const Fq6B<V1, D1>& a, const Fq6B<V2, D2>& b) {
  using R = decltype(sel(c, a.c0.c0, b.c0.c0));
  return Fq6B<R::val, R::dig>{sel(c, a.c0, b.c0), sel(c, a.c1, b.c1), sel(c, a.c2, b.c2)};
}

template <uint64_t V1, uint64_t D1, uint64_t V2, uint64_t D2>
BLS_HD auto operator-(const Fq6B<V1, D1>& a, const Fq6B<V2, D2>& b) {
  using R = decltype(a.c0.c0 - b.c0.c0);
  return Fq6B<R::val, R::dig>{a.c0 - b.c0, a.c1 - b.c1, a.c2 - b.c2};
}
// v a = (xi a2, a0, a1)   (v^3 = xi)
template <uint64_t V, uint64_t D>
BLS_HD auto f6v(const Fq6B<V, D>& a) {
  const auto x = xi(a.c2);
  using X = decltype(x.c0);
  return Fq6B<X::val, X::dig>{x, relax<X::val, X::dig>(a.c0), relax<X::val, X::dig>(a.c1)};
}
// the common bound of three Fp2 values
template <uint64_t V0, uint64_t D0, uint64_t V1, uint64_t D1, uint64_t V2, uint64_t D2>
BLS_HD auto fq6b(const Fq2B<V0, D0>& c0, const Fq2B<V1, D1>& c1, const Fq2B<V2, D2>& c2) {
  constexpr uint64_t V = V0 > V1 ? (V0 > V2 ? V0 : V2) : (V1 > V2 ? V1 : V2);
  constexpr uint64_t D = D0 > D1 ? (D0 > D2 ? D0 : D2) : (D1 > D2 ? D1 : D2);
  return Fq6B<V, D>{relax<V, D>(c0), relax<V, D>(c1), relax<V, D>(c2)};
}

// canonical packed <-> bounded digit form
BLS_HD Fq2B<1, fqb_detail::MASK> fq2b_canon(const Fp2& a) { return {fqb_canon(a.c0), fqb_canon(a.c1)}; }
template <uint64_t V, uint64_t D>
BLS_HD Fp2 fq2b_pack(const Fq2B<V, D>& a) {
  return Fp2{fq_pack(a.c0.x), fq_pack(a.c1.x)};
}

}  // namespace bls
