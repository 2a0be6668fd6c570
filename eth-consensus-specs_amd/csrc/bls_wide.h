// Wavefront-cooperative ("wide") Fp arithmetic for the latency-bound one-item
// chains of the per-call path (north_star (a): multi-limb carries across the
// lanes of a wavefront).
//
// Why.  In the lane form (bls_fq.h) one lane owns a whole value and a product
// is ~500 wave instructions: a chain of N dependent products takes N x ~1 us
// whatever the other 63 lanes do.  That is the right trade for batches (64
// items per wave) and the wrong one for a single Verify, whose hash_to_G2,
// signature check and key check are chains of thousands of dependent products.
//
// Layout ("D layout").  A value is 14 radix-2^29 digits of the Montgomery form
// (R = 2^406, the same representation as bls_fq.h) spread over the lanes of a
// 32-lane half-wave: lane k of the half holds digit (k mod 16) when k mod 16 <
// 14, else 0 -- i.e. both 16-lane rows of the half hold the digits.  The two
// halves of a wave hold two independent values (two items, or two chains of one
// item), so every operation below runs both at once.  One VGPR per value.
//
// Product x y R^-1 mod p (wmul / wdot2), per half:
//   1. column sums: lane k accumulates c_k = sum_i x_i y_{k-i} in 64 bits --
//      x_i is a row broadcast (DPP row_newbcast:i; both rows hold x), y walks up
//      one lane per step (DPP wave_shr:1): 14 steps of (two DPP moves, one
//      v_mad_u64_u32).
//   2. carry-save normalisation (wnorm64: two rounds of d_k = (d_k mod 2^29) +
//      (d_{k-1} >> 29), one DPP move each): digits <= 2^29 + 64, same value.
//   3. m = (T mod R) (-p^-1) mod R as a 14-column half product by the constant
//      NINV29 (scalar operands), normalised, lanes >= 14 dropped (mod R).
//   4. T + m p (14 more steps), normalised: the low 14 digits then sum to 0 or
//      exactly R (they are = 0 mod R and below 2 R), so the carry into digit 14
//      is "any low digit nonzero" -- one wave ballot, no carry chain.
//   5. digits 14..27 move down to lanes 0..13 of both rows (v_permlane16_swap + two DPP row shifts: whigh).
// ~140 wave instructions per product pair instead of ~500 per lane product:
// ~3.5x lower latency per product, ~8x per Fp2 product (wdot2 forms a whole
// Fp2 coefficient with one reduction).  Nothing is sequential across digits
// except the DPP walk; no lane ever holds more than one digit of a value.
//
// Bounds ("W form"): digits <= 2^29 + 64 (digit 13 small), value < 2.0001 p for
// products whose operand values multiply to < p R (R/p ~ 2^25.3).  Column sums
// stay below 2^63 for one product of W-form operands and for wdot2 (28 terms);
// sums of two W values must be normalised (wnorm) before they enter a product.
// Subtractions add Q29_K1 = 64 p in borrowed digits (each >= 2^29 + 2^25), so the
// subtrahend must be a W value below 62 p.
//
// All control flow is uniform across the wave; results are checked against the
// lane form on the device (bls_test_wide_selftest, tests/test_gpu_percall.py).
#pragma once
#include <utility>

#include "bls_fq.h"

namespace bls {
namespace wide {

constexpr uint32_t WM = 0x1fffffffu;
// -p^-1 mod 2^406 in radix 2^29 (digit 0 is P29_NINV); n' p = -1 mod R is checked in tests/test_hostcheck.py
constexpr uint32_t NINV29[14] = {0x1ffcfffdu, 0x0f9fffe7u, 0x1444fa22u, 0x15b725b3u, 0x10b48286u,
                                 0x17786471u, 0x0d305bbcu, 0x01d1d65bu, 0x1819eccau, 0x1713467au,
                                 0x1a2cc5bfu, 0x1d55f928u, 0x0b06106fu, 0x1f13d067u};

__device__ __forceinline__ int wlane() { return (int)(threadIdx.x & 63u); }
__device__ __forceinline__ int wpos() { return (int)(threadIdx.x & 31u); }  // lane within the half
__device__ __forceinline__ int wdig() { return (int)(threadIdx.x & 15u); }  // digit index in D layout
__device__ __forceinline__ int whalf() { return (int)((threadIdx.x >> 5) & 1u); }

// DPP wave_shr:1 -- lane l gets lane l - 1, lane 0 gets 0 (lane 32 gets lane 31, which is always 0 here).  The
// move stays a separate v_mov_b32_dpp: folded by the compiler's DPP combine into the consuming VALU op
// (v_add_u32_dpp ... wave_shr:1) it produced results shifted by one more lane in some contexts on gfx950
// (found by tools/h2c_wide_debug.py: a carry-save normalisation came out as shr1(d & M + shr1(d >> 29))).
// an opaque copy: keeps each DPP move a separate instruction (the compiler's DPP combine folded wave_shr moves
// into their VALU consumers and shifted a normalisation by one more lane on gfx950)
// (a plain asm measured the same as the volatile one: tools/fe_stages.py, round 4)
#define BLS_WIDE_FENCE(r) asm volatile("" : "+v"(r))
__device__ __forceinline__ uint32_t shr1(uint32_t v) {
  uint32_t r = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xF, 0xF, true);  // bound_ctrl: invalid -> 0
  BLS_WIDE_FENCE(r);
  return r;
}
// DPP row_newbcast:I -- every lane of a 16-lane row gets lane I of that row
template <int I>
__device__ __forceinline__ uint32_t rbc(uint32_t v) {
  uint32_t r = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x150 + I, 0xF, 0xF, true);
  BLS_WIDE_FENCE(r);  // no DPP combine (see shr1)
  return r;
}
template <class F, int... I>
__device__ __forceinline__ void for14_(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <class F>
__device__ __forceinline__ void for14(F&& f) {
  for14_(f, std::make_integer_sequence<int, 14>{});
}

// d_k = (d_k mod 2^29) + (d_{k-1} >> 29): same value, digits <= 2^29 - 1 + (max digit >> 29)
__device__ __forceinline__ uint32_t wnorm(uint32_t d) { return (d & WM) + shr1(d >> 29); }

// 64-bit column sums (< 2^63) -> 32-bit digits <= 2^29 + 64, same value (two carry-save rounds)
__device__ __forceinline__ uint32_t wnorm64(uint64_t c) {
  const uint64_t h = c >> 29;  // < 2^34
  const uint64_t hs = ((uint64_t)shr1((uint32_t)(h >> 32)) << 32) | shr1((uint32_t)h);
  const uint64_t c1 = (uint64_t)((uint32_t)c & WM) + hs;  // < 2^35
  return ((uint32_t)c1 & WM) + shr1((uint32_t)(c1 >> 29));
}

// acc += x y as column sums (lane k of the half: sum_i x_i y_{k-i}); x, y in D layout
__device__ __forceinline__ void wmac(uint64_t& acc, uint32_t x, uint32_t y) {
  uint32_t s = wpos() < 14 ? y : 0u;  // y's digits of row 0 only
  for14([&](auto I) {
    constexpr int i = decltype(I)::value;
    if (i) s = shr1(s);
    acc += (uint64_t)rbc<i>(x) * s;
  });
}

// columns 14..27 of a half (lanes 14, 15 of its first row, 0..11 of its second) -> digits 0..13 of BOTH rows, lanes
// 14, 15 zero (columns 28, 29 are zero: the value is below 2^(29 x 28)).  v_permlane16_swap puts the first row's
// columns in both rows of one register and the second row's in both rows of another; row_shl:14 / row_shr:2 (zero
// fill) then line them up -- four VALU operations where a ds_bpermute cost ~250 cycles of LDS-path latency on the
// chain (tools/microbench/widerate.hip).
__device__ __forceinline__ uint32_t whigh(uint32_t u) {
  const auto sw = __builtin_amdgcn_permlane16_swap(u, u, false, false);  // [0]: first rows, [1]: second rows
  uint32_t a = (uint32_t)__builtin_amdgcn_mov_dpp((int)sw[0], 0x10E, 0xF, 0xF, true);  // row_shl:14
  uint32_t b = (uint32_t)__builtin_amdgcn_mov_dpp((int)sw[1], 0x112, 0xF, 0xF, true);  // row_shr:2
  BLS_WIDE_FENCE(a);
  BLS_WIDE_FENCE(b);
  return a | b;  // disjoint lanes
}

// Montgomery reduction of column sums (< 2^63, value T < p R): T R^-1 mod p in W form (value < 2.0001 p)
__device__ __forceinline__ uint32_t wredc(uint64_t acc) {
  const int k = wpos();
  const uint32_t t = wnorm64(acc);
  uint64_t am = 0;
  uint32_t s = k < 14 ? t : 0u;
  for14([&](auto I) {
    constexpr int i = decltype(I)::value;
    if (i) s = shr1(s);
    am += (uint64_t)NINV29[i] * s;
  });
  const uint32_t mn = wnorm64(am);
  const uint32_t m = k < 14 ? mn : 0u;  // m = -T p^-1 mod R, < R (1 + 2^-23)
  uint64_t au = t;
  s = m;
  for14([&](auto I) {
    constexpr int i = decltype(I)::value;
    if (i) s = shr1(s);
    au += (uint64_t)P29[i] * s;
  });
  const uint32_t u = wnorm64(au);
  // the low 14 digits sum to 0 or R: the carry into digit 14 is "any of them nonzero"
  const uint64_t bal = __builtin_amdgcn_ballot_w64(k < 14 && u != 0u);
  const bool lowc = ((bal >> (threadIdx.x & 32u)) & 0x3fffull) != 0;
  const uint32_t u2 = u + ((k == 14 && lowc) ? 1u : 0u);
  return whigh(u2);
}

__device__ __forceinline__ uint32_t wmul(uint32_t x, uint32_t y) {
  uint64_t a = 0;
  wmac(a, x, y);
  return wredc(a);
}
__device__ __forceinline__ uint32_t wsqr(uint32_t x) { return wmul(x, x); }
// (x y + u v) R^-1 with one reduction
__device__ __forceinline__ uint32_t wdot2(uint32_t x, uint32_t y, uint32_t u, uint32_t v) {
  uint64_t a = 0;
  wmac(a, x, y);
  wmac(a, u, v);
  return wredc(a);
}

// carry-save round on column sums (same value, columns < 2^29 + 2^35): lets a dot product take two more wmac
// terms (the column bound 2^63 of wredc holds for at most two wmac between rounds)
__device__ __forceinline__ void wacc_norm(uint64_t& acc) {
  const uint64_t h = acc >> 29;  // < 2^34
  acc = (acc & WM) + (((uint64_t)shr1((uint32_t)(h >> 32)) << 32) | shr1((uint32_t)h));
}

// per-lane constants of a kernel: the subtraction constant 64 p (Q29_K1) and R mod p (one) in D layout
struct WK {
  uint32_t k1, one, zero;
};
__device__ __forceinline__ WK wk_init() {
  const int j = wdig();
  const Fq o = fq_unpack(FP_ONE);
  uint32_t k1 = 0, one = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    k1 = j == i ? Q29_K1[i] : k1;
    one = j == i ? o.d[i] : one;
  }
  return WK{k1, one, 0u};
}

__device__ __forceinline__ uint32_t wadd(uint32_t a, uint32_t b) { return wnorm(a + b); }
// a - b (b a W value below 62 p): a + 64 p - b digit-wise, normalised
__device__ __forceinline__ uint32_t wsub(const WK& K, uint32_t a, uint32_t b) { return wnorm(a + (K.k1 - b)); }
__device__ __forceinline__ uint32_t wneg(const WK& K, uint32_t b) { return wnorm(K.k1 - b); }
// small multiple of a W value, normalised (k <= 7 per step keeps a digit below 2^32)
template <uint32_t KM>
__device__ __forceinline__ uint32_t wmuls(uint32_t a) {
  if constexpr (KM <= 7u)
    return wnorm(a * KM);
  else if constexpr ((KM & 1u) == 0u)
    return wmuls<KM / 2>(wmuls<2>(a));
  else  // the sum of two normalised values is normalised again before it can enter a product
    return wnorm(wmuls<KM / 2>(wmuls<2>(a)) + a);
}

// ---- conversions (kernel edges; lane-local work, not on the chain) ----------
// this half's value as a lane-local Fq (every lane of the half gets all 14 digits)
__device__ __forceinline__ Fq w_to_fq(uint32_t v) {
  Fq r;
  const bool hi = whalf() != 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)v, i);
    const uint32_t up = (uint32_t)__builtin_amdgcn_readlane((int)v, 32 + i);
    r.d[i] = hi ? up : lo;
  }
  return r;
}
// a lane-local Fq (the same in every lane of a half, or different per half) -> D layout
__device__ __forceinline__ uint32_t w_from_fq(const Fq& a) {
  const int j = wdig();
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) v = j == i ? a.d[i] : v;
  return v;
}
__device__ __forceinline__ uint32_t w_from_fp(const Fp& a) { return w_from_fq(fq_unpack(a)); }
// canonical packed Montgomery Fp of this half's value
__device__ __forceinline__ Fp w_to_fp(uint32_t v) { return fq_pack(w_to_fq(v)); }
__device__ __forceinline__ bool w_is_zero(uint32_t v) { return fp_is_zero(w_to_fp(v)); }
__device__ __forceinline__ bool w_eq(const WK& K, uint32_t a, uint32_t b) { return w_is_zero(wsub(K, a, b)); }
// the other half's value (lane l gets lane l ^ 32)
// (v_permlane32_swap: [0] holds the first half in both halves, [1] the second; a VALU move, not the LDS path)
__device__ __forceinline__ uint32_t wswap(uint32_t v) {
  const auto sw = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return whalf() ? (uint32_t)sw[0] : (uint32_t)sw[1];
}

// a^e on two waves of a workgroup whose waves all call it (it holds two workgroup barriers): wave 0 forms the
// squarings a^(2^i) and hands each to wave 1 through an LDS ring of PW_RING slots, wave 1 multiplies in those of
// the set bits of e (LSB first) -- the chain is the nbits - 1 squarings alone, not the squarings plus a window
// method's products (sswu's (p - 3) / 4: 378 squarings, 228 set bits).  ring: PW_RING x 64 words of LDS, cnt: two
// ints of LDS (squarings published, ring slots released); every wave returns a^e.
constexpr int PW_RING = 32;
__device__ __forceinline__ uint32_t wpow_2w(uint32_t a, const uint32_t* e, int nbits, uint32_t* ring, int* cnt,
                                            int w) {
  const int l = wlane();
  if (threadIdx.x == 0) {
    cnt[0] = 0;
    cnt[1] = 0;
  }
  __syncthreads();
  if (w == 0) {  // the squarer: slot i % PW_RING <- a^(2^i), once wave 1 has released index i - PW_RING
    uint32_t sq = a;
#pragma unroll 1
    for (int i = 0; i < nbits; ++i) {
      if (i >= PW_RING)
        while (__hip_atomic_load(&cnt[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= i - PW_RING)
          __builtin_amdgcn_s_sleep(1);
      ring[(i % PW_RING) * 64 + l] = sq;
      if (l == 0) __hip_atomic_store(&cnt[0], i + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (i + 1 < nbits) sq = wsqr(sq);
    }
  } else if (w == 1) {  // the multiplier: r = prod of a^(2^i) over the set bits i
    uint32_t r = 0;
    bool started = false;
#pragma unroll 1
    for (int i = 0; i < nbits; ++i) {
      if (!((e[i >> 5] >> (i & 31)) & 1u)) continue;
      if (l == 0) __hip_atomic_store(&cnt[1], i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);  // below i: done
      while (__hip_atomic_load(&cnt[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= i)
        __builtin_amdgcn_s_sleep(1);
      const uint32_t v = ring[(i % PW_RING) * 64 + l];
      r = started ? wmul(r, v) : v;
      started = true;
      if (l == 0) __hip_atomic_store(&cnt[1], i + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    ring[l] = r;  // every slot is released: the squarer is done with the ring
  }
  __syncthreads();
  const uint32_t r = ring[l];
  __syncthreads();  // (the ring is free again for the caller's next use)
  return r;
}

// a^e for a fixed exponent (little-endian u32 limbs, bit nbits-1 set), sliding window w = 3 (as fq_pow_w3)
__device__ __forceinline__ uint32_t wpow(uint32_t a, const uint32_t* e, int nbits) {
  const uint32_t a2 = wsqr(a);
  const uint32_t t1 = a, t3 = wmul(t1, a2), t5 = wmul(t3, a2), t7 = wmul(t5, a2);
  uint32_t r = t1;
  bool started = false;
  int i = nbits - 1;
  while (i >= 0) {
    if (!((e[i >> 5] >> (i & 31)) & 1u)) {
      r = wsqr(r);
      --i;
      continue;
    }
    int j = i - 2 < 0 ? 0 : i - 2;
    while (!((e[j >> 5] >> (j & 31)) & 1u)) ++j;
    uint32_t w = 0;
    for (int k = i; k >= j; --k) w = (w << 1) | ((e[k >> 5] >> (k & 31)) & 1u);
    const uint32_t m = w == 1u ? t1 : (w == 3u ? t3 : (w == 5u ? t5 : t7));
    if (!started) {
      r = m;
      started = true;
    } else {
      for (int k = i; k >= j; --k) r = wsqr(r);
      r = wmul(r, m);
    }
    i = j - 1;
  }
  return r;
}

// ---- Fp2 in pair form: (c0, c1) as two D-layout values per half -----------
struct W2 {
  uint32_t c0, c1;
};
__device__ __forceinline__ W2 w2add(W2 a, W2 b) { return W2{wadd(a.c0, b.c0), wadd(a.c1, b.c1)}; }
__device__ __forceinline__ W2 w2sub(const WK& K, W2 a, W2 b) { return W2{wsub(K, a.c0, b.c0), wsub(K, a.c1, b.c1)}; }
__device__ __forceinline__ W2 w2neg(const WK& K, W2 a) { return W2{wneg(K, a.c0), wneg(K, a.c1)}; }
template <uint32_t KM>
__device__ __forceinline__ W2 w2muls(W2 a) {
  return W2{wmuls<KM>(a.c0), wmuls<KM>(a.c1)};
}
__device__ __forceinline__ W2 w2conj(const WK& K, W2 a) { return W2{a.c0, wneg(K, a.c1)}; }
// c0 = a0 b0 + a1 (64p - b1), c1 = a0 b1 + a1 b0: one reduction per coefficient
__device__ __forceinline__ W2 w2mul(const WK& K, W2 a, W2 b) {
  return W2{wdot2(a.c0, b.c0, a.c1, wneg(K, b.c1)), wdot2(a.c0, b.c1, a.c1, b.c0)};
}
// (a0 + a1)(a0 - a1), 2 a0 a1
__device__ __forceinline__ W2 w2sqr(const WK& K, W2 a) {
  return W2{wmul(wadd(a.c0, a.c1), wsub(K, a.c0, a.c1)), wmul(a.c0, wadd(a.c1, a.c1))};
}
__device__ __forceinline__ W2 w2mulfp(W2 a, uint32_t b) { return W2{wmul(a.c0, b), wmul(a.c1, b)}; }
// a (1 + u): the Fp2 non-residue xi
__device__ __forceinline__ W2 w2xi(const WK& K, W2 a) { return W2{wsub(K, a.c0, a.c1), wadd(a.c0, a.c1)}; }
__device__ __forceinline__ W2 w2_from_fp2(const Fp2& a) { return W2{w_from_fp(a.c0), w_from_fp(a.c1)}; }
__device__ __forceinline__ Fp2 w2_to_fp2(W2 a) { return Fp2{w_to_fp(a.c0), w_to_fp(a.c1)}; }
__device__ __forceinline__ bool w2_is_zero(W2 a) { return w_is_zero(a.c0) && w_is_zero(a.c1); }
__device__ __forceinline__ W2 w2swap(W2 a) { return W2{wswap(a.c0), wswap(a.c1)}; }
__device__ __forceinline__ W2 w2sel(bool c, W2 a, W2 b) { return W2{c ? a.c0 : b.c0, c ? a.c1 : b.c1}; }

// ---- Fp2 in F2 layout: one VGPR, c0 in half 0 and c1 in half 1 (D layout each) ----
// An Fp2 product is ONE wdot2 per half (both halves at once): half 0 forms c0 = a0 b0 + a1 (kn - b1), half 1
// c1 = a0 b1 + a1 b0, each reading the other half's coefficients through one v_permlane32_swap (wswap).  kn is a
// multiple of p in borrowed digits covering b1 (the 4096p of bls_fq_g2.h for b1 < 4096p).
__device__ __forceinline__ uint32_t wf_mul(uint32_t kn, uint32_t a, uint32_t b) {
  const bool h = whalf() != 0;
  const uint32_t sa = wswap(a), sb = wswap(b);
  const uint32_t nb1 = wnorm(kn - sb);
  return wdot2(h ? sa : a, b, h ? a : sa, h ? sb : nb1);
}
// acc += a b (F2 layout, unreduced column sums; kn covering b1), then a carry-save round: any number of these
// terms can share one wredc while their values sum below p R
__device__ __forceinline__ void wf_mac(uint64_t& acc, uint32_t kn, uint32_t a, uint32_t b) {
  const bool h = whalf() != 0;
  const uint32_t sa = wswap(a), sb = wswap(b);
  const uint32_t nb1 = wnorm(kn - sb);
  wmac(acc, h ? sa : a, b);
  wmac(acc, h ? a : sa, h ? sb : nb1);
  wacc_norm(acc);
}
// acc += a c for an Fp constant c held in both halves (the Fp2 a times a real scalar: one wmac)
__device__ __forceinline__ void wf_mac_fp(uint64_t& acc, uint32_t a, uint32_t c) {
  wmac(acc, a, c);
  wacc_norm(acc);
}
// (a0 + a1)(a0 - a1 + ks) in half 0, a0 (2 a1) in half 1 (ks covering a1)
__device__ __forceinline__ uint32_t wf_sqr(uint32_t ks, uint32_t a) {
  const bool h = whalf() != 0;
  const uint32_t sa = wswap(a);
  const uint32_t x = h ? sa : wadd(a, sa);
  const uint32_t y = h ? wmuls<2>(a) : wnorm(a + (ks - sa));
  return wmul(x, y);
}
// a xi = (a0 - a1) + (a0 + a1) u  (k covering a1)
__device__ __forceinline__ uint32_t wf_xi(uint32_t k, uint32_t a) {
  const bool h = whalf() != 0;
  const uint32_t sa = wswap(a);
  const uint32_t d = wnorm(a + (k - sa)), s = wadd(a, sa);
  return h ? s : d;
}
// conj(a) (k covering a1)
__device__ __forceinline__ uint32_t wf_conj(uint32_t k, uint32_t a) {
  const uint32_t n = wnorm(k - a);
  return whalf() ? n : a;
}
// an Fp2 constant / lane-local Fp2 value in F2 layout
__device__ __forceinline__ uint32_t wf_from_fp2(const Fp2& a) {
  const bool h = whalf() != 0;
  return w_from_fq(fq_unpack(h ? a.c1 : a.c0));
}
// canonical packed Fp2 on every lane
__device__ __forceinline__ Fp2 wf_to_fp2(uint32_t v) {
  Fq c0, c1;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    c0.d[i] = (uint32_t)__builtin_amdgcn_readlane((int)v, i);
    c1.d[i] = (uint32_t)__builtin_amdgcn_readlane((int)v, 32 + i);
  }
  return Fp2{fq_pack(c0), fq_pack(c1)};
}

}  // namespace wide
}  // namespace bls
