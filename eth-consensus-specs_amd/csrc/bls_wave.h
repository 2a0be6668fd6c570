// Wave-cooperative execution of wave programs (tables from tools/wavec.py,
// bls_waveprog.h).
//
// One 64-lane workgroup owns one item.  Its Fp values live in an LDS slot
// array (48 B per slot).  A program level is a set of independent Montgomery
// products: lane j forms operand A and B as small-integer linear
// combinations of slots, multiplies, and writes its product slot; a "lin"
// level only forms and stores the linear combination.  Levels are separated
// by a workgroup barrier (the workgroup is one wave, so the barrier is only
// an LDS visibility / compiler ordering point).  An Fp12 product costs the
// wave ~1 multiplication of latency instead of 54 sequential ones.
#pragma once
#include "bls_tower.h"
#include "bls_waveprog.h"

namespace bls {

struct WaveProg {
  const uint32_t* terms;
  const uint32_t (*levels)[5];  // {unused, nitems, na, nb, base}; item kind in bit 31 of its dest word
  int nlevels;
  int scratch;
};

#define WAVE_PROG(NAME) \
  WaveProg { WP_##NAME##_TERMS, WP_##NAME##_LEVELS, WP_##NAME##_NLEVELS, WP_##NAME##_SCRATCH }

__device__ __forceinline__ Fp lds_get(const Fp* slots, int s) { return slots[s]; }

// Linear combinations are accumulated lazily: a 13-limb (416-bit) running sum
// that starts at OFF = 256*p (so subtracting up to 256 p's never goes
// negative) and takes each term with one add/sub carry chain -- no modular
// reduction per term.  The sum stays below 2^390, which fp_mul_digits accepts
// directly; only results stored to a slot are reduced (wave_reduce).
struct Acc {
  uint32_t l[13];
};

// 256 * p  (= p << 8), 13 limbs
__device__ __forceinline__ void acc_init(Acc& a) {
#pragma unroll
  for (int i = 0; i < 13; i++) {
    const uint32_t lo = i < 12 ? P_LIMBS[i] : 0u;
    const uint32_t prev = i > 0 ? P_LIMBS[i - 1] : 0u;
    a.l[i] = (lo << 8) | (i > 0 ? (prev >> 24) : 0u);
  }
}

__device__ __forceinline__ void acc_add(Acc& a, const uint32_t* x, int n) {
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < 13; i++) a.l[i] = __builtin_addc(a.l[i], i < n ? x[i] : 0u, c, &c);
}
__device__ __forceinline__ void acc_sub(Acc& a, const uint32_t* x, int n) {
  unsigned b = 0;
#pragma unroll
  for (int i = 0; i < 13; i++) a.l[i] = __builtin_subc(a.l[i], i < n ? x[i] : 0u, b, &b);
}

// y = m * x (13 limbs) for a small m
__device__ __forceinline__ void mul_small13(uint32_t y[13], const Fp& x, uint32_t m) {
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint64_t t = (uint64_t)x.l[i] * m + carry;
    y[i] = (uint32_t)t;
    carry = (uint32_t)(t >> 32);
  }
  y[12] = carry;
}

__device__ __forceinline__ void wave_lincomb(Acc& acc, const Fp* slots, const int* fb, const uint32_t* t, int n) {
  acc_init(acc);
  for (int k = 0; k < n; k++) {
    const uint32_t w = t[k];
    if (!w) break;
    const int fr = (int)(w >> 20);
    const int ix = (int)((w >> 8) & 0xfffu);
    const int c = (int)(w & 0xffu) - 128;
    const Fp x = slots[fb[fr] + ix];
    const uint32_t m = (uint32_t)(c < 0 ? -c : c);
    if (m == 1) {
      if (c < 0)
        acc_sub(acc, x.l, 12);
      else
        acc_add(acc, x.l, 12);
    } else {
      uint32_t y[13];
      mul_small13(y, x, m);
      if (c < 0)
        acc_sub(acc, y, 13);
      else
        acc_add(acc, y, 13);
    }
  }
}

// canonical residue of an accumulator (< 2^390): subtract q*p with q from
// the top bits (q may undershoot by a few), then up to 3 conditional p's.
__device__ __forceinline__ Fp wave_reduce(const Acc& a) {
  // q ~= floor(a / p) via the top 64 bits: a >> 350 and p >> 350 (31 bits)
  const uint64_t top = ((uint64_t)a.l[12] << 34) | ((uint64_t)a.l[11] << 2) | (a.l[10] >> 30);
  const uint64_t ptop = (((uint64_t)P_LIMBS[11]) << 2) | (P_LIMBS[10] >> 30);  // p >> 350
  uint32_t q = (uint32_t)(top / (ptop + 1));
  uint32_t r[13];
  uint32_t carry = 0;
  unsigned b = 0;
#pragma unroll
  for (int i = 0; i < 13; i++) {
    const uint64_t t = (uint64_t)(i < 12 ? P_LIMBS[i] : 0u) * q + carry;
    carry = (uint32_t)(t >> 32);
    r[i] = __builtin_subc(a.l[i], (uint32_t)t, b, &b);
  }
  Fp v;
#pragma unroll
  for (int i = 0; i < 12; i++) v.l[i] = r[i];
  // r < 4p here (r[12] == 0)
  v = fp_reduce_once(v);
  v = fp_reduce_once(v);
  v = fp_reduce_once(v);
  return v;
}

// Run program `p` with frame bases fb[] (slot indices; the last frame is the
// program's scratch).  All 64 lanes of the workgroup must call it.
__device__ __noinline__ void wave_run(const WaveProg p, Fp* slots, const int* fb) {
  const int lane = threadIdx.x;
  for (int lv = 0; lv < p.nlevels; lv++) {
    const uint32_t nitems = p.levels[lv][1], na = p.levels[lv][2], nb = p.levels[lv][3], base = p.levels[lv][4];
    if ((uint32_t)lane < nitems) {
      const uint32_t* t = p.terms + base + (size_t)lane * (1 + na + nb);
      const uint32_t d = t[0];
      Acc a;
      wave_lincomb(a, slots, fb, t + 1, (int)na);
      Fp out;
      if (d >> 31) {  // product item: both operands unreduced (< 2^390)
        Acc b;
        wave_lincomb(b, slots, fb, t + 1 + na, (int)nb);
        uint32_t x[14], y[14];
        fp_unpack29_wide(x, a.l);
        fp_unpack29_wide(y, b.l);
        out = fp_mul_digits(x, y);
      } else {  // linear item (partial sum / output): canonical residue
        out = wave_reduce(a);
      }
      slots[fb[(d >> 20) & 0xfu] + ((d >> 8) & 0xfffu)] = out;
    }
    __syncthreads();
  }
}

}  // namespace bls
