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

// |c| * x for 1 <= |c| <= 31 (double-and-add), reduced
__device__ __forceinline__ Fp fp_mul_u5(const Fp& x, uint32_t c) {
  if (c == 1) return x;
  Fp r = fp_zero();
  Fp y = x;
  bool first = true;
  while (c) {
    if (c & 1u) {
      r = first ? y : fp_add(r, y);
      first = false;
    }
    c >>= 1;
    if (c) y = fp_dbl(y);
  }
  return r;
}

// sum_k coef_k * slot[frame_k base + index_k]
__device__ __forceinline__ Fp wave_lincomb(const Fp* slots, const int* fb, const uint32_t* t, int n) {
  Fp acc = fp_zero();
  for (int k = 0; k < n; k++) {
    const uint32_t w = t[k];
    if (!w) break;
    const int fr = (int)(w >> 20);
    const int ix = (int)((w >> 8) & 0xfffu);
    const int c = (int)(w & 0xffu) - 128;
    Fp x = slots[fb[fr] + ix];
    const uint32_t m = (uint32_t)(c < 0 ? -c : c);
    if (m != 1) x = fp_mul_u5(x, m);
    acc = c < 0 ? fp_sub(acc, x) : fp_add(acc, x);
  }
  return acc;
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
      Fp a = wave_lincomb(slots, fb, t + 1, (int)na);
      if (d >> 31) {  // product item; otherwise a linear (partial-sum / output) item
        Fp b = wave_lincomb(slots, fb, t + 1 + na, (int)nb);
        a = fp_mul(a, b);
      }
      slots[fb[(d >> 20) & 0xfu] + ((d >> 8) & 0xfffu)] = a;
    }
    __syncthreads();
  }
}

}  // namespace bls
