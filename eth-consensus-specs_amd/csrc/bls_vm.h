// Wave-program interpreter (tables from tools/wavec.py, bls_waveprog.h).
//
// One 64-lane workgroup runs a program for G items at once.  Every Fp value
// lives in an LDS slot (48 B).  LDS layout of a workgroup:
//   slots[0 .. WP_NCONST)              constant pool, loaded once
//   slots[item0 + g*stride + ix]        slot ix of item g's region (the
//                                       region layouts WL_* come from wavec)
// A program level is a set of independent ops; work index k of a level maps
// to (op j = k / G, item g = k % G), so the G lanes of one op read the same
// table words and take the same branch.  Levels are separated by a barrier.
//
// Linear combinations are accumulated lazily in a 13-limb (416-bit) running
// sum that starts at OFF = 256 p: every term costs one add/sub carry chain
// and no modular reduction (wavec bounds the coefficient mass per form so the
// sum stays in [0, 2^390)); fp_mul_digits accepts such operands directly and
// only values stored by lin/sel ops are reduced (vm_reduce).
#pragma once
#include "bls_tower.h"
#include "bls_waveprog.h"

namespace bls {

constexpr int VM_MAXT = 12;  // wavec MAX_TERMS
constexpr int VM_NT = 64;    // lanes per workgroup

struct VmProg {
  const uint32_t* terms;
  const uint32_t (*levels)[4];  // {nitems, na, nb, base}
  int nlevels;
};

#define VM_PROG(NAME) \
  ::bls::VmProg { WP_##NAME##_TERMS, WP_##NAME##_LEVELS, WP_##NAME##_NLEVELS }

// Table words carry absolute slot indices (programs are bound to a layout by
// wavec): [31:24] coef + 128 | [23] const pool | [22:0] slot within the item
// region (or pool index).  ibase = item0 + g * stride.
__device__ __forceinline__ int vm_slot(uint32_t w, int ibase) {
  const int ix = (int)(w & 0x7fffffu);
  return (w & 0x800000u) ? ix : ibase + ix;
}

struct Acc {
  uint32_t l[13];
};

__device__ __forceinline__ void acc_init(Acc& a) {  // 256 p
#pragma unroll
  for (int i = 0; i < 13; i++) {
    const uint32_t lo = i < 12 ? P_LIMBS[i] : 0u;
    const uint32_t prev = i > 0 ? P_LIMBS[i - 1] : 0u;
    a.l[i] = (lo << 8) | (i > 0 ? (prev >> 24) : 0u);
  }
}

// acc += c * x for a small signed c (|c| < 128), one carry chain
__device__ __forceinline__ void acc_term(Acc& acc, const Fp& x, int c) {
  const uint32_t m = (uint32_t)(c < 0 ? -c : c);
  uint32_t y[13];
  if (m == 1u) {
#pragma unroll
    for (int i = 0; i < 12; i++) y[i] = x.l[i];
    y[12] = 0;
  } else {
    uint32_t carry = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
      const uint64_t t = (uint64_t)x.l[i] * m + carry;
      y[i] = (uint32_t)t;
      carry = (uint32_t)(t >> 32);
    }
    y[12] = carry;
  }
  // subtract as add of the complement with carry-in 1
  const uint32_t neg = c < 0 ? 0xffffffffu : 0u;
  unsigned cy = neg & 1u;
#pragma unroll
  for (int i = 0; i < 13; i++) acc.l[i] = __builtin_addc(acc.l[i], y[i] ^ neg, cy, &cy);
}

__device__ __forceinline__ void vm_lincomb(Acc& acc, const Fp* slots, int ibase, const uint32_t* w, int n) {
  acc_init(acc);
#pragma unroll
  for (int k = 0; k < VM_MAXT; k++) {
    if (k < n && w[k]) {
      const Fp x = slots[vm_slot(w[k], ibase)];
      acc_term(acc, x, (int)(w[k] >> 24) - 128);
    }
  }
}

// canonical residue of an accumulator (< 2^390): q = floor(top / (ptop + 1))
// estimated in double precision (never above floor(a / p)), then up to three
// conditional subtractions.
__device__ __forceinline__ Fp vm_reduce(const Acc& a) {
  const uint64_t top = ((uint64_t)a.l[12] << 34) | ((uint64_t)a.l[11] << 2) | (a.l[10] >> 30);  // a >> 350
  constexpr uint64_t PTOP = (((uint64_t)P_LIMBS[11]) << 2) | (P_LIMBS[10] >> 30);                // p >> 350
  constexpr double INV = 1.0 / (double)(PTOP + 1);
  const double qd = (double)top * INV - 1e-6;
  const uint32_t q = qd > 0.0 ? (uint32_t)qd : 0u;
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
  v = fp_reduce_once(v);
  v = fp_reduce_once(v);
  v = fp_reduce_once(v);
  return v;
}

// Load up to VM_MAXT term words (predicated; all loads issued together).
__device__ __forceinline__ void vm_load_terms(uint32_t* w, const uint32_t* src, int n) {
#pragma unroll
  for (int k = 0; k < VM_MAXT; k++) w[k] = k < n ? src[k] : 0u;
}

// Run program p for G items whose regions start at item0 + g * stride.
// pred[g]: per-item predicate (sel: bit 0) or table index (lut).  All 64
// lanes of the workgroup must call it.
template <int G>
__device__ __noinline__ void vm_run(const VmProg p, Fp* slots, int item0, int stride, const uint32_t* pred) {
  const int lane = threadIdx.x;
  for (int lv = 0; lv < p.nlevels; lv++) {
    const uint32_t nitems = p.levels[lv][0], na = p.levels[lv][1], nb = p.levels[lv][2], base = p.levels[lv][3];
    const uint32_t total = nitems * G, sw = 1 + na + nb;
    for (uint32_t k = lane; k < total; k += VM_NT) {
      const uint32_t j = k / G, g = k % G;
      const int ibase = item0 + (int)g * stride;
      const uint32_t* t = p.terms + base + j * sw;
      const uint32_t d = t[0];
      const uint32_t kind = d >> 30;
      uint32_t wa[VM_MAXT], wb[VM_MAXT];
      Fp out;
      if (kind == 1u) {  // mul
        vm_load_terms(wa, t + 1, (int)na);
        vm_load_terms(wb, t + 1 + na, (int)nb);
        Acc a, b;
        vm_lincomb(a, slots, ibase, wa, (int)na);
        vm_lincomb(b, slots, ibase, wb, (int)nb);
        uint32_t x[14], y[14];
        fp_unpack29_wide(x, a.l);
        fp_unpack29_wide(y, b.l);
        out = fp_mul_digits(x, y);
      } else if (kind == 3u) {  // lut
        const uint32_t w = t[1];
        const int stride_t = (int)(w >> 24) - 128;
        out = slots[vm_slot(w, ibase) + (int)pred[g] * stride_t];
      } else {  // lin / sel
        const bool pick_b = kind == 2u && !(pred[g] & 1u);
        const uint32_t* src = pick_b ? t + 1 + na : t + 1;
        const int n = pick_b ? (int)nb : (int)na;
        vm_load_terms(wa, src, n);
        Acc a;
        vm_lincomb(a, slots, ibase, wa, n);
        out = vm_reduce(a);
      }
      slots[vm_slot(d & 0x3fffffffu, ibase)] = out;
    }
    __syncthreads();
  }
}

// Constant pool -> slots[0 .. WP_NCONST)
__device__ __forceinline__ void vm_load_consts(Fp* slots) {
  for (int i = threadIdx.x; i < WP_NCONST; i += VM_NT) {
    Fp v;
#pragma unroll
    for (int k = 0; k < 12; k++) v.l[k] = WP_CONST_POOL[i].l[k];
    slots[i] = v;
  }
  __syncthreads();
}

}  // namespace bls
