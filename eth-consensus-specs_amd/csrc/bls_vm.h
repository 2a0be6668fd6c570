// Wave-program interpreter (tables from tools/wavec.py, bls_waveprog.h).
//
// One 64-lane workgroup runs a program for G items at once.  Every Fp value
// lives in an LDS slot as 14 radix-2^29 digits (Fd, 64 B, canonical residue
// in Montgomery form R = 2^406) -- the operand format of the product, so no
// unpacking happens on the hot path.  LDS layout of a workgroup:
//   slots[0 .. WP_NCONST)          constant pool, loaded once
//   slots[item0 + g*stride + ix]   slot ix of item g's region (the region
//                                  layouts WL_* come from wavec)
// A program level is a set of independent ops; work index k of a level maps
// to (op j = k / G, item g = k % G), so the G lanes of one op read the same
// table words.  Levels are separated by a barrier.
//
// A linear combination sum c_t x_t is accumulated per digit in signed 64-bit
// lanes: one v_mad_i64_i32 per digit and term, whatever the sign or size of
// the coefficient (no branches, no carry chains).  The accumulators start at
// 256 p (wavec bounds the negative coefficient mass by 190 and the positive
// one so the total stays in [0, 2^390)) written with large digits, so every
// digit stays non-negative and one parallel carry step turns them into
// product operands.
#pragma once
#include "bls_tower.h"
#include "bls_waveprog.h"

namespace bls {

constexpr int VM_MAXT = 12;  // wavec MAX_TERMS
constexpr int VM_NT = 64;    // lanes per workgroup

BLS_HD Fd fd_from_fp(const Fp& a) {
  Fd r;
  fp_unpack29(r.d, a);
  r.d[14] = 0;
  r.d[15] = 0;
  return r;
}
BLS_HD Fp fp_from_fd(const Fd& a) { return fp_pack29(a.d); }
BLS_HD bool fd_is_zero(const Fd& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) o |= a.d[i];
  return o == 0;
}
BLS_HD Fd fd_zero() {
  Fd r;
#pragma unroll
  for (int i = 0; i < 16; i++) r.d[i] = 0;
  return r;
}

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

// digits of 256 p
struct Off256 {
  uint32_t d[14];
};
constexpr Off256 vm_off256() {
  Off256 o{};
  uint64_t carry = 0;
  for (int i = 0; i < 14; i++) {
    const uint64_t v = ((uint64_t)P29[i] << 8) + carry;
    o.d[i] = (uint32_t)(v & 0x1fffffffu);
    carry = v >> 29;
  }
  return o;
}
constexpr Off256 VM_OFF = vm_off256();

// 256 p again, in a redundant digit form with digits 0..12 >= 2^37 (each
// 2^37 lent to digit i is taken back as 2^8 from digit i+1): accumulators
// started here stay non-negative digit by digit (a form's negative mass is
// at most 190 (2^29 - 1) < 2^37 per digit), so one carry step without a
// sequential chain normalises them (vm_normalise_fast).
struct OffR {
  int64_t d[14];
};
constexpr OffR vm_offr() {
  OffR o{};
  for (int i = 0; i < 14; i++) {
    o.d[i] = (int64_t)VM_OFF.d[i];
    if (i < 13) o.d[i] += (int64_t)1 << 37;
    if (i > 0) o.d[i] -= 256;
  }
  return o;
}
constexpr OffR VM_OFFR = vm_offr();

struct Acc {
  int64_t d[14];
};

// n is uniform across the wave (the level's operand width); padding words
// (0) read slot ibase with coefficient 0, so the loop body has no
// lane-dependent branch and loads of term k+1 can overlap the mads of term k.
__device__ __forceinline__ void vm_lincomb(Acc& acc, const Fd* slots, int ibase, const uint32_t* w, int n) {
#pragma unroll
  for (int i = 0; i < 14; i++) acc.d[i] = VM_OFFR.d[i];
#pragma unroll
  for (int k = 0; k < VM_MAXT; k++) {
    if (k < n) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const __attribute__((address_space(3))) u32x4* q =
          (const __attribute__((address_space(3))) u32x4*)(slots + vm_slot(w[k], ibase));
      u32x4 v0 = q[0], v1 = q[1], v2 = q[2], v3 = q[3];  // 4 x ds_read_b128
      asm volatile("" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));  // keep the loads whole
      const uint32_t x[14] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y, v2.z, v2.w, v3.x, v3.y};
      const int32_t c = w[k] ? (int32_t)(w[k] >> 24) - 128 : 0;
#pragma unroll
      for (int i = 0; i < 14; i++) acc.d[i] += (int64_t)(int32_t)x[i] * (int64_t)c;
    }
  }
}

// carry pass: signed digit sums (total in [0, 2^390)) -> digits < 2^29
__device__ __forceinline__ void vm_normalise(uint32_t x[14], const Acc& a) {
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const int64_t v = a.d[i] + c;
    x[i] = (uint32_t)v & 0x1fffffffu;
    c = v >> 29;
  }
}

// one parallel carry step for accumulators with every digit in [0, 2^38):
// x_i = (a_i mod 2^29) + (a_{i-1} >> 29), i.e. digits < 2^29 + 2^9, which
// fp_mul_digits_raw accepts (its 64-bit column sums stay below 2^63).
__device__ __forceinline__ void vm_normalise_fast(uint32_t x[14], const Acc& a) {
  uint32_t hi_prev = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const uint32_t lo32 = (uint32_t)a.d[i], hi32 = (uint32_t)((uint64_t)a.d[i] >> 32);
    if (i < 13) {
      x[i] = (lo32 & 0x1fffffffu) + hi_prev;
      hi_prev = __builtin_amdgcn_alignbit(hi32, lo32, 29);
    } else {
      x[i] = lo32 + hi_prev;  // the top digit has no high part (value < 2^390)
    }
  }
}

// r - p if r >= p (digits < 2^29, r < 2p)
__device__ __forceinline__ void vm_reduce_once(uint32_t r[14]) {
  uint32_t t[14];
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const int32_t v = (int32_t)r[i] - (int32_t)P29[i] - br;
    t[i] = (uint32_t)v & 0x1fffffffu;
    br = v < 0 ? 1 : 0;
  }
  const bool keep = br != 0;
#pragma unroll
  for (int i = 0; i < 14; i++) r[i] = keep ? r[i] : t[i];
}

// canonical residue of a normalised value x < 2^390: q = floor(top / (ptop + 1))
// estimated in double precision (never above floor(x / p)), x - q p by one
// more digit pass, then up to two conditional subtractions.
__device__ __forceinline__ void vm_reduce(uint32_t x[14]) {
  const uint64_t top = ((uint64_t)x[13] << 27) | (x[12] >> 2);  // x >> 350
  constexpr uint64_t PTOP = (((uint64_t)P_LIMBS[11]) << 2) | (P_LIMBS[10] >> 30);
  constexpr double INV = 1.0 / (double)(PTOP + 1);
  const double qd = (double)top * INV - 1e-6;
  const int32_t q = qd > 0.0 ? (int32_t)qd : 0;
  Acc a;
#pragma unroll
  for (int i = 0; i < 14; i++) a.d[i] = (int64_t)x[i] - (int64_t)q * (int64_t)P29[i];
  vm_normalise(x, a);
  vm_reduce_once(x);
  vm_reduce_once(x);
}

// Load up to VM_MAXT term words (predicated; all loads issued together).
__device__ __forceinline__ void vm_load_terms(uint32_t* w, const uint32_t* src, int n) {
#pragma unroll
  for (int k = 0; k < VM_MAXT; k++) w[k] = k < n ? src[k] : 0u;
}

// max over the 64 lanes (all active): DPP within rows of 16, then the four
// row results by readlane -> a wave-uniform (scalar) value.
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
  uint32_t o;
  o = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  v = o > v ? o : v;
  o = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  v = o > v ? o : v;
  o = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  v = o > v ? o : v;
  o = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);  // row_mirror
  v = o > v ? o : v;
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
  const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
  const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
  const uint32_t r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
  const uint32_t a = r0 > r1 ? r0 : r1, b = r2 > r3 ? r2 : r3;
  return a > b ? a : b;
}

// Run program p for G items whose regions start at item0 + g * stride.
// pred[g]: per-item predicate (sel: bit 0) or table index (lut).  All 64
// lanes of the workgroup must call it.  Each pass of a level pads operand
// lists only to the widest op of that pass (wave max of the per-op widths
// stored in the destination words), so the term loops are uniform.
template <int G>
__device__ __noinline__ void vm_run(const VmProg p, Fd* slots, int item0, int stride, const uint32_t* pred) {
  const int lane = threadIdx.x;
  for (int lv = 0; lv < p.nlevels; lv++) {
    const uint32_t nitems = p.levels[lv][0], na = p.levels[lv][1], nb = p.levels[lv][2], base = p.levels[lv][3];
    const uint32_t total = nitems * G, sw = 1 + na + nb;
    const uint32_t npass = (total + VM_NT - 1) / VM_NT;
    for (uint32_t ps = 0; ps < npass; ps++) {
      const uint32_t k = (uint32_t)lane + ps * VM_NT;
      const bool active = k < total;
      const uint32_t j = k / G, g = k % G;
      const int ibase = item0 + (int)g * stride;
      const uint32_t* t = p.terms + base + j * sw;
      const uint32_t d = active ? t[0] : 0u;
      const uint32_t kind = d >> 30;
      const uint32_t na_i = (d >> 26) & 15u, nb_i = (d >> 22) & 15u;
      const bool pick_b = kind == 2u && !(pred[active ? g : 0] & 1u);
      // uniform operand widths of this pass, per code path: the wave max of
      // the ops' own widths when several items share the pass (throughput),
      // the level width for one item (latency: no cross-lane reduction)
      uint32_t wa_mul = na, wb_mul = nb, w_lin = na > nb ? na : nb;
      if (G > 1) {
        wa_mul = wave_max(kind == 1u ? na_i : 0u);
        wb_mul = wave_max(kind == 1u ? nb_i : 0u);
        w_lin = wave_max((kind == 0u || kind == 2u) && active ? (pick_b ? nb_i : na_i) : 0u);
      }
      if (!active) continue;
      uint32_t wa[VM_MAXT];
      Fd out;
      if (kind == 1u) {  // mul: rows are zero-padded to the level widths, so
        uint32_t x[14], y[14];  // the loads need no per-op count
        {
          vm_load_terms(wa, t + 1, (int)na);
          Acc a;
          vm_lincomb(a, slots, ibase, wa, (int)wa_mul);
          vm_normalise_fast(x, a);
        }
        {
          vm_load_terms(wa, t + 1 + na, (int)nb);
          Acc b;
          vm_lincomb(b, slots, ibase, wa, (int)wb_mul);
          vm_normalise_fast(y, b);
        }
        fp_mul_digits_raw(out.d, x, y);
        vm_reduce_once(out.d);
      } else if (kind == 3u) {  // lut
        const uint32_t w = t[1];
        const int stride_t = (int)(w >> 24) - 128;
        out = slots[vm_slot(w, ibase) + (int)pred[g] * stride_t];
      } else {  // lin / sel
        const uint32_t* src = pick_b ? t + 1 + na : t + 1;
        vm_load_terms(wa, src, (int)(pick_b ? nb_i : na_i));  // zero-filled past this op's list
        Acc a;
        vm_lincomb(a, slots, ibase, wa, (int)w_lin);
        vm_normalise(out.d, a);
        vm_reduce(out.d);
      }
      {  // the 64 meaningful bytes, as four ds_write_b128 (the slot's last 16 B are padding)
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        __attribute__((address_space(3))) u32x4* q =
            (__attribute__((address_space(3))) u32x4*)(slots + vm_slot(d & 0x3fffffu, ibase));
        q[0] = u32x4{out.d[0], out.d[1], out.d[2], out.d[3]};
        q[1] = u32x4{out.d[4], out.d[5], out.d[6], out.d[7]};
        q[2] = u32x4{out.d[8], out.d[9], out.d[10], out.d[11]};
        q[3] = u32x4{out.d[12], out.d[13], 0u, 0u};
      }
    }
    __syncthreads();
  }
}

// Constant pool -> slots[0 .. WP_NCONST)
__device__ __forceinline__ void vm_load_consts(Fd* slots) {
  for (int i = threadIdx.x; i < WP_NCONST; i += VM_NT) {
    Fd v;
#pragma unroll
    for (int k = 0; k < 16; k++) v.d[k] = WP_CONST_POOL[i].d[k];
    slots[i] = v;
  }
  __syncthreads();
}

}  // namespace bls
