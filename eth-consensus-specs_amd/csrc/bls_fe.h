// Lane-parallel final exponentiation: the per-lane phase executor and the
// schedule (SURVEY.md §8(a) internal piece (7): f^((p^12 - 1) / r), easy part
// (p^6 - 1)(p^2 + 1), hard part through (x - 1)^2 (x + p)(x^2 + p^2 - 1) + 3,
// i.e. the check computes FE(f)^3, which is 1 iff FE(f) is: gcd(3, r) = 1).
//
// One 64-lane wave keeps every Fp of the computation in an LDS slot as 14
// radix-2^29 digits (bls_fq.h, N form: digits 0..12 exact, value below a small
// multiple of p -- never reduced until the final comparison) and advances them
// in phases separated by barriers.  In a phase each active lane does ONE of
//   PROD  dst = (x_1 + .. + x_nx)(y_1 + .. + y_ny) / R   (fq_mul on the
//         carry-save normalised sums: up to 54 independent products per phase,
//         e.g. the whole Fp12 product = 3 Fp6 x 6 Fp2 x 3 Fp Karatsuba levels)
//   LIN   dst = sum c_t x_t + K p   (64-bit digit accumulators, one exact carry
//         chain; K p covers the negative mass so the chain ends non-negative)
//   LIN32 dst = sum +-x_t + 16 p   (u32 digit sums; the cyclotomic squaring,
//         whose products already carry their coefficients)
//   INV   dst = src^-1 (lane 0: one safegcd inversion, bls_fp_inv.h)
// The phase tables (who does what, which slots) come from tools/gen_fe.py,
// which checks every bound of the whole schedule on integers and is checked
// against the oracle by tests/test_fe_tables.py.  The cyclotomic squaring is
// ONE product phase (18 Fp2-square products + 12 doublings 2 z as products by
// 2) and one LIN phase, so a chain step costs one Montgomery product of latency
// instead of the wave program's ~4 us per level (bls_wave_kernels.hip
// k_final_check_vm: 3.0 ms per check, one workgroup).
//
// The code here is __host__ __device__: tests/hostcheck runs the same schedule
// with the 64 lanes in a loop (FeHost) and the digit-form bound checks of
// bls_fq.h compiled in.
#pragma once
#include "bls_fq.h"
#include "bls_fp_inv.h"
#include "bls_fe_tables.h"

namespace bls {

// 14 digits + 6 pad words: 80 B, so slot s starts in 16-B bank group (5 s) mod 16 and the 16-B accesses of lanes
// reading different slots spread over the banks (at 64 B every fourth slot shared a group: 54.9 % of the kernel's
// LDS cycles were bank conflicts, profiles/r03s_pmc_lds.md -- the layout that fixed the VM slots)
struct alignas(16) FeSlot {
  uint32_t d[20];
};

// slot of a table reference: frame 0 absolute (products, temporaries, constants), 1/2/3 the banks A/B/D
BLS_HD int fe_addr(uint32_t r, int a, int b, int d) {
  const int fr = (int)(r >> 8) & 3, ix = (int)(r & 255u);
  const int bank = fr == 1 ? a : (fr == 2 ? b : d);
  return fr == 0 ? FE_ABS_BASE + ix : 12 * bank + ix;
}
BLS_HD uint32_t fe_term(const uint32_t* w, int t) { return (w[1 + (t >> 1)] >> (16 * (t & 1))) & 0xffffu; }

BLS_HD Fq fe_ld(const FeSlot* s, int slot) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = s[slot].d[i];
  return r;
}
BLS_HD void fe_st(FeSlot* s, int slot, const Fq& v) {
#pragma unroll
  for (int i = 0; i < 14; i++) s[slot].d[i] = v.d[i];
}

template <int NX, int NY>
BLS_HD void fe_prod(FeSlot* s, const uint32_t* w, int a, int b, int d) {
  // at most four loads in flight: fully unrolled, the scheduler hoisted all 16 of the Fp12 product's loads
  // (224 registers) and spilled
  Fq x = fq_zero(), y = fq_zero();
#pragma unroll 4
  for (int t = 0; t < NX; t++) x = fq_add(x, fe_ld(s, fe_addr(fe_term(w, t), a, b, d)));
#pragma unroll 4
  for (int t = 0; t < NY; t++) y = fq_add(y, fe_ld(s, fe_addr(fe_term(w, NX + t), a, b, d)));
  fe_st(s, fe_addr(w[0] & 1023u, a, b, d), fq_mul(fq_norm(x), fq_norm(y)));
}

template <int NT>
BLS_HD void fe_lin(FeSlot* s, const uint32_t* w, int a, int b, int d) {
  const int64_t K = (int64_t)((w[0] >> 10) & 1023u);
  int64_t acc[14];
#pragma unroll
  for (int i = 0; i < 14; i++) acc[i] = K * (int64_t)P29[i];
#pragma unroll 4
  for (int t = 0; t < NT; t++) {
    const uint32_t tw = fe_term(w, t);
    const int64_t c = (int64_t)(tw >> 10) - 32;
    const Fq x = fe_ld(s, fe_addr(tw, a, b, d));
#pragma unroll
    for (int i = 0; i < 14; i++) acc[i] += c * (int64_t)x.d[i];
  }
  Fq r;
  int64_t cy = 0;
#pragma unroll
  for (int i = 0; i < 13; i++) {
    const int64_t v = acc[i] + cy;
    r.d[i] = (uint32_t)v & Q29_MASK;
    cy = v >> 29;  // arithmetic: digit sums may be negative, the total is not
  }
  const int64_t top = acc[13] + cy;
#ifdef BLS_FQ_CHECK
  assert(top >= 0 && top < ((int64_t)1 << 31));
#endif
  r.d[13] = (uint32_t)top;
  fe_st(s, fe_addr(w[0] & 1023u, a, b, d), r);
}

// sum of +-1 x_t in u32 digits (LIN32): the offset 16 p with every digit below the top raised by b 2^29 (b =
// the number of subtracted terms, bits 10..19) keeps every digit non-negative and below 2^32 (gen_fe.py checks
// npos + b + 1 <= 8), then the exact carry chain
template <int NT>
BLS_HD void fe_lin32(FeSlot* s, const uint32_t* w, int a, int b, int d) {
  const uint32_t bw = (w[0] >> 10) & 1023u;
  uint32_t acc[14];
  acc[0] = FE_K32[0] + (bw << 29);
#pragma unroll
  for (int i = 1; i < 13; i++) acc[i] = FE_K32[i] + (bw << 29) - bw;
  acc[13] = FE_K32[13] - bw;
#ifdef BLS_FQ_CHECK
  int64_t chk[14];
  for (int i = 0; i < 14; i++) chk[i] = acc[i];
#endif
#pragma unroll 4
  for (int t = 0; t < NT; t++) {
    const uint32_t tw = fe_term(w, t);
    const uint32_t neg = (tw >> 10) < 32u ? 0xffffffffu : 0u;  // coefficient -1 (31) or +1 (33); padding: 0 (32)
    const uint32_t zero = (tw >> 10) == 32u ? 0u : 0xffffffffu;
    const Fq x = fe_ld(s, fe_addr(tw, a, b, d));
#pragma unroll
    for (int i = 0; i < 14; i++) acc[i] += ((x.d[i] & zero) ^ neg) - neg;
#ifdef BLS_FQ_CHECK
    for (int i = 0; i < 14; i++) chk[i] += neg ? -(int64_t)(x.d[i] & zero) : (int64_t)(x.d[i] & zero);
#endif
  }
#ifdef BLS_FQ_CHECK
  for (int i = 0; i < 14; i++) assert(chk[i] >= 0 && chk[i] < ((int64_t)1 << 32) && (uint32_t)chk[i] == acc[i]);
#endif
  Fq r;
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 13; i++) {
    const uint32_t v = acc[i] + cy;
    r.d[i] = v & Q29_MASK;
    cy = v >> 29;
  }
  r.d[13] = acc[13] + cy;
  fe_st(s, fe_addr(w[0] & 1023u, a, b, d), r);
}

BLS_HD void fe_inv(FeSlot* s, const uint32_t* w, int a, int b, int d) {
  const Fp v = fq_pack(fe_ld(s, fe_addr(fe_term(w, 0), a, b, d)));  // canonical
  fe_st(s, fe_addr(w[0] & 1023u, a, b, d), fq_unpack(fp_inv_sg_i(v)));
}

// one lane's part of a phase (its descriptor words w); KIND (bits 29..31): 1 PROD, 2 LIN, 3 INV, 4 LIN32 (idle
// lanes: kind 0)
template <int KIND, int NX, int NY>
BLS_HD void fe_lane(FeSlot* s, const uint32_t* w, int a, int b, int d) {
  if ((w[0] >> 29) != (uint32_t)KIND) return;
  if constexpr (KIND == 1)
    fe_prod<NX, NY>(s, w, a, b, d);
  else if constexpr (KIND == 2)
    fe_lin<NX>(s, w, a, b, d);
  else if constexpr (KIND == 4)
    fe_lin32<NX>(s, w, a, b, d);
  else
    fe_inv(s, w, a, b, d);
}

// descriptor words of a phase actually used by a lane (1 + ceil(terms / 2))
template <int NX, int NY>
struct FeDesc {
  static constexpr int W = 1 + (NX + NY + 1) / 2;
  uint32_t w[W];
};
template <int NX, int NY>
BLS_HD FeDesc<NX, NY> fe_desc(int phase, int lane) {
  FeDesc<NX, NY> r;
#pragma unroll
  for (int k = 0; k < FeDesc<NX, NY>::W; k++) r.w[k] = FE_DESC[((size_t)phase * 64 + lane) * FE_NW + k];
  return r;
}

#define FE_PH(NAME, I, a, b, d) \
  this->self().template ph<FE_KIND_##NAME##_##I, FE_NT_##NAME##_##I, FE_NY_##NAME##_##I>(FE_PH_##NAME##_##I, a, b, d)

// The operations as phase lists; Ex provides ph<KIND, NX, NY>(phase, a, b, d) (one phase on every lane, then a
// barrier) and may replace any operation (the device executor serves mul / cyc from registers).
template <class Ex>
struct FeOps {
  BLS_HD Ex& self() { return *static_cast<Ex*>(this); }
  BLS_HD void mul(int a, int b, int d) {
    FE_PH(MUL, 0, a, b, d);
    FE_PH(MUL, 1, a, b, d);
    FE_PH(MUL, 2, a, b, d);
  }
  BLS_HD void cyc(int a, int d) {
    FE_PH(CYC, 0, a, 0, d);
    FE_PH(CYC, 1, a, 0, d);
  }
  BLS_HD void conj(int a, int d) { FE_PH(CONJ, 0, a, 0, d); }
  BLS_HD void frob1(int a, int d) {
    FE_PH(FROB1, 0, a, 0, d);
    FE_PH(FROB1, 1, a, 0, d);
  }
  BLS_HD void frob2(int a, int d) { FE_PH(FROB2, 0, a, 0, d); }
  BLS_HD void easy(int a, int d) {
    FE_PH(EASY_FRONT, 0, a, 0, d);
    FE_PH(EASY_FRONT, 1, a, 0, d);
    FE_PH(EASY_FRONT, 2, a, 0, d);
    FE_PH(EASY_INV, 0, 0, 0, 0);
    FE_PH(EASY_INV, 1, 0, 0, 0);
    FE_PH(EASY_INV, 2, 0, 0, 0);
    FE_PH(EASY_INV, 3, 0, 0, 0);
    FE_PH(EASY_INV, 4, 0, 0, 0);
    FE_PH(EASY_INV, 5, 0, 0, 0);
    FE_PH(EASY_INV, 6, 0, 0, 0);
    FE_PH(EASY_INV, 7, 0, 0, 0);
    FE_PH(EASY_INV, 8, 0, 0, 0);
    FE_PH(EASY_INV, 9, 0, 0, 0);
    FE_PH(EASY_INV, 10, 0, 0, 0);
  }
  BLS_HD void easy_back(int a, int d) {
    FE_PH(EASY_BACK, 0, a, 0, d);
    FE_PH(EASY_BACK, 1, a, 0, d);
  }
};

// The schedule of one check: bank 0 holds f on entry (the product of the partials), bank 1 holds f^(3 h (p^6
// - 1)(p^2 + 1)) on exit.
template <class Ex>
BLS_HD void fe_powx(Ex& ex, int src, int dst) {  // dst = src^x = conj(src^|x|) (x < 0, cyclotomic src)
  int acc = src;
  for (int i = 62; i >= 0; --i) {  // the bits of |x| after the leading one
    ex.cyc(acc, dst);
    acc = dst;
    if ((X_ABS >> i) & 1ull) ex.mul(dst, src, dst);
  }
  ex.conj(dst, dst);
}

template <class Ex>
BLS_HD void fe_schedule(Ex& ex) {
  // easy part: t = conj(f) / f = conj(f)^2 / (f conj(f)), then t^(p^2) t
  ex.easy(0, 2);           // bank 2 = conj(f)^2; N = f conj(f) in Fp6 -> N^-1 (temporaries)
  ex.easy_back(2, 0);      // bank 0 = conj(f)^2 N^-1
  ex.frob2(0, 1);
  ex.mul(1, 0, 0);         // bank 0 = t
  // hard part (the order of bls_wave_kernels.hip k_final_check_vm)
  fe_powx(ex, 0, 1);       // 1 = t^x
  ex.conj(0, 3);
  ex.mul(3, 1, 2);         // 2 = a = t^(x-1)
  fe_powx(ex, 2, 1);       // 1 = a^x
  ex.conj(2, 3);
  ex.mul(1, 3, 2);         // 2 = a = t^((x-1)^2)
  fe_powx(ex, 2, 1);       // 1 = a^x
  ex.frob1(2, 3);          // 3 = a^p
  ex.mul(3, 1, 3);         // 3 = b = a^(x+p)
  fe_powx(ex, 3, 1);       // 1 = b^x
  fe_powx(ex, 1, 4);       // 4 = b^(x^2)
  ex.frob2(3, 5);          // 5 = b^(p^2)
  ex.mul(4, 5, 1);
  ex.conj(3, 4);           // 4 = b^-1
  ex.mul(1, 4, 1);         // 1 = c = b^(x^2+p^2-1)
  ex.cyc(0, 5);
  ex.mul(5, 0, 5);         // 5 = t^3
  ex.mul(1, 5, 1);         // 1 = c t^3
}

// Host executor (tests/hostcheck): the 64 lanes of every phase in a loop, straight from the tables.
struct FeHost : FeOps<FeHost> {
  FeSlot* s;
  template <int KIND, int NX, int NY>
  void ph(int phase, int a, int b, int d) {
    for (int lane = 0; lane < 64; lane++) {
      const FeDesc<NX, NY> w = fe_desc<NX, NY>(phase, lane);
      fe_lane<KIND, NX, NY>(s, w.w, a, b, d);
    }
  }
};

// constants into their slots; returns nothing (host and device: lane-strided)
BLS_HD void fe_load_consts(FeSlot* s, int lane, int nlanes) {
  for (int i = lane; i < FE_NCONST; i += nlanes) {
#pragma unroll
    for (int k = 0; k < 14; k++) s[FE_ABS_BASE + FE_CS + i].d[k] = FE_CONSTS[i][k];
  }
}

}  // namespace bls
