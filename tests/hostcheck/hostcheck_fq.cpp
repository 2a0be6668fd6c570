// TEST HARNESS ONLY: host build of the redundant digit-form arithmetic (bls_fq.h, bls_fq_g1.h, bls_fq_g2.h) with
// its 128-bit column, value and subtraction-precondition checks compiled in (BLS_FQ_CHECK).  A separate
// translation unit from hostcheck.cpp so the two compile in parallel.
#define BLS_FQ_CHECK 1
#define BLS_HD __host__ __device__ inline  // no forced inlining in this (host-only, checked) unit
#include "bls_ops.h"
#include "bls_fq_g1.h"
#include "bls_fq_g2.h"
#include "bls_fqb.h"
#include <string.h>
using namespace bls;

static Fp in_fp(const uint8_t* b) { return fp_to_mont(raw_from_be48(b)); }
static void out_fp(uint8_t* b, const Fp& a) { raw_to_be48(fp_from_mont(a), b); }
static Fp2 in_fp2(const uint8_t* b) { return Fp2{in_fp(b), in_fp(b + 48)}; }
static void out_fp2(uint8_t* b, const Fp2& a) { out_fp(b, a.c0); out_fp(b + 48, a.c1); }

// registry-gather formulas in the digit form (bls_fq_g1.h): pts = n affine points (x || y, 96 B each), the first
// `split` summed into one accumulator and the rest into another by g1q_add_aff, then g1q_add; out = affine sum
// (x || y) or 96 zero bytes for the identity
extern "C" void hc_fq_gather(const uint8_t* pts, uint32_t n, uint32_t split, uint8_t* o) {
  const G1Q id{fq_zero(), fq_unpack(FP_ONE), fq_zero()};
  G1Q a = id, b = id;
  for (uint32_t k = 0; k < n; ++k) {
    const Fq x = fq_unpack(in_fp(pts + 96 * k)), y = fq_unpack(in_fp(pts + 96 * k + 48));
    if (k < split)
      a = g1q_add_aff(a, x, y);
    else
      b = g1q_add_aff(b, x, y);
  }
  const G1Q s = g1q_add(a, b);
  const Fp X = fq_pack(s.x), Y = fq_pack(s.y), Z = fq_pack(s.z);
  if (fp_is_zero(Z)) {
    memset(o, 0, 96);
    return;
  }
  const Fp zi = fp_inv(Z);
  out_fp(o, fp_mul(X, zi));
  out_fp(o + 48, fp_mul(Y, zi));
}
// one-reduction dot product of raw digit vectors: r = (x y + u v) / 2^406, digits (fq_mul_dot2)
extern "C" void hc_fq_dot2_digits(const uint32_t* x, const uint32_t* y, const uint32_t* u, const uint32_t* v,
                                  uint32_t* r) {
  Fq a, b, c, d;
  memcpy(a.d, x, 56);
  memcpy(b.d, y, 56);
  memcpy(c.d, u, 56);
  memcpy(d.d, v, 56);
  const Fq o = fq_mul_dot2(a, b, c, d);
  memcpy(r, o.d, 56);
}
// Fp2 products: the untyped chain form (fq2_mul) and the bound-typed one (Fq2B operator*, operands at the
// Miller accumulation's bounds), both on canonical inputs a, b (96 B each); out = fq2_mul || Fq2B product
extern "C" void hc_fq2_mul_forms(const uint8_t* a, const uint8_t* b, uint8_t* o) {
  const Fq2 x = fq2_unpack(in_fp2(a)), y = fq2_unpack(in_fp2(b));
  out_fp2(o, fq2_pack(fq2_mul(x, y)));
  const Fq2B<256, 0x20000000ull + 64> xb{{x.c0}, {x.c1}};
  const Fq2B<4096, 0x20000000ull + 64> yb{{y.c0}, {y.c1}};
  out_fp2(o + 96, fq2b_pack(xb * yb));
}
// one digit-form product of raw digit vectors (14 x u32 each): r = x y / 2^406, digits
extern "C" void hc_fq_mul_digits(const uint32_t* x, const uint32_t* y, uint32_t* r) {
  Fq a, b;
  memcpy(a.d, x, 56);
  memcpy(b.d, y, 56);
  const Fq c = fq_mul(a, b);
  memcpy(r, c.d, 56);
}

// r * P by the digit-form double-and-add of k_sig_lane2 (bls_fq_g1.h g1q_dbl / g1q_add), 64-bit r; out affine
extern "C" void hc_fq_g1_mul64(const uint8_t* p, uint64_t r, uint8_t* o) {
  const G1Q A{fq_unpack(in_fp(p)), fq_unpack(in_fp(p + 48)), fq_unpack(FP_ONE)};
  G1Q R{fq_zero(), fq_unpack(FP_ONE), fq_zero()};
  if ((r >> 63) & 1ull) R = A;
  for (int b = 62; b >= 0; --b) {
    R = g1q_dbl(R);
    if ((r >> b) & 1ull) R = g1q_add(R, A);
  }
  const Fp X = fq_pack(R.x), Y = fq_pack(R.y), Z = fq_pack(R.z);
  if (fp_is_zero(Z)) {
    memset(o, 0, 96);
    return;
  }
  const Fp zi = fp_inv(Z);
  out_fp(o, fp_mul(X, zi));
  out_fp(o + 48, fp_mul(Y, zi));
}

// [|x|] q through the digit-form Jacobian chain of the hash_to_G2 kernels (bls_fq_g2.h), q affine in, affine out;
// returns the exception flag
extern "C" int hc_fq_j2_mul_xabs(const uint8_t* q, uint8_t* o) {
  const Fq2 z = fq2_unpack(fp2_one());
  const J2Q J{fq2_mul(fq2_unpack(in_fp2(q)), z), fq2_mul(fq2_unpack(in_fp2(q + 96)), fq2_sqr(z)), z};
  bool exc = false;
  const J2Q M = j2q_mul_xabs(J, exc);
  const Fp2 X = fq2_pack(fq2_mul(M.x, M.z)), Y = fq2_pack(M.y), Z = fq2_pack(fq2_mul(fq2_sqr(M.z), M.z));
  const Fp2 zi = fp2_inv(Z);
  out_fp2(o, fp2_mul(X, zi));
  out_fp2(o + 96, fp2_mul(Y, zi));
  return exc ? 1 : 0;
}

// 2p + q through the digit-form Jacobian doubling and addition (bls_fq_g2.h), p, q affine; returns the exception
// flag (q = -2p: h = 0)
extern "C" int hc_fq_j2_dbl_add(const uint8_t* p, const uint8_t* q, uint8_t* o) {
  const Fq2 one = fq2_unpack(fp2_one());
  const J2Q P{fq2_unpack(in_fp2(p)), fq2_unpack(in_fp2(p + 96)), one};
  const J2Q Q{fq2_unpack(in_fp2(q)), fq2_unpack(in_fp2(q + 96)), one};
  bool exc = false;
  const J2Q R = j2q_add(j2q_dbl(P), Q, exc);
  const Fp2 X = fq2_pack(R.x), Y = fq2_pack(R.y), Z = fq2_pack(R.z);
  if (!exc) {
    const Fp2 zi = fp2_inv(Z), zi2 = fp2_mul(zi, zi);
    out_fp2(o, fp2_mul(X, zi2));
    out_fp2(o + 96, fp2_mul(Y, fp2_mul(zi2, zi)));
  }
  return exc ? 1 : 0;
}
