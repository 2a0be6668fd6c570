// Short-Weierstrass points on E1: y^2 = x^3 + 4 (over Fp) and the M-type
// twist E2: y^2 = x^3 + 4(1+i) (over Fp2).  Jacobian coordinates
// (x = X/Z^2, y = Y/Z^3, Z = 0 is the identity), templated on the field so
// G1 and G2 share one implementation.  ZCash compressed encodings with the
// decode rules of py_ecc/milagro (SURVEY.md §8(a) "Edge-semantics rows").
#pragma once
#include "bls_tower.h"

namespace bls {

// ---- field-generic overloads -------------------------------------------
BLS_HD Fp fadd(const Fp& a, const Fp& b) { return fp_add(a, b); }
BLS_HD Fp2 fadd(const Fp2& a, const Fp2& b) { return fp2_add(a, b); }
BLS_HD Fp fsub(const Fp& a, const Fp& b) { return fp_sub(a, b); }
BLS_HD Fp2 fsub(const Fp2& a, const Fp2& b) { return fp2_sub(a, b); }
BLS_HD Fp fmul(const Fp& a, const Fp& b) { return fp_mul(a, b); }
BLS_HD Fp2 fmul(const Fp2& a, const Fp2& b) { return fp2_mul(a, b); }
BLS_HD Fp fsqr(const Fp& a) { return fp_sqr(a); }
BLS_HD Fp2 fsqr(const Fp2& a) { return fp2_sqr(a); }
BLS_HD Fp fdbl(const Fp& a) { return fp_dbl(a); }
BLS_HD Fp2 fdbl(const Fp2& a) { return fp2_dbl(a); }
BLS_HD Fp fneg(const Fp& a) { return fp_neg(a); }
BLS_HD Fp2 fneg(const Fp2& a) { return fp2_neg(a); }
BLS_HD bool fis_zero(const Fp& a) { return fp_is_zero(a); }
BLS_HD bool fis_zero(const Fp2& a) { return fp2_is_zero(a); }
BLS_HD bool feq(const Fp& a, const Fp& b) { return fp_eq(a, b); }
BLS_HD bool feq(const Fp2& a, const Fp2& b) { return fp2_eq(a, b); }
BLS_HD Fp finv(const Fp& a) { return fp_inv(a); }
BLS_HD Fp2 finv(const Fp2& a) { return fp2_inv(a); }
BLS_HD void fset_zero(Fp& a) { a = fp_zero(); }
BLS_HD void fset_zero(Fp2& a) { a = fp2_zero(); }
BLS_HD void fset_one(Fp& a) { a = FP_ONE; }
BLS_HD void fset_one(Fp2& a) { a = fp2_one(); }

template <class F>
struct Jac {
  F x, y, z;
};
template <class F>
struct Aff {
  F x, y;
  bool inf;
};
// homogeneous projective G1 point (x = X/Z, y = Y/Z; identity (0 : 1 : 0))
struct G1P {
  Fp x, y, z;
};
typedef Jac<Fp> G1J;
typedef Jac<Fp2> G2J;
typedef Aff<Fp> G1A;
typedef Aff<Fp2> G2A;

template <class F>
BLS_HD Jac<F> jac_identity() {
  Jac<F> r;
  fset_one(r.x);
  fset_one(r.y);
  fset_zero(r.z);
  return r;
}

template <class F>
BLS_HD bool jac_is_inf(const Jac<F>& p) {
  return fis_zero(p.z);
}

template <class F>
BLS_HD Jac<F> jac_from_aff(const Aff<F>& a) {
  if (a.inf) return jac_identity<F>();
  Jac<F> r;
  r.x = a.x;
  r.y = a.y;
  fset_one(r.z);
  return r;
}

template <class F>
BLS_HD Jac<F> jac_neg(const Jac<F>& p) {
  return Jac<F>{p.x, fneg(p.y), p.z};
}

// dbl-2009-l (a = 0)
template <class F>
BLS_HDNI Jac<F> jac_dbl(const Jac<F>& p) {
  F A = fsqr(p.x);
  F B = fsqr(p.y);
  F C = fsqr(B);
  F D = fdbl(fsub(fsub(fsqr(fadd(p.x, B)), A), C));
  F E = fadd(fdbl(A), A);
  F Fv = fsqr(E);
  Jac<F> r;
  r.x = fsub(Fv, fdbl(D));
  F C8 = fdbl(fdbl(fdbl(C)));
  r.y = fsub(fmul(E, fsub(D, r.x)), C8);
  r.z = fdbl(fmul(p.y, p.z));
  return r;
}

// add-2007-bl with the exceptional cases handled
template <class F>
BLS_HDNI Jac<F> jac_add(const Jac<F>& p, const Jac<F>& q) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  F z1z1 = fsqr(p.z);
  F z2z2 = fsqr(q.z);
  F u1 = fmul(p.x, z2z2);
  F u2 = fmul(q.x, z1z1);
  F s1 = fmul(fmul(p.y, q.z), z2z2);
  F s2 = fmul(fmul(q.y, p.z), z1z1);
  F h = fsub(u2, u1);
  F rr = fdbl(fsub(s2, s1));
  if (fis_zero(h)) {
    if (fis_zero(rr)) return jac_dbl(p);
    return jac_identity<F>();
  }
  F i = fsqr(fdbl(h));
  F j = fmul(h, i);
  F v = fmul(u1, i);
  Jac<F> r;
  r.x = fsub(fsub(fsqr(rr), j), fdbl(v));
  r.y = fsub(fmul(rr, fsub(v, r.x)), fdbl(fmul(s1, j)));
  r.z = fmul(fsub(fsub(fsqr(fadd(p.z, q.z)), z1z1), z2z2), h);
  return r;
}

// madd-2007-bl: p + affine q
template <class F>
BLS_HDNI Jac<F> jac_add_aff(const Jac<F>& p, const Aff<F>& q) {
  if (q.inf) return p;
  if (jac_is_inf(p)) return jac_from_aff(q);
  F z1z1 = fsqr(p.z);
  F u2 = fmul(q.x, z1z1);
  F s2 = fmul(fmul(q.y, p.z), z1z1);
  F h = fsub(u2, p.x);
  F rr = fdbl(fsub(s2, p.y));
  if (fis_zero(h)) {
    if (fis_zero(rr)) return jac_dbl(p);
    return jac_identity<F>();
  }
  F hh = fsqr(h);
  F i = fdbl(fdbl(hh));
  F j = fmul(h, i);
  F v = fmul(p.x, i);
  Jac<F> r;
  r.x = fsub(fsub(fsqr(rr), j), fdbl(v));
  r.y = fsub(fmul(rr, fsub(v, r.x)), fdbl(fmul(p.y, j)));
  r.z = fsub(fsub(fsqr(fadd(p.z, h)), z1z1), hh);
  return r;
}

template <class F>
BLS_HDNI Aff<F> jac_to_aff(const Jac<F>& p) {
  Aff<F> r;
  if (jac_is_inf(p)) {
    fset_zero(r.x);
    fset_zero(r.y);
    r.inf = true;
    return r;
  }
  F zi = finv(p.z);
  F zi2 = fsqr(zi);
  r.x = fmul(p.x, zi2);
  r.y = fmul(fmul(p.y, zi2), zi);
  r.inf = false;
  return r;
}

template <class F>
BLS_HDNI bool jac_eq(const Jac<F>& p, const Jac<F>& q) {
  bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  if (pi || qi) return pi && qi;
  F z1z1 = fsqr(p.z);
  F z2z2 = fsqr(q.z);
  if (!feq(fmul(p.x, z2z2), fmul(q.x, z1z1))) return false;
  return feq(fmul(fmul(p.y, q.z), z2z2), fmul(fmul(q.y, p.z), z1z1));
}

// [k]p for a 64-bit k (MSB-first double-and-add)
template <class F>
BLS_HDNI Jac<F> jac_mul_u64(const Jac<F>& p, uint64_t k) {
  Jac<F> r = jac_identity<F>();
  for (int i = 63; i >= 0; --i) {
    r = jac_dbl(r);
    if ((k >> i) & 1ull) r = jac_add(r, p);
  }
  return r;
}

// [k]p for a 256-bit scalar given as 8 little-endian u32 limbs
template <class F>
BLS_HDNI Jac<F> jac_mul_u256(const Jac<F>& p, const uint32_t* k) {
  int top = 255;
  while (top >= 0 && !((k[top >> 5] >> (top & 31)) & 1u)) --top;
  if (top < 0) return jac_identity<F>();
  Jac<F> r = p;
  for (int i = top - 1; i >= 0; --i) {
    r = jac_dbl(r);
    if ((k[i >> 5] >> (i & 31)) & 1u) r = jac_add(r, p);
  }
  return r;
}

// [|x|]p, x = -0xd201000000010000 (63 doublings, 5 additions)
template <class F>
BLS_HDNI Jac<F> jac_mul_xabs(const Jac<F>& p) {
  Jac<F> r = p;
  for (int i = 62; i >= 0; --i) {
    r = jac_dbl(r);
    if ((X_ABS >> i) & 1ull) r = jac_add(r, p);
  }
  return r;
}

// ---- on-curve checks ------------------------------------------------------
BLS_HDNI bool g1_aff_on_curve(const Fp& x, const Fp& y) {
  return fp_eq(fp_sqr(y), fp_add(fp_mul(fp_sqr(x), x), FP_B1));
}
BLS_HDNI bool g2_aff_on_curve(const Fp2& x, const Fp2& y) {
  return fp2_eq(fp2_sqr(y), fp2_add(fp2_mul(fp2_sqr(x), x), FP2_B2));
}

// ---- endomorphisms & subgroup checks --------------------------------------
// psi(x, y) = (conj(x) cx, conj(y) cy); Jacobian: conj each coordinate.
BLS_HDNI G2J g2_psi(const G2J& p) {
  return G2J{fp2_mul(fp2_conj(p.x), PSI_CX), fp2_mul(fp2_conj(p.y), PSI_CY), fp2_conj(p.z)};
}
BLS_HDNI G2J g2_psi2(const G2J& p) { return G2J{fp2_mul(p.x, PSI2_CX), fp2_mul(p.y, PSI2_CY), p.z}; }

// P in G2  <=>  psi(P) == [x]P  (x = -|x|)
BLS_HDNI bool g2_in_subgroup(const G2J& p) {
  if (jac_is_inf(p)) return true;
  G2J xp = jac_neg(jac_mul_xabs(p));
  return jac_eq(g2_psi(p), xp);
}

// P in G1  <=>  phi(P) == [-x^2]P,  phi(x, y) = (beta x, y)
BLS_HDNI bool g1_in_subgroup(const G1J& p) {
  if (jac_is_inf(p)) return true;
  G1J x2p = jac_mul_xabs(jac_mul_xabs(p));  // [x^2]P
  G1J phi{fp_mul(p.x, FP_BETA), p.y, p.z};
  return jac_eq(phi, jac_neg(x2p));
}

// ---- serialisation ----------------------------------------------------------
enum DecodeStatus : int {
  DEC_OK = 0,
  DEC_INFINITY = 1,   // valid encoding of the identity
  DEC_BAD_FLAGS = 2,  // c_flag clear, or b_flag / a_flag inconsistent
  DEC_NOT_FIELD = 3,  // coordinate >= p
  DEC_NOT_ON_CURVE = 4,
};

BLS_HDNI bool fp2_lex_largest(const Fp2& y_mont) {
  Fp y0 = fp_from_mont(y_mont.c0), y1 = fp_from_mont(y_mont.c1);
  if (!fp_is_zero(y1)) return raw_gt_half(y1);
  return raw_gt_half(y0);
}

// 48 bytes -> affine G1 (py_ecc pubkey_to_G1 / decompress_G1 rules)
BLS_HDNI int g1_decompress(G1A& out, const uint8_t* b) {
  const uint8_t f = b[0];
  const bool c_flag = f & 0x80, b_flag = f & 0x40, a_flag = f & 0x20;
  out.inf = false;
  if (!c_flag) return DEC_BAD_FLAGS;
  uint8_t tmp[48];
  for (int i = 0; i < 48; i++) tmp[i] = b[i];
  tmp[0] &= 0x1f;
  Fp x = raw_from_be48(tmp);
  const bool x_zero = fp_is_zero(x);
  if (b_flag != x_zero) return DEC_BAD_FLAGS;
  if (x_zero) {
    if (a_flag) return DEC_BAD_FLAGS;
    out.inf = true;
    out.x = fp_zero();
    out.y = fp_zero();
    return DEC_INFINITY;
  }
  if (!raw_lt_p(x)) return DEC_NOT_FIELD;
  Fp xm = fp_to_mont(x);
  Fp rhs = fp_add(fp_mul(fp_sqr(xm), xm), FP_B1);
  Fp y;
  if (!fp_sqrt(y, rhs)) return DEC_NOT_ON_CURVE;
  if (raw_gt_half(fp_from_mont(y)) != a_flag) y = fp_neg(y);
  out.x = xm;
  out.y = y;
  return DEC_OK;
}

// 96 bytes (x.c1 || x.c0) -> affine G2 (py_ecc signature_to_G2 rules)
BLS_HDNI int g2_decompress(G2A& out, const uint8_t* b) {
  const uint8_t f = b[0];
  const bool c_flag = f & 0x80, b_flag = f & 0x40, a_flag = f & 0x20;
  out.inf = false;
  if (!c_flag) return DEC_BAD_FLAGS;
  uint8_t tmp[48];
  for (int i = 0; i < 48; i++) tmp[i] = b[i];
  tmp[0] &= 0x1f;
  Fp x1 = raw_from_be48(tmp);
  Fp x0 = raw_from_be48(b + 48);
  const bool x_zero = fp_is_zero(x1) && fp_is_zero(x0);
  if (b_flag != x_zero) return DEC_BAD_FLAGS;
  if (x_zero) {
    if (a_flag) return DEC_BAD_FLAGS;
    out.inf = true;
    out.x = fp2_zero();
    out.y = fp2_zero();
    return DEC_INFINITY;
  }
  if (!raw_lt_p(x1) || !raw_lt_p(x0)) return DEC_NOT_FIELD;
  Fp2 xm{fp_to_mont(x0), fp_to_mont(x1)};
  Fp2 rhs = fp2_add(fp2_mul(fp2_sqr(xm), xm), FP2_B2);
  Fp2 y;
  if (!fp2_sqrt(y, rhs)) return DEC_NOT_ON_CURVE;
  if (fp2_lex_largest(y) != a_flag) y = fp2_neg(y);
  out.x = xm;
  out.y = y;
  return DEC_OK;
}

BLS_HDNI void g1_compress(uint8_t* out, const G1A& p) {
  if (p.inf) {
    out[0] = 0xc0;
    for (int i = 1; i < 48; i++) out[i] = 0;
    return;
  }
  raw_to_be48(fp_from_mont(p.x), out);
  out[0] |= 0x80;
  if (raw_gt_half(fp_from_mont(p.y))) out[0] |= 0x20;
}

BLS_HDNI void g2_compress(uint8_t* out, const G2A& p) {
  if (p.inf) {
    out[0] = 0xc0;
    for (int i = 1; i < 96; i++) out[i] = 0;
    return;
  }
  raw_to_be48(fp_from_mont(p.x.c1), out);
  raw_to_be48(fp_from_mont(p.x.c0), out + 48);
  out[0] |= 0x80;
  if (fp2_lex_largest(p.y)) out[0] |= 0x20;
}

BLS_HD G1A g1_generator() { return G1A{G1_GEN_X, G1_GEN_Y, false}; }
BLS_HD G2A g2_generator() { return G2A{G2_GEN_X, G2_GEN_Y, false}; }

}  // namespace bls
