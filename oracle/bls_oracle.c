/*
 * bls_oracle.c -- BLS12-381 CPU restatement in plain C.  TEST INFRASTRUCTURE
 * ONLY: it is the fast parity checker (tests/) and the CPU baseline leg of
 * bench.py (cpu_baseline, kind "port").  The product path
 * (eth-consensus-specs_amd/) never links or calls it.
 *
 * What it restates (the reference reaches these through third-party wheels,
 * milagro_bls_binding==1.9.0 / py_arkworks_bls12381==0.3.8 / py_ecc==8.0.0,
 * pinned at reference pyproject.toml:19-21, none vendored or importable here):
 *   - the eth2spec.utils.bls wrapper semantics (reference
 *     tests/core/pyspec/eth2spec/utils/bls.py:141-221,395-397, written E/ below):
 *     Verify / FastAggregateVerify / AggregateVerify return 0 on every decode,
 *     subgroup, infinity and empty-list rejection; Aggregate / AggregatePKs /
 *     Sign / SkToPk report failure (the shim raises);
 *   - ciphersuite BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_ (IETF BLS
 *     draft-04, reference specs/phase0/beacon-chain.md:688-703);
 *   - RFC 9380 hash_to_G2: expand_message_xmd SHA-256 (§5.3.1), hash_to_field
 *     (§5.2), simplified SWU on E2' (§6.6.2), 3-isogeny (App. E.3),
 *     clear_cofactor by the psi method (App. G.3 / §8.8.2);
 *   - ZCash compressed encodings with the py_ecc decode rules (SURVEY.md §8(a)
 *     edge-semantics rows);
 *   - optimal-ate Miller loop (homogeneous projective twist coordinates, lines
 *     scaled by subfield factors the final exponentiation removes) and the
 *     final exponentiation (p^12-1)/r with the hard part computed as
 *     3(p^4-p^2+1)/r = (x-1)^2 (x+p) (x^2+p^2-1) + 3 (the cube does not change
 *     the "== 1" verdict because gcd(3, r) = 1).
 *
 * Independence from the device code: 6 x 64-bit limbs with CIOS Montgomery
 * (R = 2^384) instead of the device's 12 x 32-bit / radix-2^29 forms,
 * Fermat inversion, its own SHA-256.  It is pinned by tests/test_oracle_c.py
 * against the Python oracle (oracle/bls_oracle.py) and the committed golden
 * fixtures (tests/golden/ JSON files: reference verdicts, the deposit-cli Verify
 * known answer, trusted-setup points, eth2 BLS sign vectors).
 *
 * Not constant time.  Not for production keys.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t u64;
typedef unsigned __int128 u128;

typedef struct { u64 l[6]; } fp;
typedef struct { fp c0, c1; } fp2;
typedef struct { fp2 c0, c1, c2; } fp6;
typedef struct { fp6 c0, c1; } fp12;
typedef struct { fp x, y, z; } g1j;  /* Jacobian, z == 0 is infinity */
typedef struct { fp2 x, y, z; } g2j;

/* ------------------------------------------------------------------------- */
/* Fp: Montgomery form, R = 2^384                                            */
/* ------------------------------------------------------------------------- */
static const fp P = {{0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL, 0x64774b84f38512bfULL,
                      0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL}};
static u64 PINV;  /* -p^-1 mod 2^64 */
static fp R1, R2;  /* R mod p, R^2 mod p */
static fp FP_ZERO;

static int fp_geq_p(const fp* a) {
  for (int i = 5; i >= 0; i--) {
    if (a->l[i] > P.l[i]) return 1;
    if (a->l[i] < P.l[i]) return 0;
  }
  return 1;
}
static u64 sub6(u64* r, const u64* a, const u64* b) {
  u64 br = 0;
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)a[i] - b[i] - br;
    r[i] = (u64)d;
    br = (u64)(d >> 64) & 1;
  }
  return br;
}
static void fp_add(fp* r, const fp* a, const fp* b) {
  u64 c = 0;
  for (int i = 0; i < 6; i++) {
    u128 s = (u128)a->l[i] + b->l[i] + c;
    r->l[i] = (u64)s;
    c = (u64)(s >> 64);
  }
  if (fp_geq_p(r)) sub6(r->l, r->l, P.l);
}
static void fp_sub(fp* r, const fp* a, const fp* b) {
  if (sub6(r->l, a->l, b->l)) {
    u64 c = 0;
    for (int i = 0; i < 6; i++) {
      u128 s = (u128)r->l[i] + P.l[i] + c;
      r->l[i] = (u64)s;
      c = (u64)(s >> 64);
    }
  }
}
static int fp_is_zero(const fp* a) {
  u64 x = 0;
  for (int i = 0; i < 6; i++) x |= a->l[i];
  return x == 0;
}
static int fp_eq(const fp* a, const fp* b) { return memcmp(a, b, sizeof(fp)) == 0; }
static void fp_neg(fp* r, const fp* a) {
  if (fp_is_zero(a)) *r = *a;
  else sub6(r->l, P.l, a->l);
}
static void fp_mul(fp* r, const fp* a, const fp* b) {
  u64 t[8] = {0};
  for (int i = 0; i < 6; i++) {
    u64 c = 0;
    for (int j = 0; j < 6; j++) {
      u128 uv = (u128)a->l[j] * b->l[i] + t[j] + c;
      t[j] = (u64)uv;
      c = (u64)(uv >> 64);
    }
    u128 uv = (u128)t[6] + c;
    t[6] = (u64)uv;
    t[7] = (u64)(uv >> 64);
    u64 m = t[0] * PINV;
    uv = (u128)m * P.l[0] + t[0];
    c = (u64)(uv >> 64);
    for (int j = 1; j < 6; j++) {
      uv = (u128)m * P.l[j] + t[j] + c;
      t[j - 1] = (u64)uv;
      c = (u64)(uv >> 64);
    }
    uv = (u128)t[6] + c;
    t[5] = (u64)uv;
    t[6] = t[7] + (u64)(uv >> 64);
  }
  fp out;
  memcpy(out.l, t, 48);
  if (t[6] || fp_geq_p(&out)) sub6(out.l, out.l, P.l);
  *r = out;
}
static void fp_sqr(fp* r, const fp* a) { fp_mul(r, a, a); }
static void fp_dbl(fp* r, const fp* a) { fp_add(r, a, a); }
/* a^e, e given as little-endian u64 limbs (n of them) */
static void fp_pow(fp* r, const fp* a, const u64* e, int n) {
  fp acc = R1, b = *a;
  for (int i = 0; i < n; i++)
    for (int k = 0; k < 64; k++) {
      if ((e[i] >> k) & 1) fp_mul(&acc, &acc, &b);
      fp_sqr(&b, &b);
    }
  *r = acc;
}
static u64 E_PM2[6], E_SQRT[6], E_LEG[6];
static void fp_inv(fp* r, const fp* a) { fp_pow(r, a, E_PM2, 6); }
static void fp_from_u64(fp* r, u64 v) {
  fp t = FP_ZERO;
  t.l[0] = v;
  fp_mul(r, &t, &R2);
}
/* big-endian 48 bytes (value < 2^384) -> plain limbs */
static void limbs_from_be48(u64* l, const uint8_t* b) {
  for (int i = 0; i < 6; i++) {
    u64 v = 0;
    for (int k = 0; k < 8; k++) v = (v << 8) | b[(5 - i) * 8 + k];
    l[i] = v;
  }
}
static void limbs_to_be48(uint8_t* b, const u64* l) {
  for (int i = 0; i < 6; i++)
    for (int k = 0; k < 8; k++) b[(5 - i) * 8 + k] = (uint8_t)(l[i] >> (56 - 8 * k));
}
static void fp_to_mont(fp* r, const u64* plain) {
  fp t;
  memcpy(t.l, plain, 48);
  fp_mul(r, &t, &R2);
}
static void fp_from_mont(u64* plain, const fp* a) {
  fp one = FP_ZERO, t;
  one.l[0] = 1;
  fp_mul(&t, a, &one);
  memcpy(plain, t.l, 48);
}
static void fp_from_hex(fp* r, const char* h) {
  uint8_t b[48] = {0};
  size_t n = strlen(h);
  for (size_t i = 0; i < n; i++) {
    char c = h[n - 1 - i];
    int v = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : c - 'A' + 10;
    b[47 - i / 2] |= (uint8_t)(v << (4 * (i & 1)));
  }
  u64 l[6];
  limbs_from_be48(l, b);
  fp_to_mont(r, l);
}
/* integer comparisons on canonical values */
static int fp_gt_half(const fp* a) { /* a > (p-1)/2 */
  u64 v[6], h[6];
  fp_from_mont(v, a);
  memcpy(h, P.l, 48);
  for (int i = 0; i < 5; i++) h[i] = (h[i] >> 1) | (h[i + 1] << 63);
  h[5] >>= 1;
  for (int i = 5; i >= 0; i--) {
    if (v[i] > h[i]) return 1;
    if (v[i] < h[i]) return 0;
  }
  return 0;
}
static int fp_is_square(const fp* a) {
  if (fp_is_zero(a)) return 1;
  fp t;
  fp_pow(&t, a, E_LEG, 6);
  return fp_eq(&t, &R1);
}
static int fp_sqrt(fp* r, const fp* a) {
  fp s, c;
  fp_pow(&s, a, E_SQRT, 6);
  fp_sqr(&c, &s);
  if (!fp_eq(&c, a)) return 0;
  *r = s;
  return 1;
}

/* ------------------------------------------------------------------------- */
/* Fp2 = Fp[i]/(i^2+1)                                                       */
/* ------------------------------------------------------------------------- */
static fp2 F2_ZERO, F2_ONE;
static void f2_add(fp2* r, const fp2* a, const fp2* b) { fp_add(&r->c0, &a->c0, &b->c0); fp_add(&r->c1, &a->c1, &b->c1); }
static void f2_sub(fp2* r, const fp2* a, const fp2* b) { fp_sub(&r->c0, &a->c0, &b->c0); fp_sub(&r->c1, &a->c1, &b->c1); }
static void f2_neg(fp2* r, const fp2* a) { fp_neg(&r->c0, &a->c0); fp_neg(&r->c1, &a->c1); }
static void f2_dbl(fp2* r, const fp2* a) { f2_add(r, a, a); }
static void f2_conj(fp2* r, const fp2* a) { r->c0 = a->c0; fp_neg(&r->c1, &a->c1); }
static int f2_is_zero(const fp2* a) { return fp_is_zero(&a->c0) && fp_is_zero(&a->c1); }
static int f2_eq(const fp2* a, const fp2* b) { return fp_eq(&a->c0, &b->c0) && fp_eq(&a->c1, &b->c1); }
static void f2_mul(fp2* r, const fp2* a, const fp2* b) {
  fp t0, t1, s0, s1, m;
  fp_mul(&t0, &a->c0, &b->c0);
  fp_mul(&t1, &a->c1, &b->c1);
  fp_add(&s0, &a->c0, &a->c1);
  fp_add(&s1, &b->c0, &b->c1);
  fp_mul(&m, &s0, &s1);
  fp_sub(&r->c0, &t0, &t1);
  fp_sub(&m, &m, &t0);
  fp_sub(&r->c1, &m, &t1);
}
static void f2_sqr(fp2* r, const fp2* a) {
  fp s, d, m;
  fp_add(&s, &a->c0, &a->c1);
  fp_sub(&d, &a->c0, &a->c1);
  fp_mul(&m, &a->c0, &a->c1);
  fp_mul(&r->c0, &s, &d);
  fp_dbl(&r->c1, &m);
}
static void f2_mul_fp(fp2* r, const fp2* a, const fp* b) { fp_mul(&r->c0, &a->c0, b); fp_mul(&r->c1, &a->c1, b); }
static void f2_mul_xi(fp2* r, const fp2* a) { /* (1+i) a */
  fp t;
  fp_sub(&t, &a->c0, &a->c1);
  fp_add(&r->c1, &a->c0, &a->c1);
  r->c0 = t;
}
static void f2_inv(fp2* r, const fp2* a) {
  fp n, t;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  fp_inv(&n, &n);
  fp_mul(&r->c0, &a->c0, &n);
  fp_mul(&t, &a->c1, &n);
  fp_neg(&r->c1, &t);
}
static void f2_from_u64(fp2* r, u64 a, u64 b) { fp_from_u64(&r->c0, a); fp_from_u64(&r->c1, b); }
static void f2_pow_big(fp2* r, const fp2* a, const u64* e, int n) {
  fp2 acc = F2_ONE, b = *a;
  for (int i = 0; i < n; i++)
    for (int k = 0; k < 64; k++) {
      if ((e[i] >> k) & 1) f2_mul(&acc, &acc, &b);
      f2_sqr(&b, &b);
    }
  *r = acc;
}
static int f2_is_square(const fp2* a) {
  fp n, t;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  return fp_is_square(&n);
}
static fp INV2;
/* some square root (norm method, same choice as oracle/bls_oracle.py f2_sqrt) */
static int f2_sqrt(fp2* r, const fp2* a) {
  fp2 cand;
  if (fp_is_zero(&a->c1)) {
    fp s, na;
    if (fp_sqrt(&s, &a->c0)) { cand.c0 = s; cand.c1 = FP_ZERO; *r = cand; return 1; }
    fp_neg(&na, &a->c0);
    if (fp_sqrt(&s, &na)) { cand.c0 = FP_ZERO; cand.c1 = s; *r = cand; return 1; }
    return 0;
  }
  fp n, t, x0, x1;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  if (!fp_sqrt(&n, &n)) return 0;
  fp_add(&t, &a->c0, &n);
  fp_mul(&t, &t, &INV2);
  if (!fp_sqrt(&x0, &t)) {
    fp_sub(&t, &a->c0, &n);
    fp_mul(&t, &t, &INV2);
    if (!fp_sqrt(&x0, &t)) return 0;
  }
  fp_dbl(&t, &x0);
  fp_inv(&t, &t);
  fp_mul(&x1, &a->c1, &t);
  cand.c0 = x0;
  cand.c1 = x1;
  fp2 chk;
  f2_sqr(&chk, &cand);
  if (!f2_eq(&chk, a)) return 0;
  *r = cand;
  return 1;
}
static int f2_lex_largest(const fp2* y) {
  if (!fp_is_zero(&y->c1)) return fp_gt_half(&y->c1);
  return fp_gt_half(&y->c0);
}
static int f2_sgn0(const fp2* a) {
  u64 v0[6], v1[6];
  fp_from_mont(v0, &a->c0);
  fp_from_mont(v1, &a->c1);
  int s0 = (int)(v0[0] & 1), z0 = fp_is_zero(&a->c0), s1 = (int)(v1[0] & 1);
  return s0 | (z0 & s1);
}

/* ------------------------------------------------------------------------- */
/* Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v)                          */
/* ------------------------------------------------------------------------- */
static void f6_add(fp6* r, const fp6* a, const fp6* b) {
  f2_add(&r->c0, &a->c0, &b->c0); f2_add(&r->c1, &a->c1, &b->c1); f2_add(&r->c2, &a->c2, &b->c2);
}
static void f6_sub(fp6* r, const fp6* a, const fp6* b) {
  f2_sub(&r->c0, &a->c0, &b->c0); f2_sub(&r->c1, &a->c1, &b->c1); f2_sub(&r->c2, &a->c2, &b->c2);
}
static void f6_neg(fp6* r, const fp6* a) { f2_neg(&r->c0, &a->c0); f2_neg(&r->c1, &a->c1); f2_neg(&r->c2, &a->c2); }
static void f6_mul(fp6* r, const fp6* a, const fp6* b) {
  fp2 t0, t1, t2, s, u, c0, c1, c2;
  f2_mul(&t0, &a->c0, &b->c0);
  f2_mul(&t1, &a->c1, &b->c1);
  f2_mul(&t2, &a->c2, &b->c2);
  /* c0 = t0 + xi((a1+a2)(b1+b2) - t1 - t2) */
  f2_add(&s, &a->c1, &a->c2); f2_add(&u, &b->c1, &b->c2); f2_mul(&s, &s, &u);
  f2_sub(&s, &s, &t1); f2_sub(&s, &s, &t2); f2_mul_xi(&s, &s); f2_add(&c0, &t0, &s);
  /* c1 = (a0+a1)(b0+b1) - t0 - t1 + xi t2 */
  f2_add(&s, &a->c0, &a->c1); f2_add(&u, &b->c0, &b->c1); f2_mul(&s, &s, &u);
  f2_sub(&s, &s, &t0); f2_sub(&s, &s, &t1); f2_mul_xi(&u, &t2); f2_add(&c1, &s, &u);
  /* c2 = (a0+a2)(b0+b2) - t0 - t2 + t1 */
  f2_add(&s, &a->c0, &a->c2); f2_add(&u, &b->c0, &b->c2); f2_mul(&s, &s, &u);
  f2_sub(&s, &s, &t0); f2_sub(&s, &s, &t2); f2_add(&c2, &s, &t1);
  r->c0 = c0; r->c1 = c1; r->c2 = c2;
}
static void f6_mul_v(fp6* r, const fp6* a) {
  fp2 t;
  f2_mul_xi(&t, &a->c2);
  r->c2 = a->c1;
  r->c1 = a->c0;
  r->c0 = t;
}
static void f6_inv(fp6* r, const fp6* a) {
  fp2 t0, t1, t2, u, det;
  f2_sqr(&t0, &a->c0); f2_mul(&u, &a->c1, &a->c2); f2_mul_xi(&u, &u); f2_sub(&t0, &t0, &u);
  f2_sqr(&t1, &a->c2); f2_mul_xi(&t1, &t1); f2_mul(&u, &a->c0, &a->c1); f2_sub(&t1, &t1, &u);
  f2_sqr(&t2, &a->c1); f2_mul(&u, &a->c0, &a->c2); f2_sub(&t2, &t2, &u);
  f2_mul(&det, &a->c2, &t1); f2_mul(&u, &a->c1, &t2); f2_add(&det, &det, &u); f2_mul_xi(&det, &det);
  f2_mul(&u, &a->c0, &t0); f2_add(&det, &det, &u);
  f2_inv(&det, &det);
  f2_mul(&r->c0, &t0, &det); f2_mul(&r->c1, &t1, &det); f2_mul(&r->c2, &t2, &det);
}
static fp12 F12_ONE;
static void f12_mul(fp12* r, const fp12* a, const fp12* b) {
  fp6 t0, t1, s, u;
  f6_mul(&t0, &a->c0, &b->c0);
  f6_mul(&t1, &a->c1, &b->c1);
  f6_add(&s, &a->c0, &a->c1);
  f6_add(&u, &b->c0, &b->c1);
  f6_mul(&s, &s, &u);
  f6_sub(&s, &s, &t0);
  f6_sub(&r->c1, &s, &t1);
  f6_mul_v(&t1, &t1);
  f6_add(&r->c0, &t0, &t1);
}
static void f12_sqr(fp12* r, const fp12* a) {
  /* complex squaring: (a0 + a1 w)^2 = (a0^2 + v a1^2) + 2 a0 a1 w */
  fp6 m, s, u, t;
  f6_mul(&m, &a->c0, &a->c1);
  f6_add(&s, &a->c0, &a->c1);
  f6_mul_v(&u, &a->c1);
  f6_add(&u, &a->c0, &u);
  f6_mul(&s, &s, &u);           /* (a0+a1)(a0+v a1) = a0^2 + v a1^2 + (1+v) a0 a1 */
  f6_sub(&s, &s, &m);
  f6_mul_v(&t, &m);
  f6_sub(&r->c0, &s, &t);
  f6_add(&r->c1, &m, &m);
}
static void f12_conj(fp12* r, const fp12* a) { r->c0 = a->c0; f6_neg(&r->c1, &a->c1); }
static void f12_inv(fp12* r, const fp12* a) {
  fp6 t0, t1;
  f6_mul(&t0, &a->c0, &a->c0);
  f6_mul(&t1, &a->c1, &a->c1);
  f6_mul_v(&t1, &t1);
  f6_sub(&t0, &t0, &t1);
  f6_inv(&t0, &t0);
  f6_mul(&r->c0, &a->c0, &t0);
  f6_mul(&t1, &a->c1, &t0);
  f6_neg(&r->c1, &t1);
}
static int f12_eq(const fp12* a, const fp12* b) { return memcmp(a, b, sizeof(fp12)) == 0; }
/* w-basis coefficient access: c[0..5] = a0.c0, a1.c0, a0.c1, a1.c1, a0.c2, a1.c2 */
static fp2* f12_coef(fp12* a, int k) {
  fp6* h = (k & 1) ? &a->c1 : &a->c0;
  return (k >> 1) == 0 ? &h->c0 : (k >> 1) == 1 ? &h->c1 : &h->c2;
}
static fp2 GAMMA1[6], GAMMA2[6]; /* xi^(k(p-1)/6), and its p^2 analogue */
static void f12_frob(fp12* r, const fp12* a) {
  fp12 t = *a;
  for (int k = 0; k < 6; k++) {
    fp2* c = f12_coef(&t, k);
    f2_conj(c, c);
    f2_mul(c, c, &GAMMA1[k]);
  }
  *r = t;
}
static void f12_frob2(fp12* r, const fp12* a) {
  fp12 t = *a;
  for (int k = 0; k < 6; k++) {
    fp2* c = f12_coef(&t, k);
    f2_mul(c, c, &GAMMA2[k]);
  }
  *r = t;
}

/* ------------------------------------------------------------------------- */
/* Curves: E1 y^2 = x^3 + 4, E2 y^2 = x^3 + 4(1+i)                           */
/* ------------------------------------------------------------------------- */
static fp B1;
static fp2 B2, B2x3;   /* 4(1+i), 3 * 4(1+i) */
static const u64 X_ABS = 0xd201000000010000ULL;

#define DEF_JAC(PFX, F, T, ADD, SUB, MUL, SQR, DBL, NEG, ISZ, EQ, ONE)                      \
  static int PFX##_is_inf(const T* p) { return ISZ(&p->z); }                                \
  static void PFX##_dbl(T* r, const T* p) {                                                 \
    if (ISZ(&p->z)) { *r = *p; return; }                                                    \
    F a, b, c, d, e, f, t, x3, y3, z3;                                                      \
    SQR(&a, &p->x); SQR(&b, &p->y); SQR(&c, &b);                                            \
    ADD(&d, &p->x, &b); SQR(&d, &d); SUB(&d, &d, &a); SUB(&d, &d, &c); DBL(&d, &d);         \
    DBL(&e, &a); ADD(&e, &e, &a); SQR(&f, &e);                                              \
    DBL(&t, &d); SUB(&x3, &f, &t);                                                          \
    SUB(&t, &d, &x3); MUL(&y3, &e, &t); DBL(&c, &c); DBL(&c, &c); DBL(&c, &c);              \
    SUB(&y3, &y3, &c);                                                                      \
    MUL(&z3, &p->y, &p->z); DBL(&z3, &z3);                                                  \
    r->x = x3; r->y = y3; r->z = z3;                                                        \
  }                                                                                         \
  static void PFX##_add(T* r, const T* p, const T* q) {                                     \
    if (ISZ(&p->z)) { *r = *q; return; }                                                    \
    if (ISZ(&q->z)) { *r = *p; return; }                                                    \
    F z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t, x3, y3, z3;                            \
    SQR(&z1z1, &p->z); SQR(&z2z2, &q->z);                                                   \
    MUL(&u1, &p->x, &z2z2); MUL(&u2, &q->x, &z1z1);                                         \
    MUL(&s1, &p->y, &q->z); MUL(&s1, &s1, &z2z2);                                           \
    MUL(&s2, &q->y, &p->z); MUL(&s2, &s2, &z1z1);                                           \
    SUB(&h, &u2, &u1); SUB(&rr, &s2, &s1);                                                  \
    if (ISZ(&h)) {                                                                          \
      if (ISZ(&rr)) { PFX##_dbl(r, p); return; }                                            \
      memset(r, 0, sizeof(T)); r->x = ONE; r->y = ONE; return;                              \
    }                                                                                       \
    DBL(&i, &h); SQR(&i, &i); MUL(&j, &h, &i); DBL(&rr, &rr); MUL(&v, &u1, &i);             \
    SQR(&x3, &rr); SUB(&x3, &x3, &j); SUB(&x3, &x3, &v); SUB(&x3, &x3, &v);                 \
    SUB(&t, &v, &x3); MUL(&y3, &rr, &t); MUL(&t, &s1, &j); DBL(&t, &t); SUB(&y3, &y3, &t);  \
    ADD(&z3, &p->z, &q->z); SQR(&z3, &z3); SUB(&z3, &z3, &z1z1); SUB(&z3, &z3, &z2z2);      \
    MUL(&z3, &z3, &h);                                                                      \
    r->x = x3; r->y = y3; r->z = z3;                                                        \
  }                                                                                         \
  static void PFX##_neg(T* r, const T* p) { r->x = p->x; NEG(&r->y, &p->y); r->z = p->z; }  \
  static void PFX##_mul_u64(T* r, const T* p, u64 k) {                                      \
    T acc; memset(&acc, 0, sizeof(T)); acc.x = ONE; acc.y = ONE;                            \
    for (int b = 63; b >= 0; b--) {                                                         \
      PFX##_dbl(&acc, &acc);                                                                \
      if ((k >> b) & 1) PFX##_add(&acc, &acc, p);                                           \
    }                                                                                       \
    *r = acc;                                                                               \
  }                                                                                         \
  static void PFX##_mul_big(T* r, const T* p, const u64* k, int n) {                        \
    T acc; memset(&acc, 0, sizeof(T)); acc.x = ONE; acc.y = ONE;                            \
    for (int i = n - 1; i >= 0; i--)                                                        \
      for (int b = 63; b >= 0; b--) {                                                       \
        PFX##_dbl(&acc, &acc);                                                              \
        if ((k[i] >> b) & 1) PFX##_add(&acc, &acc, p);                                      \
      }                                                                                     \
    *r = acc;                                                                               \
  }                                                                                         \
  static int PFX##_eq(const T* p, const T* q) {                                             \
    int ip = ISZ(&p->z), iq = ISZ(&q->z);                                                   \
    if (ip || iq) return ip && iq;                                                          \
    F z1z1, z2z2, a, b;                                                                     \
    SQR(&z1z1, &p->z); SQR(&z2z2, &q->z);                                                   \
    MUL(&a, &p->x, &z2z2); MUL(&b, &q->x, &z1z1);                                           \
    if (!EQ(&a, &b)) return 0;                                                              \
    MUL(&a, &p->y, &z2z2); MUL(&a, &a, &q->z); MUL(&b, &q->y, &z1z1); MUL(&b, &b, &p->z);   \
    return EQ(&a, &b);                                                                      \
  }                                                                                         \
  static void PFX##_affine(F* x, F* y, const T* p) {                                        \
    F zi, zi2;                                                                              \
    F##_inv_(&zi, &p->z); SQR(&zi2, &zi); MUL(x, &p->x, &zi2);                              \
    MUL(&zi2, &zi2, &zi); MUL(y, &p->y, &zi2);                                              \
  }

#define fp_inv_ fp_inv
#define fp2_inv_ f2_inv
DEF_JAC(g1, fp, g1j, fp_add, fp_sub, fp_mul, fp_sqr, fp_dbl, fp_neg, fp_is_zero, fp_eq, R1)
DEF_JAC(g2, fp2, g2j, f2_add, f2_sub, f2_mul, f2_sqr, f2_dbl, f2_neg, f2_is_zero, f2_eq, F2_ONE)

static g1j G1_GEN, G1_NEG_GEN;
static g2j G2_GEN;
static u64 R_LIMBS[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL, 0x73eda753299d7d48ULL};

static int g1_on_curve_aff(const fp* x, const fp* y) {
  fp l, r;
  fp_sqr(&l, y);
  fp_sqr(&r, x);
  fp_mul(&r, &r, x);
  fp_add(&r, &r, &B1);
  return fp_eq(&l, &r);
}
static int g1_in_subgroup(const g1j* p) {
  g1j t;
  g1_mul_big(&t, p, R_LIMBS, 4);
  return g1_is_inf(&t);
}
static fp2 PSI_CX, PSI_CY;
static void g2_psi(g2j* r, const g2j* p) {
  f2_conj(&r->x, &p->x);
  f2_mul(&r->x, &r->x, &PSI_CX);
  f2_conj(&r->y, &p->y);
  f2_mul(&r->y, &r->y, &PSI_CY);
  f2_conj(&r->z, &p->z);
}
/* [x]P with x = -X_ABS */
static void g2_mul_x(g2j* r, const g2j* p) {
  g2j t;
  g2_mul_u64(&t, p, X_ABS);
  g2_neg(r, &t);
}
/* P in G2 iff psi(P) == [x]P (Scott, eprint 2021/1130 §4); cross-checked
 * against [r]P == O by tests/test_oracle_c.py */
static int g2_in_subgroup(const g2j* p) {
  g2j a, b;
  g2_psi(&a, p);
  g2_mul_x(&b, p);
  return g2_eq(&a, &b);
}

/* ------------------------------------------------------------------------- */
/* ZCash encodings (py_ecc pubkey_to_G1 / signature_to_G2 rules)             */
/* ------------------------------------------------------------------------- */
static u64 LIMB_P_GE_CHECK(const u64* v) { /* v >= p */
  for (int i = 5; i >= 0; i--) {
    if (v[i] > P.l[i]) return 1;
    if (v[i] < P.l[i]) return 0;
  }
  return 1;
}
/* 1 ok (point, possibly infinity), 0 invalid */
static int g1_decompress(g1j* out, const uint8_t* in) {
  int c = in[0] >> 7 & 1, b = in[0] >> 6 & 1, a = in[0] >> 5 & 1;
  if (!c) return 0;
  uint8_t t[48];
  memcpy(t, in, 48);
  t[0] &= 0x1f;
  u64 xl[6];
  limbs_from_be48(xl, t);
  int xz = 1;
  for (int i = 0; i < 6; i++) xz &= xl[i] == 0;
  if (b != xz) return 0;
  if (xz) {
    if (a) return 0;
    memset(out, 0, sizeof(*out));
    out->x = R1; out->y = R1;
    return 1;
  }
  if (LIMB_P_GE_CHECK(xl)) return 0;
  fp x, y, r;
  fp_to_mont(&x, xl);
  fp_sqr(&r, &x);
  fp_mul(&r, &r, &x);
  fp_add(&r, &r, &B1);
  if (!fp_sqrt(&y, &r)) return 0;
  if (fp_gt_half(&y) != a) fp_neg(&y, &y);
  out->x = x; out->y = y; out->z = R1;
  return 1;
}
static void g1_compress(uint8_t* out, const g1j* p) {
  if (g1_is_inf(p)) { memset(out, 0, 48); out[0] = 0xc0; return; }
  fp x, y;
  g1_affine(&x, &y, p);
  u64 l[6];
  fp_from_mont(l, &x);
  limbs_to_be48(out, l);
  out[0] |= 0x80 | (fp_gt_half(&y) ? 0x20 : 0);
}
static int g2_decompress(g2j* out, const uint8_t* in) {
  int c = in[0] >> 7 & 1, b = in[0] >> 6 & 1, a = in[0] >> 5 & 1;
  if (!c) return 0;
  uint8_t t[48];
  memcpy(t, in, 48);
  t[0] &= 0x1f;
  u64 x1l[6], x0l[6];
  limbs_from_be48(x1l, t);
  limbs_from_be48(x0l, in + 48);
  int xz = 1;
  for (int i = 0; i < 6; i++) xz &= (x1l[i] | x0l[i]) == 0;
  if (b != xz) return 0;
  if (xz) {
    if (a) return 0;
    memset(out, 0, sizeof(*out));
    out->x = F2_ONE; out->y = F2_ONE;
    return 1;
  }
  if (LIMB_P_GE_CHECK(x1l) || LIMB_P_GE_CHECK(x0l)) return 0;
  fp2 x, y, r;
  fp_to_mont(&x.c0, x0l);
  fp_to_mont(&x.c1, x1l);
  f2_sqr(&r, &x);
  f2_mul(&r, &r, &x);
  f2_add(&r, &r, &B2);
  if (!f2_sqrt(&y, &r)) return 0;
  if (f2_lex_largest(&y) != a) f2_neg(&y, &y);
  out->x = x; out->y = y; out->z = F2_ONE;
  return 1;
}
static void g2_compress(uint8_t* out, const g2j* p) {
  if (g2_is_inf(p)) { memset(out, 0, 96); out[0] = 0xc0; return; }
  fp2 x, y;
  g2_affine(&x, &y, p);
  u64 l[6];
  fp_from_mont(l, &x.c1);
  limbs_to_be48(out, l);
  fp_from_mont(l, &x.c0);
  limbs_to_be48(out + 48, l);
  out[0] |= 0x80 | (f2_lex_largest(&y) ? 0x20 : 0);
}

/* ------------------------------------------------------------------------- */
/* SHA-256 (FIPS 180-4) and expand_message_xmd (RFC 9380 §5.3.1)             */
/* ------------------------------------------------------------------------- */
typedef struct { uint32_t h[8]; uint8_t buf[64]; size_t n; uint64_t len; } sha256;
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
    0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
    0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
    0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
    0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
    0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
    0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha_block(sha256* s, const uint8_t* p) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | p[4 * i + 2] << 8 | p[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = s->h[0], b = s->h[1], c = s->h[2], d = s->h[3], e = s->h[4], f = s->h[5], g = s->h[6], h = s->h[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = h + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
    uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  s->h[0] += a; s->h[1] += b; s->h[2] += c; s->h[3] += d; s->h[4] += e; s->h[5] += f; s->h[6] += g; s->h[7] += h;
}
static void sha_init(sha256* s) {
  static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(s->h, iv, 32);
  s->n = 0;
  s->len = 0;
}
static void sha_update(sha256* s, const uint8_t* p, size_t n) {
  s->len += n;
  while (n) {
    size_t k = 64 - s->n < n ? 64 - s->n : n;
    memcpy(s->buf + s->n, p, k);
    s->n += k; p += k; n -= k;
    if (s->n == 64) { sha_block(s, s->buf); s->n = 0; }
  }
}
static void sha_final(sha256* s, uint8_t out[32]) {
  uint64_t bits = s->len * 8;
  uint8_t pad = 0x80, z = 0;
  sha_update(s, &pad, 1);
  while (s->n != 56) sha_update(s, &z, 1);
  uint8_t l[8];
  for (int i = 0; i < 8; i++) l[i] = (uint8_t)(bits >> (56 - 8 * i));
  sha_update(s, l, 8);
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(s->h[i] >> (24 - 8 * k));
}
static int expand_message_xmd(uint8_t* out, size_t len, const uint8_t* msg, size_t mlen, const uint8_t* dst,
                              size_t dlen) {
  size_t ell = (len + 31) / 32;
  if (dlen > 255 || ell > 255) return 0;
  uint8_t dlb = (uint8_t)dlen, zeros[64] = {0}, b0[32], bi[32], lib[3] = {(uint8_t)(len >> 8), (uint8_t)len, 0};
  sha256 s;
  sha_init(&s);
  sha_update(&s, zeros, 64);
  sha_update(&s, msg, mlen);
  sha_update(&s, lib, 3);
  sha_update(&s, dst, dlen);
  sha_update(&s, &dlb, 1);
  sha_final(&s, b0);
  uint8_t one = 1;
  sha_init(&s);
  sha_update(&s, b0, 32);
  sha_update(&s, &one, 1);
  sha_update(&s, dst, dlen);
  sha_update(&s, &dlb, 1);
  sha_final(&s, bi);
  size_t off = 0;
  for (size_t i = 1;; i++) {
    size_t k = len - off < 32 ? len - off : 32;
    memcpy(out + off, bi, k);
    off += k;
    if (off >= len) break;
    uint8_t x[32], ib = (uint8_t)(i + 1);
    for (int j = 0; j < 32; j++) x[j] = b0[j] ^ bi[j];
    sha_init(&s);
    sha_update(&s, x, 32);
    sha_update(&s, &ib, 1);
    sha_update(&s, dst, dlen);
    sha_update(&s, &dlb, 1);
    sha_final(&s, bi);
  }
  return 1;
}

/* ------------------------------------------------------------------------- */
/* hash_to_G2 (RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_)                      */
/* ------------------------------------------------------------------------- */
static fp TWO384; /* 2^384 mod p, Montgomery form */
/* 64 big-endian bytes -> element mod p */
static void fp_from_be64(fp* r, const uint8_t* b) {
  u64 hi[6] = {0}, lo[6];
  uint8_t t[48] = {0};
  memcpy(t + 32, b, 16);
  limbs_from_be48(hi, t);
  limbs_from_be48(lo, b + 16);
  while (LIMB_P_GE_CHECK(lo)) sub6(lo, lo, P.l);
  fp h, l;
  fp_to_mont(&h, hi);
  fp_to_mont(&l, lo);
  fp_mul(&h, &h, &TWO384);
  fp_add(r, &h, &l);
}
static fp2 SSWU_A, SSWU_B, SSWU_Z, SSWU_MBA, SSWU_BZA; /* -B/A, B/(Z A) */
static void map_to_curve_sswu(fp2* xo, fp2* yo, const fp2* u) {
  fp2 zu2, den, x1, x2, gx1, gx2, t, y;
  f2_sqr(&zu2, u);
  f2_mul(&zu2, &zu2, &SSWU_Z);
  f2_sqr(&den, &zu2);
  f2_add(&den, &den, &zu2);
  if (f2_is_zero(&den)) {
    x1 = SSWU_BZA;
  } else {
    f2_inv(&t, &den);
    f2_add(&t, &t, &F2_ONE);
    f2_mul(&x1, &SSWU_MBA, &t);
  }
  f2_sqr(&gx1, &x1); f2_add(&gx1, &gx1, &SSWU_A); f2_mul(&gx1, &gx1, &x1); f2_add(&gx1, &gx1, &SSWU_B);
  f2_mul(&x2, &zu2, &x1);
  f2_sqr(&gx2, &x2); f2_add(&gx2, &gx2, &SSWU_A); f2_mul(&gx2, &gx2, &x2); f2_add(&gx2, &gx2, &SSWU_B);
  if (f2_is_square(&gx1)) { *xo = x1; f2_sqrt(&y, &gx1); }
  else { *xo = x2; f2_sqrt(&y, &gx2); }
  if (f2_sgn0(u) != f2_sgn0(&y)) f2_neg(&y, &y);
  *yo = y;
}
static fp2 ISO_XNUM[4], ISO_XDEN[3], ISO_YNUM[4], ISO_YDEN[4];
static void poly(fp2* r, const fp2* c, int n, const fp2* x) {
  fp2 acc = F2_ZERO;
  for (int i = n - 1; i >= 0; i--) {
    f2_mul(&acc, &acc, x);
    f2_add(&acc, &acc, &c[i]);
  }
  *r = acc;
}
static void iso_map(g2j* out, const fp2* x, const fp2* y) {
  fp2 xn, xd, yn, yd;
  poly(&xn, ISO_XNUM, 4, x);
  poly(&xd, ISO_XDEN, 3, x);
  poly(&yn, ISO_YNUM, 4, x);
  poly(&yd, ISO_YDEN, 4, x);
  if (f2_is_zero(&xd) || f2_is_zero(&yd)) {
    memset(out, 0, sizeof(*out));
    out->x = F2_ONE; out->y = F2_ONE;
    return;
  }
  f2_inv(&xd, &xd);
  f2_inv(&yd, &yd);
  f2_mul(&out->x, &xn, &xd);
  f2_mul(&yn, &yn, &yd);
  f2_mul(&out->y, y, &yn);
  out->z = F2_ONE;
}
/* Budroni-Pintore: [x^2-x-1]P + [x-1]psi(P) + psi^2(2P) */
static void clear_cofactor(g2j* r, const g2j* p) {
  g2j t1, t2, t3, s;
  g2_mul_x(&t1, p);
  g2_psi(&t2, p);
  g2_dbl(&t3, p);
  g2_psi(&t3, &t3);
  g2_psi(&t3, &t3);
  g2_neg(&s, &t2);
  g2_add(&t3, &t3, &s);
  g2_add(&t2, &t1, &t2);
  g2_mul_x(&t2, &t2);
  g2_add(&t3, &t3, &t2);
  g2_neg(&s, &t1);
  g2_add(&t3, &t3, &s);
  g2_neg(&s, p);
  g2_add(r, &t3, &s);
}
static int hash_to_g2(g2j* out, const uint8_t* msg, size_t mlen, const uint8_t* dst, size_t dlen) {
  uint8_t ub[256];
  if (!expand_message_xmd(ub, 256, msg, mlen, dst, dlen)) return 0;
  g2j q[2];
  for (int i = 0; i < 2; i++) {
    fp2 u, x, y;
    fp_from_be64(&u.c0, ub + 128 * i);
    fp_from_be64(&u.c1, ub + 128 * i + 64);
    map_to_curve_sswu(&x, &y, &u);
    iso_map(&q[i], &x, &y);
  }
  g2j s;
  g2_add(&s, &q[0], &q[1]);
  clear_cofactor(out, &s);
  return 1;
}
static const uint8_t DST_POP[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
#define DST_POP_LEN 43

/* ------------------------------------------------------------------------- */
/* Pairing                                                                   */
/* ------------------------------------------------------------------------- */
/* f <- f * l where l = l0 + l2 w^2 + l3 w^3 (w-basis), i.e. a0 = (l0, l2, 0),
 * a1 = (0, l3, 0). */
static void f12_mul_line(fp12* f, const fp2* l0, const fp2* l2, const fp2* l3) {
  fp12 l;
  memset(&l, 0, sizeof(l));
  l.c0.c0 = *l0;
  l.c0.c1 = *l2;
  l.c1.c1 = *l3;
  f12_mul(f, f, &l);
}
/* Homogeneous projective doubling on E2 with the tangent line at (xp, yp):
 * line (scaled by subfield factors) = -I + (-3 X^2 xp) w^2 + (2YZ yp) w^3
 * with I = 3b'Z^2 - Y^2. */
static void dbl_step(fp2* X, fp2* Y, fp2* Z, fp12* f, const fp* xp, const fp* yp) {
  fp2 a, b, c, e, ff, g, h, i, j, t, l0, l2, l3;
  f2_mul(&a, X, Y);
  f2_mul_fp(&a, &a, &INV2);          /* XY/2 */
  f2_sqr(&b, Y);                     /* B = Y^2 */
  f2_sqr(&c, Z);                     /* C = Z^2 */
  f2_mul(&e, &c, &B2x3);             /* E = 3b'C */
  f2_dbl(&ff, &e); f2_add(&ff, &ff, &e); /* F = 3E */
  f2_add(&g, &b, &ff); f2_mul_fp(&g, &g, &INV2); /* G = (B+F)/2 */
  f2_add(&h, Y, Z); f2_sqr(&h, &h); f2_sub(&h, &h, &b); f2_sub(&h, &h, &c); /* H = 2YZ */
  f2_sub(&i, &e, &b);                /* I = E - B */
  f2_sqr(&j, X);                     /* J = X^2 */
  /* line */
  f2_neg(&l0, &i);
  f2_dbl(&l2, &j); f2_add(&l2, &l2, &j); f2_mul_fp(&l2, &l2, xp); f2_neg(&l2, &l2);
  f2_mul_fp(&l3, &h, yp);
  /* point */
  f2_sub(&t, &b, &ff); f2_mul(X, &a, &t);
  f2_sqr(&t, &e); f2_dbl(&l0, &t); f2_add(&t, &t, &l0); /* 3E^2 */
  f2_sqr(Y, &g); f2_sub(Y, Y, &t);
  f2_mul(Z, &b, &h);
  f2_neg(&l0, &i);
  f12_mul_line(f, &l0, &l2, &l3);
}
/* Mixed addition T + Q (Q affine) with the chord line at (xp, yp):
 * u = yq Z - Y, v = xq Z - X; line = (u xq - v yq) + (-u xp) w^2 + (v yp) w^3 */
static void add_step(fp2* X, fp2* Y, fp2* Z, fp12* f, const fp2* xq, const fp2* yq, const fp* xp, const fp* yp) {
  fp2 u, v, uu, vv, vvv, r, a, t, l0, l2, l3;
  f2_mul(&u, yq, Z); f2_sub(&u, &u, Y);
  f2_mul(&v, xq, Z); f2_sub(&v, &v, X);
  f2_mul(&l0, &u, xq); f2_mul(&t, &v, yq); f2_sub(&l0, &l0, &t);
  f2_mul_fp(&l2, &u, xp); f2_neg(&l2, &l2);
  f2_mul_fp(&l3, &v, yp);
  f2_sqr(&uu, &u); f2_sqr(&vv, &v); f2_mul(&vvv, &v, &vv);
  f2_mul(&r, &vv, X);
  f2_mul(&a, &uu, Z); f2_sub(&a, &a, &vvv); f2_sub(&a, &a, &r); f2_sub(&a, &a, &r);
  f2_mul(&t, &vvv, Y);
  f2_sub(&r, &r, &a); f2_mul(Y, &u, &r); f2_sub(Y, Y, &t);
  f2_mul(X, &v, &a);
  f2_mul(Z, &vvv, Z);
  f12_mul_line(f, &l0, &l2, &l3);
}
/* f *= f_{|x|,Q}(P) for affine P, Q (both finite); conjugation for x < 0 is
 * applied by the caller once on the product. */
static void miller_acc(fp12* f, const fp* xp, const fp* yp, const fp2* xq, const fp2* yq) {
  fp2 X = *xq, Y = *yq, Z = F2_ONE;
  fp12 g = F12_ONE;
  for (int b = 62; b >= 0; b--) {
    f12_sqr(&g, &g);
    dbl_step(&X, &Y, &Z, &g, xp, yp);
    if ((X_ABS >> b) & 1) add_step(&X, &Y, &Z, &g, xq, yq, xp, yp);
  }
  f12_mul(f, f, &g);
}
/* shared-squaring multi-Miller loop over n pairs (affine, finite) */
typedef struct { fp xp, yp; fp2 xq, yq; } pair_aff;
static void multi_miller(fp12* out, const pair_aff* ps, int n) {
  fp2* T = (fp2*)malloc(sizeof(fp2) * 3 * (size_t)(n ? n : 1));
  for (int k = 0; k < n; k++) { T[3 * k] = ps[k].xq; T[3 * k + 1] = ps[k].yq; T[3 * k + 2] = F2_ONE; }
  fp12 g = F12_ONE;
  for (int b = 62; b >= 0; b--) {
    f12_sqr(&g, &g);
    for (int k = 0; k < n; k++) dbl_step(&T[3 * k], &T[3 * k + 1], &T[3 * k + 2], &g, &ps[k].xp, &ps[k].yp);
    if ((X_ABS >> b) & 1)
      for (int k = 0; k < n; k++)
        add_step(&T[3 * k], &T[3 * k + 1], &T[3 * k + 2], &g, &ps[k].xq, &ps[k].yq, &ps[k].xp, &ps[k].yp);
  }
  free(T);
  f12_conj(out, &g);
}
/* a^|x| then conjugate: a^x for a in the cyclotomic subgroup */
static void f12_pow_x(fp12* r, const fp12* a) {
  fp12 acc = *a;
  for (int b = 62; b >= 0; b--) {
    f12_sqr(&acc, &acc);
    if ((X_ABS >> b) & 1) f12_mul(&acc, &acc, a);
  }
  f12_conj(r, &acc);
}
/* f^(3 (p^12-1)/r) */
static void final_exp(fp12* r, const fp12* f) {
  fp12 t, a, b, c, d;
  f12_inv(&t, f);
  f12_conj(&a, f);
  f12_mul(&a, &a, &t);        /* f^(p^6-1) */
  f12_frob2(&t, &a);
  f12_mul(&a, &t, &a);        /* ^(p^2+1): now in the cyclotomic subgroup */
  /* hard part: (x-1)^2 (x+p) (x^2+p^2-1) + 3 */
  f12_pow_x(&b, &a); f12_conj(&t, &a); f12_mul(&b, &b, &t);  /* a^(x-1) */
  f12_pow_x(&c, &b); f12_conj(&t, &b); f12_mul(&b, &c, &t);  /* a^((x-1)^2) */
  f12_pow_x(&c, &b); f12_frob(&t, &b); f12_mul(&b, &c, &t);  /* ^(x+p) */
  f12_pow_x(&c, &b); f12_pow_x(&c, &c);                        /* b^(x^2) */
  f12_frob2(&t, &b); f12_mul(&c, &c, &t);
  f12_conj(&t, &b); f12_mul(&c, &c, &t);                       /* ^(x^2+p^2-1) */
  f12_sqr(&d, &a); f12_mul(&d, &d, &a);                        /* a^3 */
  f12_mul(r, &c, &d);
}

/* ------------------------------------------------------------------------- */
/* init                                                                      */
/* ------------------------------------------------------------------------- */
static pthread_once_t ONCE = PTHREAD_ONCE_INIT;
static void shr(u64* r, const u64* a, int s) {
  for (int i = 0; i < 6; i++) r[i] = (a[i] >> s) | (i < 5 && s ? a[i + 1] << (64 - s) : 0);
}
static void do_init(void) {
  u64 inv = 1;
  for (int i = 0; i < 7; i++) inv *= 2 - P.l[0] * inv;
  PINV = (u64)0 - inv;
  /* R mod p by doubling 1, then R^2 = R * 2^384 by more doublings (plain adds) */
  fp one = FP_ZERO;
  one.l[0] = 1;
  fp x = one;
  for (int i = 0; i < 384; i++) fp_add(&x, &x, &x);
  R1 = x;
  for (int i = 0; i < 384; i++) fp_add(&x, &x, &x);
  R2 = x;
  /* exponents */
  u64 t[6];
  memcpy(E_PM2, P.l, 48);
  E_PM2[0] -= 2;
  memcpy(t, P.l, 48);
  t[0] += 1; /* p+1 has no carry out of limb 0 (p ends in ...aaab) */
  shr(E_SQRT, t, 2);
  memcpy(t, P.l, 48);
  t[0] -= 1;
  shr(E_LEG, t, 1);
  F2_ZERO.c0 = FP_ZERO; F2_ZERO.c1 = FP_ZERO;
  F2_ONE.c0 = R1; F2_ONE.c1 = FP_ZERO;
  memset(&F12_ONE, 0, sizeof(F12_ONE));
  F12_ONE.c0.c0 = F2_ONE;
  fp two;
  fp_from_u64(&two, 2);
  fp_inv(&INV2, &two);
  fp_from_u64(&B1, 4);
  f2_from_u64(&B2, 4, 4);
  f2_from_u64(&B2x3, 12, 12);
  /* 2^384 mod p: R1 is 2^384 mod p in plain form; to Montgomery */
  fp_to_mont(&TWO384, R1.l);
  /* Frobenius constants gamma_k = xi^(k(p-1)/6) */
  fp2 xi;
  f2_from_u64(&xi, 1, 1);
  u64 e6[6];
  memcpy(t, P.l, 48);
  t[0] -= 1;
  /* (p-1)/6: divide by 2 then by 3 (p-1 is divisible by 6) */
  shr(e6, t, 1);
  {
    u128 rem = 0;
    for (int i = 5; i >= 0; i--) {
      u128 cur = (rem << 64) | e6[i];
      e6[i] = (u64)(cur / 3);
      rem = cur % 3;
    }
  }
  fp2 g1;
  f2_pow_big(&g1, &xi, e6, 6);
  GAMMA1[0] = F2_ONE;
  for (int k = 1; k < 6; k++) f2_mul(&GAMMA1[k], &GAMMA1[k - 1], &g1);
  /* p^2-Frobenius: (c w^k)^(p^2) = c * gamma_k * conj(gamma_k) (c in Fp2 fixed by p^2) */
  for (int k = 0; k < 6; k++) {
    fp2 cj;
    f2_conj(&cj, &GAMMA1[k]);
    f2_mul(&GAMMA2[k], &GAMMA1[k], &cj);
  }
  /* psi constants: 1/xi^((p-1)/3) = 1/gamma_2, 1/xi^((p-1)/2) = 1/gamma_3 */
  f2_inv(&PSI_CX, &GAMMA1[2]);
  f2_inv(&PSI_CY, &GAMMA1[3]);
  /* generators */
  static const uint8_t g1b[48] = {0x97, 0xf1, 0xd3, 0xa7, 0x31, 0x97, 0xd7, 0x94, 0x26, 0x95, 0x63, 0x8c,
                                  0x4f, 0xa9, 0xac, 0x0f, 0xc3, 0x68, 0x8c, 0x4f, 0x97, 0x74, 0xb9, 0x05,
                                  0xa1, 0x4e, 0x3a, 0x3f, 0x17, 0x1b, 0xac, 0x58, 0x6c, 0x55, 0xe8, 0x3f,
                                  0xf9, 0x7a, 0x1a, 0xef, 0xfb, 0x3a, 0xf0, 0x0a, 0xdb, 0x22, 0xc6, 0xbb};
  static const uint8_t g2b[96] = {
      0x93, 0xe0, 0x2b, 0x60, 0x52, 0x71, 0x9f, 0x60, 0x7d, 0xac, 0xd3, 0xa0, 0x88, 0x27, 0x4f, 0x65,
      0x59, 0x6b, 0xd0, 0xd0, 0x99, 0x20, 0xb6, 0x1a, 0xb5, 0xda, 0x61, 0xbb, 0xdc, 0x7f, 0x50, 0x49,
      0x33, 0x4c, 0xf1, 0x12, 0x13, 0x94, 0x5d, 0x57, 0xe5, 0xac, 0x7d, 0x05, 0x5d, 0x04, 0x2b, 0x7e,
      0x02, 0x4a, 0xa2, 0xb2, 0xf0, 0x8f, 0x0a, 0x91, 0x26, 0x08, 0x05, 0x27, 0x2d, 0xc5, 0x10, 0x51,
      0xc6, 0xe4, 0x7a, 0xd4, 0xfa, 0x40, 0x3b, 0x02, 0xb4, 0x51, 0x0b, 0x64, 0x7a, 0xe3, 0xd1, 0x77,
      0x0b, 0xac, 0x03, 0x26, 0xa8, 0x05, 0xbb, 0xef, 0xd4, 0x80, 0x56, 0xc8, 0xc1, 0x21, 0xbd, 0xb8};
  g1_decompress(&G1_GEN, g1b);
  g1_neg(&G1_NEG_GEN, &G1_GEN);
  g2_decompress(&G2_GEN, g2b);
  /* SSWU constants on E2': A' = 240 i, B' = 1012 (1 + i), Z = -(2 + i) */
  f2_from_u64(&SSWU_A, 0, 240);
  f2_from_u64(&SSWU_B, 1012, 1012);
  f2_from_u64(&SSWU_Z, 2, 1);
  f2_neg(&SSWU_Z, &SSWU_Z);
  fp2 ai, zai;
  f2_inv(&ai, &SSWU_A);
  f2_mul(&SSWU_MBA, &SSWU_B, &ai);
  f2_neg(&SSWU_MBA, &SSWU_MBA);
  f2_mul(&zai, &SSWU_Z, &SSWU_A);
  f2_inv(&zai, &zai);
  f2_mul(&SSWU_BZA, &SSWU_B, &zai);
  /* 3-isogeny constants (RFC 9380 App. E.3) */
  static const char* const K1 =
      "5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6";
  static const char* const K2 =
      "11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a";
  static const char* const K3 =
      "11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e";
  static const char* const K4 =
      "8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d";
  static const char* const K5 =
      "171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1";
  static const char* const K6 =
      "1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706";
  static const char* const K7 =
      "5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be";
  static const char* const K8 =
      "11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c";
  static const char* const K9 =
      "8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f";
  static const char* const K10 =
      "124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10";
  memset(ISO_XNUM, 0, sizeof(ISO_XNUM));
  fp_from_hex(&ISO_XNUM[0].c0, K1); fp_from_hex(&ISO_XNUM[0].c1, K1);
  fp_from_hex(&ISO_XNUM[1].c1, K2);
  fp_from_hex(&ISO_XNUM[2].c0, K3); fp_from_hex(&ISO_XNUM[2].c1, K4);
  fp_from_hex(&ISO_XNUM[3].c0, K5);
  memset(ISO_YNUM, 0, sizeof(ISO_YNUM));
  fp_from_hex(&ISO_YNUM[0].c0, K6); fp_from_hex(&ISO_YNUM[0].c1, K6);
  fp_from_hex(&ISO_YNUM[1].c1, K7);
  fp_from_hex(&ISO_YNUM[2].c0, K8); fp_from_hex(&ISO_YNUM[2].c1, K9);
  fp_from_hex(&ISO_YNUM[3].c0, K10);
  fp m;
  /* XDEN = [(0,-72), (12,-12), (1,0)] ; YDEN = [(-432,-432), (0,-216), (18,-18), (1,0)] */
  memset(ISO_XDEN, 0, sizeof(ISO_XDEN));
  fp_from_u64(&m, 72); fp_neg(&ISO_XDEN[0].c1, &m);
  fp_from_u64(&ISO_XDEN[1].c0, 12); fp_from_u64(&m, 12); fp_neg(&ISO_XDEN[1].c1, &m);
  ISO_XDEN[2].c0 = R1;
  memset(ISO_YDEN, 0, sizeof(ISO_YDEN));
  fp_from_u64(&m, 432); fp_neg(&ISO_YDEN[0].c0, &m); ISO_YDEN[0].c1 = ISO_YDEN[0].c0;
  fp_from_u64(&m, 216); fp_neg(&ISO_YDEN[1].c1, &m);
  fp_from_u64(&ISO_YDEN[2].c0, 18); fp_from_u64(&m, 18); fp_neg(&ISO_YDEN[2].c1, &m);
  ISO_YDEN[3].c0 = R1;
}
static void init(void) { pthread_once(&ONCE, do_init); }

/* ------------------------------------------------------------------------- */
/* BLS POP ciphersuite with the wrapper semantics (E/utils/bls.py)           */
/* ------------------------------------------------------------------------- */
static int sk_from_be32(u64* k, const uint8_t* sk) {
  for (int i = 0; i < 4; i++) {
    u64 v = 0;
    for (int j = 0; j < 8; j++) v = (v << 8) | sk[(3 - i) * 8 + j];
    k[i] = v;
  }
  int zero = (k[0] | k[1] | k[2] | k[3]) == 0;
  for (int i = 3; i >= 0; i--) {
    if (k[i] < R_LIMBS[i]) return !zero;
    if (k[i] > R_LIMBS[i]) return 0;
  }
  return 0; /* == r */
}
/* KeyValidate: decode OK, not infinity, in G1 (E/utils/bls.py:395-397) */
static int key_validate_pt(g1j* out, const uint8_t* pk) {
  if (!g1_decompress(out, pk)) return 0;
  if (g1_is_inf(out)) return 0;
  return g1_in_subgroup(out);
}
static int sig_decode(g2j* out, const uint8_t* sig) {
  if (!g2_decompress(out, sig)) return 0;
  return g2_in_subgroup(out);
}
/* e(pk, H(m)) * e(-G1, sig) == 1 ; pk finite; sig may be infinity */
static int core_verify_pt(const g1j* pk, const uint8_t* msg, size_t mlen, const g2j* sig) {
  g2j h;
  hash_to_g2(&h, msg, mlen, DST_POP, DST_POP_LEN);
  pair_aff ps[2];
  int n = 0;
  if (!g2_is_inf(&h)) {
    g1_affine(&ps[n].xp, &ps[n].yp, pk);
    g2_affine(&ps[n].xq, &ps[n].yq, &h);
    n++;
  }
  if (!g2_is_inf(sig)) {
    g1_affine(&ps[n].xp, &ps[n].yp, &G1_NEG_GEN);
    g2_affine(&ps[n].xq, &ps[n].yq, sig);
    n++;
  }
  fp12 f, e;
  multi_miller(&f, ps, n);
  final_exp(&e, &f);
  return f12_eq(&e, &F12_ONE);
}

int oc_key_validate(const uint8_t* pk48) {
  init();
  g1j p;
  return key_validate_pt(&p, pk48);
}
int oc_verify(const uint8_t* pk48, const uint8_t* msg, size_t mlen, const uint8_t* sig96) {
  init();
  g1j pk;
  g2j s;
  if (!key_validate_pt(&pk, pk48)) return 0;
  if (!sig_decode(&s, sig96)) return 0;
  return core_verify_pt(&pk, msg, mlen, &s);
}
int oc_fast_aggregate_verify(const uint8_t* pks48, size_t n, const uint8_t* msg, size_t mlen, const uint8_t* sig96) {
  init();
  if (n == 0) return 0;
  g1j agg, p;
  memset(&agg, 0, sizeof(agg));
  agg.x = R1; agg.y = R1;
  for (size_t i = 0; i < n; i++) {
    if (!key_validate_pt(&p, pks48 + 48 * i)) return 0;
    g1_add(&agg, &agg, &p);
  }
  if (g1_is_inf(&agg)) return 0;
  g2j s;
  if (!sig_decode(&s, sig96)) return 0;
  return core_verify_pt(&agg, msg, mlen, &s);
}
int oc_aggregate_verify(const uint8_t* pks48, size_t n, const uint8_t* msgs, const size_t* lens, const uint8_t* sig96) {
  init();
  if (n == 0) return 0;
  pair_aff* ps = (pair_aff*)malloc(sizeof(pair_aff) * (n + 1));
  size_t k = 0, off = 0;
  int ok = 1;
  for (size_t i = 0; i < n && ok; i++) {
    g1j p;
    g2j h;
    if (!key_validate_pt(&p, pks48 + 48 * i)) { ok = 0; break; }
    hash_to_g2(&h, msgs + off, lens[i], DST_POP, DST_POP_LEN);
    off += lens[i];
    if (g2_is_inf(&h)) continue;
    g1_affine(&ps[k].xp, &ps[k].yp, &p);
    g2_affine(&ps[k].xq, &ps[k].yq, &h);
    k++;
  }
  g2j s;
  if (ok && !sig_decode(&s, sig96)) ok = 0;
  if (ok) {
    if (!g2_is_inf(&s)) {
      g1_affine(&ps[k].xp, &ps[k].yp, &G1_NEG_GEN);
      g2_affine(&ps[k].xq, &ps[k].yq, &s);
      k++;
    }
    fp12 f, e;
    multi_miller(&f, ps, (int)k);
    final_exp(&e, &f);
    ok = f12_eq(&e, &F12_ONE);
  }
  free(ps);
  return ok;
}
/* 1 and out96, or 0 (empty / undecodable / non-G2 signature: the shim raises) */
int oc_aggregate(const uint8_t* sigs96, size_t n, uint8_t* out96) {
  init();
  if (n == 0) return 0;
  g2j agg, s;
  memset(&agg, 0, sizeof(agg));
  agg.x = F2_ONE; agg.y = F2_ONE;
  for (size_t i = 0; i < n; i++) {
    if (!sig_decode(&s, sigs96 + 96 * i)) return 0;
    g2_add(&agg, &agg, &s);
  }
  g2_compress(out96, &agg);
  return 1;
}
int oc_aggregate_pks(const uint8_t* pks48, size_t n, uint8_t* out48) {
  init();
  if (n == 0) return 0;
  g1j agg, p;
  memset(&agg, 0, sizeof(agg));
  agg.x = R1; agg.y = R1;
  for (size_t i = 0; i < n; i++) {
    if (!key_validate_pt(&p, pks48 + 48 * i)) return 0;
    g1_add(&agg, &agg, &p);
  }
  g1_compress(out48, &agg);
  return 1;
}
int oc_sign(const uint8_t* sk32, const uint8_t* msg, size_t mlen, uint8_t* out96) {
  init();
  u64 k[4];
  if (!sk_from_be32(k, sk32)) return 0;
  g2j h, s;
  hash_to_g2(&h, msg, mlen, DST_POP, DST_POP_LEN);
  g2_mul_big(&s, &h, k, 4);
  g2_compress(out96, &s);
  return 1;
}
int oc_sk_to_pk(const uint8_t* sk32, uint8_t* out48) {
  init();
  u64 k[4];
  if (!sk_from_be32(k, sk32)) return 0;
  g1j p;
  g1_mul_big(&p, &G1_GEN, k, 4);
  g1_compress(out48, &p);
  return 1;
}
int oc_hash_to_g2(const uint8_t* msg, size_t mlen, const uint8_t* dst, size_t dlen, uint8_t* out96) {
  init();
  g2j h;
  if (!hash_to_g2(&h, msg, mlen, dst, dlen)) return 0;
  g2_compress(out96, &h);
  return 1;
}
/* Decode (no checks beyond the encoding) and run the G2 subgroup test two
 * ways; for cross-checking the psi test.  Returns -1 on decode failure,
 * else (psi_test << 1) | r_test. */
int oc_g2_subgroup_both(const uint8_t* sig96) {
  init();
  g2j s, t;
  if (!g2_decompress(&s, sig96)) return -1;
  g2_mul_big(&t, &s, R_LIMBS, 4);
  return (g2_in_subgroup(&s) << 1) | g2_is_inf(&t);
}
/* e(P, Q) final-exponentiated (cubed, see header) as 576 bytes (w-basis,
 * each coefficient c0 || c1 big-endian) -- for bilinearity tests. */
int oc_pairing(const uint8_t* pk48, const uint8_t* sig96, uint8_t* out576) {
  init();
  g1j p;
  g2j q;
  if (!g1_decompress(&p, pk48) || !g2_decompress(&q, sig96)) return 0;
  fp12 f = F12_ONE, e;
  if (!g1_is_inf(&p) && !g2_is_inf(&q)) {
    pair_aff pa;
    g1_affine(&pa.xp, &pa.yp, &p);
    g2_affine(&pa.xq, &pa.yq, &q);
    multi_miller(&f, &pa, 1);
  }
  final_exp(&e, &f);
  for (int k = 0; k < 6; k++) {
    fp2* c = f12_coef(&e, k);
    u64 l[6];
    fp_from_mont(l, &c->c0);
    limbs_to_be48(out576 + 96 * k, l);
    fp_from_mont(l, &c->c1);
    limbs_to_be48(out576 + 96 * k + 48, l);
  }
  return 1;
}

/* ------------------------------------------------------------------------- */
/* CPU baseline: registry-resident FastAggregateVerify batches on threads    */
/* ------------------------------------------------------------------------- */
/* Registry: affine keys, 96 bytes each (x || y big-endian, canonical),
 * already decoded and KeyValidated (registry load is not
 * part of the per-verification metric). */
int oc_registry_generate(u64 first_sk, size_t n, uint8_t* out96) {
  init();
  g1j p, step = G1_GEN;
  g1_mul_u64(&p, &G1_GEN, first_sk);
  for (size_t i = 0; i < n; i++) {
    fp x, y;
    u64 l[6];
    g1_affine(&x, &y, &p);
    fp_from_mont(l, &x);
    limbs_to_be48(out96 + 96 * i, l);
    fp_from_mont(l, &y);
    limbs_to_be48(out96 + 96 * i + 48, l);
    g1_add(&p, &p, &step);
  }
  return 1;
}
/* Jacobian + affine (z2 = 1) addition, madd-2007-bl, with the doubling /
 * inverse special cases. */
static void g1_add_aff(g1j* r, const g1j* p, const fp* x2, const fp* y2) {
  if (g1_is_inf(p)) { r->x = *x2; r->y = *y2; r->z = R1; return; }
  fp z1z1, u2, s2, h, hh, i, j, rr, v, t, x3, y3, z3;
  fp_sqr(&z1z1, &p->z);
  fp_mul(&u2, x2, &z1z1);
  fp_mul(&s2, y2, &p->z);
  fp_mul(&s2, &s2, &z1z1);
  fp_sub(&h, &u2, &p->x);
  fp_sub(&rr, &s2, &p->y);
  if (fp_is_zero(&h)) {
    if (fp_is_zero(&rr)) { g1_dbl(r, p); return; }
    memset(r, 0, sizeof(*r)); r->x = R1; r->y = R1; return;
  }
  fp_sqr(&hh, &h);
  fp_dbl(&i, &hh); fp_dbl(&i, &i);
  fp_mul(&j, &h, &i);
  fp_dbl(&rr, &rr);
  fp_mul(&v, &p->x, &i);
  fp_sqr(&x3, &rr); fp_sub(&x3, &x3, &j); fp_sub(&x3, &x3, &v); fp_sub(&x3, &x3, &v);
  fp_sub(&t, &v, &x3); fp_mul(&y3, &rr, &t); fp_mul(&t, &p->y, &j); fp_dbl(&t, &t); fp_sub(&y3, &y3, &t);
  fp_add(&z3, &p->z, &h); fp_sqr(&z3, &z3); fp_sub(&z3, &z3, &z1z1); fp_sub(&z3, &z3, &hh);
  r->x = x3; r->y = y3; r->z = z3;
}
static void reg_point(g1j* p, const uint8_t* r96) {
  u64 l[6];
  limbs_from_be48(l, r96);
  fp_to_mont(&p->x, l);
  limbs_from_be48(l, r96 + 48);
  fp_to_mont(&p->y, l);
  p->z = R1;
}

typedef struct {
  const uint8_t* reg;
  const uint32_t* idx;
  const uint64_t* offs;
  const uint8_t* msgs;
  const uint8_t* sigs;
  uint8_t* out;
  size_t lo, hi;
  int mode; /* 0 per call, 1 RLC */
  const uint8_t* seed;
  fp12 f;   /* RLC: product of this thread's Miller values */
  g2j S;    /* RLC: sum r_i sigma_i */
  int bad;
} fav_job;

static u64 rlc_scalar(const uint8_t* seed, size_t i, const uint8_t* msg, const uint8_t* sig) {
  sha256 s;
  uint8_t d[32], ib[8];
  for (int k = 0; k < 8; k++) ib[k] = (uint8_t)(i >> (8 * k));
  sha_init(&s);
  sha_update(&s, seed, 32);
  sha_update(&s, ib, 8);
  sha_update(&s, msg, 32);
  sha_update(&s, sig, 96);
  sha_final(&s, d);
  u64 r = 0;
  for (int k = 0; k < 8; k++) r |= (u64)d[k] << (8 * k);
  return r | 1;
}

static void* fav_worker(void* arg) {
  fav_job* j = (fav_job*)arg;
  j->f = F12_ONE;
  memset(&j->S, 0, sizeof(j->S));
  j->S.x = F2_ONE; j->S.y = F2_ONE;
  j->bad = 0;
  for (size_t b = j->lo; b < j->hi; b++) {
    g1j apk, p;
    memset(&apk, 0, sizeof(apk));
    apk.x = R1; apk.y = R1;
    for (uint64_t k = j->offs[b]; k < j->offs[b + 1]; k++) {
      reg_point(&p, j->reg + 96 * (size_t)j->idx[k]);
      g1_add_aff(&apk, &apk, &p.x, &p.y);
    }
    const uint8_t* msg = j->msgs + 32 * b;
    const uint8_t* sig = j->sigs + 96 * b;
    g2j s;
    int ok = j->offs[b + 1] > j->offs[b] && !g1_is_inf(&apk) && sig_decode(&s, sig);
    if (ok && j->mode == 0) {
      ok = core_verify_pt(&apk, msg, 32, &s);
    } else if (ok) {
      u64 r = rlc_scalar(j->seed, b, msg, sig);
      g1j rp;
      g2j rs, h;
      g1_mul_u64(&rp, &apk, r);
      g2_mul_u64(&rs, &s, r);
      g2_add(&j->S, &j->S, &rs);
      hash_to_g2(&h, msg, 32, DST_POP, DST_POP_LEN);
      if (!g2_is_inf(&h)) {
        pair_aff pa;
        g1_affine(&pa.xp, &pa.yp, &rp);
        g2_affine(&pa.xq, &pa.yq, &h);
        fp12 m;
        multi_miller(&m, &pa, 1);
        f12_mul(&j->f, &j->f, &m);
      }
    }
    if (!ok) j->bad = 1;
    j->out[b] = (uint8_t)ok;
  }
  return NULL;
}

/* Synthetic signatures for the baseline sample: out96[b] = sk_b * H(msg_b),
 * sks32 big-endian, msgs 32 bytes each; `threads` worker threads. */
typedef struct { const uint8_t *sks, *msgs; uint8_t* out; size_t lo, hi; int ok; } sign_job;
static void* sign_worker(void* arg) {
  sign_job* j = (sign_job*)arg;
  j->ok = 1;
  for (size_t b = j->lo; b < j->hi; b++) {
    u64 k[4];
    if (!sk_from_be32(k, j->sks + 32 * b)) { j->ok = 0; continue; }
    g2j h, s;
    hash_to_g2(&h, j->msgs + 32 * b, 32, DST_POP, DST_POP_LEN);
    g2_mul_big(&s, &h, k, 4);
    g2_compress(j->out + 96 * b, &s);
  }
  return NULL;
}
int oc_sign_batch(const uint8_t* sks32, const uint8_t* msgs32, size_t B, int threads, uint8_t* out96) {
  init();
  if (threads < 1) threads = 1;
  sign_job* jobs = (sign_job*)calloc((size_t)threads, sizeof(sign_job));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; t++) {
    jobs[t] = (sign_job){sks32, msgs32, out96, B * t / threads, B * (t + 1) / threads, 1};
    pthread_create(&th[t], NULL, sign_worker, &jobs[t]);
  }
  int ok = 1;
  for (int t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    ok &= jobs[t].ok;
  }
  free(jobs);
  free(th);
  return ok;
}

/* B registry-indexed FastAggregateVerify calls on `threads` threads.
 * mode 0: per call (each its own final exponentiation, reference-equivalent);
 * mode 1: one random-linear-combination batch check (per-call re-check of the
 * batch when it fails).  Returns 1 (all verdicts written) or 0. */
int oc_fav_batch_resident(const uint8_t* reg96, const uint32_t* idx, const uint64_t* offs, size_t B,
                          const uint8_t* msgs32, const uint8_t* sigs96, const uint8_t* seed32, int mode,
                          int threads, uint8_t* out) {
  init();
  if (threads < 1) threads = 1;
  if ((size_t)threads > B) threads = B ? (int)B : 1;
  fav_job* jobs = (fav_job*)calloc((size_t)threads, sizeof(fav_job));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; t++) {
    jobs[t] = (fav_job){reg96, idx, offs, msgs32, sigs96, out, B * t / threads, B * (t + 1) / threads, mode, seed32};
    pthread_create(&th[t], NULL, fav_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  if (mode == 1) {
    fp12 f = F12_ONE;
    g2j S;
    memset(&S, 0, sizeof(S));
    S.x = F2_ONE; S.y = F2_ONE;
    int bad = 0;
    for (int t = 0; t < threads; t++) {
      f12_mul(&f, &f, &jobs[t].f);
      g2_add(&S, &S, &jobs[t].S);
      bad |= jobs[t].bad;
    }
    int ok = 0;
    if (!g2_is_inf(&S)) {
      pair_aff pa;
      g1_affine(&pa.xp, &pa.yp, &G1_NEG_GEN);
      g2_affine(&pa.xq, &pa.yq, &S);
      fp12 m, e;
      multi_miller(&m, &pa, 1);
      f12_mul(&f, &f, &m);
      final_exp(&e, &f);
      ok = f12_eq(&e, &F12_ONE);
    }
    (void)bad;
    if (!ok) { /* batch failed: per-call re-check (bisection is a GPU-side optimisation) */
      for (int t = 0; t < threads; t++) {
        jobs[t].mode = 0;
        pthread_create(&th[t], NULL, fav_worker, &jobs[t]);
      }
      for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    }
  }
  free(jobs);
  free(th);
  return 1;
}
