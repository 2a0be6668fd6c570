// TEST HARNESS ONLY: ASan + UBSan driver for the host build of the device headers (tests/hostcheck/*.cpp, the
// same bls_*.h the gfx950 kernels compile).  SURVEY.md §5 ("Race detection / sanitizers").  The Python suite
// checks these functions' values against the oracle; this driver runs them again with every out-of-bounds
// access, overflowing shift, misaligned load or signed overflow turned into an abort, and checks them against
// algebraic identities (no oracle needed):
//   Fp / Fp2 / Fp12: commutativity, a * a^-1 = 1, squaring = product, Frobenius orders, the inline tower
//     (bls_tower_inline.h) against the out-of-line one, square roots;
//   curve: generator decoding, subgroup checks, key / signature validation and their rejections;
//   pairing: FE(ML([2]P, Q)) = FE(ML(P, Q))^2, and the lane-parallel FE check (bls_fe.h) on e([2]P,Q) e(P,Q)^-2;
//   hashing and signatures: hash_to_G2 lands in G2, sign / verify through core_verify, lane SSWU = reference SSWU;
//   digit form (bls_fq*.h, built with its column checks): gather split invariance, the [|x|] chains against the
//     packed ones, the digit-form G1 scalar chain against the packed one.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

extern "C" {
void hc_f2mul_i(const uint8_t* a, const uint8_t* b, uint8_t* o);
void hc_f12sqr_i(const uint8_t* a, uint8_t* o);
void hc_f12line_i(const uint8_t* f, const uint8_t* l0, const uint8_t* l2, const uint8_t* l3, uint8_t* o);
void hc_fp_mul(const uint8_t* a, const uint8_t* b, uint8_t* o);
void hc_fp_add(const uint8_t* a, const uint8_t* b, uint8_t* o);
void hc_fp_sub(const uint8_t* a, const uint8_t* b, uint8_t* o);
void hc_fp_inv(const uint8_t* a, uint8_t* o);
void hc_fp_inv_sg(const uint8_t* a, uint8_t* o);
void hc_fp_sqr(const uint8_t* a, uint8_t* o);
int hc_fp_is_square(const uint8_t* a);
void hc_fp_pow_w3(const uint8_t* a, const uint32_t* e, int nbits, uint8_t* o);
void hc_fp2_mul(const uint8_t* a, const uint8_t* b, uint8_t* o);
void hc_fp2_sqr(const uint8_t* a, uint8_t* o);
void hc_fp2_inv(const uint8_t* a, uint8_t* o);
int hc_fp2_sqrt(const uint8_t* a, uint8_t* o);
int hc_fp2_sqrt_lane(const uint8_t* a, uint8_t* o);
void hc_fp12_mul(const uint8_t* a, const uint8_t* b, uint8_t* o);
void hc_fp12_sqr(const uint8_t* a, uint8_t* o);
void hc_fp12_inv(const uint8_t* a, uint8_t* o);
void hc_fp12_frob1(const uint8_t* a, uint8_t* o);
void hc_fp12_frob2(const uint8_t* a, uint8_t* o);
void hc_fp12_mul_line(const uint8_t* f, const uint8_t* l0, const uint8_t* l2, const uint8_t* l3, uint8_t* o);
void hc_final_exp(const uint8_t* a, uint8_t* o);
void hc_miller_loop(const uint8_t* p, const uint8_t* q, uint8_t* o);
int hc_g1_decompress(const uint8_t* b, uint8_t* o);
int hc_g2_decompress(const uint8_t* b, uint8_t* o);
int hc_g2_decompress_lane(const uint8_t* b, uint8_t* o);
int hc_g1_in_subgroup(const uint8_t* p);
int hc_g2_in_subgroup(const uint8_t* q);
void hc_map_to_curve(const uint8_t* u, uint8_t* o);
void hc_map_to_curve_lane(const uint8_t* u, uint8_t* o);
void hc_hash_to_g2(const uint8_t* m, uint32_t ml, const uint8_t* d, uint32_t dl, uint8_t* o96);
int hc_key_validate(const uint8_t* pk);
int hc_sig_validate(const uint8_t* s);
int hc_core_verify(const uint8_t* pk, const uint8_t* m, uint32_t ml, const uint8_t* d, uint32_t dl, const uint8_t* sig);
void hc_g2_mul_u256(const uint8_t* q, const uint32_t* k, uint8_t* o96);
void hc_g1_mul_u256(const uint8_t* p, const uint32_t* k, uint8_t* o48);
int hc_j2_mul_xabs(const uint8_t* q, uint8_t* o);
int hc_fe_check(const uint8_t* f, int n, uint8_t* out);
void hc_fq_gather(const uint8_t* pts, uint32_t n, uint32_t split, uint8_t* o);
void hc_fq_g1_mul64(const uint8_t* p, uint64_t r, uint8_t* o);
int hc_fq_j2_mul_xabs(const uint8_t* q, uint8_t* o);
}

static int fails = 0;
#define CHECK(c)                                                                    \
  do {                                                                              \
    if (!(c)) {                                                                     \
      fprintf(stderr, "san_hostcheck: FAILED %s (line %d)\n", #c, __LINE__);        \
      fails++;                                                                      \
    }                                                                               \
  } while (0)

static uint64_t rs = 0x5eed5eed12345678ull;
static uint8_t rb() {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return (uint8_t)(rs >> 32);
}
// a random canonical Fp (top byte below p's 0x1a), big-endian
static void rfp(uint8_t* b) {
  for (int i = 0; i < 48; i++) b[i] = rb();
  b[0] &= 0x0f;
}
static void rfpn(uint8_t* b, int n) {
  for (int i = 0; i < n; i++) rfp(b + 48 * i);
}
static void unhex(uint8_t* out, const char* h) {
  for (size_t i = 0; 2 * i < strlen(h); i++) {
    unsigned v;
    sscanf(h + 2 * i, "%2x", &v);
    out[i] = (uint8_t)v;
  }
}
static bool eq(const uint8_t* a, const uint8_t* b, size_t n) { return memcmp(a, b, n) == 0; }
// hc_fp12_* layout (w-basis interleaved: c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2) -> hc_fe_check's tower order
// (c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2), 96 bytes per Fp2
static void to_tower(uint8_t* out, const uint8_t* in) {
  static const int src[6] = {0, 2, 4, 1, 3, 5};
  for (int k = 0; k < 6; k++) memcpy(out + 96 * k, in + 96 * src[k], 96);
}
static void one_fp(uint8_t* b) {
  memset(b, 0, 48);
  b[47] = 1;
}
static void one_fp12(uint8_t* b) {
  memset(b, 0, 576);
  b[47] = 1;
}
// p - 2 as little-endian u32 limbs (381 bits)
static const uint32_t PM2[12] = {0xffffaaa9u, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                                 0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};

static const char* G1_GEN =
    "97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb";
static const char* G2_GEN =
    "93e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e024aa2b2f08f0a"
    "91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8";
static const char DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";

int main() {
  uint8_t a[48], b[48], c[48], d[48], one[48];
  one_fp(one);
  // ---- Fp
  for (int it = 0; it < 20; it++) {
    rfp(a);
    rfp(b);
    hc_fp_mul(a, b, c);
    hc_fp_mul(b, a, d);
    CHECK(eq(c, d, 48));
    hc_fp_sqr(a, c);
    hc_fp_mul(a, a, d);
    CHECK(eq(c, d, 48));
    hc_fp_inv(a, c);
    hc_fp_mul(a, c, d);
    CHECK(eq(d, one, 48));
    hc_fp_inv_sg(a, d);
    CHECK(eq(c, d, 48));
    hc_fp_pow_w3(a, PM2, 381, d);
    CHECK(eq(c, d, 48));
    hc_fp_sub(a, b, c);
    hc_fp_add(c, b, d);
    CHECK(eq(a, d, 48));
    hc_fp_sqr(a, c);
    CHECK(hc_fp_is_square(c) == 1);
  }
  // ---- Fp2
  uint8_t a2[96], b2[96], c2[96], d2[96], e2[96];
  for (int it = 0; it < 10; it++) {
    rfpn(a2, 2);
    rfpn(b2, 2);
    hc_fp2_mul(a2, b2, c2);
    hc_f2mul_i(a2, b2, d2);
    CHECK(eq(c2, d2, 96));
    hc_fp2_mul(a2, a2, c2);
    hc_fp2_sqr(a2, d2);
    CHECK(eq(c2, d2, 96));
    hc_fp2_inv(a2, c2);
    hc_fp2_mul(a2, c2, d2);
    static const uint8_t zero48[48] = {0};
    CHECK(eq(d2, one, 48) && eq(d2 + 48, zero48, 48));
    hc_fp2_sqr(a2, c2);
    CHECK(hc_fp2_sqrt(c2, d2) == 1);
    hc_fp2_sqr(d2, e2);
    CHECK(eq(c2, e2, 96));
    CHECK(hc_fp2_sqrt_lane(c2, d2) == 1);
    hc_fp2_sqr(d2, e2);
    CHECK(eq(c2, e2, 96));
  }
  // ---- Fp12
  static uint8_t f[576], g[576], h[576], k[576], o12[576];
  one_fp12(o12);
  for (int it = 0; it < 3; it++) {
    rfpn(f, 12);
    rfpn(g, 12);
    hc_fp12_mul(f, g, h);
    hc_fp12_mul(g, f, k);
    CHECK(eq(h, k, 576));
    hc_fp12_sqr(f, h);
    hc_fp12_mul(f, f, k);
    CHECK(eq(h, k, 576));
    hc_f12sqr_i(f, k);
    CHECK(eq(h, k, 576));
    hc_fp12_inv(f, h);
    hc_fp12_mul(f, h, k);
    CHECK(eq(k, o12, 576));
    memcpy(h, f, 576);
    for (int i = 0; i < 12; i++) {
      hc_fp12_frob1(h, k);
      memcpy(h, k, 576);
    }
    CHECK(eq(h, f, 576));
    for (int i = 0; i < 6; i++) {
      hc_fp12_frob2(h, k);
      memcpy(h, k, 576);
    }
    CHECK(eq(h, f, 576));
    rfpn(a2, 2);
    rfpn(b2, 2);
    rfpn(c2, 2);
    hc_fp12_mul_line(f, a2, b2, c2, h);
    hc_f12line_i(f, a2, b2, c2, k);
    CHECK(eq(h, k, 576));
  }
  // ---- curve decoding and validation
  uint8_t g1c[48], g2c[96], P[96], Q[192], P2[96], s48[48], s96[96];
  unhex(g1c, G1_GEN);
  unhex(g2c, G2_GEN);
  CHECK(hc_g1_decompress(g1c, P) == 0);
  CHECK(hc_g2_decompress(g2c, Q) == 0);
  uint8_t Ql[192];
  CHECK(hc_g2_decompress_lane(g2c, Ql) == 0 && eq(Q, Ql, 192));
  CHECK(hc_g1_in_subgroup(P) == 1 && hc_g2_in_subgroup(Q) == 1);
  CHECK(hc_key_validate(g1c) == 1 && hc_sig_validate(g2c) == 1);
  memset(s48, 0, 48);
  s48[0] = 0xc0;
  CHECK(hc_key_validate(s48) == 0);
  s48[0] = 0x40;
  CHECK(hc_key_validate(s48) == 0);
  memset(s96, 0, 96);
  CHECK(hc_sig_validate(s96) == 0);
  s96[0] = 0xc0;
  s96[1] = 0x10;
  CHECK(hc_sig_validate(s96) == 0);
  // ---- pairing: e([2]P, Q) = e(P, Q)^2, and the lane-parallel FE check
  uint32_t two[8] = {2, 0, 0, 0, 0, 0, 0, 0};
  hc_g1_mul_u256(P, two, s48);
  CHECK(hc_g1_decompress(s48, P2) == 0);
  static uint8_t m1[576], m2[576], e1[576], e2b[576], fe2[1152], feo[576];
  hc_miller_loop(P, Q, m1);
  hc_miller_loop(P2, Q, m2);
  hc_final_exp(m1, e1);
  hc_final_exp(m2, e2b);
  hc_fp12_sqr(e1, h);
  CHECK(eq(h, e2b, 576));
  CHECK(!eq(e1, o12, 576));
  to_tower(fe2, m2);
  hc_fp12_sqr(m1, h);
  hc_fp12_inv(h, k);
  to_tower(fe2 + 576, k);
  CHECK(hc_fe_check(fe2, 2, feo) == 1);
  to_tower(k, m1);
  CHECK(hc_fe_check(k, 1, feo) == 0);
  // ---- hashing, SSWU, signatures
  uint8_t msg[32], hm[96], H[192], pk[48], sig[96];
  for (int i = 0; i < 32; i++) msg[i] = (uint8_t)(3 * i + 1);
  hc_hash_to_g2(msg, 32, (const uint8_t*)DST, sizeof DST - 1, hm);
  CHECK(hc_g2_decompress(hm, H) == 0 && hc_g2_in_subgroup(H) == 1);
  uint32_t sk[8] = {0x1234567u, 0x89abcdefu, 7, 0, 0, 0, 0, 0};
  hc_g1_mul_u256(P, sk, pk);
  hc_g2_mul_u256(H, sk, sig);
  CHECK(hc_core_verify(pk, msg, 32, (const uint8_t*)DST, sizeof DST - 1, sig) == 1);
  msg[0] ^= 1;
  CHECK(hc_core_verify(pk, msg, 32, (const uint8_t*)DST, sizeof DST - 1, sig) == 0);
  for (int it = 0; it < 4; it++) {
    uint8_t u[96], x1[192], x2[192];
    rfpn(u, 2);
    hc_map_to_curve(u, x1);
    hc_map_to_curve_lane(u, x2);
    CHECK(eq(x1, x2, 192));
  }
  // ---- digit form
  uint8_t j1[192], j2[192];
  CHECK(hc_j2_mul_xabs(Q, j1) == 0);
  CHECK(hc_fq_j2_mul_xabs(Q, j2) == 0);
  CHECK(eq(j1, j2, 192));
  enum { NPT = 9 };
  static uint8_t pts[96 * NPT];
  for (int i = 0; i < NPT; i++) {
    uint32_t kk[8] = {(uint32_t)(i + 1) * 0x9e3779b9u, 0, 0, 0, 0, 0, 0, 0};
    uint8_t c48[48];
    hc_g1_mul_u256(P, kk, c48);
    CHECK(hc_g1_decompress(c48, pts + 96 * i) == 0);
  }
  uint8_t s0[96], s1[96];
  hc_fq_gather(pts, NPT, 0, s0);
  hc_fq_gather(pts, NPT, NPT / 2, s1);
  CHECK(eq(s0, s1, 96));
  uint8_t q64[96], r48[48], r96[96];
  const uint64_t r = 0xd201000000010000ull;
  hc_fq_g1_mul64(P, r, q64);
  uint32_t rk[8] = {(uint32_t)r, (uint32_t)(r >> 32), 0, 0, 0, 0, 0, 0};
  hc_g1_mul_u256(P, rk, r48);
  CHECK(hc_g1_decompress(r48, r96) == 0 && eq(q64, r96, 96));
  if (fails) return 1;
  printf("san_hostcheck ok\n");
  return 0;
}
