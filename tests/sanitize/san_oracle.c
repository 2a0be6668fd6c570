/* TEST HARNESS ONLY: AddressSanitizer / UndefinedBehaviorSanitizer (and, in a
 * second build, ThreadSanitizer) driver for oracle/bls_oracle.c -- the C
 * restatement that tests/ and bench.py's cpu_baseline leg use as the checker.
 * SURVEY.md §5 ("Race detection / sanitizers"): the CPU code runs under the
 * sanitizers in the CPU suite (tests/test_sanitize_cpu.py).
 *
 * Every oc_* entry point is driven through its edge cases with known answers:
 *   - SkToPk(1) = the G1 generator (E/test/helpers/keys.py:4);
 *   - the staking-deposit-cli Verify known answer
 *     (E/test/capella/block_processing/test_process_bls_to_execution_change.py:257-288),
 *     and the same with one flipped message bit;
 *   - the decode edge cases of SURVEY.md §8(a) (infinity, 0x40, c010.., x >= p);
 *   - FastAggregateVerify / AggregateVerify / Aggregate / AggregatePKs, their
 *     empty-list rejections (E/utils/bls.py:154-213);
 *   - the multi-threaded registry paths (oc_registry_generate, oc_sign_batch,
 *     oc_fav_batch_resident in both modes, with one bad item). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oc_key_validate(const uint8_t* pk48);
int oc_verify(const uint8_t* pk48, const uint8_t* msg, size_t mlen, const uint8_t* sig96);
int oc_fast_aggregate_verify(const uint8_t* pks48, size_t n, const uint8_t* msg, size_t mlen, const uint8_t* sig96);
int oc_aggregate_verify(const uint8_t* pks48, size_t n, const uint8_t* msgs, const size_t* lens, const uint8_t* sig96);
int oc_aggregate(const uint8_t* sigs96, size_t n, uint8_t* out96);
int oc_aggregate_pks(const uint8_t* pks48, size_t n, uint8_t* out48);
int oc_sign(const uint8_t* sk32, const uint8_t* msg, size_t mlen, uint8_t* out96);
int oc_sk_to_pk(const uint8_t* sk32, uint8_t* out48);
int oc_hash_to_g2(const uint8_t* msg, size_t mlen, const uint8_t* dst, size_t dlen, uint8_t* out96);
int oc_g2_subgroup_both(const uint8_t* sig96);
int oc_pairing(const uint8_t* pk48, const uint8_t* sig96, uint8_t* out576);
int oc_registry_generate(uint64_t first_sk, size_t n, uint8_t* out96);
int oc_sign_batch(const uint8_t* sks32, const uint8_t* msgs32, size_t B, int threads, uint8_t* out96);
int oc_fav_batch_resident(const uint8_t* reg96, const uint32_t* idx, const uint64_t* offs, size_t B,
                          const uint8_t* msgs32, const uint8_t* sigs96, const uint8_t* seed32, int mode, int threads,
                          uint8_t* out);

static int fails = 0;
#define CHECK(c)                                               \
  do {                                                         \
    if (!(c)) {                                                \
      fprintf(stderr, "san_oracle: FAILED %s (line %d)\n", #c, __LINE__); \
      fails++;                                                 \
    }                                                          \
  } while (0)

static void unhex(uint8_t* out, const char* h) {
  size_t n = strlen(h) / 2;
  for (size_t i = 0; i < n; i++) {
    unsigned v;
    sscanf(h + 2 * i, "%2x", &v);
    out[i] = (uint8_t)v;
  }
}

static void sk32(uint8_t* b, uint64_t v) {
  memset(b, 0, 32);
  for (int i = 0; i < 8; i++) b[31 - i] = (uint8_t)(v >> (8 * i));
}

static const char* G1_GEN =
    "97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb";
static const char* KA_PK =
    "86248e64705987236ec3c41f6a81d96f98e7b85e842a1d71405b216fa75a9917512f3c94c85779a9729c927ea2aa9ed1";
static const char* KA_SIG =
    "8cf4219884b326a04f6664b680cd9a99ad70b5280745af1147477aa9f8b4a2b2b38b8688c6a74a06f275ad4e14c5c0c70e2ed37a15ece5bf"
    "7c0724a376ad4c03c79e14dd9f633a3d54abc1ce4e73bec3524a789ab9a69d4d06686a8a67c9e4dc";
static const char* KA_MSG = "ea9b5656a364bc4d92aca5806b91a76fe538217e39e258d1b9874e776cb49904";
static const char* P_HEX =
    "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab";

int main(int argc, char** argv) {
  const int threads_only = argc > 1 && strcmp(argv[1], "threads") == 0;
  uint8_t sk[32], pk[48], g1[48], sig[96], msg[32], kpk[48], ksig[96], kmsg[32];
  unhex(g1, G1_GEN);
  unhex(kpk, KA_PK);
  unhex(ksig, KA_SIG);
  unhex(kmsg, KA_MSG);
  for (int i = 0; i < 32; i++) msg[i] = (uint8_t)(i * 7 + 1);

  if (!threads_only) {
    /* keys and the known answers */
    sk32(sk, 1);
    CHECK(oc_sk_to_pk(sk, pk) == 1 && memcmp(pk, g1, 48) == 0);
    sk32(sk, 0);
    CHECK(oc_sk_to_pk(sk, pk) != 1); /* sk = 0 is rejected */
    CHECK(oc_verify(kpk, kmsg, 32, ksig) == 1);
    kmsg[5] ^= 0x10;
    CHECK(oc_verify(kpk, kmsg, 32, ksig) == 0);
    kmsg[5] ^= 0x10;

    /* decode edges */
    uint8_t e48[48], e96[96];
    CHECK(oc_key_validate(g1) == 1);
    memset(e48, 0, 48);
    e48[0] = 0xc0;
    CHECK(oc_key_validate(e48) == 0); /* infinity pk */
    e48[0] = 0x40;
    CHECK(oc_key_validate(e48) == 0); /* no compression flag */
    e48[0] = 0xc0;
    e48[1] = 0x10;
    CHECK(oc_key_validate(e48) == 0); /* c010..: infinity with other bits */
    unhex(e48, P_HEX);
    e48[0] |= 0x80;
    CHECK(oc_key_validate(e48) == 0); /* x = p */
    memset(e96, 0, 96);
    e96[0] = 0xc0;
    CHECK(oc_verify(g1, msg, 32, e96) == 0); /* infinity signature */
    memset(e96, 0, 96);
    CHECK(oc_verify(g1, msg, 32, e96) == 0); /* 0x00 x 96 */

    /* sign / verify / aggregates over sk = 1, 2, 3 */
    uint8_t pks[3 * 48], sigs[3 * 96], agg[96], aggpk[48], s6[96], pk6[48];
    for (int k = 0; k < 3; k++) {
      sk32(sk, (uint64_t)k + 1);
      CHECK(oc_sk_to_pk(sk, pks + 48 * k) == 1);
      CHECK(oc_sign(sk, msg, 32, sigs + 96 * k) == 1);
      CHECK(oc_verify(pks + 48 * k, msg, 32, sigs + 96 * k) == 1);
    }
    CHECK(oc_verify(pks, msg, 31, sigs) == 0); /* another message */
    sk32(sk, 6);
    CHECK(oc_sign(sk, msg, 32, s6) == 1 && oc_sk_to_pk(sk, pk6) == 1);
    CHECK(oc_aggregate(sigs, 3, agg) == 1 && memcmp(agg, s6, 96) == 0);
    CHECK(oc_aggregate_pks(pks, 3, aggpk) == 1 && memcmp(aggpk, pk6, 48) == 0);
    CHECK(oc_aggregate(sigs, 0, agg) != 1);    /* Aggregate([]) raises */
    CHECK(oc_aggregate_pks(pks, 0, aggpk) != 1); /* AggregatePKs([]) raises */
    CHECK(oc_fast_aggregate_verify(pks, 3, msg, 32, s6) == 1);
    CHECK(oc_fast_aggregate_verify(pks, 2, msg, 32, s6) == 0);
    CHECK(oc_fast_aggregate_verify(pks, 0, msg, 32, s6) == 0); /* empty list */
    uint8_t msgs[64];
    size_t lens[2] = {32, 32};
    memcpy(msgs, msg, 32);
    for (int i = 0; i < 32; i++) msgs[32 + i] = (uint8_t)(msg[i] ^ 0x5a);
    uint8_t s1[96], s2[96], av[192], avs[96];
    sk32(sk, 1);
    CHECK(oc_sign(sk, msgs, 32, s1) == 1);
    sk32(sk, 2);
    CHECK(oc_sign(sk, msgs + 32, 32, s2) == 1);
    memcpy(av, s1, 96);
    memcpy(av + 96, s2, 96);
    CHECK(oc_aggregate(av, 2, avs) == 1);
    CHECK(oc_aggregate_verify(pks, 2, msgs, lens, avs) == 1);
    CHECK(oc_aggregate_verify(pks, 0, msgs, lens, avs) == 0);
    lens[1] = 31;
    CHECK(oc_aggregate_verify(pks, 2, msgs, lens, avs) == 0);

    /* hash_to_G2, subgroup, pairing */
    static const char DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
    uint8_t h[96], f[576];
    CHECK(oc_hash_to_g2(msg, 32, (const uint8_t*)DST, sizeof DST - 1, h) == 1);
    CHECK(oc_g2_subgroup_both(h) != 0);
    CHECK(oc_hash_to_g2((const uint8_t*)"", 0, (const uint8_t*)DST, sizeof DST - 1, h) == 1);
    CHECK(oc_pairing(g1, s6, f) == 1);
  }

  /* registry paths on threads: generate, sign, FAV batches in both modes with one bad item */
  enum { NREG = 96, B = 6, PER = 12 };
  uint8_t* reg = (uint8_t*)malloc(96 * NREG);
  CHECK(oc_registry_generate(1, NREG, reg) == 1);
  uint32_t idx[B * PER];
  uint64_t offs[B + 1];
  uint8_t sks[B * 32], msgs32[B * 32], bsigs[B * 96], seed[32], out[B];
  for (int j = 0; j < B; j++) {
    uint64_t s = 0;
    offs[j] = (uint64_t)j * PER;
    for (int k = 0; k < PER; k++) {
      idx[j * PER + k] = (uint32_t)((j * 13 + k * 7) % NREG);
      s += idx[j * PER + k] + 1; /* sk_i = i + 1 */
    }
    sk32(sks + 32 * j, s);
    for (int i = 0; i < 32; i++) msgs32[32 * j + i] = (uint8_t)(j * 31 + i);
  }
  offs[B] = (uint64_t)B * PER;
  for (int i = 0; i < 32; i++) seed[i] = (uint8_t)(0x5e + i);
  CHECK(oc_sign_batch(sks, msgs32, B, 3, bsigs) == 1);
  bsigs[96 * 2 + 50] ^= 1; /* item 2: a different (probably undecodable or wrong) signature */
  for (int mode = 0; mode < 2; mode++) {
    memset(out, 0xee, B);
    CHECK(oc_fav_batch_resident(reg, idx, offs, B, msgs32, bsigs, seed, mode, 3, out) == 1);
    for (int j = 0; j < B; j++) CHECK(out[j] == (j == 2 ? 0 : 1));
  }
  free(reg);
  if (fails) return 1;
  printf("san_oracle ok%s\n", threads_only ? " (threads)" : "");
  return 0;
}
