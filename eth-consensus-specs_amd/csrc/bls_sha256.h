// SHA-256 (FIPS 180-4) and expand_message_xmd (RFC 9380 §5.3.1) for
// hash_to_G2.  A 32-byte signing root under the 43-byte POP DST costs
// 3 + 2 + 8*2 = 21 block compressions; the first block of msg_prime is the
// all-zero Z_pad, whose chaining value is a constant, so 20 are computed.
#pragma once
#include "bls_field_types.h"

namespace bls {

static constexpr uint32_t SHA256_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

static constexpr uint32_t SHA256_IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                          0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

BLS_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// One compression of a 16-word big-endian block.
BLS_HDNI void sha256_compress(uint32_t st[8], const uint32_t blk[16]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = blk[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + SHA256_K[i] + wi;
    uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}

// Streaming SHA-256 over bytes (messages here are short; simplicity over speed).
struct Sha256 {
  uint32_t st[8];
  uint32_t blk[16];
  uint32_t nbuf;  // bytes in blk
  uint64_t total;
};

BLS_HD void sha256_init(Sha256& s) {
  for (int i = 0; i < 8; i++) s.st[i] = SHA256_IV[i];
  for (int i = 0; i < 16; i++) s.blk[i] = 0;
  s.nbuf = 0;
  s.total = 0;
}

BLS_HDNI void sha256_byte(Sha256& s, uint8_t v) {
  const uint32_t wi = s.nbuf >> 2, sh = 24 - 8 * (s.nbuf & 3);
  s.blk[wi] |= (uint32_t)v << sh;
  s.nbuf++;
  s.total++;
  if (s.nbuf == 64) {
    sha256_compress(s.st, s.blk);
    for (int i = 0; i < 16; i++) s.blk[i] = 0;
    s.nbuf = 0;
  }
}

BLS_HDNI void sha256_update(Sha256& s, const uint8_t* p, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) sha256_byte(s, p[i]);
}

BLS_HDNI void sha256_final(Sha256& s, uint8_t out[32]) {
  const uint64_t bits = s.total * 8;
  sha256_byte(s, 0x80);
  while (s.nbuf != 56) sha256_byte(s, 0);
  for (int i = 7; i >= 0; --i) sha256_byte(s, (uint8_t)(bits >> (8 * i)));
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)(s.st[i] >> 24);
    out[4 * i + 1] = (uint8_t)(s.st[i] >> 16);
    out[4 * i + 2] = (uint8_t)(s.st[i] >> 8);
    out[4 * i + 3] = (uint8_t)s.st[i];
  }
}

// expand_message_xmd(msg, DST, 256) -> 256 uniform bytes (ell = 8).
BLS_HDNI void expand_message_xmd_256(uint8_t out[256], const uint8_t* msg, uint32_t msg_len, const uint8_t* dst,
                                   uint32_t dst_len) {
  Sha256 s;
  sha256_init(s);
  for (int i = 0; i < 64; i++) sha256_byte(s, 0);  // Z_pad
  sha256_update(s, msg, msg_len);
  sha256_byte(s, 1);  // I2OSP(256, 2)
  sha256_byte(s, 0);
  sha256_byte(s, 0);  // I2OSP(0, 1)
  sha256_update(s, dst, dst_len);
  sha256_byte(s, (uint8_t)dst_len);
  uint8_t b0[32];
  sha256_final(s, b0);
  uint8_t bi[32];
  for (int i = 1; i <= 8; i++) {
    sha256_init(s);
    if (i == 1) {
      sha256_update(s, b0, 32);
    } else {
      for (int j = 0; j < 32; j++) sha256_byte(s, b0[j] ^ bi[j]);
    }
    sha256_byte(s, (uint8_t)i);
    sha256_update(s, dst, dst_len);
    sha256_byte(s, (uint8_t)dst_len);
    sha256_final(s, bi);
    for (int j = 0; j < 32; j++) out[32 * (i - 1) + j] = bi[j];
  }
}

}  // namespace bls
