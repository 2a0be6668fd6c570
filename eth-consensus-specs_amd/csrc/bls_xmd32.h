// hash_to_field for a 32-byte message under the POP DST, register-resident.
//
// expand_message_xmd (RFC 9380 §5.3.1) of msg (32 B) with DST =
// "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_" (43 B) and len_in_bytes = 256:
//   b0  = H(Z_pad(64) || msg || 01 00 || 00 || DST || 2b)      143 B -> 3 blocks
//   b1  = H(b0 || 01 || DST || 2b)                              77 B -> 2 blocks
//   b_i = H((b0 ^ b_{i-1}) || i || DST || 2b),  i = 2..8
// Every block position is fixed, so the block words are either message /
// chaining words or compile-time constants: the Z_pad block's chaining value
// (XMD_H1), b0's third block and every b_i's second block are constant (their
// message schedules plus round constants are folded into XMD_KW0 / XMD_KWB),
// and b_i's first block is x(8 words) || (i << 24 | DST[0..2]) || DST[3..30].
// 18 compressions, all words in registers with constant indices -- the
// byte-streaming version (bls_sha256.h, any message length) kept its block
// buffer in a private array: 2,144 B of scratch per lane in the h2c kernel.
// Constants are computed at compile time from the DST (constexpr SHA-256).
#pragma once
#include "bls_fp.h"
#include "bls_sha256.h"

namespace bls {

namespace xmd32 {

constexpr uint8_t DST[43] = {'B', 'L', 'S', '_', 'S', 'I', 'G', '_', 'B', 'L', 'S', '1', '2', '3', '8',
                             '1', 'G', '2', '_', 'X', 'M', 'D', ':', 'S', 'H', 'A', '-', '2', '5', '6',
                             '_', 'S', 'S', 'W', 'U', '_', 'R', 'O', '_', 'P', 'O', 'P', '_'};

struct W16 {
  uint32_t w[16];
};
struct W64 {
  uint32_t w[64];
};
struct H8 {
  uint32_t h[8];
};

constexpr uint32_t rotr_c(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// bytes [from, from + 64) of a byte string given by a generator -> 16 big-endian words
template <class F>
constexpr W16 words(F byte_at, int from) {
  W16 r{};
  for (int i = 0; i < 64; ++i) r.w[i / 4] |= (uint32_t)byte_at(from + i) << (24 - 8 * (i % 4));
  return r;
}
// message schedule + round constants of a constant block
constexpr W64 kw(const W16& b) {
  W64 s{};
  for (int i = 0; i < 16; ++i) s.w[i] = b.w[i];
  for (int i = 16; i < 64; ++i) {
    const uint32_t w15 = s.w[i - 15], w2 = s.w[i - 2];
    s.w[i] = s.w[i - 16] + (rotr_c(w15, 7) ^ rotr_c(w15, 18) ^ (w15 >> 3)) + s.w[i - 7] +
             (rotr_c(w2, 17) ^ rotr_c(w2, 19) ^ (w2 >> 10));
  }
  for (int i = 0; i < 64; ++i) s.w[i] += SHA256_K[i];
  return s;
}
constexpr H8 compress_c(H8 st, const W64& kwv) {
  uint32_t a = st.h[0], b = st.h[1], c = st.h[2], d = st.h[3], e = st.h[4], f = st.h[5], g = st.h[6], h = st.h[7];
  for (int i = 0; i < 64; ++i) {
    const uint32_t t1 = h + (rotr_c(e, 6) ^ rotr_c(e, 11) ^ rotr_c(e, 25)) + ((e & f) ^ (~e & g)) + kwv.w[i];
    const uint32_t t2 = (rotr_c(a, 2) ^ rotr_c(a, 13) ^ rotr_c(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  st.h[0] += a;
  st.h[1] += b;
  st.h[2] += c;
  st.h[3] += d;
  st.h[4] += e;
  st.h[5] += f;
  st.h[6] += g;
  st.h[7] += h;
  return st;
}

// b0's message (bytes 0..191 after padding); msg bytes (32..63 of block 2) read as 0 here
constexpr uint8_t b0_byte(int p) {
  if (p < 64) return 0;                 // Z_pad
  if (p < 96) return 0;                 // msg (not constant; these words are replaced)
  if (p == 96) return 0x01;             // I2OSP(256, 2)
  if (p == 97 || p == 98) return 0x00;  // ... and I2OSP(0, 1)
  if (p < 99 + 43) return DST[p - 99];
  if (p == 142) return 43;              // I2OSP(len(DST), 1)
  if (p == 143) return 0x80;
  if (p >= 184) return (uint8_t)((uint64_t)(143 * 8) >> (8 * (191 - p)));
  return 0;
}
// b_i's message (bytes 0..127 after padding); x bytes (0..31) read as 0, i at byte 32 read as 0
constexpr uint8_t bi_byte(int p) {
  if (p < 33) return 0;
  if (p < 33 + 43) return DST[p - 33];
  if (p == 76) return 43;
  if (p == 77) return 0x80;
  if (p >= 120) return (uint8_t)((uint64_t)(77 * 8) >> (8 * (127 - p)));
  return 0;
}
constexpr H8 iv() {
  H8 r{};
  for (int i = 0; i < 8; ++i) r.h[i] = SHA256_IV[i];
  return r;
}
constexpr W16 ZERO16{};
constexpr H8 H1 = compress_c(iv(), kw(ZERO16));        // chaining value after the Z_pad block
constexpr W16 B0_BLK2 = words(b0_byte, 64);             // words 8..15 used (0..7 = msg)
constexpr W64 KW_B0_BLK3 = kw(words(b0_byte, 128));     // constant third block of b0
constexpr W16 BI_BLKA = words(bi_byte, 0);              // words 9..15 used; word 8 = i << 24 | DST[0..2]
constexpr W64 KW_BI_BLKB = kw(words(bi_byte, 64));      // constant second block of every b_i

}  // namespace xmd32

// one compression with the schedule computed from 16 register words (constant indices only)
BLS_HD void sha256_compress_w(uint32_t st[8], const uint32_t blk[16]) {
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
      const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      wi = w[i & 15] + (rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3)) + w[(i + 9) & 15] +
           (rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10));
      w[i & 15] = wi;
    }
    const uint32_t t1 = h + (rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25)) + ((e & f) ^ (~e & g)) + SHA256_K[i] + wi;
    const uint32_t t2 = (rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
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
// one compression of a constant block (schedule + round constants precomputed)
BLS_HD void sha256_compress_kw(uint32_t st[8], const uint32_t kw[64]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    const uint32_t t1 = h + (rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25)) + ((e & f) ^ (~e & g)) + kw[i];
    const uint32_t t2 = (rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
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

// 16 big-endian words (64 bytes) mod p -> Montgomery form, as fp_from_be64_mod
BLS_HD Fp fp_from_be64w_mod(const uint32_t w[16]) {
  Fp lo, hi = fp_zero();
#pragma unroll
  for (int i = 0; i < 12; i++) lo.l[i] = w[15 - i];
#pragma unroll
  for (int i = 0; i < 4; i++) hi.l[i] = w[3 - i];
  return fp_add(fp_mul_i(lo, FP_R2), fp_mul_i(hi, FP_2P384_R2));
}

// a wave-uniform word kept in a VGPR: on the device an identity DPP move hides its uniformity from the
// compiler, so the compressions of one message run as VALU code (v_alignbit rotates, v_xor3, v_bitop3, v_add3)
// instead of scalar code that sends every rotate through a VALU v_alignbit and a v_readfirstlane back
BLS_HD uint32_t xmd_vector(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xE4, 0xF, 0xF, false);  // quad_perm [0,1,2,3]
#else
  return v;
#endif
}

template <bool UNIFORM = false>
BLS_HD void hash_to_field_fp2_m32(Fp2 u[2], const uint8_t* msg32) {
  uint32_t blk[16], st[8], b0[8], bi[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint8_t* q = msg32 + 4 * j;
    blk[j] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
    if (UNIFORM) blk[j] = xmd_vector(blk[j]);
  }
#pragma unroll
  for (int j = 8; j < 16; j++) blk[j] = xmd32::B0_BLK2.w[j];
#pragma unroll
  for (int j = 0; j < 8; j++) st[j] = xmd32::H1.h[j];
  sha256_compress_w(st, blk);
  sha256_compress_kw(st, xmd32::KW_B0_BLK3.w);
#pragma unroll
  for (int j = 0; j < 8; j++) {
    b0[j] = st[j];
    bi[j] = 0;
  }
  // b_{2k+1}, b_{2k+2} -> the 64-byte string of field element k, reduced at once; a rolled loop over k with
  // every array index a compile-time constant (an unrolled 8-step loop of 16 compressions was not unrolled by the
  // compiler and its indexed word arrays went to private memory)
  Fp el0 = fp_zero(), el1 = fp_zero(), el2 = fp_zero(), el3 = fp_zero();
#pragma unroll 1
  for (int k = 0; k < 4; k++) {
    uint32_t e[16];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t i = 2 * k + h + 1;
#pragma unroll
      for (int j = 0; j < 8; j++) blk[j] = b0[j] ^ bi[j];  // b_0 ^ b_{i-1} (b1: b_0 itself, bi = 0)
      blk[8] = (i << 24) | (xmd32::BI_BLKA.w[8] & 0x00ffffffu);
#pragma unroll
      for (int j = 9; j < 16; j++) blk[j] = xmd32::BI_BLKA.w[j];
#pragma unroll
      for (int j = 0; j < 8; j++) st[j] = SHA256_IV[j];
      sha256_compress_w(st, blk);
      sha256_compress_kw(st, xmd32::KW_BI_BLKB.w);
#pragma unroll
      for (int j = 0; j < 8; j++) {
        bi[j] = st[j];
        e[8 * h + j] = st[j];
      }
    }
    const Fp v = fp_from_be64w_mod(e);
    el0 = fp_select(k == 0, v, el0);
    el1 = fp_select(k == 1, v, el1);
    el2 = fp_select(k == 2, v, el2);
    el3 = fp_select(k == 3, v, el3);
  }
  u[0] = Fp2{el0, el1};
  u[1] = Fp2{el2, el3};
}

}  // namespace bls
