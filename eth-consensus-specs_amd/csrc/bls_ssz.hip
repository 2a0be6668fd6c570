// SHA-256 node hashing for signing roots and SSZ merkleization (SURVEY.md
// §8(f) item 3): the step right before the verify path.
//   compute_signing_root(obj, domain) = hash_tree_root(SigningData(obj_root, domain))
//                                     = SHA-256(obj_root || domain)
//   (specs/phase0/beacon-chain.md:953-962, SigningData :317-320)
//   merkleize(chunks, limit): pairwise SHA-256 up a tree padded with zero
//   chunks to the next power of two (ssz/simple-serialize.md, "merkleize").
// One lane per 64-byte node: two compressions, the second a constant padding
// block (message length 512 bits).
#include "bls_kernels.h"
#include "bls_sha256.h"

namespace bls {

__device__ __forceinline__ void node_hash(const uint8_t* l, const uint8_t* r, uint8_t* out) {
  uint32_t blk[16];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    blk[k] = ((uint32_t)l[4 * k] << 24) | ((uint32_t)l[4 * k + 1] << 16) | ((uint32_t)l[4 * k + 2] << 8) | l[4 * k + 3];
    blk[8 + k] = ((uint32_t)r[4 * k] << 24) | ((uint32_t)r[4 * k + 1] << 16) | ((uint32_t)r[4 * k + 2] << 8) | r[4 * k + 3];
  }
  uint32_t st[8];
#pragma unroll
  for (int k = 0; k < 8; k++) st[k] = SHA256_IV[k];
  sha256_compress(st, blk);
#pragma unroll
  for (int k = 0; k < 16; k++) blk[k] = 0;
  blk[0] = 0x80000000u;
  blk[15] = 512;
  sha256_compress(st, blk);
#pragma unroll
  for (int k = 0; k < 8; k++) {
    out[4 * k] = (uint8_t)(st[k] >> 24);
    out[4 * k + 1] = (uint8_t)(st[k] >> 16);
    out[4 * k + 2] = (uint8_t)(st[k] >> 8);
    out[4 * k + 3] = (uint8_t)st[k];
  }
}

// out[i] = SHA-256(left[32 i ..] || right[rstride i ..])  (rstride 0: one shared right half, e.g. a domain)
__global__ void __launch_bounds__(64) k_sha256_pairs(const uint8_t* left, const uint8_t* right, size_t rstride,
                                                     size_t n, uint8_t* out) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i < n) node_hash(left + 32 * i, right + rstride * i, out + 32 * i);
}

// one tree level: out[j] = H(in[2j] || in[2j+1]), the missing right sibling of an odd tail = zero[0]
__global__ void __launch_bounds__(64) k_merkle_level(const uint8_t* in, size_t n_in, const uint8_t* zero,
                                                     uint8_t* out) {
  const size_t j = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t n_out = (n_in + 1) / 2;
  if (j >= n_out) return;
  const uint8_t* r = 2 * j + 1 < n_in ? in + 32 * (2 * j + 1) : zero;
  node_hash(in + 64 * j, r, out + 32 * j);
}

// zero[0] <- H(zero[0] || zero[0]): the zero-subtree root one level up
__global__ void k_zero_up(uint8_t* zero) {
  if (threadIdx.x || blockIdx.x) return;
  uint8_t t[32];
  node_hash(zero, zero, t);
  for (int k = 0; k < 32; k++) zero[k] = t[k];
}

hipError_t launch_sha256_pairs(hipStream_t st, const uint8_t* left, const uint8_t* right, size_t rstride, size_t n,
                               uint8_t* out) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_sha256_pairs, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, left, right, rstride, n, out);
  return hipGetLastError();
}

// depth levels over n >= 1 chunks in a (ping-pong with b); zero: 32 zeroed device bytes (clobbered).
// Returns the buffer holding the root.
hipError_t launch_merkleize(hipStream_t st, uint8_t* a, uint8_t* b, size_t n, int depth, uint8_t* zero,
                            uint8_t** root) {
  uint8_t *cur = a, *nxt = b;
  for (int l = 0; l < depth; l++) {
    hipLaunchKernelGGL(k_merkle_level, dim3((unsigned)(((n + 1) / 2 + 63) / 64)), dim3(64), 0, st, cur, n, zero, nxt);
    hipLaunchKernelGGL(k_zero_up, dim3(1), dim3(64), 0, st, zero);
    n = (n + 1) / 2;
    uint8_t* t = cur;
    cur = nxt;
    nxt = t;
  }
  *root = cur;
  return hipGetLastError();
}

}  // namespace bls
