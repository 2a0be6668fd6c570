// gfx950 kernels of the BLS12-381 backend.  One lane owns one item
// (verification, key, signature, pair) unless noted; reductions (aggregate
// pubkeys, sum of r_i*sig_i, Miller-product) are LDS trees inside a
// workgroup followed by a second pass over the per-workgroup partials.
#include <cstdlib>

#include "bls_kernels.h"
#include "bls_fq_g1.h"

namespace bls {

__device__ static const uint8_t DST_POP_DEV[43] = {
    'B', 'L', 'S', '_', 'S', 'I', 'G', '_', 'B', 'L', 'S', '1', '2', '3', '8', '1', 'G', '2', '_', 'X', 'M', 'D',
    ':', 'S', 'H', 'A', '-', '2', '5', '6', '_', 'S', 'S', 'W', 'U', '_', 'R', 'O', '_', 'P', 'O', 'P', '_'};

static __device__ __forceinline__ size_t gtid() { return (size_t)blockIdx.x * blockDim.x + threadIdx.x; }

// ---------------------------------------------------------------- decode --
// [|x|] P by the complete projective formulas in the digit form (bls_fq_g1.h: g1q_dbl / g1q_add, the chain of
// k_sig_lane2); the base is affine (x, y) when AFF, else the projective point b.
template <bool AFF>
static __device__ __forceinline__ G1Q g1q_mul_xabs(const G1Q& b) {
  G1Q m = b;
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    m = g1q_dbl(m);
    if ((X_ABS >> i) & 1ull) m = AFF ? g1q_add_aff(m, b.x, b.y) : g1q_add(m, b);
  }
  return m;
}

// KeyValidate (E/utils/bls.py:395-397; py_ecc pubkey_to_G1 decode rules, identity rejected, subgroup check) of one
// 48-byte key, every product in the redundant digit form of bls_fq.h and inlined (the packed form's out-of-line
// square root and Jacobian chains cost this kernel a 1,552-B private segment):
//   decode: flags, x < p, y = (x^3 + 4)^((p+1)/4) (fq_pow_w3), y^2 == x^3 + 4, the sign bit picks y or -y;
//   subgroup (bls_curve.h g1_in_subgroup): phi(P) == -[x^2] P with phi(x, y) = (beta x, y), i.e. for
//   [|x|]([|x|] P) = (X : Y : Z):  beta x Z == X  and  y Z + Y == 0  (Z == 0, the identity, fails the second).
__global__ void __launch_bounds__(64) k_key_validate(const uint8_t* pks48, size_t n, G1A* out, int* ok) {
  const size_t i = gtid();
  if (i >= n) return;
  // 48 big-endian bytes; records are 48 B apart, so word loads stay 4-byte aligned
  const uint32_t* w = reinterpret_cast<const uint32_t*>(pks48 + 48 * i);
  Fp x;
#pragma unroll
  for (int k = 0; k < 12; k++) x.l[11 - k] = __builtin_bswap32(w[k]);
  const uint32_t flags = x.l[11] >> 24;
  const bool c_flag = flags & 0x80, b_flag = flags & 0x40, a_flag = flags & 0x20;
  x.l[11] &= 0x1fffffffu;
  G1A a{fp_zero(), fp_zero(), true};
  int v = 0;
  // the identity (b_flag) and every malformed encoding fail KeyValidate
  if (c_flag && !b_flag && !fp_is_zero(x) && raw_lt_p(x)) {
    const Fq xm = fq_mul(fq_unpack(x), fq_unpack(FP_R2));  // Montgomery form, N
    const Fq rhs = fq_add(fq_mul(fq_sqr(xm), xm), fq_unpack(FP_B1));
    Fq y = fq_pow_w3(rhs, EXP_SQRT, EXP_SQRT_BITS);
    if (fp_eq(fq_pack(fq_sqr(y)), fq_pack(rhs))) {
      Fp yc = fq_pack_n(y);
      Fq one = fq_zero();
      one.d[0] = 1;
      if (raw_gt_half(fq_pack_n(fq_mul(y, one))) != a_flag) yc = fp_neg(yc);
      const Fp xc = fq_pack_n(xm);
      y = fq_unpack(yc);
      const G1Q P{xm, y, fq_unpack(FP_ONE)};
      const G1Q Q = g1q_mul_xabs<false>(g1q_mul_xabs<true>(P));
      const bool eq_x = fp_eq(fq_pack(fq_mul(fq_mul(xm, fq_unpack(FP_BETA)), Q.z)), fq_pack(Q.x));
      const bool eq_y = fp_is_zero(fq_pack(fq_add(fq_mul(y, Q.z), Q.y)));
      if (eq_x && eq_y) {
        a = G1A{xc, yc, false};
        v = 1;
      }
    }
  }
  out[i] = a;
  ok[i] = v;
}

// ------------------------------------------------------------ reductions --
// Sum of affine G1 points (only entries with ok != 0 when ok is given) into
// one Jacobian partial per workgroup.
template <int NT>
__global__ void __launch_bounds__(NT) k_g1_sum_aff(const G1A* in, const int* ok, size_t n, G1J* out) {
  __shared__ G1J sh[NT];
  G1J acc = jac_identity<Fp>();
  for (size_t i = (size_t)blockIdx.x * NT + threadIdx.x; i < n; i += (size_t)gridDim.x * NT) {
    if (!ok || ok[i]) acc = jac_add_aff(acc, in[i]);
  }
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int s = NT / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) sh[threadIdx.x] = jac_add(sh[threadIdx.x], sh[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = sh[0];
}

// The sum of up to G1Q_SUM_MAX points in ONE workgroup (the per-call aggregate key, AggregatePKs, multi_exp
// totals): each lane adds its points with the complete mixed additions of the registry gather in the redundant
// digit form (bls_fq_g1.h g1q_add_aff), then a tree over the workgroup's lanes through LDS (g1q_add); the
// projective (X : Y : Z) leaves as the Jacobian (X Z, Y Z^2, Z), packed.  One launch instead of two, and digit-form
// products instead of packed ones (k_g1_sum_aff + k_jac_sum: 0.20-0.29 ms for 512 keys).
constexpr int G1Q_SUM_NT = 256;
constexpr size_t G1Q_SUM_MAX = 8 * G1Q_SUM_NT;
__global__ void __launch_bounds__(G1Q_SUM_NT) k_g1_sum_q(const G1A* in, const int* ok, size_t n, G1J* out) {
  __shared__ uint32_t sh[42][G1Q_SUM_NT];  // [word][lane]: a G1Q is 3 x 14 digits
  const int t = (int)threadIdx.x;
  const Fq zero = fq_zero();
  G1Q acc{zero, fq_unpack(FP_ONE), zero};  // the identity (0 : 1 : 0)
  for (size_t i = (size_t)t; i < n; i += G1Q_SUM_NT) {
    if ((ok && !ok[i]) || in[i].inf) continue;
    acc = g1q_add_aff(acc, fq_unpack(in[i].x), fq_unpack(in[i].y));
  }
  for (int s = G1Q_SUM_NT / 2; s > 0; s >>= 1) {
    if (t >= s && t < 2 * s) {
      const uint32_t* w = reinterpret_cast<const uint32_t*>(&acc);
#pragma unroll
      for (int k = 0; k < 42; ++k) sh[k][t - s] = w[k];
    }
    __syncthreads();
    if (t < s) {
      G1Q o;
      uint32_t* w = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
      for (int k = 0; k < 42; ++k) w[k] = sh[k][t];
      acc = g1q_add(acc, o);
    }
    __syncthreads();
  }
  if (t == 0) {
    G1J r;
    const Fp z = fq_pack(acc.z);
    if (fp_is_zero(z)) {
      r = jac_identity<Fp>();
    } else {
      r.x = fq_pack(fq_mul(acc.x, acc.z));
      r.y = fq_pack(fq_mul(fq_mul(acc.y, acc.z), acc.z));
      r.z = z;
    }
    *out = r;
  }
}

template <class F, int NT>
__global__ void __launch_bounds__(NT) k_jac_sum(const Jac<F>* in, size_t n, Jac<F>* out) {
  __shared__ Jac<F> sh[NT];
  Jac<F> acc = jac_identity<F>();
  for (size_t i = (size_t)blockIdx.x * NT + threadIdx.x; i < n; i += (size_t)gridDim.x * NT) acc = jac_add(acc, in[i]);
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int s = NT / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) sh[threadIdx.x] = jac_add(sh[threadIdx.x], sh[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = sh[0];
}

__global__ void __launch_bounds__(64) k_g2_sum_aff(const G2A* in, const int* ok, size_t n, G2J* out) {
  __shared__ G2J sh[64];
  G2J acc = jac_identity<Fp2>();
  for (size_t i = (size_t)blockIdx.x * 64 + threadIdx.x; i < n; i += (size_t)gridDim.x * 64) {
    if (!ok || ok[i]) acc = jac_add(acc, jac_from_aff(in[i]));
  }
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 32; s > 0; s >>= 1) {
    if (threadIdx.x < s) sh[threadIdx.x] = jac_add(sh[threadIdx.x], sh[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = sh[0];
}

// ------------------------------------------------------------- encoding --
__global__ void k_g1_compress(const G1J* in, uint8_t* out48, int* is_inf) {
  if (threadIdx.x || blockIdx.x) return;
  G1A a = jac_to_aff(in[0]);
  g1_compress(out48, a);
  if (is_inf) *is_inf = a.inf;
}

__global__ void k_g2_compress(const G2J* in, uint8_t* out96) {
  if (threadIdx.x || blockIdx.x) return;
  g2_compress(out96, jac_to_aff(in[0]));
}

// Per-call path (bls_verify / bls_fast_aggregate_verify): the pairs
// (apk, H(m)) and (-G1, sigma) for k_miller2_vm.  apk is the validated key
// (n == 1) or the sum of the validated keys; *live = 0 if any key failed
// KeyValidate, the sum is the identity, or the signature failed its checks.
// pz != nullptr: P[0] keeps the sum's Jacobian X, Y and pz[0] its Z (1 for n == 1) -- no inversion; the wide
// Miller loop scales its lines by Z^3 instead.
__global__ void k_percall_pairs(const G1A* keys, const int* key_ok, size_t n, const G1J* apk_sum, const int* sig_ok,
                                G1A* P, int* live, Fp* pz) {
  if (threadIdx.x || blockIdx.x) return;
  int ok = sig_ok[0];
  for (size_t i = 0; i < n; i++) ok = ok && key_ok[i];
  G1A a;
  if (n == 1) {
    a = keys[0];
    if (pz) pz[0] = FP_ONE;
  } else if (pz) {
    const G1J& j = apk_sum[0];
    a = G1A{j.x, j.y, jac_is_inf(j)};
    pz[0] = j.z;
  } else {
    a = jac_to_aff(apk_sum[0]);
  }
  ok = ok && !a.inf;
  P[0] = a;
  P[1] = g1_neg_generator();
  *live = ok;
}

__global__ void __launch_bounds__(64) k_hash_many(const uint8_t* msgs, const uint64_t* offs, size_t n,
                                                  const uint8_t* dst, uint32_t dst_len, G2A* out) {
  size_t i = gtid();
  if (i >= n) return;
  const uint8_t* d = dst ? dst : DST_POP_DEV;
  uint32_t dl = dst ? dst_len : 43;
  out[i] = jac_to_aff(hash_to_g2(msgs + offs[i], (uint32_t)(offs[i + 1] - offs[i]), d, dl));
}

__global__ void k_g2_compress_aff(const G2A* in, uint8_t* out96) {
  if (threadIdx.x || blockIdx.x) return;
  g2_compress(out96, in[0]);
}

// --------------------------------------------------------------- signing --
// sk: 32 bytes big-endian -> 8 LE u32 limbs; valid iff 0 < sk < r
static __device__ bool sk_parse(uint32_t k[8], const uint8_t* sk) {
  for (int i = 0; i < 8; i++) {
    const uint8_t* q = sk + 28 - 4 * i;
    k[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
  static constexpr uint32_t R_LIMBS[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                                          0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
  uint32_t nz = 0;
  for (int i = 0; i < 8; i++) nz |= k[i];
  if (!nz) return false;
  for (int i = 7; i >= 0; --i) {
    if (k[i] != R_LIMBS[i]) return k[i] < R_LIMBS[i];
  }
  return false;  // == r
}

__global__ void __launch_bounds__(64) k_sign_many(const uint8_t* sks32, const uint8_t* msgs, const uint64_t* offs,
                                                  size_t n, uint8_t* out96, int* ok) {
  size_t i = gtid();
  if (i >= n) return;
  uint32_t k[8];
  if (!sk_parse(k, sks32 + 32 * i)) {
    ok[i] = 0;
    return;
  }
  G2J h = hash_to_g2(msgs + offs[i], (uint32_t)(offs[i + 1] - offs[i]), DST_POP_DEV, 43);
  g2_compress(out96 + 96 * i, jac_to_aff(jac_mul_u256(h, k)));
  ok[i] = 1;
}

__global__ void __launch_bounds__(64) k_sk_to_pk_many(const uint8_t* sks32, size_t n, uint8_t* out48, int* ok) {
  size_t i = gtid();
  if (i >= n) return;
  uint32_t k[8];
  if (!sk_parse(k, sks32 + 32 * i)) {
    ok[i] = 0;
    return;
  }
  g1_compress(out48 + 48 * i, jac_to_aff(jac_mul_u256(jac_from_aff(g1_generator()), k)));
  ok[i] = 1;
}

// ------------------------------------------------------- FAV batch path --
// Aggregate pubkeys: L lanes per aggregate, 64 / L aggregates per workgroup.
// Each lane adds its strided share of the registry points with the complete
// projective mixed addition (Renes-Costello-Batina alg. 8, 11 products, no
// exceptional cases), then an LDS tree of complete additions (alg. 7), all in
// the redundant digit form (bls_fq_g1.h: g1q_add_aff, g1q_add).  The tree costs
// log2(L) full additions of the whole wave, so for mainnet-sized committees
// L = 16 (32 mixed additions per lane + 4 tree levels) beats 64 lanes (8 + 6
// levels: the tree was ~45 % of the wave's time).
template <int L>
__global__ void __launch_bounds__(64) k_fav_gather_q(const uint32_t* idx, const uint64_t* offs, size_t B,
                                                     const RegKey* reg, uint32_t reg_n, G1P* apk, int* status,
                                                     const int* only) {
  constexpr int IPW = 64 / L;
  __shared__ G1Q sh[64];
  __shared__ int bad[IPW];
  const int sub = (int)threadIdx.x / L, ln = (int)threadIdx.x % L;
  const size_t b = (size_t)blockIdx.x * IPW + sub;
  // only (launch_fav_gather_redo): just the flagged aggregates, the others keep what k_fav_gather_aff wrote; a
  // workgroup with none of them leaves at once (a uniform exit, before any barrier)
  if (only) {
    bool any = false;
    for (int s = 0; s < IPW; ++s) {
      const size_t bb = (size_t)blockIdx.x * IPW + s;
      any |= bb < B && only[bb] != 0;
    }
    if (!any) return;
  }
  const bool mine = b < B && (!only || only[b] != 0);
  if ((int)threadIdx.x < IPW) bad[threadIdx.x] = 0;
  __syncthreads();
  G1Q acc{fq_zero(), fq_unpack(FP_ONE), fq_zero()};  // identity (0 : 1 : 0)
  int mybad = 0;
  uint64_t lo = 0, hi = 0;
  if (mine) {
    lo = offs[b];
    hi = offs[b + 1];
    // software pipeline: the record of key j + L and the index of key j + 2L are in flight while key j is added
    // (an out-of-range index reads record 0 and is flagged; every load is unconditional)
    uint64_t j = lo + ln;
    uint32_t k1 = j < hi ? idx[j] : 0u;
    const uint32_t* rw = reinterpret_cast<const uint32_t*>(reg + (k1 < reg_n ? k1 : 0u));
    uint4 r[6];
#pragma unroll
    for (int w = 0; w < 6; ++w) r[w] = reinterpret_cast<const uint4*>(rw)[w];
    uint32_t k2 = j + L < hi ? idx[j + L] : 0u;
#pragma unroll 1
    for (; j < hi; j += L) {
      uint4 cr[6];
#pragma unroll
      for (int w = 0; w < 6; ++w) cr[w] = r[w];
      const uint32_t ck = k1;
      k1 = k2;
      const uint4* nr = reinterpret_cast<const uint4*>(reg + (k1 < reg_n ? k1 : 0u));
#pragma unroll
      for (int w = 0; w < 6; ++w) r[w] = nr[w];
      k2 = j + 2 * L < hi ? idx[j + 2 * L] : 0u;
      Fp x, y;
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        reinterpret_cast<uint4*>(x.l)[w] = cr[w];
        reinterpret_cast<uint4*>(y.l)[w] = cr[3 + w];
      }
      if (ck >= reg_n || !(x.l[11] & REG_VALID)) {
        mybad = 1;
      } else {
        x.l[11] &= ~REG_VALID;
        acc = g1q_add_aff(acc, fq_unpack(x), fq_unpack(y));
      }
    }
  }
  if (mybad) atomicOr(&bad[sub], 1);
  sh[threadIdx.x] = acc;
  __syncthreads();
#pragma unroll 1
  for (int s = L / 2; s > 0; s >>= 1) {
    if (ln < s) sh[threadIdx.x] = g1q_add(sh[threadIdx.x], sh[threadIdx.x + s]);
    __syncthreads();
  }
  if (ln == 0 && mine) {  // canonical projective aggregate key; the identity is invalid (KeyValidate of the sum)
    const G1Q& a = sh[threadIdx.x];
    const G1P o{fq_pack(a.x), fq_pack(a.y), fq_pack(a.z)};
    apk[b] = o;
    status[b] = (hi > lo && !bad[sub] && !fp_is_zero(o.z)) ? 1 : 0;
  }
}

// Registry entries from decoded keys (bls_registry_load / _append): the
// KeyValidate verdict goes into x's spare top bit; valid[i] = 1/0 for the host.
__global__ void __launch_bounds__(256) k_reg_pack(const G1A* a, const int* ok, size_t n, RegKey* reg, uint8_t* valid) {
  const size_t i = gtid();
  if (i >= n) return;
  RegKey e{a[i].x, a[i].y};
  const bool v = ok[i] != 0;
  if (!v) e = RegKey{fp_zero(), fp_zero()};
  e.x.l[11] |= v ? REG_VALID : 0u;
  reg[i] = e;
  valid[i] = v ? 1 : 0;
}

// (5) AggregateVerify batches (bls_aggregate_verify_batch).  Item b owns the
//     n_b pairs (pk_bj, m_bj) at pair indices io[b] .. io[b+1] and one
//     signature; its pairs are laid out at io[b] + b + j, followed by the
//     signature pair at io[b+1] + b.  With a random 64-bit r_b per item the
//     item's pairs are (r_b pk_bj, H(m_bj)) and (-r_b G1, sigma_b): their
//     Miller product is the item's check raised to r_b, so the product over
//     all items is the batch's random-linear-combination check and any
//     item's own segment is its individual check (fallback).
__global__ void __launch_bounds__(64) k_av_items(size_t B, const uint64_t* io, const int* pk_ok, const int* sig_ok,
                                                 const G2A* sig, const uint64_t* rsc, int* status, G1A* P2, G2A* Q2) {
  const size_t b = gtid();
  if (b >= B) return;
  const uint64_t lo = io[b], hi = io[b + 1];
  int st = hi > lo && sig_ok[b];
  for (uint64_t j = lo; st && j < hi; j++) st = pk_ok[j] != 0;
  status[b] = st;
  G1A ng{fp_zero(), fp_zero(), true};
  if (st) {
    G1A g = g1_generator();
    g.y = fp_neg(g.y);
    ng = jac_to_aff(jac_mul_u64(jac_from_aff(g), rsc[b]));
  }
  P2[hi + b] = ng;
  Q2[hi + b] = sig[b];
}

__global__ void __launch_bounds__(64) k_av_pairs(size_t total, const uint32_t* pair_item, const int* status,
                                                 const uint64_t* rsc, const G1A* pk, const G2A* H, G1A* P2, G2A* Q2) {
  const size_t t = gtid();
  if (t >= total) return;
  const uint32_t b = pair_item[t];
  G1A rp{fp_zero(), fp_zero(), true};
  if (status[b]) rp = jac_to_aff(jac_mul_u64(jac_from_aff(pk[t]), rsc[b]));
  P2[t + b] = rp;
  Q2[t + b] = H[t];
}

// (6) KZG pieces: checked G1 decoding that accepts the
//     identity (validate_kzg_g1, specs/deneb/polynomial-commitments.md), and the
//     per-point products [k_i] P_i of multi_exp (summed by k_g1_sum_aff).
__global__ void __launch_bounds__(64) k_g1_decode_checked(const uint8_t* in48, size_t n, G1A* out, int* ok) {
  const size_t i = gtid();
  if (i >= n) return;
  G1A a{fp_zero(), fp_zero(), true};
  const int d = g1_decompress(a, in48 + 48 * i);
  int v = 0;
  if (d == DEC_INFINITY) {
    a = G1A{fp_zero(), fp_zero(), true};
    v = 1;
  } else if (d == DEC_OK) {
    v = g1_in_subgroup(jac_from_aff(a)) ? 1 : 0;
  }
  if (!v) a = G1A{fp_zero(), fp_zero(), true};
  out[i] = a;
  ok[i] = v;
}

// scalars: 32-byte big-endian integers; out[i] = [k_i] P_i (affine), live[i] = 0 for the identity
__global__ void __launch_bounds__(64) k_g1_scale(const G1A* P, const uint8_t* k32, size_t n, G1A* out, int* live) {
  const size_t i = gtid();
  if (i >= n) return;
  uint32_t k[8];
  for (int w = 0; w < 8; w++) {
    const uint8_t* b = k32 + 32 * i + 28 - 4 * w;
    k[w] = ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
  }
  G1A r{fp_zero(), fp_zero(), true};
  if (!P[i].inf) r = jac_to_aff(jac_mul_u256(jac_from_aff(P[i]), k));
  out[i] = r;
  live[i] = r.inf ? 0 : 1;
}

// Verdicts: valid iff the per-item checks passed and bisection did not isolate it.
__global__ void k_verdicts(const int* status, const uint8_t* bad, size_t B, uint8_t* out) {
  size_t i = gtid();
  if (i < B) out[i] = (status[i] && !bad[i]) ? 1 : 0;
}

__global__ void k_status_to_u8(const int* status, size_t B, uint8_t* out) {
  size_t i = gtid();
  if (i < B) out[i] = status[i] ? 1 : 0;
}

// Fp12 <-> 576 big-endian bytes (w-basis order c0..c5, each Fp2 as c0||c1)
__global__ void k_fp12_to_bytes(const Fp12* f, uint8_t* out) {
  if (threadIdx.x || blockIdx.x) return;
  const Fp2* c[6] = {&f->c0.c0, &f->c1.c0, &f->c0.c1, &f->c1.c1, &f->c0.c2, &f->c1.c2};
  for (int k = 0; k < 6; k++) {
    raw_to_be48(fp_from_mont(c[k]->c0), out + 96 * k);
    raw_to_be48(fp_from_mont(c[k]->c1), out + 96 * k + 48);
  }
}

__global__ void k_fp12_from_bytes(const uint8_t* in, size_t n, Fp12* f) {
  size_t i = gtid();
  if (i >= n) return;
  const uint8_t* b = in + 576 * i;
  Fp12 r;
  Fp2* c[6] = {&r.c0.c0, &r.c1.c0, &r.c0.c1, &r.c1.c1, &r.c0.c2, &r.c1.c2};
  for (int k = 0; k < 6; k++) {
    c[k]->c0 = fp_to_mont(raw_from_be48(b + 96 * k));
    c[k]->c1 = fp_to_mont(raw_from_be48(b + 96 * k + 48));
  }
  f[i] = r;
}

// Synthetic registry: pk_i = (first + i) * G1, affine, valid.  One lane
// walks a chunk of consecutive multiples (mixed additions of G1) and
// normalises the chunk with one inversion (Montgomery's batch trick).
__global__ void __launch_bounds__(64) k_registry_generate(uint64_t first, size_t n, uint32_t chunk, G1J* tmpJ,
                                                          RegKey* reg, uint8_t* out48) {
  size_t t = gtid();
  size_t lo = t * chunk;
  if (lo >= n) return;
  size_t hi = lo + chunk < n ? lo + chunk : n;
  uint64_t k0 = first + lo;
  uint32_t k[8] = {(uint32_t)k0, (uint32_t)(k0 >> 32), 0, 0, 0, 0, 0, 0};
  const G1A g = g1_generator();
  G1J p = jac_mul_u256(jac_from_aff(g), k);
  // forward pass: store points, prefix products of Z in reg[].x (scratch)
  Fp acc = FP_ONE;
  for (size_t i = lo; i < hi; i++) {
    tmpJ[i] = p;
    acc = fp_mul(acc, p.z);
    reg[i].y = acc;  // prefix product up to i
    p = jac_add_aff(p, g);
  }
  Fp inv = fp_inv(acc);
  for (size_t i = hi; i-- > lo;) {
    Fp prev = (i > lo) ? reg[i - 1].y : FP_ONE;
    Fp zi = fp_mul(inv, prev);  // 1/Z_i
    inv = fp_mul(inv, tmpJ[i].z);
    Fp zi2 = fp_sqr(zi);
    G1A a{fp_mul(tmpJ[i].x, zi2), fp_mul(fp_mul(tmpJ[i].y, zi2), zi), false};
    RegKey e{a.x, a.y};
    e.x.l[11] |= REG_VALID;
    reg[i] = e;
    if (out48) g1_compress(out48 + 48 * i, a);
  }
}

// ======================================================= host launchers ==
static inline unsigned nblk(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

#define LAUNCH(k, g, b, st, ...)                              \
  do {                                                        \
    hipLaunchKernelGGL(k, dim3(g), dim3(b), 0, st, __VA_ARGS__); \
    hipError_t e__ = hipGetLastError();                       \
    if (e__ != hipSuccess) return e__;                        \
  } while (0)

hipError_t launch_key_validate(hipStream_t st, const uint8_t* pks, size_t n, G1A* out, int* ok) {
  if (!n) return hipSuccess;
  LAUNCH(k_key_validate, nblk(n, 64), 64, st, pks, n, out, ok);
  return hipSuccess;
}

// Two-pass sums; tmp must hold >= 1 + nblk entries.
hipError_t launch_g1_sum_aff(hipStream_t st, const G1A* in, const int* ok, size_t n, G1J* tmp, G1J* out) {
  if (n <= G1Q_SUM_MAX) {
    LAUNCH(k_g1_sum_q, 1, G1Q_SUM_NT, st, in, ok, n, out);
    return hipSuccess;
  }
  unsigned g = nblk(n, 64);
  if (g > 1024) g = 1024;
  if (g == 0) g = 1;
  LAUNCH((k_g1_sum_aff<64>), g, 64, st, in, ok, n, tmp);
  LAUNCH((k_jac_sum<Fp, 64>), 1, 64, st, tmp, (size_t)g, out);
  return hipSuccess;
}
hipError_t launch_g2_sum_aff(hipStream_t st, const G2A* in, const int* ok, size_t n, G2J* tmp, G2J* out) {
  unsigned g = nblk(n, 64);
  if (g > 1024) g = 1024;
  if (g == 0) g = 1;
  LAUNCH(k_g2_sum_aff, g, 64, st, in, ok, n, tmp);
  LAUNCH((k_jac_sum<Fp2, 64>), 1, 64, st, tmp, (size_t)g, out);
  return hipSuccess;
}
hipError_t launch_g1_compress(hipStream_t st, const G1J* in, uint8_t* out48, int* is_inf) {
  LAUNCH(k_g1_compress, 1, 64, st, in, out48, is_inf);
  return hipSuccess;
}
hipError_t launch_g2_compress(hipStream_t st, const G2J* in, uint8_t* out96) {
  LAUNCH(k_g2_compress, 1, 64, st, in, out96);
  return hipSuccess;
}
hipError_t launch_percall_pairs(hipStream_t st, const G1A* keys, const int* key_ok, size_t n, const G1J* apk_sum,
                                const int* sig_ok, G1A* P, int* live, Fp* pz) {
  LAUNCH(k_percall_pairs, 1, 64, st, keys, key_ok, n, apk_sum, sig_ok, P, live, pz);
  return hipSuccess;
}
hipError_t launch_hash_many(hipStream_t st, const uint8_t* msgs, const uint64_t* offs, size_t n, const uint8_t* dst,
                            uint32_t dst_len, G2A* out) {
  if (!n) return hipSuccess;
  LAUNCH(k_hash_many, nblk(n, 64), 64, st, msgs, offs, n, dst, dst_len, out);
  return hipSuccess;
}
hipError_t launch_sign_many(hipStream_t st, const uint8_t* sks, const uint8_t* msgs, const uint64_t* offs, size_t n,
                            uint8_t* out, int* ok) {
  if (!n) return hipSuccess;
  LAUNCH(k_sign_many, nblk(n, 64), 64, st, sks, msgs, offs, n, out, ok);
  return hipSuccess;
}
hipError_t launch_sk_to_pk_many(hipStream_t st, const uint8_t* sks, size_t n, uint8_t* out, int* ok) {
  if (!n) return hipSuccess;
  LAUNCH(k_sk_to_pk_many, nblk(n, 64), 64, st, sks, n, out, ok);
  return hipSuccess;
}
hipError_t launch_fav_gather(hipStream_t st, const uint32_t* idx, const uint64_t* offs, size_t B, const RegKey* reg,
                             uint32_t reg_n, G1P* apk, int* status) {
  if (!B) return hipSuccess;
  // lanes per aggregate: 16 from 1,024 aggregates up (C2 and the C3 epoch of 2,048: 32 mixed additions per lane and
  // a 4-level tree beat 8 + 6 levels of 64 lanes -- C3 +4 %, profiles/r03u_inv_gather_ab.txt), else 64 (a few
  // aggregates spread over more lanes: shorter chains)
  if (B >= 1024)
    LAUNCH(k_fav_gather_q<16>, (unsigned)((B + 3) / 4), 64, st, idx, offs, B, reg, reg_n, apk, status,
           (const int*)nullptr);
  else
    LAUNCH(k_fav_gather_q<64>, (unsigned)B, 64, st, idx, offs, B, reg, reg_n, apk, status, (const int*)nullptr);
  return hipSuccess;
}
// the aggregates k_fav_gather_aff flagged (redo[b]): complete formulas, the others left as they are
hipError_t launch_fav_gather_redo(hipStream_t st, const uint32_t* idx, const uint64_t* offs, size_t B,
                                  const RegKey* reg, uint32_t reg_n, G1P* apk, int* status, const int* redo) {
  if (!B) return hipSuccess;
  LAUNCH(k_fav_gather_q<16>, (unsigned)((B + 3) / 4), 64, st, idx, offs, B, reg, reg_n, apk, status, redo);
  return hipSuccess;
}
hipError_t launch_av_items(hipStream_t st, size_t B, const uint64_t* io, const int* pk_ok, const int* sig_ok,
                           const G2A* sig, const uint64_t* rsc, int* status, G1A* P2, G2A* Q2) {
  if (!B) return hipSuccess;
  LAUNCH(k_av_items, nblk(B, 64), 64, st, B, io, pk_ok, sig_ok, sig, rsc, status, P2, Q2);
  return hipSuccess;
}
hipError_t launch_av_pairs(hipStream_t st, size_t total, const uint32_t* pair_item, const int* status,
                           const uint64_t* rsc, const G1A* pk, const G2A* H, G1A* P2, G2A* Q2) {
  if (!total) return hipSuccess;
  LAUNCH(k_av_pairs, nblk(total, 64), 64, st, total, pair_item, status, rsc, pk, H, P2, Q2);
  return hipSuccess;
}
hipError_t launch_g1_decode_checked(hipStream_t st, const uint8_t* in48, size_t n, G1A* out, int* ok) {
  if (!n) return hipSuccess;
  LAUNCH(k_g1_decode_checked, nblk(n, 64), 64, st, in48, n, out, ok);
  return hipSuccess;
}
hipError_t launch_g1_scale(hipStream_t st, const G1A* P, const uint8_t* k32, size_t n, G1A* out, int* live) {
  if (!n) return hipSuccess;
  LAUNCH(k_g1_scale, nblk(n, 64), 64, st, P, k32, n, out, live);
  return hipSuccess;
}
hipError_t launch_verdicts(hipStream_t st, const int* status, const uint8_t* bad, size_t B, uint8_t* out) {
  if (!B) return hipSuccess;
  LAUNCH(k_verdicts, nblk(B, 256), 256, st, status, bad, B, out);
  return hipSuccess;
}
hipError_t launch_status_to_u8(hipStream_t st, const int* status, size_t B, uint8_t* out) {
  if (!B) return hipSuccess;
  LAUNCH(k_status_to_u8, nblk(B, 256), 256, st, status, B, out);
  return hipSuccess;
}
hipError_t launch_fp12_to_bytes(hipStream_t st, const Fp12* f, uint8_t* out) {
  LAUNCH(k_fp12_to_bytes, 1, 64, st, f, out);
  return hipSuccess;
}
hipError_t launch_fp12_from_bytes(hipStream_t st, const uint8_t* in, size_t n, Fp12* f) {
  if (!n) return hipSuccess;
  LAUNCH(k_fp12_from_bytes, nblk(n, 64), 64, st, in, n, f);
  return hipSuccess;
}
hipError_t launch_registry_generate(hipStream_t st, uint64_t first, size_t n, G1J* tmpJ, RegKey* reg,
                                    uint8_t* out48) {
  if (!n) return hipSuccess;
  const uint32_t chunk = 32;
  size_t threads = (n + chunk - 1) / chunk;
  LAUNCH(k_registry_generate, nblk(threads, 64), 64, st, first, n, chunk, tmpJ, reg, out48);
  return hipSuccess;
}
hipError_t launch_reg_pack(hipStream_t st, const G1A* a, const int* ok, size_t n, RegKey* reg, uint8_t* valid) {
  if (!n) return hipSuccess;
  LAUNCH(k_reg_pack, nblk(n, 256), 256, st, a, ok, n, reg, valid);
  return hipSuccess;
}
hipError_t launch_g2_compress_aff(hipStream_t st, const G2A* in, uint8_t* out96) {
  LAUNCH(k_g2_compress_aff, 1, 64, st, in, out96);
  return hipSuccess;
}

}  // namespace bls
