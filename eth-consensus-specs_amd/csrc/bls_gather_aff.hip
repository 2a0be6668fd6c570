// Registry gather of the FAV batch path with affine additions that share one
// inversion per tree level (Montgomery's trick) -- the aggregate public keys
// apk_b = sum_j registry[idx_j] of SURVEY.md §8(d) (E/utils/bls.py:167-177:
// FastAggregateVerify aggregates its pubkeys before the pairing check).
//
// Work per addition (FME = one 381-bit Montgomery product):
//   complete projective mixed addition (k_fav_gather_q)            11
//   affine addition, inversion shared over the level's m pairs     6 + 84 / m
//     lambda = (y2 - y1) / (x2 - x1): 3 products of the batch inversion (prefix
//     product, and the walk back's two) + 1; x3 = lambda^2 - x1 - x2: 1;
//     y3 = lambda (x1 - x3) - y1: 1; one safegcd inversion (~84 FME) per level.
// A lane owns a contiguous run of its aggregate's keys (all of them for full
// batches: one lane per aggregate) and halves its point list level by level
// while a level has >= 16 pairs, then adds the <= 31 points left into a
// projective accumulator with the complete mixed formulas (bls_fq_g1.h).  A
// 512-key committee: 496 affine additions in 5 levels + 15 mixed additions =
// ~3,560 FME against ~5,620 for 511 mixed additions.
//
// The level lists live in per-lane scratch in HBM (a point is one 128-B slot,
// seven 16-B loads off one address); the level-0 list is read straight from the
// registry's 128-B records, twice (forward and walk-back passes).  The kernel
// fits two waves per SIMD (256 registers): one wave alone issues at most every
// other VALU slot of its SIMD (MI355X_MICROARCH.md), so a kernel that holds a
// SIMD alone wastes the half its partner would use.
//
// Exceptional cases: x1 == x2 (P1 = +-P2: a doubling or the identity) makes a
// level's product of denominators 0 mod p, which the one canonical check before
// the inversion sees.  The aggregate is then flagged (redo[b]) and recomputed by
// k_fav_gather_q's complete formulas (launch_fav_gather_redo), which have no
// exceptional case; its verdict never depends on the affine path.  Registry
// keys are distinct validators, so only adversarial committees (duplicate
// indices, keys chosen as sums of other keys) take that path.
#include <cstdlib>

#include "bls_kernels.h"
#include "bls_fp_inv.h"
#include "bls_fq_g1.h"
#include "bls_fqb.h"

namespace bls {

namespace {

using FqS = FqB<2, fqb_detail::MASK>;  // a stored coordinate: the fold's output (value < 1.32 p, exact digits)

constexpr uint32_t FOLD_C = 0x13b06ba5u;  // floor(2^409 / p): q = d13 FOLD_C / 2^32 <= d13 2^377 / p

// x - q p, q = floor(d13 2^377 / p) (q p <= x), the digits carried through one signed chain.  Value bound: with
// digits 0..12 <= D < 2^31, x < (d13 + 4.0001) 2^377, and q p > d13 2^377 - p (1 + d13 2^-32), so x - q p < 1.32 p
// for V <= 2^20; the chain leaves exact 29-bit digits 0..12 and digit 13 = floor((x - q p) / 2^377) <= 17.
template <uint64_t V, uint64_t D>
__device__ __forceinline__ FqS fold(const FqB<V, D>& a) {
  static_assert(D < (1ull << 31) && V <= (1ull << 20), "fold: digit or value bound outside its proof");
  const uint32_t q = (uint32_t)(((uint64_t)a.x.d[13] * FOLD_C) >> 32);
  Fq r;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 13; i++) {
    const int64_t t = (int64_t)a.x.d[i] - (int64_t)q * (int64_t)P29[i] + c;
    r.d[i] = (uint32_t)t & Q29_MASK;
    c = t >> 29;
  }
  r.d[13] = (uint32_t)((int64_t)a.x.d[13] - (int64_t)q * (int64_t)P29[13] + c);
  return {r};
}

struct Pt {
  FqS x, y;
};

// Per-lane scratch, slot-major: slot e of lane g is 128 B at ((e * NL + g) * 32) words (x in words 0..13, y in
// 16..29; prefix products 64 B, words 0..13), so a point is seven 16-B loads off one address.  Regions: A (level
// outputs 0, 2, 4, ..: CH / 2 points), Bq (levels 1, 3, ..: CH / 4 points), P (prefix products: CH / 2 values).
struct AffScr {
  uint32_t* base;
  size_t nl, g;  // lanes of the launch, this lane
  int ch;        // keys per chunk (a power of two)
  __device__ uint32_t* buf_a() const { return base; }
  __device__ uint32_t* buf_b() const { return base + (size_t)(ch / 2) * 32 * nl; }
  __device__ uint32_t* buf_p() const { return base + (size_t)(ch / 2 + ch / 4) * 32 * nl; }
  __device__ uint32_t* pt(uint32_t* b, int slot) const { return b + ((size_t)slot * nl + g) * 32; }
  __device__ const uint32_t* pt(const uint32_t* b, int slot) const { return b + ((size_t)slot * nl + g) * 32; }
  __device__ uint32_t* pre(int slot) const { return buf_p() + ((size_t)slot * nl + g) * 16; }
};

__device__ __forceinline__ Fq ld14(const uint32_t* a) {
  Fq r;
  const uint4* q = reinterpret_cast<const uint4*>(a);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint4 v = q[k];
    r.d[4 * k] = v.x;
    r.d[4 * k + 1] = v.y;
    r.d[4 * k + 2] = v.z;
    r.d[4 * k + 3] = v.w;
  }
  const uint2 t = reinterpret_cast<const uint2*>(a)[6];
  r.d[12] = t.x;
  r.d[13] = t.y;
  return r;
}
__device__ __forceinline__ void st14(uint32_t* a, const Fq& v) {
  uint4* q = reinterpret_cast<uint4*>(a);
#pragma unroll
  for (int k = 0; k < 3; k++) q[k] = make_uint4(v.d[4 * k], v.d[4 * k + 1], v.d[4 * k + 2], v.d[4 * k + 3]);
  reinterpret_cast<uint2*>(a)[6] = make_uint2(v.d[12], v.d[13]);
}

// registry key k's coordinate (affine, canonical; word 0 = x, 12 = y of the 128-B record); x's top bit is the
// registry's validity flag
__device__ __forceinline__ FqS ld_key_x(const RegKey* reg, uint32_t reg_n, uint32_t k, bool& ok) {
  const uint4* r = reinterpret_cast<const uint4*>(reg + (k < reg_n ? k : 0u));
  Fp x;
#pragma unroll
  for (int w = 0; w < 3; ++w) reinterpret_cast<uint4*>(x.l)[w] = r[w];
  ok = k < reg_n && (x.l[11] & REG_VALID);
  x.l[11] &= ~REG_VALID;
  return relax<2, fqb_detail::MASK>(fqb_canon(x));
}
__device__ __forceinline__ FqS ld_key_y(const RegKey* reg, uint32_t reg_n, uint32_t k) {
  const uint4* r = reinterpret_cast<const uint4*>(reg + (k < reg_n ? k : 0u));
  Fp y;
#pragma unroll
  for (int w = 0; w < 3; ++w) reinterpret_cast<uint4*>(y.l)[w] = r[3 + w];
  return relax<2, fqb_detail::MASK>(fqb_canon(y));
}

// coordinate c (0 = x, 1 = y) of point j of a level's list: the registry (level 0: key k = idx[k0 + j], loaded by
// the caller one step ahead) or the scratch list
template <bool REG>
__device__ __forceinline__ FqS ld_c(uint32_t k, const RegKey* reg, uint32_t reg_n, const uint32_t* src,
                                    const AffScr& s, int j, int c, bool& bad) {
  if constexpr (REG) {
    if (c) return ld_key_y(reg, reg_n, k);
    bool ok;
    const FqS x = ld_key_x(reg, reg_n, k, ok);
    bad |= !ok;
    return x;
  } else {
    return FqS{ld14(s.pt(src, j) + 16 * c)};
  }
}
template <bool REG>
__device__ __forceinline__ uint32_t key_of(const uint32_t* idx, uint64_t k0, int j) {
  if constexpr (REG) return idx[k0 + j];
  return 0u;
}

// One level: the list of m points (>= 32) -> ceil(m / 2) points in dst (pairs added, an odd last point copied).
// The walk back loads each coordinate only where it is next used, so at most x1, x1 + x2, y1, lambda, inv and one
// product's state are live (the kernel fits two waves per SIMD without spilling).  Software pipelining: the
// forward pass loads pair i + 1's x while pair i's product runs; at level 0 both passes load the next pair's
// registry indices one step ahead, so a record load waits for one memory latency, not two.
template <bool REG>
__device__ __forceinline__ int aff_level(const uint32_t* idx, uint64_t k0, const RegKey* reg, uint32_t reg_n,
                                         const uint32_t* src, uint32_t* dst, const AffScr& s, int m, bool& bad,
                                         bool& exc) {
  const int np = m >> 1;
  // forward: pre[i] = prod_{k < i} (x_2k+1 - x_2k); the level's keys are validated here (REG)
  FqN acc{fq_unpack(FP_ONE)};
  uint32_t ka = key_of<REG>(idx, k0, 0), kb = key_of<REG>(idx, k0, 1);
  FqS nx1 = ld_c<REG>(ka, reg, reg_n, src, s, 0, 0, bad), nx2 = ld_c<REG>(kb, reg, reg_n, src, s, 1, 0, bad);
  ka = key_of<REG>(idx, k0, 2);
  kb = key_of<REG>(idx, k0, 3);
#pragma unroll 1
  for (int i = 0; i < np; i++) {
    const FqS x1 = nx1, x2 = nx2;
    if (i + 1 < np) {
      nx1 = ld_c<REG>(ka, reg, reg_n, src, s, 2 * i + 2, 0, bad);
      nx2 = ld_c<REG>(kb, reg, reg_n, src, s, 2 * i + 3, 0, bad);
      if (i + 2 < np) {
        ka = key_of<REG>(idx, k0, 2 * i + 4);
        kb = key_of<REG>(idx, k0, 2 * i + 5);
      }
    }
    if (i) st14(s.pre(i), acc.x);
    acc = acc * (x2 - x1);
  }
  // one inversion for the level; a zero product means some x1 == x2 (an exceptional pair): the aggregate is redone
  // by the complete formulas
  const Fp pk = fq_pack_n(acc.x);
  exc |= fp_is_zero(pk);
  FqN inv{fq_unpack(fp_inv_sg_i(pk))};
  bool dummy = false;
  ka = key_of<REG>(idx, k0, 2 * np - 2);
  kb = key_of<REG>(idx, k0, 2 * np - 1);
#pragma unroll 1
  for (int i = np - 1; i >= 0; i--) {
    const uint32_t k1 = ka, k2 = kb;
    if (i) {
      ka = key_of<REG>(idx, k0, 2 * i - 2);
      kb = key_of<REG>(idx, k0, 2 * i - 1);
    }
    const FqS x1 = ld_c<REG>(k1, reg, reg_n, src, s, 2 * i, 0, dummy);
    const FqS x2 = ld_c<REG>(k2, reg, reg_n, src, s, 2 * i + 1, 0, dummy);
    const auto sx = x1 + x2;
    const FqN inv_i = i ? inv * FqN{ld14(s.pre(i))} : inv;
    if (i) inv = inv * (x2 - x1);
    const FqS y1 = ld_c<REG>(k1, reg, reg_n, src, s, 2 * i, 1, dummy);
    const FqS y2 = ld_c<REG>(k2, reg, reg_n, src, s, 2 * i + 1, 1, dummy);
    const FqN lam = (y2 - y1) * inv_i;
    const FqS x3 = fold(norm(sqr(lam) - sx));
    uint32_t* o = s.pt(dst, i);
    st14(o, x3.x);
    st14(o + 16, fold(norm(lam * (x1 - x3) - y1)).x);
  }
  if (m & 1) {
    const uint32_t k = key_of<REG>(idx, k0, m - 1);
    uint32_t* o = s.pt(dst, np);
    st14(o, ld_c<REG>(k, reg, reg_n, src, s, m - 1, 0, bad).x);
    st14(o + 16, ld_c<REG>(k, reg, reg_n, src, s, m - 1, 1, bad).x);
  }
  return np + (m & 1);
}

// the chunk of keys idx[k0 .. k0 + m) (m <= s.ch) added into the projective accumulator
__device__ __forceinline__ void aff_chunk(const uint32_t* idx, uint64_t k0, int m, const RegKey* reg, uint32_t reg_n,
                          const AffScr& s, G1Q& acc, bool& bad, bool& exc) {
  const uint32_t* cur = nullptr;
  if (m >= 32) {
    m = aff_level<true>(idx, k0, reg, reg_n, nullptr, s.buf_a(), s, m, bad, exc);
    cur = s.buf_a();
    bool in_a = true;
#pragma unroll 1
    while (m >= 32) {
      uint32_t* dst = in_a ? s.buf_b() : s.buf_a();
      m = aff_level<false>(idx, k0, reg, reg_n, cur, dst, s, m, bad, exc);
      cur = dst;
      in_a = !in_a;
    }
  }
  // the <= 31 points left: complete mixed additions on canonical coordinates (k_fav_gather_q's inputs)
#pragma unroll 1
  for (int j = 0; j < m; j++) {
    FqS x, y;
    if (cur) {
      x = ld_c<false>(0u, reg, reg_n, cur, s, j, 0, bad);
      y = ld_c<false>(0u, reg, reg_n, cur, s, j, 1, bad);
    } else {
      const uint32_t k = idx[k0 + j];
      x = ld_c<true>(k, reg, reg_n, cur, s, j, 0, bad);
      y = ld_c<true>(k, reg, reg_n, cur, s, j, 1, bad);
    }
    acc = g1q_add_aff(acc, fq_unpack(fq_pack_n(x.x)), fq_unpack(fq_pack_n(y.x)));
  }
}

}  // namespace

// L lanes per aggregate, 64 / L aggregates per workgroup; lane ln of aggregate b owns the ln-th of L contiguous runs
// of its keys, processed in chunks of s.ch keys.  Output as k_fav_gather_q: canonical projective apk[b], status[b]
// (keys valid, non-empty, sum not the identity); redo[b] = 1 when an exceptional pair occurred (status 0 until
// launch_fav_gather_redo recomputes it).
template <int L>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) k_fav_gather_aff(const uint32_t* idx, const uint64_t* offs, size_t B,
                                                       const RegKey* reg, uint32_t reg_n, G1P* apk, int* status,
                                                       uint32_t* scr, int ch, int* redo) {
  constexpr int IPW = 64 / L;
  __shared__ G1Q sh[L > 1 ? 64 : 1];
  __shared__ int flags[IPW];
  const int sub = (int)threadIdx.x / L, ln = (int)threadIdx.x % L;
  const size_t b = (size_t)blockIdx.x * IPW + sub;
  if ((int)threadIdx.x < IPW) flags[threadIdx.x] = 0;
  if constexpr (L > 1) __syncthreads();
  const AffScr s{scr, (size_t)gridDim.x * 64, (size_t)blockIdx.x * 64 + threadIdx.x, ch};
  G1Q acc{fq_zero(), fq_unpack(FP_ONE), fq_zero()};  // identity (0 : 1 : 0)
  bool bad = false, exc = false;
  uint64_t lo = 0, hi = 0;
  if (b < B) {
    lo = offs[b];
    hi = offs[b + 1];
    const uint64_t n = hi - lo;
    const uint64_t s0 = lo + n * (uint64_t)ln / L, s1 = lo + n * (uint64_t)(ln + 1) / L;
#pragma unroll 1
    for (uint64_t k0 = s0; k0 < s1; k0 += (uint64_t)ch) {
      const uint64_t left = s1 - k0;
      aff_chunk(idx, k0, left < (uint64_t)ch ? (int)left : ch, reg, reg_n, s, acc, bad, exc);
    }
  }
  if (bad || exc) atomicOr(&flags[sub], (bad ? 1 : 0) | (exc ? 2 : 0));
  if constexpr (L > 1) {
    sh[threadIdx.x] = acc;
    __syncthreads();
#pragma unroll 1
    for (int st = L / 2; st > 0; st >>= 1) {
      if (ln < st) sh[threadIdx.x] = g1q_add(sh[threadIdx.x], sh[threadIdx.x + st]);
      __syncthreads();
    }
    if (ln == 0) acc = sh[threadIdx.x];
  } else {
    __syncthreads();
  }
  if (ln == 0 && b < B) {  // canonical projective aggregate key; the identity is invalid (KeyValidate of the sum)
    const G1P o{fq_pack(acc.x), fq_pack(acc.y), fq_pack(acc.z)};
    const int f = flags[sub];
    apk[b] = o;
    status[b] = (hi > lo && !f && !fp_is_zero(o.z)) ? 1 : 0;
    redo[b] = (f & 2) ? 1 : 0;
  }
}

// Scratch words of k_fav_gather_aff for B aggregates (launch_fav_gather_aff's chunk size for that B); 0 when the
// batch takes the complete-formula kernel alone.
static void aff_shape(size_t B, int* L, int* ch, size_t* nl) {
  // full batches (C2): one lane per aggregate; C3's 2,048 / C5's 1,024: four (the launch's latency is what the
  // smaller batches see); below 1,024 the complete-formula kernel (AggregateVerify-sized calls, bisection leaves)
  static const int lanes = getenv("BLS_GATHER_L") ? atoi(getenv("BLS_GATHER_L")) : 1;
  *L = B >= 4096 ? (lanes == 2 || lanes == 4 ? lanes : 1) : 0;
  if (!*L) {
    *ch = 0;
    *nl = 0;
    return;
  }
  const size_t ipw = 64 / (size_t)*L;
  *nl = (B + ipw - 1) / ipw * 64;
  // chunk: 512 keys (a mainnet committee in one chunk), smaller when the lanes are many (the C4 firehose's 125,000
  // one-key items) so the scratch stays <= ~1 GiB: 128 B per key of chunk per lane
  int c = 512;
  while (c > 32 && (size_t)c * 128 * *nl > ((size_t)1 << 30)) c >>= 1;
  *ch = c;
}

size_t fav_gather_aff_words(size_t B) {
  int L, ch;
  size_t nl;
  aff_shape(B, &L, &ch, &nl);
  return L ? (size_t)ch * 32 * nl : 0;  // (CH/2 + CH/4) x 32 + CH/2 x 16 words per lane
}

hipError_t launch_fav_gather_aff(hipStream_t st, const uint32_t* idx, const uint64_t* offs, size_t B,
                                 const RegKey* reg, uint32_t reg_n, G1P* apk, int* status, uint32_t* scr, int* redo) {
  if (!B) return hipSuccess;
  int L, ch;
  size_t nl;
  aff_shape(B, &L, &ch, &nl);
  if (!L) return hipErrorInvalidValue;
  const dim3 grid((unsigned)(nl / 64));
  if (L == 1)
    hipLaunchKernelGGL(k_fav_gather_aff<1>, grid, dim3(64), 0, st, idx, offs, B, reg, reg_n, apk, status, scr, ch, redo);
  else if (L == 2)
    hipLaunchKernelGGL(k_fav_gather_aff<2>, grid, dim3(64), 0, st, idx, offs, B, reg, reg_n, apk, status, scr, ch, redo);
  else
    hipLaunchKernelGGL(k_fav_gather_aff<4>, grid, dim3(64), 0, st, idx, offs, B, reg, reg_n, apk, status, scr, ch, redo);
  return hipGetLastError();
}

}  // namespace bls
