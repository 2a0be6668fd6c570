// S = sum_i r_i sigma_i for the RLC batch check (Pippenger, 8-bit windows).
//
// The 64-bit scalars split into 8 windows; the (item, window) pairs with a
// nonzero digit d are counting-sorted into 8 x 255 buckets (atomic histogram,
// one block-wide prefix scan, atomic scatter).  Seven launches:
//   k_msm_count, k_msm_scan, k_msm_scatter   the sort
//   k_msm_bucketc   each bucket's points summed in C strided chunks (C = 8 for
//                   a C2 batch: one lane pair per chunk, ~5 mixed additions
//                   each, 16,384 chunks = 512 waves, the point loads one step
//                   ahead; fewer for smaller batches, msm_chunks), the chunks
//                   then folded into the bucket sum B_{w,d} in LDS
//   k_msm_usum      U_b = sum_{d : bit k of d} B_{w,d}  (b = 8w + k): one
//                   wave per b, 32 lane pairs adding 4 bucket sums each, then a
//                   5-level LDS tree (a 16-wave wide-arithmetic variant
//                   measured C2 -4 %: profiles/r04o_usum_ab.txt)
//   k_msm_upairs    the 64 pairs (-2^b G1, U_b), U_b affine: the Miller loop
//                   of (-G1, S) with S = sum_b 2^b U_b is, after the final
//                   exponentiation, the product of e(-2^b G1, U_b) -- so the
//                   U_b join the batch's own pairs (lines + f accumulation)
//                   and the 63-doubling weighted sum S (round 4:
//                   k_msm_weighted_wide, one 16-wave workgroup, ~0.7 ms) and
//                   its one-pair Miller loop (k_miller_wide, ~0.5 ms) leave
//                   the latency chain.  The -2^b G1 are entries of the
//                   bisection's fixed-base comb (bls_bisect.hip).
// ~8 additions per signature instead of a 64-step double-and-add.  (The
// previous form ran one lane pair per bucket -- 64 waves, ~40 dependent
// additions with unprefetched loads -- and 13 tree launches: ~6.8 ms per C2
// batch.)
#include "bls_kernels.h"
#include "bls_fp_inv.h"
#include "bls_pp_lane.h"


namespace bls {

constexpr int MSM_W = 8, MSM_NB = MSM_W * 256;

// cnt[MSM_NB] must be zero on entry.
__global__ void __launch_bounds__(256) k_msm_count(size_t B, const int* status, const int* status2, const uint64_t* rsc,
                                                   uint32_t* cnt) {
  const size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= B * MSM_W) return;
  const size_t i = k / MSM_W;
  const int w = (int)(k % MSM_W);
  if (!status[i] || !status2[i]) return;
  const uint32_t d = (uint32_t)(rsc[i] >> (8 * w)) & 0xffu;
  if (d) atomicAdd(&cnt[w * 256 + d], 1u);
}

// off[b] = exclusive prefix of cnt; cur[b] = off[b] (scatter cursor); one 256-thread block, 8 buckets per thread
__global__ void __launch_bounds__(256) k_msm_scan(const uint32_t* cnt, uint32_t* off, uint32_t* cur) {
  constexpr int PER = MSM_NB / 256;
  __shared__ uint32_t part[256];
  const int t = threadIdx.x;
  uint32_t loc[PER], sum = 0;
#pragma unroll
  for (int i = 0; i < PER; i++) {
    loc[i] = cnt[t * PER + i];
    sum += loc[i];
  }
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {  // inclusive Hillis-Steele scan of the per-thread sums
    const uint32_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t base = part[t] - sum;
#pragma unroll
  for (int i = 0; i < PER; i++) {
    off[t * PER + i] = base;
    cur[t * PER + i] = base;
    base += loc[i];
  }
  if (t == 255) off[MSM_NB] = part[255];
}

__global__ void __launch_bounds__(256) k_msm_scatter(size_t B, const int* status, const int* status2,
                                                     const uint64_t* rsc, uint32_t* cur, uint32_t* lst) {
  const size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= B * MSM_W) return;
  const size_t i = k / MSM_W;
  const int w = (int)(k % MSM_W);
  if (!status[i] || !status2[i]) return;
  const uint32_t d = (uint32_t)(rsc[i] >> (8 * w)) & 0xffu;
  if (d) lst[atomicAdd(&cur[w * 256 + d], 1u)] = (uint32_t)i;
}

constexpr int MSM_CMAX = 8;  // chunks per bucket, at most (msm_chunks)
// chunks per bucket for a batch of B items: ~B / 255 points per bucket (8 windows of 255 nonzero digits); enough
// chunks that a bucket's chain stays short on full batches, few enough that a C3- or C5-size batch is not mostly
// fold tree and idle lanes (8 chunks of ~1 point each plus a 3-level fold at 2,048 items)
static int msm_chunks(size_t B) {
  const size_t per = B / 255;
  return per >= 32 ? 8 : per >= 12 ? 4 : per >= 4 ? 2 : 1;
}
using P2 = PP<Fp2>;

// ----------------------------------------------------------- lane form --
// Bucket, U and weighted sums on lane pairs (bls_pp_lane.h pp2_*: complete
// projective formulas, each dependency level split between lanes 2k / 2k+1).
namespace {
// a point through LDS or HBM as six packed Fp: lane 0 of a pair writes x, y.c0, lane 1 y.c1, z
__device__ __forceinline__ void p2_store(Fp* o, const P2& p, bool hi) {  // selects, not a branch: no stack copy
  Fp* d = o + (hi ? 3 : 0);
  d[0] = fp_select(hi, p.y.c1, p.x.c0);
  d[1] = fp_select(hi, p.z.c0, p.x.c1);
  d[2] = fp_select(hi, p.z.c1, p.y.c0);
}
__device__ __forceinline__ P2 p2_load(const Fp* in) {
  return P2{Fp2{in[0], in[1]}, Fp2{in[2], in[3]}, Fp2{in[4], in[5]}};
}
}  // namespace

// chunk c of bucket b (lane pair (b, c)): csum[b C + c] = sum of the bucket's points k = off[b] + c + j C
template <int MSM_C>
__global__ void __launch_bounds__(64) k_msm_bucketc(const uint32_t* off, const uint32_t* lst, const G2A* sig,
                                                    Fp* csum) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  const int pi = t >> 1;
  const bool hi = (t & 1) != 0;
  // every lane reaches the fold's barriers: the grid covers the MSM_NB * MSM_C lane pairs exactly
  static_assert((2 * MSM_NB * MSM_C) % 64 == 0 && MSM_C <= 32, "k_msm_bucketc: whole waves, chunks within a wave");
  const int b = pi / MSM_C, c = pi % MSM_C;
  P2 R{fp2_zero(), fp2_one(), fp2_zero()};
  const uint32_t end = off[b + 1];
  uint32_t k = off[b] + c;
  // the next point is in flight while this one is added (both lanes of a pair run the same trip count)
  G2A q = sig[k < end ? lst[k] : 0u];
  uint32_t li = k + MSM_C < end ? lst[k + MSM_C] : 0u;
#pragma unroll 1
  for (; k < end; k += MSM_C) {
    const G2A cq = q;
    q = sig[li];
    li = k + 2 * MSM_C < end ? lst[k + 2 * MSM_C] : 0u;
    R = pp2_add_aff(R, cq.x, cq.y, hi);
  }
  // the bucket's MSM_C chunk sums (lane pairs C b' .. C b' + C - 1 of this wave) folded by a log2(C)-level LDS tree, so the
  // U sums read one point per bucket instead of re-adding its chunks once per set bit of the digit
  __shared__ Fp sm[32 * 6];
  const int lp = threadIdx.x >> 1;  // lane pair in the wave
#pragma unroll 1
  for (int s = MSM_C / 2; s >= 1; s >>= 1) {
    if (c >= s && c < 2 * s) p2_store(sm + 6 * (lp - s), R, hi);
    __syncthreads();
    if (c < s) R = pp2_add(R, p2_load(sm + 6 * lp), hi);
    __syncthreads();
  }
  if (c == 0) p2_store(csum + (size_t)b * 6, R, hi);
}

// U_b for b = blockIdx.x (w = b / 8, bit k = b % 8): one wave of 32 lane pairs; pair j adds the bucket sums of
// the digits d_j, d_{j+32}, d_{j+64}, d_{j+96} (d_i = the i-th digit with bit k set), then a 5-level LDS tree.
// (128 pairs over four waves with a 7-level tree ran one addition shorter but held 4x the waves at barriers:
// 16 % -> 9 % of a C3 epoch's wave time after the bucket fold, profiles/r04n2_c3_timeline.txt.)
constexpr int USUM_PAIRS = 32;
__global__ void __launch_bounds__(64) k_msm_usum(const Fp* csum, Fp* U) {
  __shared__ Fp sm[(USUM_PAIRS / 2) * 6];
  const int b = blockIdx.x, w = b >> 3, kb = b & 7;
  const int j = threadIdx.x >> 1;
  const bool hi = (threadIdx.x & 1) != 0;
  auto bucket = [&](int i) {
    const int d = ((i >> kb) << (kb + 1)) | (1 << kb) | (i & ((1 << kb) - 1));
    return csum + (size_t)(w * 256 + d) * 6;
  };
  P2 R = p2_load(bucket(j));
#pragma unroll 1
  for (int t = 1; t < 128 / USUM_PAIRS; ++t) R = pp2_add(R, p2_load(bucket(j + USUM_PAIRS * t)), hi);
#pragma unroll 1
  for (int s = USUM_PAIRS / 2; s >= 1; s >>= 1) {
    if (j >= s && j < 2 * s) p2_store(sm + 6 * (j - s), R, hi);
    __syncthreads();
    if (j < s) R = pp2_add(R, p2_load(sm + 6 * j), hi);
    __syncthreads();
  }
  if (j == 0) p2_store(U + 6 * b, R, hi);
}

// lane b < 64: pair (-2^b G1, U_b) at P[b], Q[b], ok[b] = 1 (U_b = the identity: Q[b].inf, a skipped pair).
// -2^b G1 = comb[256 (b / 8) + 2^(b % 8)] (comb[256 w + d] = d 2^(8 w) (-G1)).
__global__ void __launch_bounds__(64) k_msm_upairs(const Fp* U, const G1A* comb, G1A* P, G2A* Q, int* ok) {
  const int b = threadIdx.x;
  const Fp* u = U + 6 * b;
  const Fp2 X{u[0], u[1]}, Y{u[2], u[3]}, Z{u[4], u[5]};
  G2A q{fp2_zero(), fp2_zero(), true};
  if (!fp2_is_zero(Z)) {  // homogeneous projective (RCB): x = X / Z, y = Y / Z
    const Fp ni = fp_inv_sg_i(fp_add(fp_sqr_i(Z.c0), fp_sqr_i(Z.c1)));  // 1 / norm(Z)
    const Fp2 zi{fp_mul_i(Z.c0, ni), fp_neg(fp_mul_i(Z.c1, ni))};
    q = G2A{f2mul(X, zi), f2mul(Y, zi), false};
  }
  Q[b] = q;
  P[b] = comb[256 * (b >> 3) + (1 << (b & 7))];
  ok[b] = 1;
}

// Scratch: cnt[MSM_NB] | off[MSM_NB + 1] | cur[MSM_NB] (u32), lst[8 B] (u32);
// points (packed Fp, 6 per point, in units of Fd slots): chunk sums [MSM_NB * MSM_CMAX] | U [64].
size_t msm_scratch_u32(size_t B) { return (size_t)3 * MSM_NB + 1 + MSM_W * B; }
size_t msm_scratch_fd() { return ((size_t)(MSM_NB * MSM_CMAX + 64) * 6 * sizeof(Fp) + sizeof(Fd) - 1) / sizeof(Fd); }

hipError_t launch_msm_upairs(hipStream_t st, size_t B, const int* status, const int* status2, const uint64_t* rsc,
                             const G2A* sig, uint32_t* scr, Fd* pts, const G1A* comb, G1A* P, G2A* Q, int* ok) {
  uint32_t* cnt = scr;
  uint32_t* off = cnt + MSM_NB;
  uint32_t* cur = off + MSM_NB + 1;
  uint32_t* lst = cur + MSM_NB;
  Fp* csum = reinterpret_cast<Fp*>(pts);
  Fp* U = csum + (size_t)MSM_NB * MSM_CMAX * 6;
  hipError_t e = hipMemsetAsync(cnt, 0, MSM_NB * sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  const unsigned nb = (unsigned)((B * MSM_W + 255) / 256);
  if (B) {
    hipLaunchKernelGGL(k_msm_count, dim3(nb), dim3(256), 0, st, B, status, status2, rsc, cnt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_msm_scan, dim3(1), dim3(256), 0, st, cnt, off, cur);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (B) {
    hipLaunchKernelGGL(k_msm_scatter, dim3(nb), dim3(256), 0, st, B, status, status2, rsc, cur, lst);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  switch (msm_chunks(B)) {
    case 8: hipLaunchKernelGGL(k_msm_bucketc<8>, dim3(2 * MSM_NB * 8 / 64), dim3(64), 0, st, off, lst, sig, csum); break;
    case 4: hipLaunchKernelGGL(k_msm_bucketc<4>, dim3(2 * MSM_NB * 4 / 64), dim3(64), 0, st, off, lst, sig, csum); break;
    case 2: hipLaunchKernelGGL(k_msm_bucketc<2>, dim3(2 * MSM_NB * 2 / 64), dim3(64), 0, st, off, lst, sig, csum); break;
    default: hipLaunchKernelGGL(k_msm_bucketc<1>, dim3(2 * MSM_NB / 64), dim3(64), 0, st, off, lst, sig, csum);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_msm_usum, dim3(64), dim3(2 * USUM_PAIRS), 0, st, csum, U);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_msm_upairs, dim3(1), dim3(64), 0, st, U, comb, P, Q, ok);
  return hipGetLastError();
}

}  // namespace bls
