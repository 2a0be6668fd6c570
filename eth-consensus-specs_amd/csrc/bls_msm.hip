// S = sum_i r_i sigma_i for the RLC batch check (Pippenger, 8-bit windows).
//
// The 64-bit scalars split into 8 windows; the (item, window) pairs with a
// nonzero digit d are counting-sorted into 8 x 255 buckets (atomic histogram,
// one prefix pass, atomic scatter), and each bucket's points are added by a
// lane pair (k_msm_bucket2, one mixed addition per step).  The bucket reduction is parallel:
//   U_b = sum_{d : bit k of d} B_{w,d}   (b = 8w + k; 64 sums of 128 buckets,
//                                          a 7-level pairwise tree), then
//   S   = sum_b 2^b U_b                   (a 6-level tree of A + [2^k] B).
// ~8 additions per signature instead of a 64-step double-and-add; the chain
// runs on its own high-priority stream beside the Miller loops of the
// (r_i apk_i, H_i) pairs.
#include "bls_kernels.h"
#include "bls_pp_lane.h"
#include "bls_vm.h"

#include <stdlib.h>

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

// off[b] = exclusive prefix of cnt; cur[b] = off[b] (scatter cursor).
__global__ void k_msm_scan(const uint32_t* cnt, uint32_t* off, uint32_t* cur) {
  if (threadIdx.x || blockIdx.x) return;
  uint32_t s = 0;
  for (int b = 0; b < MSM_NB; b++) {
    off[b] = s;
    cur[b] = s;
    s += cnt[b];
  }
  off[MSM_NB] = s;
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

// U-tree input: ubase[(8w + k) * 128 + j] = B_{w, d_j} with d_j the j-th digit
// having bit k set (bit k inserted into j).
__global__ void __launch_bounds__(256) k_msm_gather_bits(const Fd* bsum, Fd* ubase) {
  const int t = blockIdx.x * 256 + threadIdx.x;  // (b, j, coordinate)
  if (t >= 64 * 128 * 6) return;
  const int c = t % 6, j = (t / 6) % 128, b = t / (6 * 128);
  const int w = b >> 3, k = b & 7;
  const int d = ((j >> k) << (k + 1)) | (1 << k) | (j & ((1 << k) - 1));
  ubase[t] = bsum[(size_t)(w * 256 + d) * 6 + c];
}

// ----------------------------------------------------------- lane form --
// The bucket sums and both reduction trees on lane pairs (bls_pp_lane.h pp2_*)
// instead of wave programs: a bucket is ~40 sequential mixed additions, a tree
// node one addition (after k doublings), so a 64-lane workgroup spent most of
// its time staging slots and on per-level barriers for 4 items.  Same points
// in the same projective form (complete formulas), same Fd staging.
namespace {
__device__ __forceinline__ PP<Fp2> msm_load(const Fd* in) {
  return PP<Fp2>{Fp2{fp_from_fd(in[0]), fp_from_fd(in[1])}, Fp2{fp_from_fd(in[2]), fp_from_fd(in[3])},
                 Fp2{fp_from_fd(in[4]), fp_from_fd(in[5])}};
}
__device__ __forceinline__ void msm_store(Fd* o, const PP<Fp2>& p, bool hi) {
  if (!hi) {
    o[0] = fd_from_fp(p.x.c0);
    o[1] = fd_from_fp(p.x.c1);
    o[2] = fd_from_fp(p.y.c0);
  } else {
    o[3] = fd_from_fp(p.y.c1);
    o[4] = fd_from_fp(p.z.c0);
    o[5] = fd_from_fp(p.z.c1);
  }
}
}  // namespace

// bucket b = (lane pair index): bsum[b] = sum of its points (identity (0 : 1 : 0) if empty)
__global__ void __launch_bounds__(64) k_msm_bucket2(const uint32_t* off, const uint32_t* lst, const G2A* sig,
                                                    Fd* bsum) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  const int b = t >> 1;
  const bool hi = (t & 1) != 0;
  if (b >= MSM_NB) return;
  PP<Fp2> R{fp2_zero(), fp2_one(), fp2_zero()};
  const uint32_t lo = off[b], hi_end = off[b + 1];
  // both lanes of a pair run the same trip count (the pair's bucket)
#pragma unroll 1
  for (uint32_t k = lo; k < hi_end; ++k) {
    const G2A& q = sig[lst[k]];
    R = pp2_add_aff(R, q.x, q.y, hi);
  }
  msm_store(bsum + (size_t)b * 6, R, hi);
}

// out[j] = in[2j] + [2^k] in[2j+1] (k = 0: plain sum), one lane pair per output
__global__ void __launch_bounds__(64) k_msm_tree2(const Fd* in, int nout, int k, Fd* out) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  const int j = t >> 1;
  const bool hi = (t & 1) != 0;
  if (j >= nout) return;
  const PP<Fp2> A = msm_load(in + (size_t)(2 * j) * 6);
  PP<Fp2> Bp = msm_load(in + (size_t)(2 * j + 1) * 6);
#pragma unroll 1
  for (int s = 0; s < k; ++s) Bp = pp2_dbl(Bp, hi);
  msm_store(out + (size_t)j * 6, pp2_add(A, Bp, hi), hi);
}

// projective S -> affine (identity if Z = 0)
__global__ void __launch_bounds__(64) k_msm_affine(const Fd* pt, G2A* out) {
  __shared__ Fd s[WP_NCONST + WL_MA_STRIDE];
  const int lane = threadIdx.x;
  vm_load_consts(s);
  const int item0 = WP_NCONST;
  if (lane < 6) s[item0 + WL_MA_P + lane] = pt[lane];
  __syncthreads();
  vm_run<1>(VM_PROG(MA_NORM), s, item0, 0, nullptr);
  if (lane == 0) s[item0 + WL_MA_NI] = fd_from_fp(fp_inv(fp_from_fd(s[item0 + WL_MA_N])));
  __syncthreads();
  vm_run<1>(VM_PROG(MA_INVFIN), s, item0, 0, nullptr);
  vm_run<1>(VM_PROG(MA_TOAFF), s, item0, 0, nullptr);
  if (lane == 0) {
    G2A r;
    r.inf = fd_is_zero(s[item0 + WL_MA_N]);
    r.x = Fp2{fp_from_fd(s[item0 + WL_MA_XY]), fp_from_fd(s[item0 + WL_MA_XY + 1])};
    r.y = Fp2{fp_from_fd(s[item0 + WL_MA_XY + 2]), fp_from_fd(s[item0 + WL_MA_XY + 3])};
    if (r.inf) r.x = r.y = fp2_zero();
    *out = r;
  }
}

// Scratch: cnt[MSM_NB] | off[MSM_NB + 1] | cur[MSM_NB] (u32), lst[8 B] (u32);
// points (Fd): bsum[MSM_NB * 6] | tree ping [64 * 128 * 6] | pong [64 * 64 * 6].
size_t msm_scratch_u32(size_t B) { return (size_t)3 * MSM_NB + 1 + MSM_W * B; }
size_t msm_scratch_fd() { return (size_t)MSM_NB * 6 + 64 * 128 * 6 + 64 * 64 * 6; }

hipError_t launch_msm(hipStream_t st, size_t B, const int* status, const int* status2, const uint64_t* rsc,
                      const G2A* sig, uint32_t* scr, Fd* pts, G2A* out) {
  uint32_t* cnt = scr;
  uint32_t* off = cnt + MSM_NB;
  uint32_t* cur = off + MSM_NB + 1;
  uint32_t* lst = cur + MSM_NB;
  Fd* bsum = pts;
  Fd* ping = bsum + (size_t)MSM_NB * 6;
  Fd* pong = ping + (size_t)64 * 128 * 6;
  hipError_t e = hipMemsetAsync(cnt, 0, MSM_NB * sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  const unsigned nb = (unsigned)((B * MSM_W + 255) / 256);
  if (B) {
    hipLaunchKernelGGL(k_msm_count, dim3(nb), dim3(256), 0, st, B, status, status2, rsc, cnt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_msm_scan, dim3(1), dim3(64), 0, st, cnt, off, cur);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (B) {
    hipLaunchKernelGGL(k_msm_scatter, dim3(nb), dim3(256), 0, st, B, status, status2, rsc, cur, lst);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_msm_bucket2, dim3(2 * MSM_NB / 64), dim3(64), 0, st, off, lst, sig, bsum);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_msm_gather_bits, dim3(64 * 128 * 6 / 256), dim3(256), 0, st, bsum, ping);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // U tree: 64 x 128 -> 64 (7 levels of pairwise sums; sets stay contiguous)
  Fd* a = ping;
  Fd* b = pong;
  for (int n = 64 * 64; n >= 64; n >>= 1) {
    hipLaunchKernelGGL(k_msm_tree2, dim3((2 * n + 63) / 64), dim3(64), 0, st, a, n, 0, b);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    Fd* t = a;
    a = b;
    b = t;
  }
  // weighted tree: sum_b 2^b U_b, 64 -> 1
  int k = 1;
  for (int n = 32; n >= 1; n >>= 1, k <<= 1) {
    hipLaunchKernelGGL(k_msm_tree2, dim3((2 * n + 63) / 64), dim3(64), 0, st, a, n, k, b);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    Fd* t = a;
    a = b;
    b = t;
  }
  hipLaunchKernelGGL(k_msm_affine, dim3(1), dim3(64), 0, st, a, out);
  return hipGetLastError();
}

}  // namespace bls
