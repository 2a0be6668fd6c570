// Kernels of the bisection fallback of a failing FAV batch (bls_capi.hip fav_bisect), which reuses the batch's own
// Miller kernels for its per-item values:
//   k_neg_g1_comb_table  once per context: comb[256 w + d] = d 2^(8 w) (-G1), affine (d = 1 .. 255, w = 0 .. 7)
//   k_neg_rg1            -r_i G1 from the comb: eight complete mixed additions per item (fixed base, no doublings)
//   k_verdicts_res       verdict = status && the item's leaf passed (or inherited its ancestors' pass)
// The gated final-exponentiation checks of the tree levels are k_fe_check_gated (bls_fe.hip), the leaf and node
// products k_fp12_chunk_prod2 / k_fp12_chunk_prod (bls_wave_kernels.hip).
#include "bls_kernels.h"
#include "bls_fq_g1.h"
#include "bls_fp_inv.h"

namespace bls {

namespace {
inline unsigned nblk(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }
}  // namespace

constexpr int COMB_W = 8, COMB_D = 256;  // 8-bit windows of the 64-bit RLC scalar

__global__ void __launch_bounds__(64) k_neg_g1_comb_table(G1A* tab) {
  const int t = (int)(blockIdx.x * 64 + threadIdx.x);
  if (t >= COMB_W * COMB_D) return;
  const int w = t / COMB_D, d = t % COMB_D;
  G1A g = g1_generator();
  const G1Q A{fq_unpack(g.x), fq_unpack(fp_neg(g.y)), fq_unpack(FP_ONE)};
  const uint64_t k = (uint64_t)d << (8 * w);
  G1Q R{fq_zero(), fq_unpack(FP_ONE), fq_zero()};
#pragma unroll 1
  for (int b = 63; b >= 0; --b) {  // complete formulas: the identity start and d = 0 need no special case
    R = g1q_dbl(R);
    if ((k >> b) & 1ull) R = g1q_add(R, A);
  }
  const Fp z = fq_pack(R.z);
  G1A o{fp_zero(), fp_zero(), true};
  if (!fp_is_zero(z)) {
    const Fp zi = fp_inv_sg_i(z);
    o = G1A{fp_mul_i(fq_pack(R.x), zi), fp_mul_i(fq_pack(R.y), zi), false};
  }
  tab[t] = o;
}

// -r_i G1 = sum_w d_w 2^(8 w) (-G1), r_i = sum_w d_w 2^(8 w): the table entries are affine, so each window is one
// complete mixed addition (RCB alg. 8, g1q_add_aff; the identity start needs no case) -- 8 x 12 products per item
// where a double-and-add chain on -G1 would take ~64 doublings and ~32 additions.  Items with status 0 are skipped
// (their leaf is 1 on both sides, bls_capi.hip fav_bisect).
__global__ void __launch_bounds__(64) k_neg_rg1(size_t B, const int* status, const uint64_t* rsc, const G1A* tab,
                                                G1P* out) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= B) return;
  if (!status[i]) {
    out[i] = G1P{fp_zero(), FP_ONE, fp_zero()};
    return;
  }
  const uint64_t r = rsc[i];
  G1Q R{fq_zero(), fq_unpack(FP_ONE), fq_zero()};
#pragma unroll 1
  for (int w = 0; w < COMB_W; ++w) {
    const uint32_t d = (uint32_t)(r >> (8 * w)) & (COMB_D - 1);
    const G1A& t = tab[w * COMB_D + (d ? d : 1)];
    const G1Q S = g1q_add_aff(R, fq_unpack(t.x), fq_unpack(t.y));
    if (d) R = S;
  }
  out[i] = G1P{fq_pack(R.x), fq_pack(R.y), fq_pack(R.z)};
}

__global__ void k_verdicts_res(const int* status, const int* res, size_t B, uint8_t* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) out[i] = (status[i] && res[i]) ? 1 : 0;
}

size_t neg_g1_comb_entries() { return (size_t)COMB_W * COMB_D; }

hipError_t launch_neg_g1_comb_table(hipStream_t st, G1A* tab) {
  hipLaunchKernelGGL(k_neg_g1_comb_table, dim3(nblk(neg_g1_comb_entries(), 64)), dim3(64), 0, st, tab);
  return hipGetLastError();
}

hipError_t launch_neg_rg1(hipStream_t st, size_t B, const int* status, const uint64_t* rsc, const G1A* tab, G1P* tmp,
                          G1A* out) {
  if (!B) return hipSuccess;
  hipLaunchKernelGGL(k_neg_rg1, dim3(nblk(B, 64)), dim3(64), 0, st, B, status, rsc, tab, tmp);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_g1_affine(st, B, status, tmp, out);
}

hipError_t launch_verdicts_res(hipStream_t st, const int* status, const int* res, size_t B, uint8_t* out) {
  if (!B) return hipSuccess;
  hipLaunchKernelGGL(k_verdicts_res, dim3(nblk(B, 256)), dim3(256), 0, st, status, res, B, out);
  return hipGetLastError();
}

}  // namespace bls
