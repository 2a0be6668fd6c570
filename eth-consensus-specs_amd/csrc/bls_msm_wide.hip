// k_msm_weighted_wide: the last stage of the RLC MSM (bls_msm.hip), S = sum_b 2^b U_b over the 64 bit-sums U_b,
// in wavefront-cooperative F2-layout arithmetic (bls_wide.h) with the complete projective formulas of
// bls_pp_lane.h (Renes-Costello-Batina, a = 0, 3b = 12 (1 + i)), so an identity U_b (a bit no scalar sets, small
// batches) needs no special case.  One workgroup of 16 waves: wave j first forms T_j = sum_i 2^(16 i) U_{j+16 i}
// by Horner (48 doublings, 3 additions), then a 4-level LDS tree folds node j + s into node j weighted by 2^s.
// The longest chain is 63 doublings and 7 additions of one wave -- the lane-pair kernel (k_msm_weighted) ran the
// same chain in per-lane arithmetic at ~25 us per doubling.
#include "bls_kernels.h"
#include "bls_lane.h"
#include "bls_wide.h"
#include "bls_wide_g2.h"

namespace bls {

using namespace wide;

namespace {
struct P2F {  // homogeneous projective (X : Y : Z), F2 layout; every coordinate a product output (< 1.1 p)
  uint32_t x, y, z;
};

// 3 b t = 12 xi t (t below 62 p: the xi subtraction against 64 p)
__device__ __forceinline__ uint32_t wf_b3(const WKG& K, uint32_t t) { return wmuls<12>(wf_xi(K.k1, t)); }

// bls_pp_lane.h pp_dbl: t0 = Y^2, t1 = Y Z, t2 = 3b Z^2, z8 = 8 t0, w = t0 - 3 t2,
//   X3 = 2 w X Y,  Y3 = w (t0 + t2) + t2 z8,  Z3 = t1 z8   (Y3 as one reduction of two products)
// bounds (units of p): t0, t1, Z^2, XY < 1.1; t2 < 790; w < 4100 (against 4096 p); every output a product
__device__ __forceinline__ P2F p2f_dbl(const WKG& K, const P2F& p) {
  const uint32_t kn = K.kneg;
  const uint32_t t0 = wf_sqr(K.k1, p.y);
  const uint32_t t1 = wf_mul(kn, p.y, p.z);
  const uint32_t t2 = wf_b3(K, wf_sqr(K.k1, p.z));
  const uint32_t u = wf_mul(kn, p.x, p.y);
  const uint32_t z8 = wmuls<8>(t0);
  const uint32_t w = wsubk(kn, t0, wmuls<3>(t2));
  P2F r;
  uint64_t acc = 0;
  wf_mac(acc, kn, w, wadd(t0, t2));
  wf_mac(acc, kn, t2, z8);
  r.y = wredc(acc);
  r.x = wf_mul(kn, w, wmuls<2>(u));
  r.z = wf_mul(kn, t1, z8);
  return r;
}

// bls_pp_lane.h pp_add / pp_finish with the cross terms as sums of products (t3 = X1 Y2 + Y1 X2, ...):
//   X3 = t3 t1' - t4 y3',  Y3 = t1' z3 + y3' 3 t0,  Z3 = z3 t4 + 3 t0 t3   (t1' = t1 - 3b t2, z3 = t1 + 3b t2,
//   y3' = 3b y3), each output one reduction; the big operands (y3' < 790 p) go first, the negated t4 (< 256 p)
//   second, inside kneg's 4096 p
__device__ __forceinline__ P2F p2f_add(const WKG& K, const P2F& p, const P2F& q) {
  const uint32_t kn = K.kneg;
  const uint32_t t0 = wf_mul(kn, p.x, q.x);
  const uint32_t t1 = wf_mul(kn, p.y, q.y);
  const uint32_t t2 = wf_mul(kn, p.z, q.z);
  uint64_t a3 = 0, a4 = 0, ay = 0;
  wf_mac(a3, kn, p.x, q.y);
  wf_mac(a3, kn, p.y, q.x);
  wf_mac(a4, kn, p.y, q.z);
  wf_mac(a4, kn, p.z, q.y);
  wf_mac(ay, kn, p.x, q.z);
  wf_mac(ay, kn, p.z, q.x);
  const uint32_t t3 = wredc(a3), t4 = wredc(a4), y3 = wf_b3(K, wredc(ay));
  const uint32_t bt2 = wf_b3(K, t2);
  const uint32_t t0x3 = wmuls<3>(t0);
  const uint32_t z3 = wadd(t1, bt2);
  const uint32_t t1m = wsubk(K.k1024, t1, bt2);
  P2F r;
  uint64_t ax = 0, ayy = 0, az = 0;
  wf_mac(ax, kn, t3, t1m);
  wf_mac(ax, kn, y3, wsubk(K.k256, 0u, t4));
  wf_mac(ayy, kn, t1m, z3);
  wf_mac(ayy, kn, y3, t0x3);
  wf_mac(az, kn, z3, t4);
  wf_mac(az, kn, t0x3, t3);
  r.x = wredc(ax);
  r.y = wredc(ayy);
  r.z = wredc(az);
  return r;
}

// a packed projective point of the lane kernels (x.c0, x.c1, y.c0, y.c1, z.c0, z.c1) into F2 layout
__device__ __forceinline__ P2F p2f_load(const Fp* in) {
  return P2F{wf_from_fp2(Fp2{in[0], in[1]}), wf_from_fp2(Fp2{in[2], in[3]}), wf_from_fp2(Fp2{in[4], in[5]})};
}
}  // namespace

__global__ void __launch_bounds__(1024) k_msm_weighted_wide(const Fp* U, G2A* out) {
  __shared__ uint32_t sm[8][3 * 64];
  const WKG K = wkg_init();
  const int lane = wlane(), j = (int)(threadIdx.x >> 6);
  P2F T = p2f_load(U + 6 * (j + 48));
#pragma unroll 1
  for (int i = 32; i >= 0; i -= 16) {
#pragma unroll 1
    for (int d = 0; d < 16; ++d) T = p2f_dbl(K, T);
    T = p2f_add(K, T, p2f_load(U + 6 * (j + i)));
  }
#pragma unroll 1
  for (int s = 8; s >= 1; s >>= 1) {
    if (j >= s && j < 2 * s) {
      sm[j - s][lane] = T.x;
      sm[j - s][64 + lane] = T.y;
      sm[j - s][128 + lane] = T.z;
    }
    __syncthreads();
    if (j < s) {
      P2F Bp{sm[j][lane], sm[j][64 + lane], sm[j][128 + lane]};
#pragma unroll 1
      for (int d = 0; d < s; ++d) Bp = p2f_dbl(K, Bp);
      T = p2f_add(K, T, Bp);
    }
    __syncthreads();
  }
  if (j == 0) {  // (X : Y : Z) -> (X / Z, Y / Z); Z = 0 is the identity
    const uint32_t sq = wsqr(T.z);
    const Fp nl = w_to_fp(wadd(sq, wswap(sq)));  // norm(Z)
    const uint32_t ni = w_from_fp(fp_inv_sg_i(nl));
    const uint32_t zi = wmul(wf_conj(K.k1, T.z), ni);
    const Fp2 x = wf_to_fp2(wf_mul(K.kneg, T.x, zi)), y = wf_to_fp2(wf_mul(K.kneg, T.y, zi));
    if (lane == 0) {
      G2A r;
      r.inf = fp_is_zero(nl);
      r.x = r.inf ? fp2_zero() : x;
      r.y = r.inf ? fp2_zero() : y;
      *out = r;
    }
  }
}

hipError_t launch_msm_weighted_wide(hipStream_t st, const Fp* U, G2A* out) {
  hipLaunchKernelGGL(k_msm_weighted_wide, dim3(1), dim3(1024), 0, st, U, out);
  return hipGetLastError();
}

}  // namespace bls
