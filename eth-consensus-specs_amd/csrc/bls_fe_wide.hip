// k_fe_wide: the final-exponentiation check in wavefront-cooperative arithmetic (bls_wide.h, F2 layout) on six
// waves, easy and hard part -- the per-call path's check.  Same schedule, same answer as k_fe_check
// (bls_fe.hip), which stays the batch / bisection check.
#include "bls_kernels.h"
#include "bls_lane.h"
#include "bls_wide.h"
#include "bls_wide_g2.h"

namespace bls {

using namespace wide;

// ---- final-exponentiation check: easy part lane-parallel, hard part in F2 layout on six waves ----------
// Wave 0 runs the product of the partials and the easy part with the lane-parallel phase executor of bls_fe.h
// (the other waves only keep the barriers); the result t = f^((p^6 - 1)(p^2 + 1)) then moves into six LDS rows
// of F2-layout values (wave k owns the w^k coefficient), and the hard part -- four x-power chains of cyclotomic
// squarings (Granger-Scott: per w^k one or two Fp2 products), Fp12 products (six per wave), Frobenius maps and
// conjugations, in fe_schedule's order -- runs with every wave forming its coefficient of each result.  Every
// bank value is brought below 2.0001p after each operation (a product by R mod p), so the cyclotomic
// formula's 3 t - 2 a and the products' xi terms subtract small values against 64p.
// gamma1_k = xi^(k (p - 1) / 6) (A^p: w^k coefficient -> conj(c_k) gamma1_k) and gamma2_k = gamma1_k conj(gamma1_k)
// (real), per w-basis index k
__device__ static const Fp2 FE_W_G1[6] = {FROB1_0, FROB1_1, FROB1_2, FROB1_3, FROB1_4, FROB1_5};
__device__ static const Fp2 FE_W_G2[6] = {FROB2_0, FROB2_1, FROB2_2, FROB2_3, FROB2_4, FROB2_5};

struct FeWide {
  uint32_t* B;  // banks: B[(bank * 6 + k) * 64 + lane]
  int k, lane;
  WKG K;
  uint32_t two, mtwo;  // 2 and -2 (Montgomery form, both halves)
  __device__ uint32_t ld(int bank, int j) const { return B[(bank * 6 + j) * 64 + lane]; }
  // publish this wave's coefficient of bank d; an operation whose destination is also a source waits for every
  // wave's reads first, otherwise the barrier after the previous write already ordered them
  __device__ void put(int d, uint32_t v, bool inplace) {
    if (inplace) __syncthreads();
    B[(d * 6 + k) * 64 + lane] = v;
    __syncthreads();
  }
  __device__ uint32_t xi(uint32_t v) const { return wf_xi(K.k256, v); }
  __device__ uint32_t real(uint32_t v) const { return whalf() ? 0u : v; }  // v in half 0 only (a real Fp2)
  // D = A B: coefficient k = sum_{i <= k} a_i b_{k-i} + sum_{i > k} a_i (xi b_{k-i+6}), twelve wmac terms per
  // half into one reduction
  __device__ void mul(int a, int b, int d) {
    uint64_t acc = 0;
#pragma unroll 1
    for (int i = 0; i < 6; i++) {
      const int j = k - i < 0 ? k - i + 6 : k - i;
      const uint32_t bj = ld(b, j);
      wf_mac(acc, K.kneg, ld(a, i), i > k ? xi(bj) : bj);
    }
    put(d, wredc(acc), d == a || d == b);
  }
  // D = A^2, A cyclotomic (Granger-Scott on the Fp4 pairs (a_k, a_k+3), bls_fe.h / tools/gen_fe.py op_cyc):
  //   a0' = 3 (a0^2 + xi a3^2) - 2 a0,  a3' = 6 a0 a3 + 2 a3,  a2' = 3 (a1^2 + xi a4^2) - 2 a2,  a5' = 6 a1 a4 + 2 a5,
  //   a4' = 3 (a2^2 + xi a5^2) - 2 a4,  a1' = 6 xi a2 a5 + 2 a1
  // each as ONE reduction of a few products, the linear terms folded in as products by the constants +-2:
  //   a0' = a0 (3 a0 - 2) + (3 xi a3) a3,  a3' = a3 (6 a0 + 2),  a2' = a1 (3 a1) + (3 xi a4) a4 + a2 (-2),
  //   a5' = a1 (6 a4) + a5 2,  a4' = a2 (3 a2) + (3 xi a5) a5 + a4 (-2),  a1' = (6 xi a2) a5 + a1 2
  __device__ void cyc(int a, int d) {
    const int m = k == 0 || k == 3 ? 0 : (k == 2 || k == 5 ? 1 : 2);  // the pair (m, m + 3) this output needs
    const uint32_t x = ld(a, m), y = ld(a, m + 3);
    uint64_t acc = 0;
    if (k == 0) {
      wf_mac(acc, K.kneg, x, wnorm(wmuls<3>(x) + real(wnorm(K.k1 - two))));
      wf_mac(acc, K.kneg, wmuls<3>(xi(y)), y);
    } else if (k == 3) {
      wf_mac(acc, K.kneg, y, wnorm(wmuls<6>(x) + real(two)));
    } else if (k == 2 || k == 4) {
      wf_mac(acc, K.kneg, x, wmuls<3>(x));
      wf_mac(acc, K.kneg, wmuls<3>(xi(y)), y);
      wf_mac_fp(acc, ld(a, k), mtwo);
    } else if (k == 5) {
      wf_mac(acc, K.kneg, x, wmuls<6>(y));
      wf_mac_fp(acc, ld(a, 5), two);
    } else {  // k == 1
      wf_mac(acc, K.kneg, wmuls<6>(xi(x)), y);
      wf_mac_fp(acc, ld(a, 1), two);
    }
    put(d, wredc(acc), d == a);
  }
  // conjugation: the odd coefficients negated (64 p - v: sources are product outputs, below 1.1 p)
  __device__ void conj(int a, int d) {
    const uint32_t v = ld(a, k);
    put(d, (k & 1) ? wnorm(K.k1 - v) : v, d == a);
  }
  __device__ void frob1(int a, int d, uint32_t g) {  // conj(a_k) gamma1_k
    uint64_t acc = 0;
    wf_mac(acc, K.kneg, wf_conj(K.k256, ld(a, k)), g);
    put(d, wredc(acc), d == a);
  }
  __device__ void frob2(int a, int d, uint32_t g2) {  // a_k gamma2_k (gamma2_k in Fp: both halves)
    uint64_t acc = 0;
    wf_mac_fp(acc, ld(a, k), g2);
    put(d, wredc(acc), d == a);
  }
  // easy part: bank 0 = f on entry, t = f^((p^6 - 1)(p^2 + 1)) on exit (banks 1 .. 5 temporaries):
  //   g = conj(f), N = f g in Fp6 (the even coefficients n0, n2, n4 = Fp6 coefficients of v^0, v^1, v^2),
  //   N^-1 = (t0, t1, t2) / d with t0 = n0^2 - xi n2 n4, t1 = xi n4^2 - n0 n2, t2 = n2^2 - n0 n4,
  //   d = n0 t0 + xi (n4 t1 + n2 t2) (one Fp2 inversion: conj(d) / norm(d), the Fp inverse lane-local),
  //   f^(p^6 - 1) = g^2 N^-1, then t = (f^(p^6 - 1))^(p^2) f^(p^6 - 1)
  __device__ void easy(uint32_t g2) {
    const uint32_t kn = K.kneg;
    conj(0, 1);
    mul(0, 1, 2);
    {
      const uint32_t n0 = ld(2, 0), n2 = ld(2, 2), n4 = ld(2, 4);
      uint64_t acc = 0;
      if (k == 0) {
        wf_mac(acc, kn, n0, n0);
        wf_mac(acc, kn, wsubk(K.k1024, 0u, xi(n2)), n4);
      } else if (k == 2) {
        wf_mac(acc, kn, xi(n4), n4);
        wf_mac(acc, kn, wsubk(K.k1, 0u, n0), n2);
      } else if (k == 4) {
        wf_mac(acc, kn, n2, n2);
        wf_mac(acc, kn, wsubk(K.k1, 0u, n0), n4);
      }
      put(3, (k & 1) ? 0u : wredc(acc), false);
    }
    if (k == 0) {
      uint64_t acc = 0;
      wf_mac(acc, kn, ld(2, 0), ld(3, 0));
      wf_mac(acc, kn, xi(ld(2, 4)), ld(3, 2));
      wf_mac(acc, kn, xi(ld(2, 2)), ld(3, 4));
      const uint32_t d = wredc(acc);
      const uint32_t sq = wsqr(d);
      const Fp nl = w_to_fp(wadd(sq, wswap(sq)));  // norm(d) in both halves
      const uint32_t ni = w_from_fp(fp_inv_sg_i(nl));
      B[(4 * 6 + 0) * 64 + lane] = wmul(wf_conj(K.k1, d), ni);
    }
    __syncthreads();
    {
      uint64_t acc = 0;
      wf_mac(acc, kn, ld(3, k), ld(4, 0));  // odd k: a zero coefficient
      put(5, wredc(acc), false);
    }
    mul(1, 1, 2);
    mul(2, 5, 0);  // f^(p^6 - 1)
    frob2(0, 1, g2);
    mul(1, 0, 0);
  }
  // dst = src^x = conj(src^|x|): the chain ping-pongs between dst and tmp so each step has one barrier
  __device__ void powx(int src, int dst, int tmp) {
    int acc = src, o = dst;
#pragma unroll 1
    for (int i = 62; i >= 0; --i) {
      cyc(acc, o);
      acc = o;
      o = o == dst ? tmp : dst;
      if ((X_ABS >> i) & 1ull) {
        mul(acc, src, o);
        acc = o;
        o = o == dst ? tmp : dst;
      }
    }
    conj(acc, dst);
  }
};

// sel: workgroup b checks fin[sel[b]] into out[b].  nchecks != nullptr (the bisection tree's levels, bls_capi.hip
// fav_bisect): workgroup b checks fin[b] into out[b] when parent is null or parent[b / pdiv] == 0 (and counts it in
// *nchecks), else out[b] = 1 without a check.
__global__ void __launch_bounds__(384) k_fe_wide(const Fp12* fin, int n, const uint32_t* sel, int* out, uint64_t* ts,
                                                 const int* parent, uint32_t pdiv, uint32_t* nchecks) {
  if (nchecks) {
    const uint32_t b = blockIdx.x;
    fin += b;
    out += b;
    if (parent && parent[b / pdiv]) {  // uniform over the workgroup: it leaves before any barrier
      if (threadIdx.x == 0) *out = 1;
      return;
    }
    if (threadIdx.x == 0) atomicAdd(nchecks, 1u);
  }
  int nts = 0;
  auto stamp = [&]() {
    if (ts && threadIdx.x == 0) ts[nts] = wall_clock64();
    nts++;
  };
  stamp();
  __shared__ uint32_t B[7 * 6 * 64];
  __shared__ int bad;
  // wave w owns coefficient k = w with 3 and 4 swapped.  Six waves on a CU's four SIMDs: waves 0 / 4 and 1 / 5
  // share a SIMD, 2 and 3 run alone.  A cyclotomic squaring step -- the x-power chains' unit, one barrier each --
  // costs k = 0: 2 products, 1: 1 + a real one, 2 and 4: 2 + a real one, 3: 1, 5: 1 + a real one; so the shared
  // SIMDs get {0, 3} and {1, 5} and the two heaviest run alone (a step's slowest SIMD: 3 products instead of
  // 2 + 2 + a real one with k = w)
  const int lane = wlane(), wv = (int)(threadIdx.x >> 6), k = wv == 3 ? 4 : (wv == 4 ? 3 : wv);
  if (sel) {
    fin += sel[blockIdx.x];
    out += blockIdx.x;
  }
  if (threadIdx.x == 0) bad = 0;
  FeWide W;
  W.B = B;
  W.k = k;
  W.lane = lane;
  W.K = wkg_init();
  W.two = wmuls<2>(W.K.one);
  W.mtwo = wnorm(W.K.k1 - W.two);
  // the partials in F2 layout (w^k is the tower Fp2 (k & 1) * 3 + (k >> 1)), multiplied up in bank 0
  const int tp = (k & 1) * 3 + (k >> 1);
#pragma unroll 1
  for (int i = 0; i < n; i++) {
    const Fp* fp = reinterpret_cast<const Fp*>(fin + i);
    const uint32_t v = wf_from_fp2(Fp2{fp[2 * tp], fp[2 * tp + 1]});
    if (i == 0) {
      B[(0 * 6 + k) * 64 + lane] = v;
      __syncthreads();
    } else {
      W.put(1, v, false);
      W.mul(0, 1, 0);
    }
  }
  stamp();
  const uint32_t wg1 = wf_from_fp2(FE_W_G1[k]), wg2 = w_from_fp(FE_W_G2[k].c0);
  W.easy(wg2);  // bank 0 = t
  stamp();
  // hard part, bls_fe.h fe_schedule's order (banks 0..5)
  W.powx(0, 1, 6);      // 1 = t^x
  stamp();
  W.conj(0, 3);
  W.mul(3, 1, 2);    // 2 = a = t^(x-1)
  W.powx(2, 1, 6);      // 1 = a^x
  W.conj(2, 3);
  W.mul(1, 3, 2);    // 2 = a = t^((x-1)^2)
  W.powx(2, 1, 6);      // 1 = a^x
  W.frob1(2, 3, wg1);  // 3 = a^p
  W.mul(3, 1, 3);    // 3 = b = a^(x+p)
  W.powx(3, 1, 6);      // 1 = b^x
  W.powx(1, 4, 6);      // 4 = b^(x^2)
  W.frob2(3, 5, wg2);  // 5 = b^(p^2)
  W.mul(4, 5, 1);
  W.conj(3, 4);      // 4 = b^-1
  W.mul(1, 4, 1);    // 1 = c = b^(x^2+p^2-1)
  W.cyc(0, 5);
  W.mul(5, 0, 5);    // 5 = t^3
  W.mul(1, 5, 1);    // 1 = c t^3
  stamp();
  const Fp2 v = wf_to_fp2(W.ld(1, k));
  const bool ok = k == 0 ? (fp_is_one(v.c0) && fp_is_zero(v.c1)) : (fp_is_zero(v.c0) && fp_is_zero(v.c1));
  if (lane == 0 && !ok) atomicOr(&bad, 1);
  __syncthreads();
  if (threadIdx.x == 0) *out = bad ? 0 : 1;
}

hipError_t launch_fe_wide(hipStream_t st, const Fp12* f, int n, int* out, uint64_t* ts) {
  hipLaunchKernelGGL(k_fe_wide, dim3(1), dim3(384), 0, st, f, n, (const uint32_t*)nullptr, out, ts, (const int*)nullptr,
                     1u, (uint32_t*)nullptr);
  return hipGetLastError();
}

hipError_t launch_fe_wide_gated(hipStream_t st, const Fp12* node, size_t n, const int* parent, uint32_t pdiv, int* res,
                                uint32_t* nchecks) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_fe_wide, dim3((unsigned)n), dim3(384), 0, st, node, 1, (const uint32_t*)nullptr, res,
                     (uint64_t*)nullptr, parent, pdiv, nchecks);
  return hipGetLastError();
}

}  // namespace bls
