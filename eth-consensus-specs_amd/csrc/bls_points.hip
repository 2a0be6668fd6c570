// Curve-object kernels behind the reference's G1/G2/GT helpers
// (E/utils/bls.py:224-392 with E = tests/core/pyspec/eth2spec): the arkworks
// G1Point / G2Point / GT operations the spec reaches through bls.add,
// bls.neg, bls.multiply, bls.multi_exp, bls.bytes48_to_G1 / bytes96_to_G2,
// bls.G1_to_bytes48 / G2_to_bytes96 and bls.pairing_check
// (specs/altair/beacon-chain.md:592-596, specs/deneb/polynomial-commitments.md).
//
// Points cross the C ABI compressed (48 / 96 B); every kernel decodes with the
// ZCash rules of g1_decompress / g2_decompress (identity encoding accepted),
// with or without the subgroup check (arkworks from_compressed_bytes vs
// from_compressed_bytes_unchecked, multiexp_unchecked), and re-compresses its
// result.  These are one-shot operations (one per block in
// process_sync_aggregate): small launches, not the FAV throughput path.
#include "bls_kernels.h"

namespace bls {

static __device__ __forceinline__ size_t ptid() { return (size_t)blockIdx.x * blockDim.x + threadIdx.x; }

// 32-byte big-endian scalar -> 8 little-endian u32 limbs
static __device__ void k32_parse(uint32_t k[8], const uint8_t* b) {
  for (int w = 0; w < 8; w++) {
    const uint8_t* q = b + 28 - 4 * w;
    k[w] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
}

// decode: 1 = valid point (identity included), 0 = invalid encoding / not in the subgroup
template <class F>
__device__ int pt_decode(Aff<F>& a, const uint8_t* in, int subgroup);

template <>
__device__ int pt_decode<Fp>(G1A& a, const uint8_t* in, int subgroup) {
  const int d = g1_decompress(a, in);
  if (d == DEC_INFINITY) {
    a = G1A{fp_zero(), fp_zero(), true};
    return 1;
  }
  if (d != DEC_OK) return 0;
  return !subgroup || g1_in_subgroup(jac_from_aff(a));
}

template <>
__device__ int pt_decode<Fp2>(G2A& a, const uint8_t* in, int subgroup) {
  const int d = g2_decompress(a, in);
  if (d == DEC_INFINITY) {
    a = G2A{fp2_zero(), fp2_zero(), true};
    return 1;
  }
  if (d != DEC_OK) return 0;
  return !subgroup || g2_in_subgroup(jac_from_aff(a));
}

static __device__ __forceinline__ void pt_compress(uint8_t* out, const G1A& a) { g1_compress(out, a); }
static __device__ __forceinline__ void pt_compress(uint8_t* out, const G2A& a) { g2_compress(out, a); }

// n independent decodes; ok[i] = 1/0, points to `out` (identity when invalid)
template <class F, int NB>
__global__ void __launch_bounds__(64) k_pt_decode(const uint8_t* in, size_t n, int subgroup, Aff<F>* out, int* ok) {
  const size_t i = ptid();
  if (i >= n) return;
  Aff<F> a;
  const int v = pt_decode<F>(a, in + NB * i, subgroup);
  if (!v) {
    fset_zero(a.x);
    fset_zero(a.y);
    a.inf = true;
  }
  out[i] = a;
  ok[i] = v;
}

// One binary operation on compressed points, one lane (unchecked decodes):
//   op 0: a + b          op 1: [k] a (k = 256-bit big-endian scalar)
// *ok = 0 when an input encoding is invalid (the reference raises).
template <class F, int NB>
__global__ void k_pt_binop(const uint8_t* a_in, const uint8_t* b_in, const uint8_t* k32, int op, uint8_t* out,
                           int* ok) {
  if (threadIdx.x || blockIdx.x) return;
  Aff<F> a, b;
  if (!pt_decode<F>(a, a_in, 0) || (op == 0 && !pt_decode<F>(b, b_in, 0))) {
    *ok = 0;
    return;
  }
  Jac<F> r;
  if (op == 0) {
    r = jac_add(jac_from_aff(a), jac_from_aff(b));
  } else {
    uint32_t k[8];
    k32_parse(k, k32);
    r = jac_mul_u256(jac_from_aff(a), k);
  }
  pt_compress(out, jac_to_aff(r));
  *ok = 1;
}

// per-point products [k_i] P_i (multi_exp), affine
template <class F>
__global__ void __launch_bounds__(64) k_pt_scale(const Aff<F>* P, const uint8_t* k32, size_t n, Aff<F>* out) {
  const size_t i = ptid();
  if (i >= n) return;
  uint32_t k[8];
  k32_parse(k, k32 + 32 * i);
  Aff<F> r;
  fset_zero(r.x);
  fset_zero(r.y);
  r.inf = true;
  if (!P[i].inf) r = jac_to_aff(jac_mul_u256(jac_from_aff(P[i]), k));
  out[i] = r;
}

// Sum of n affine points (two-pass: workgroup partials, then one workgroup)
template <class F>
__global__ void __launch_bounds__(64) k_pt_sum(const Aff<F>* in, size_t n, Jac<F>* out) {
  __shared__ Jac<F> sh[64];
  Jac<F> acc = jac_identity<F>();
  for (size_t i = (size_t)blockIdx.x * 64 + threadIdx.x; i < n; i += (size_t)gridDim.x * 64)
    acc = jac_add_aff(acc, in[i]);
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 32; s > 0; s >>= 1) {
    if (threadIdx.x < s) sh[threadIdx.x] = jac_add(sh[threadIdx.x], sh[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = sh[0];
}

template <class F>
__global__ void __launch_bounds__(64) k_pt_sum_jac(const Jac<F>* in, size_t n, Jac<F>* out) {
  __shared__ Jac<F> sh[64];
  Jac<F> acc = jac_identity<F>();
  for (size_t i = threadIdx.x; i < n; i += 64) acc = jac_add(acc, in[i]);
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 32; s > 0; s >>= 1) {
    if (threadIdx.x < s) sh[threadIdx.x] = jac_add(sh[threadIdx.x], sh[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = sh[0];
}

template <class F>
__global__ void k_pt_compress_jac(const Jac<F>* in, uint8_t* out) {
  if (threadIdx.x || blockIdx.x) return;
  pt_compress(out, jac_to_aff(in[0]));
}

// GT: the final exponentiation of a Miller product, as 576 bytes (the
// k_fp12_to_bytes layout), and the product of two GT elements.
static __device__ void fp12_store_bytes(const Fp12& f, uint8_t* out) {
  const Fp2* c[6] = {&f.c0.c0, &f.c1.c0, &f.c0.c1, &f.c1.c1, &f.c0.c2, &f.c1.c2};
  for (int k = 0; k < 6; k++) {
    raw_to_be48(fp_from_mont(c[k]->c0), out + 96 * k);
    raw_to_be48(fp_from_mont(c[k]->c1), out + 96 * k + 48);
  }
}
static __device__ Fp12 fp12_load_bytes(const uint8_t* b) {
  Fp12 r;
  Fp2* c[6] = {&r.c0.c0, &r.c1.c0, &r.c0.c1, &r.c1.c1, &r.c0.c2, &r.c1.c2};
  for (int k = 0; k < 6; k++) {
    c[k]->c0 = fp_to_mont(raw_from_be48(b + 96 * k));
    c[k]->c1 = fp_to_mont(raw_from_be48(b + 96 * k + 48));
  }
  return r;
}

// final_exponentiation() returns e^3 (its hard part is 3 (p^4 - p^2 + 1) / r,
// which the check kernels use as is: e == 1 <=> e^3 == 1).  A GT value must be
// e itself: e = (e^3)^d with d = 3^-1 mod r = (2r + 1) / 3 (255 bits).  One
// lane, ~370 Fp12 products: GT objects are not on the verification path.
__global__ void k_gt_final_exp(const Fp12* f, uint8_t* out576) {
  if (threadIdx.x || blockIdx.x) return;
  static constexpr uint32_t D[8] = {0x00000001u, 0xaaaaaaaau, 0x55543d54u, 0xe27e6d57u,
                                    0x066be558u, 0xccd13ab0u, 0x7113a8dau, 0x4d491a37u};
  const Fp12 e3 = final_exponentiation(*f);
  Fp12 r = e3;  // bit 254 of d is its top bit
  for (int i = 253; i >= 0; --i) {
    r = fp12_sqr(r);
    if ((D[i >> 5] >> (i & 31)) & 1u) r = fp12_mul(r, e3);
  }
  fp12_store_bytes(r, out576);
}

__global__ void k_gt_mul(const uint8_t* a576, const uint8_t* b576, uint8_t* out576) {
  if (threadIdx.x || blockIdx.x) return;
  fp12_store_bytes(fp12_mul(fp12_load_bytes(a576), fp12_load_bytes(b576)), out576);
}

// ================================================================ launchers ==
static inline unsigned pblk(size_t n) { return (unsigned)((n + 63) / 64); }

hipError_t launch_pt_decode(hipStream_t st, int group, const uint8_t* in, size_t n, int subgroup, void* out, int* ok) {
  if (!n) return hipSuccess;
  if (group == 1)
    hipLaunchKernelGGL((k_pt_decode<Fp, 48>), dim3(pblk(n)), dim3(64), 0, st, in, n, subgroup, (G1A*)out, ok);
  else
    hipLaunchKernelGGL((k_pt_decode<Fp2, 96>), dim3(pblk(n)), dim3(64), 0, st, in, n, subgroup, (G2A*)out, ok);
  return hipGetLastError();
}

hipError_t launch_pt_binop(hipStream_t st, int group, const uint8_t* a, const uint8_t* b, const uint8_t* k32, int op,
                           uint8_t* out, int* ok) {
  if (group == 1)
    hipLaunchKernelGGL((k_pt_binop<Fp, 48>), dim3(1), dim3(64), 0, st, a, b, k32, op, out, ok);
  else
    hipLaunchKernelGGL((k_pt_binop<Fp2, 96>), dim3(1), dim3(64), 0, st, a, b, k32, op, out, ok);
  return hipGetLastError();
}

// sum_i [k_i] P_i over decoded points P (group 1: G1A, 2: G2A); tmp: >= n
// affine + 1024 Jacobian scratch entries of the group's type; out compressed
template <class F>
static hipError_t pt_msm(hipStream_t st, const Aff<F>* P, const uint8_t* k32, size_t n, void* tmp, uint8_t* out) {
  Aff<F>* S = (Aff<F>*)tmp;
  Jac<F>* J = (Jac<F>*)(S + n);
  unsigned g = pblk(n);
  if (g > 1024) g = 1024;
  if (g == 0) g = 1;
  hipLaunchKernelGGL(k_pt_scale<F>, dim3(pblk(n ? n : 1)), dim3(64), 0, st, P, k32, n, S);
  hipLaunchKernelGGL(k_pt_sum<F>, dim3(g), dim3(64), 0, st, S, n, J);
  hipLaunchKernelGGL(k_pt_sum_jac<F>, dim3(1), dim3(64), 0, st, J, (size_t)g, J + 1024);
  hipLaunchKernelGGL(k_pt_compress_jac<F>, dim3(1), dim3(64), 0, st, J + 1024, out);
  return hipGetLastError();
}

size_t pt_msm_scratch_bytes(int group, size_t n) {
  return group == 1 ? n * sizeof(G1A) + 1025 * sizeof(G1J) : n * sizeof(G2A) + 1025 * sizeof(G2J);
}

hipError_t launch_pt_msm(hipStream_t st, int group, const void* P, const uint8_t* k32, size_t n, void* tmp,
                         uint8_t* out) {
  return group == 1 ? pt_msm<Fp>(st, (const G1A*)P, k32, n, tmp, out)
                    : pt_msm<Fp2>(st, (const G2A*)P, k32, n, tmp, out);
}

hipError_t launch_gt_final_exp(hipStream_t st, const Fp12* f, uint8_t* out576) {
  hipLaunchKernelGGL(k_gt_final_exp, dim3(1), dim3(64), 0, st, f, out576);
  return hipGetLastError();
}

hipError_t launch_gt_mul(hipStream_t st, const uint8_t* a, const uint8_t* b, uint8_t* out) {
  hipLaunchKernelGGL(k_gt_mul, dim3(1), dim3(64), 0, st, a, b, out);
  return hipGetLastError();
}

}  // namespace bls
