// k_fe_check: the final-exponentiation check of a product of Fp12 values on
// one 64-lane wave, lane-parallel (bls_fe.h: phase executor, tables from
// tools/gen_fe.py, schedule).  Replaces the wave-program k_final_check_vm on
// every batch check, bisection round, per-call verification and RCCL
// exchange (launch_final_check_wave / launch_final_check_sel / launch_final_check_gated).
//
// The descriptors of the two operations that make up the hard part -- the
// cyclotomic squaring (315 calls) and the Fp12 product (~40) -- are loaded
// into registers once per kernel; the one-shot phases of the easy part read
// theirs from the table when they run.
#include "bls_kernels.h"
#include "bls_fe.h"

namespace bls {

namespace {

struct FeDev : FeOps<FeDev> {
  FeSlot* s;
  int lane;
  FeDesc<FE_NT_MUL_0, FE_NY_MUL_0> m0;
  FeDesc<FE_NT_MUL_1, FE_NY_MUL_1> m1;
  FeDesc<FE_NT_MUL_2, FE_NY_MUL_2> m2;
  FeDesc<FE_NT_CYC_0, FE_NY_CYC_0> c0;
  FeDesc<FE_NT_CYC_1, FE_NY_CYC_1> c1;

  __device__ void init() {
    m0 = fe_desc<FE_NT_MUL_0, FE_NY_MUL_0>(FE_PH_MUL_0, lane);
    m1 = fe_desc<FE_NT_MUL_1, FE_NY_MUL_1>(FE_PH_MUL_1, lane);
    m2 = fe_desc<FE_NT_MUL_2, FE_NY_MUL_2>(FE_PH_MUL_2, lane);
    c0 = fe_desc<FE_NT_CYC_0, FE_NY_CYC_0>(FE_PH_CYC_0, lane);
    c1 = fe_desc<FE_NT_CYC_1, FE_NY_CYC_1>(FE_PH_CYC_1, lane);
  }
  template <int KIND, int NX, int NY>
  __device__ void ph(int phase, int a, int b, int d) {
    const FeDesc<NX, NY> w = fe_desc<NX, NY>(phase, lane);
    fe_lane<KIND, NX, NY>(s, w.w, a, b, d);
    __syncthreads();
  }
  __device__ void mul(int a, int b, int d) {
    fe_lane<FE_KIND_MUL_0, FE_NT_MUL_0, FE_NY_MUL_0>(s, m0.w, a, b, d);
    __syncthreads();
    fe_lane<FE_KIND_MUL_1, FE_NT_MUL_1, FE_NY_MUL_1>(s, m1.w, a, b, d);
    __syncthreads();
    fe_lane<FE_KIND_MUL_2, FE_NT_MUL_2, FE_NY_MUL_2>(s, m2.w, a, b, d);
    __syncthreads();
  }
  __device__ void cyc(int a, int d) {
    fe_lane<FE_KIND_CYC_0, FE_NT_CYC_0, FE_NY_CYC_0>(s, c0.w, a, 0, d);
    __syncthreads();
    fe_lane<FE_KIND_CYC_1, FE_NT_CYC_1, FE_NY_CYC_1>(s, c1.w, a, 0, d);
    __syncthreads();
  }
};

}  // namespace

// Product of fin[0 .. n), final exponentiation, *out = (result == 1), on the calling 64-lane workgroup.
__device__ __forceinline__ void fe_check_body(FeSlot* s, int* bad, const Fp12* fin, int n, int* out) {
  const int lane = threadIdx.x;
  fe_load_consts(s, lane, 64);
  if (lane == 0) {
    *bad = 0;
    fe_st(s, FE_ABS_BASE + FE_CS, fq_zero());
  }
  FeDev ex;
  ex.s = s;
  ex.lane = lane;
  ex.init();
  for (int i = 0; i < n; i++) {
    if (lane < 12) fe_st(s, 12 * (i ? 1 : 0) + lane, fq_unpack(reinterpret_cast<const Fp*>(fin + i)[lane]));
    __syncthreads();
    if (i) ex.mul(0, 1, 0);
  }
  fe_schedule(ex);
  if (lane < 12) {
    const Fp v = fq_pack(fe_ld(s, 12 + lane));
    if (!(lane == 0 ? fp_is_one(v) : fp_is_zero(v))) atomicOr(bad, 1);
  }
  __syncthreads();
  if (lane == 0) *out = *bad ? 0 : 1;
}

// With sel != nullptr, workgroup b checks fin[sel[b]] alone and writes out[b] (AggregateVerify per-item checks).
__global__ void __launch_bounds__(64) k_fe_check(const Fp12* fin, int n, const uint32_t* sel, int* out) {
  __shared__ FeSlot s[FE_NSLOT];
  __shared__ int bad;
  if (sel) {
    fin += sel[blockIdx.x];
    out += blockIdx.x;
  }
  fe_check_body(s, &bad, fin, n, out);
}

// One level of the bisection tree (bls_capi.hip fav_bisect): workgroup b checks node[b] only when its parent
// failed -- parent == nullptr (the level's nodes are all checked) or parent[b / pdiv] == 0 -- and otherwise
// inherits the parent's pass (res[b] = 1) without a check.  The gate is read on the device, so the rounds of a
// bisection are launched back to back with no host round trip; *nchecks counts the checks that ran.
__global__ void __launch_bounds__(64) k_fe_check_gated(const Fp12* node, const int* parent, uint32_t pdiv, int* res,
                                                       uint32_t* nchecks) {
  __shared__ FeSlot s[FE_NSLOT];
  __shared__ int bad;
  const uint32_t b = blockIdx.x;
  if (parent && parent[b / pdiv]) {  // uniform over the workgroup: it leaves before any barrier
    if (threadIdx.x == 0) res[b] = 1;
    return;
  }
  if (threadIdx.x == 0) atomicAdd(nchecks, 1u);
  fe_check_body(s, &bad, node + b, 1, res + b);
}

// Products of consecutive chunks, out[b] = prod in[b chunk .. min(n, (b + 1) chunk)), with the lane-parallel
// Fp12 product of the final exponentiation (three phases over the 64 lanes; the wave-program product of
// k_fp12_chunk_prod runs each step on a few lanes)
__global__ void __launch_bounds__(64) k_fp12_chunk_prod_fe(const Fp12* in, size_t n, int chunk, Fp12* outp) {
  __shared__ FeSlot s[FE_NSLOT];
  const int lane = threadIdx.x;
  const size_t lo = (size_t)blockIdx.x * chunk;
  const size_t hi = lo + chunk < n ? lo + chunk : n;
  fe_load_consts(s, lane, 64);
  FeDev ex;
  ex.s = s;
  ex.lane = lane;
  ex.init();
  for (size_t i = lo; i < hi; i++) {
    if (lane < 12) fe_st(s, 12 * (i != lo ? 1 : 0) + lane, fq_unpack(reinterpret_cast<const Fp*>(in + i)[lane]));
    __syncthreads();
    if (i != lo) ex.mul(0, 1, 0);
  }
  if (lane < 12) reinterpret_cast<Fp*>(outp + blockIdx.x)[lane] = fq_pack(fe_ld(s, lane));
}

// out[b] = prod_{i in chunk b} a[i] b[i] (the bisection tree's leaves), as k_fp12_chunk_prod2
__global__ void __launch_bounds__(64) k_fp12_chunk_prod2_fe(const Fp12* a, const Fp12* b, size_t n, int chunk,
                                                             Fp12* outp) {
  __shared__ FeSlot s[FE_NSLOT];
  const int lane = threadIdx.x;
  const size_t lo = (size_t)blockIdx.x * chunk;
  const size_t hi = lo + chunk < n ? lo + chunk : n;
  fe_load_consts(s, lane, 64);
  FeDev ex;
  ex.s = s;
  ex.lane = lane;
  ex.init();
  for (size_t i = lo; i < hi; i++) {
    if (lane < 12) fe_st(s, 12 * (i != lo ? 1 : 0) + lane, fq_unpack(reinterpret_cast<const Fp*>(a + i)[lane]));
    __syncthreads();
    if (i != lo) ex.mul(0, 1, 0);
    if (lane < 12) fe_st(s, 12 + lane, fq_unpack(reinterpret_cast<const Fp*>(b + i)[lane]));
    __syncthreads();
    ex.mul(0, 1, 0);
  }
  if (lane < 12) reinterpret_cast<Fp*>(outp + blockIdx.x)[lane] = fq_pack(fe_ld(s, lane));
}

// ragged segments out[b] = prod in[io[b] + b .. io[b + 1] + b] (inclusive), as k_fp12_seg_prod
__global__ void __launch_bounds__(64) k_fp12_seg_prod_fe(const Fp12* in, const uint64_t* io, Fp12* outp) {
  __shared__ FeSlot s[FE_NSLOT];
  const int lane = threadIdx.x;
  const size_t b = blockIdx.x;
  const size_t lo = io[b] + b, hi = io[b + 1] + b + 1;
  fe_load_consts(s, lane, 64);
  FeDev ex;
  ex.s = s;
  ex.lane = lane;
  ex.init();
  for (size_t i = lo; i < hi; i++) {
    if (lane < 12) fe_st(s, 12 * (i != lo ? 1 : 0) + lane, fq_unpack(reinterpret_cast<const Fp*>(in + i)[lane]));
    __syncthreads();
    if (i != lo) ex.mul(0, 1, 0);
  }
  if (lane < 12) reinterpret_cast<Fp*>(outp + b)[lane] = fq_pack(fe_ld(s, lane));
}

hipError_t launch_fp12_chunk_prod2_fe(hipStream_t st, const Fp12* a, const Fp12* b, size_t n, int chunk, Fp12* out) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_fp12_chunk_prod2_fe, dim3((unsigned)((n + chunk - 1) / chunk)), dim3(64), 0, st, a, b, n, chunk,
                     out);
  return hipGetLastError();
}

hipError_t launch_fp12_seg_prod_fe(hipStream_t st, const Fp12* in, const uint64_t* io, size_t B, Fp12* out) {
  if (!B) return hipSuccess;
  hipLaunchKernelGGL(k_fp12_seg_prod_fe, dim3((unsigned)B), dim3(64), 0, st, in, io, out);
  return hipGetLastError();
}

hipError_t launch_fp12_chunk_prod_fe(hipStream_t st, const Fp12* in, size_t n, int chunk, Fp12* out) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_fp12_chunk_prod_fe, dim3((unsigned)((n + chunk - 1) / chunk)), dim3(64), 0, st, in, n, chunk,
                     out);
  return hipGetLastError();
}

hipError_t launch_final_check_wave(hipStream_t st, const Fp12* f, int n, int* out) {
  hipLaunchKernelGGL(k_fe_check, dim3(1), dim3(64), 0, st, f, n, (const uint32_t*)nullptr, out);
  return hipGetLastError();
}

hipError_t launch_final_check_sel(hipStream_t st, const Fp12* f, const uint32_t* sel, size_t nsel, int* out) {
  if (!nsel) return hipSuccess;
  hipLaunchKernelGGL(k_fe_check, dim3((unsigned)nsel), dim3(64), 0, st, f, 1, sel, out);
  return hipGetLastError();
}

hipError_t launch_final_check_gated(hipStream_t st, const Fp12* node, size_t n, const int* parent, uint32_t pdiv,
                                    int* res, uint32_t* nchecks) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_fe_check_gated, dim3((unsigned)n), dim3(64), 0, st, node, parent, pdiv, res, nchecks);
  return hipGetLastError();
}

}  // namespace bls
