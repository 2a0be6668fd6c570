// FastAggregateVerify batch kernels of the signature side and hash_to_G2:
//   k_h2c_sswu_iso2   lane pair per message: expand_message_xmd + hash_to_field,
//                     SSWU of u_0 / u_1, 3-isogeny, Q = iso(P0) + iso(P1)
//   k_g2x_pre1t/post1t one lane per item: cofactor clearing (two [|x|] chains in
//                     the digit-form Jacobian formulas + complete pre/post steps)
//   k_h2c_affine_b    affine H with one inversion per 8 items
//   k_sig_decode      signature decompression + RLC scalar, one lane per item
//   k_g1_affine_b     r_i apk_i to affine (after k_sig_lane2, bls_chain_lane.hip)
//   k_h2c_fallback    the reference-path hash_to_G2 for flagged items
#include <cstdlib>
#include <cstring>
#include <utility>

#include "bls_kernels.h"
#include "bls_lane.h"
#include "bls_fq_g2.h"
#include "bls_fq_g2pair.h"
#include "bls_pp_lane.h"
#include "bls_vm.h"
#include "bls_xmd32.h"
#include "bls_fp_inv.h"

namespace bls {

__device__ static const uint8_t DST_POP_FAV[43] = {
    'B', 'L', 'S', '_', 'S', 'I', 'G', '_', 'B', 'L', 'S', '1', '2', '3', '8', '1', 'G', '2', '_', 'X', 'M', 'D',
    ':', 'S', 'H', 'A', '-', '2', '5', '6', '_', 'S', 'S', 'W', 'U', '_', 'R', 'O', '_', 'P', 'O', 'P', '_'};

// hash_to_G2 staging in HBM (Fd form, HCF = 24 slots per item): Q | M | A | C,
// each a projective E2 point (X.c0, X.c1, Y.c0, Y.c1, Z.c0, Z.c1).
// flag[i] = 1 when an isogeny denominator vanished or a chain addition hit an
// exceptional case (the item is recomputed by k_h2c_fallback).
constexpr int HCF_Q = 0, HCF_M = 6, HCF_A = 12, HCF_C = 18;

// The fallback runs as ONE 64-lane workgroup striding over the flags (they
// are ~never set, so the loop is B / 64 flag loads).  Its hash_to_g2 call
// chain needs 6,000 B of private segment per lane, and the runtime sizes a
// hardware queue's scratch by the largest private segment it has run times
// the device's wave slots -- not by the grid.  Launched on every job's h2c
// stream, it gave each of those queues that reservation and six jobs in
// flight exhausted the scratch pool (HSA_STATUS_ERROR_OUT_OF_RESOURCES); the
// C ABI therefore runs it on one context-wide stream (bls_capi.hip).
__global__ void __launch_bounds__(64) k_h2c_fallback(size_t B, const uint8_t* msgs32, const int* flag, G2A* H) {
  for (size_t i = threadIdx.x; i < B; i += 64)
    if (flag[i]) H[i] = jac_to_aff(hash_to_g2(msgs32 + 32 * i, 32, DST_POP_FAV, 43));
}

__global__ void __launch_bounds__(64) k_h2c_fallback_var(size_t B, const uint8_t* msgs, const uint64_t* offs,
                                                         const int* flag, G2A* H) {
  for (size_t i = threadIdx.x; i < B; i += 64)
    if (flag[i]) H[i] = jac_to_aff(hash_to_g2(msgs + offs[i], (uint32_t)(offs[i + 1] - offs[i]), DST_POP_FAV, 43));
}

// ----------------------------------------------------------- signatures --
// RLC scalar r_i = first 8 bytes of SHA-256(seed || i (8 bytes LE) || msg || sig), nonzero.  The 168-byte input
// is three blocks whose word positions are all fixed, so the message words are loaded straight into the
// schedule registers (bls_xmd32.h sha256_compress_w, constant indices): the byte-streaming Sha256 state of
// bls_sha256.h kept its block buffer in a private segment.
static __device__ __forceinline__ uint32_t ld_be32(const uint8_t* p) {
  return __builtin_bswap32(*reinterpret_cast<const uint32_t*>(p));
}
static __device__ uint64_t rlc_scalar_fav(const uint8_t* seed32, uint64_t i, const uint8_t* msg32,
                                          const uint8_t* sig96) {
  uint32_t st[8], blk[16];
#pragma unroll
  for (int k = 0; k < 8; k++) st[k] = SHA256_IV[k];
#pragma unroll
  for (int k = 0; k < 8; k++) blk[k] = ld_be32(seed32 + 4 * k);
  blk[8] = __builtin_bswap32((uint32_t)i);
  blk[9] = __builtin_bswap32((uint32_t)(i >> 32));
#pragma unroll
  for (int k = 0; k < 6; k++) blk[10 + k] = ld_be32(msg32 + 4 * k);
  sha256_compress_w(st, blk);
  blk[0] = ld_be32(msg32 + 24);
  blk[1] = ld_be32(msg32 + 28);
#pragma unroll
  for (int k = 0; k < 14; k++) blk[2 + k] = ld_be32(sig96 + 4 * k);
  sha256_compress_w(st, blk);
#pragma unroll
  for (int k = 0; k < 10; k++) blk[k] = ld_be32(sig96 + 56 + 4 * k);
  blk[10] = 0x80000000u;
#pragma unroll
  for (int k = 11; k < 15; k++) blk[k] = 0;
  blk[15] = 168 * 8;
  sha256_compress_w(st, blk);
  const uint64_t r = ((uint64_t)st[0] << 32) | st[1];
  return r ? r : 1;
}

// (1) lane per item: signature decompression (no subgroup check yet) and the
// RLC scalar.  Independent of the registry gather, so it runs beside it.
// The identity signature can only verify against the identity key, which the
// gather rejects: it is marked invalid here.
__global__ void __launch_bounds__(64) k_sig_decode(size_t B, const uint8_t* msgs32, const uint8_t* sigs96,
                                                   const uint8_t* seed32, G2A* sig, uint64_t* rsc, int* dstat) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= B) return;
  // the hash first: nothing of the decompression is live across its three compressions
  const uint64_t r = rlc_scalar_fav(seed32, i, msgs32 + 32 * i, sigs96 + 96 * i);
  G2A q{fp2_zero(), fp2_zero(), true};
  const int st = g2_decompress_lane_w(q, sigs96 + 96 * i) == DEC_OK ? 1 : 0;
  rsc[i] = st ? r : 0;
  sig[i] = q;
  dstat[i] = st;
}

// ------------------------------------------------ batched affine conversion --
// k_g1_affine / k_h2c_affine spend one inversion per item, and a 64-lane wave
// pays a whole inversion's time whether one lane or all need it.  Here each
// lane converts AFF_K items (item w * 64 AFF_K + lane + 64 k, so every load is
// coalesced) with Montgomery's trick: prefix products of the K denominators,
// ONE inversion, then two products per item walking back -- ~1/K of the
// inversions' SIMD time.  A zero denominator (identity, or a skipped item)
// enters the products as 1 and gets the same output as the one-item kernels.
constexpr int AFF_K = 8;

// f(integral_constant<k>) for k = AFF_K - 1 .. 0: the walk-back loops of the affine kernels with compile-time k
// (as `#pragma unroll` loops the compiler left them rolled, pre[] indexed at run time in a private segment)
template <class F, int... K>
__device__ __forceinline__ void aff_walk_back(F&& f, std::integer_sequence<int, K...>) {
  (f(std::integral_constant<int, (int)sizeof...(K) - 1 - K>{}), ...);
}
// k_h2c_affine_b converts 4 items per lane: its Fp2 products beside 8 prefix products pushed it past the register
// file (112 B/lane of private memory); the extra inversion per 4 items is ~5 FME against ~40 for the conversions
constexpr int AFF_K2 = 4;

__global__ void __launch_bounds__(64) k_g1_affine_b(size_t B, const int* status, const G1P* rPj, G1A* rP) {
  const size_t base = (size_t)blockIdx.x * 64 * AFF_K + threadIdx.x;
  Fp pre[AFF_K];
  bool zero[AFF_K];
  Fp acc = FP_ONE;
#pragma unroll
  for (int k = 0; k < AFF_K; ++k) {
    const size_t i = base + 64 * k;
    const bool live = i < B && status[i];
    const Fp z = live ? rPj[i].z : FP_ONE;
    zero[k] = fp_is_zero(z);
    acc = fp_mul_i(acc, zero[k] ? FP_ONE : z);
    pre[k] = acc;
  }
  Fp inv = fp_inv_sg_i(acc);  // 1 / (z_0 ... z_{K-1})
  aff_walk_back([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const size_t i = base + 64 * k;
    const bool in = i < B;
    const bool live = in && status[i] != 0;
    const Fp zk = live ? rPj[i].z : FP_ONE;
    const Fp zi = k ? fp_mul_i(inv, pre[k ? k - 1 : 0]) : inv;
    if (in && k && !zero[k]) inv = fp_mul_i(inv, zk);
    G1A o{fp_zero(), fp_zero(), true};
    if (live) {
      const G1P q = rPj[i];
      const Fp zz = zero[k] ? fp_zero() : zi;  // fp_inv(0) = 0, as k_g1_affine
      o = G1A{fp_mul_i(q.x, zz), fp_mul_i(q.y, zz), false};
    }
    if (in) rP[i] = o;
  }, std::make_integer_sequence<int, AFF_K>{});
}

__global__ void __launch_bounds__(64) k_h2c_affine_b(size_t B, const int* status, const Fd* hf, G2A* H) {
  const size_t base = (size_t)blockIdx.x * 64 * AFF_K2 + threadIdx.x;
  Fp pre[AFF_K2];
  bool zero[AFF_K2];
  Fp acc = FP_ONE;
#pragma unroll
  for (int k = 0; k < AFF_K2; ++k) {
    const size_t i = base + 64 * k;
    Fp n = FP_ONE;
    if (i < B && (!status || status[i])) {
      const Fd* r = hf + HCF * i + HCF_A;
      n = fp2_norm(Fp2{fp_from_fd(r[4]), fp_from_fd(r[5])});
    } else if (i < B) {
      n = fp_zero();  // skipped item: identity output
    }
    zero[k] = fp_is_zero(n);
    acc = fp_mul_i(acc, zero[k] ? FP_ONE : n);
    pre[k] = acc;
  }
  Fp inv = fp_inv_sg_i(acc);
  aff_walk_back([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const size_t i = base + 64 * k;
    const bool in = i < B;
    const Fd* r = hf + HCF * (in ? i : 0) + HCF_A;
    G2A h{fp2_zero(), fp2_zero(), true};
    if (in && !zero[k]) {
      const Fp2 Z{fp_from_fd(r[4]), fp_from_fd(r[5])};
      const Fp ni = k ? fp_mul_i(inv, pre[k ? k - 1 : 0]) : inv;  // 1 / norm(Z)
      inv = k ? fp_mul_i(inv, fp2_norm(Z)) : inv;
      const Fp2 X{fp_from_fd(r[0]), fp_from_fd(r[1])}, Y{fp_from_fd(r[2]), fp_from_fd(r[3])};
      const Fp2 zi{fp_mul_i(Z.c0, ni), fp_neg(fp_mul_i(Z.c1, ni))};
      h = G2A{f2mul(X, zi), f2mul(Y, zi), false};
    }
    if (in) H[i] = h;
  }, std::make_integer_sequence<int, AFF_K2>{});
}

// ---------------------------------------------- hash_to_G2 on lane pairs --
// k_h2c_sswu_iso2, lane (item, t): hash_to_field, SSWU of u_t, 3-isogeny of its
// own point (homogeneous projective, tools/wavec.py prog_iso_pair), swap, and
// Q = iso(P0) + iso(P1) with the complete formulas (Renes-Costello-Batina).
namespace {

__device__ __forceinline__ PP<Fp2> pp2_swap(const PP<Fp2>& p) { return PP<Fp2>{cl_swap2(p.x), cl_swap2(p.y), cl_swap2(p.z)}; }
__device__ __forceinline__ PP<Fp2> pp2_sel(bool c, const PP<Fp2>& a, const PP<Fp2>& b) {
  return PP<Fp2>{cl_sel(c, a.x, b.x), cl_sel(c, a.y, b.y), cl_sel(c, a.z, b.z)};
}

// (x, y) affine on E2' -> iso(x, y) = (xnum yden : y ynum xden : xden yden) on E2 (RFC 9380 App. E.3)
// (the products run one after another: interleaved, their digit columns pushed the kernel into spills)
#define H2C_SEQ() __builtin_amdgcn_sched_barrier(0)
__device__ __forceinline__ PP<Fp2> iso_proj_lane(const Fp2& x, const Fp2& y) {
  const Fp2 xx = f2sqr(x);
  H2C_SEQ();
  const Fp2 xxx = f2mul(xx, x);
  H2C_SEQ();
  const Fp2 xnum = fadd(fadd(f2mul(ISO_XNUM_3, xxx), f2mul(ISO_XNUM_2, xx)), fadd(f2mul(ISO_XNUM_1, x), ISO_XNUM_0));
  H2C_SEQ();
  const Fp2 xden = fadd(fadd(xx, f2mul(ISO_XDEN_1, x)), ISO_XDEN_0);
  H2C_SEQ();
  const Fp2 ynum = fadd(fadd(f2mul(ISO_YNUM_3, xxx), f2mul(ISO_YNUM_2, xx)), fadd(f2mul(ISO_YNUM_1, x), ISO_YNUM_0));
  H2C_SEQ();
  const Fp2 yden = fadd(fadd(xxx, f2mul(ISO_YDEN_2, xx)), fadd(f2mul(ISO_YDEN_1, x), ISO_YDEN_0));
  H2C_SEQ();
  const Fp2 X = f2mul(xnum, yden);
  H2C_SEQ();
  const Fp2 Y = f2mul(f2mul(y, ynum), xden);
  H2C_SEQ();
  return PP<Fp2>{X, Y, f2mul(xden, yden)};
}

// lane 0 writes X, Y.c0; lane 1 Y.c1, Z (six consecutive Fd slots).  Selects, not a branch on the lane: the
// branch kept the point in a private-memory copy.
__device__ __forceinline__ void pp2_store(Fd* o, const PP<Fp2>& p, bool hi) {
  Fd* d = o + (hi ? 3 : 0);
  d[0] = fd_from_fp(fp_select(hi, p.y.c1, p.x.c0));
  d[1] = fd_from_fp(fp_select(hi, p.z.c0, p.x.c1));
  d[2] = fd_from_fp(fp_select(hi, p.z.c1, p.y.c0));
}
__device__ __forceinline__ PP<Fp2> pp2_load(const Fd* in) {
  return PP<Fp2>{Fp2{fp_from_fd(in[0]), fp_from_fd(in[1])}, Fp2{fp_from_fd(in[2]), fp_from_fd(in[3])},
                 Fp2{fp_from_fd(in[4]), fp_from_fd(in[5])}};
}

}  // namespace

// VAR = false: 32-byte messages msgs[32 i ..] (the FastAggregateVerify batches), hashed by the register-resident
// expand_message_xmd of bls_xmd32.h; VAR = true: msgs[offs[i] .. offs[i+1]) of any length (the byte-streaming
// bls_sha256.h).  status: items to skip (may be null)
template <bool VAR>
__global__ void __launch_bounds__(64) k_h2c_sswu_iso2(size_t B, const uint8_t* msgs, const uint64_t* offs,
                                                      const int* status, Fd* hf, int* flag) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = t >> 1;
  const bool hi = (t & 1) != 0;
  if (i >= B) return;  // both lanes of an item leave together
  Fd* o = hf + HCF * i + HCF_Q;
  if (status && !status[i]) {
    pp2_store(o, PP<Fp2>{fp2_zero(), fp2_zero(), fp2_zero()}, hi);
    if (!hi) flag[i] = 0;
    return;
  }
  Fp2 u[2];
  if (VAR)
    hash_to_field_fp2(u, msgs + offs[i], (uint32_t)(offs[i + 1] - offs[i]), DST_POP_FAV, 43);
  else
    hash_to_field_fp2_m32(u, msgs + 32 * i);
  H2C_SEQ();
  Fp2 x, y;
  bool rare;
  map_to_curve_sswu_lane_i(x, y, hi ? u[1] : u[0], rare);
  H2C_SEQ();
  const PP<Fp2> mine = iso_proj_lane(x, y);
  H2C_SEQ();
  const PP<Fp2> other = pp2_swap(mine);
  // an isogeny denominator vanished, or an SSWU case this kernel does not compute: k_h2c_fallback
  const uint32_t bad = (rare || fp2_is_zero(mine.z)) ? 1u : 0u;
  const uint32_t any_bad = bad | cl_swap(bad);
  const PP<Fp2> Q = pp2_add(pp2_sel(hi, other, mine), pp2_sel(hi, mine, other), hi);
  pp2_store(o, Q, hi);
  if (!hi) flag[i] = any_bad ? 1 : 0;
}

// The cofactor-clearing chains on ONE lane per item in Jacobian coordinates
// (bls_pp_lane.h j2_*: 16 instead of 2 x 12 FME per doubling and item); the
// pre/post steps stay complete projective (pp_add).  An exceptional case of
// the incomplete chain additions raises flag[i], and k_h2c_fallback recomputes
// the item with the reference-path formulas.  Items with status 0 are skipped.
__device__ __forceinline__ PP<Fp2> pp_neg2(const PP<Fp2>& p) { return PP<Fp2>{p.x, fp2_neg(p.y), p.z}; }
__device__ __forceinline__ PP<Fp2> pp_psi2x(const PP<Fp2>& p) {
  return PP<Fp2>{f2mul(fp2_conj(p.x), PSI_CX), f2mul(fp2_conj(p.y), PSI_CY), fp2_conj(p.z)};
}
__device__ __forceinline__ void pp_store1(Fd* o, const PP<Fp2>& p) {
  o[0] = fd_from_fp(p.x.c0);
  o[1] = fd_from_fp(p.x.c1);
  o[2] = fd_from_fp(p.y.c0);
  o[3] = fd_from_fp(p.y.c1);
  o[4] = fd_from_fp(p.z.c0);
  o[5] = fd_from_fp(p.z.c1);
}

// [|x|] of a projective point through the digit-form Jacobian chain (bls_fq_g2.h, base point parked in LDS): (X Z,
// Y Z^2, Z) in, (X Z, Y, Z^3) out, canonical packed.  Inline and call-free: the out-of-line chain cost each
// kernel a 1.5-2 KB private segment.
__device__ __forceinline__ PP<Fp2> pp_mul_xabs_q(const PP<Fp2>& P, bool& exc, uint32_t* lds) {
  const Fq2 z = fq2_unpack(P.z);
  const J2Q J{fq2_mul(fq2_unpack(P.x), z), fq2_mul(fq2_unpack(P.y), fq2_sqr(z)), z};
  const J2Q M = j2q_mul_xabs_lds(J, exc, lds);
  return PP<Fp2>{fq2_pack(fq2_mul(M.x, M.z)), fq2_pack(M.y), fq2_pack(fq2_mul(fq2_sqr(M.z), M.z))};
}
// the staged inputs are re-read from HBM after the chain instead of being held across it (the barrier keeps the
// compiler from reusing the first load)
#define H2C_RELOAD_BARRIER() asm volatile("" ::: "memory")

__global__ void __launch_bounds__(64) k_g2x_pre1t(size_t B, const int* status, Fd* hf, int* flag) {
  __shared__ uint32_t lds[84 * 64];
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= B || (status && !status[i])) return;
  Fd* r = hf + HCF * i;
  bool exc = false;
  pp_store1(r + HCF_M, pp_mul_xabs_q(pp2_load(r + HCF_Q), exc, lds));  // M = [|x|] Q
  // the complete-formula steps, each from points re-read from the staging slots so at most ~3 points are live
  // (held across all of them, five points spilled ~450 VGPRs)
  H2C_RELOAD_BARRIER();
  {
    const PP<Fp2> pq = pp_psi2x(pp2_load(r + HCF_Q));
    pp_store1(r + HCF_A, pp_add(pq, pp_neg2(pp2_load(r + HCF_M))));  // A = psi(Q) - M  (t1 + t2, t1 = -M)
  }
  H2C_RELOAD_BARRIER();
  {
    const PP<Fp2> Q = pp2_load(r + HCF_Q);
    const PP<Fp2> pq = pp_psi2x(Q);
    const PP<Fp2> t3{f2mul(Q.x, PSI2_CX), f2mul(Q.y, PSI2_CY), Q.z};  // psi^2(Q); psi^2(2Q) = 2 psi^2(Q)
    pp_store1(r + HCF_C, pp_add(pp_dbl(t3), pp_neg2(pq)));          // psi^2(2Q) - psi(Q)
  }
  H2C_RELOAD_BARRIER();
  {
    const PP<Fp2> mq = pp_add(pp2_load(r + HCF_M), pp_neg2(pp2_load(r + HCF_Q)));  // M - Q
    pp_store1(r + HCF_C, pp_add(pp2_load(r + HCF_C), mq));
  }
  if (exc) flag[i] = 1;
}

__global__ void __launch_bounds__(64) k_g2x_post1t(size_t B, const int* status, Fd* hf, int* flag) {
  __shared__ uint32_t lds[84 * 64];
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= B || (status && !status[i])) return;
  Fd* r = hf + HCF * i;
  bool exc = false;
  const PP<Fp2> M = pp_mul_xabs_q(pp2_load(r + HCF_A), exc, lds);
  H2C_RELOAD_BARRIER();
  pp_store1(r + HCF_A, pp_add(pp2_load(r + HCF_C), pp_neg2(M)));  // projective H over the dead A slots
  if (exc) flag[i] = 1;
}


// The same two kernels on a LANE PAIR per item (bls_fq_g2pair.h: the [|x|] chain in the F2 layout, each lane one
// coefficient of every Fp2; the complete-formula steps by pp2_add / pp2_dbl, whose products are split between the
// two lanes).  Every value is the one-lane kernels' (the same expressions per coefficient), so H and the exception
// flags are identical; the chain's latency halves and a lane holds half the point.  Both lanes write whole staged
// points (identical values), so every re-read is of the lane's own stores.
__device__ __forceinline__ PP<Fp2> pp_mul_xabs_pair(const PP<Fp2>& P, bool& exc, uint32_t* lds, bool hi) {
  const Fq z = q2p_own(P.z, hi);
  const J2P J{q2p_mul(q2p_own(P.x, hi), z, hi), q2p_mul(q2p_own(P.y, hi), q2p_sqr(z, hi), hi), z};
  const J2P M = j2p_mul_xabs_lds(J, exc, lds, hi);
  return PP<Fp2>{q2p_join(q2p_mul(M.x, M.z, hi), hi), q2p_join(M.y, hi),
                 q2p_join(q2p_mul(q2p_sqr(M.z, hi), M.z, hi), hi)};
}

__global__ void __launch_bounds__(64) k_g2x_pre2(size_t B, const int* status, Fd* hf, int* flag) {
  __shared__ uint32_t lds[42 * 64];
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = t >> 1;
  const bool hi = (t & 1) != 0;
  if (i >= B || (status && !status[i])) return;  // both lanes of an item leave together
  Fd* r = hf + HCF * i;
  bool exc = false;
  // M = [|x|] Q, staged by BOTH lanes (the same values): each lane re-reads its own stores below
  pp_store1(r + HCF_M, pp_mul_xabs_pair(pp2_load(r + HCF_Q), exc, lds, hi));
  // the complete-formula steps of k_g2x_pre1t, each from points re-read from the staging slots, products split
  // over the pair (pp2_add / pp2_dbl)
  H2C_RELOAD_BARRIER();
  {
    const PP<Fp2> pq = pp_psi2x(pp2_load(r + HCF_Q));
    pp_store1(r + HCF_A, pp2_add(pq, pp_neg2(pp2_load(r + HCF_M)), hi));  // A = psi(Q) - M
  }
  H2C_RELOAD_BARRIER();
  {
    const PP<Fp2> Q = pp2_load(r + HCF_Q);
    const PP<Fp2> pq = pp_psi2x(Q);
    const PP<Fp2> t3{f2mul(Q.x, PSI2_CX), f2mul(Q.y, PSI2_CY), Q.z};  // psi^2(Q); psi^2(2Q) = 2 psi^2(Q)
    pp_store1(r + HCF_C, pp2_add(pp2_dbl(t3, hi), pp_neg2(pq), hi));    // psi^2(2Q) - psi(Q)
  }
  H2C_RELOAD_BARRIER();
  {
    const PP<Fp2> mq = pp2_add(pp2_load(r + HCF_M), pp_neg2(pp2_load(r + HCF_Q)), hi);  // M - Q
    pp_store1(r + HCF_C, pp2_add(pp2_load(r + HCF_C), mq, hi));
  }
  if (exc && !hi) flag[i] = 1;
}

__global__ void __launch_bounds__(64) k_g2x_post2(size_t B, const int* status, Fd* hf, int* flag) {
  __shared__ uint32_t lds[42 * 64];
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = t >> 1;
  const bool hi = (t & 1) != 0;
  if (i >= B || (status && !status[i])) return;
  Fd* r = hf + HCF * i;
  bool exc = false;
  const PP<Fp2> M = pp_mul_xabs_pair(pp2_load(r + HCF_A), exc, lds, hi);
  H2C_RELOAD_BARRIER();
  pp_store1(r + HCF_A, pp2_add(pp2_load(r + HCF_C), pp_neg2(M), hi));  // projective H over the dead A slots
  if (exc && !hi) flag[i] = 1;
}

static inline unsigned nblk(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

size_t h2c_scratch_fd(size_t B) { return (size_t)HCF * B; }

// msgs: 32-byte messages (offs == nullptr) or msgs[offs[i] .. offs[i+1]); status: items to skip (may be null)
static hipError_t launch_h2c_lane2(hipStream_t st, size_t B, const uint8_t* msgs, const uint64_t* offs,
                                   const int* status, Fd* hf, G2A* H, int* flag) {
  if (offs)
    hipLaunchKernelGGL(k_h2c_sswu_iso2<true>, dim3(nblk(2 * B, 64)), dim3(64), 0, st, B, msgs, offs, status, hf, flag);
  else
    hipLaunchKernelGGL(k_h2c_sswu_iso2<false>, dim3(nblk(2 * B, 64)), dim3(64), 0, st, B, msgs, offs, status, hf, flag);
  // the cofactor clearing on a lane pair per item (k_g2x_pre2 / post2: half the chain latency) for batches below
  // BLS_H2C_PAIR_MAX items (default 4,096: the C3 epoch's 2,048 and C5's 1,024, whose pipelines wait on the hash
  // branch -- C3 +9 %), on one lane per item above (full batches are bound by total work, which the pair's operand
  // exchanges raise: C2 -1 %; profiles/r06l_h2c_pair_ab.txt)
  static const size_t pair_max = getenv("BLS_H2C_PAIR_MAX") ? (size_t)atol(getenv("BLS_H2C_PAIR_MAX")) : 4096;
  if (B < pair_max) {
    hipLaunchKernelGGL(k_g2x_pre2, dim3(nblk(2 * B, 64)), dim3(64), 0, st, B, status, hf, flag);
    hipLaunchKernelGGL(k_g2x_post2, dim3(nblk(2 * B, 64)), dim3(64), 0, st, B, status, hf, flag);
  } else {
    hipLaunchKernelGGL(k_g2x_pre1t, dim3(nblk(B, 64)), dim3(64), 0, st, B, status, hf, flag);
    hipLaunchKernelGGL(k_g2x_post1t, dim3(nblk(B, 64)), dim3(64), 0, st, B, status, hf, flag);
  }
  hipLaunchKernelGGL(k_h2c_affine_b, dim3(nblk(B, 64 * AFF_K2)), dim3(64), 0, st, B, status, hf, H);
  return hipGetLastError();
}

hipError_t launch_h2c(hipStream_t st, size_t B, const uint8_t* msgs32, const int* status, Fd* hf, G2A* H, int* flag) {
  if (!B) return hipSuccess;
  return launch_h2c_lane2(st, B, msgs32, nullptr, status, hf, H, flag);
}

hipError_t launch_h2c_msgs(hipStream_t st, size_t B, const uint8_t* msgs, const uint64_t* offs, Fd* hf, G2A* H,
                           int* flag) {
  if (!B) return hipSuccess;
  return launch_h2c_lane2(st, B, msgs, offs, nullptr, hf, H, flag);
}

hipError_t launch_h2c_fallback(hipStream_t st, size_t B, const uint8_t* msgs, const uint64_t* offs, const int* flag,
                               G2A* H) {
  if (!B) return hipSuccess;
  if (offs)
    hipLaunchKernelGGL(k_h2c_fallback_var, dim3(1), dim3(64), 0, st, B, msgs, offs, flag, H);
  else
    hipLaunchKernelGGL(k_h2c_fallback, dim3(1), dim3(64), 0, st, B, msgs, flag, H);
  return hipGetLastError();
}

hipError_t launch_sig_decode(hipStream_t st, size_t B, const uint8_t* msgs32, const uint8_t* sigs96,
                             const uint8_t* seed32, G2A* sig, uint64_t* rsc, int* dstat) {
  if (!B) return hipSuccess;
  hipLaunchKernelGGL(k_sig_decode, dim3(nblk(B, 64)), dim3(64), 0, st, B, msgs32, sigs96, seed32, sig, rsc, dstat);
  return hipGetLastError();
}

hipError_t launch_g1_affine(hipStream_t st, size_t B, const int* status, const G1P* Pj, G1A* out) {
  if (!B) return hipSuccess;
  hipLaunchKernelGGL(k_g1_affine_b, dim3(nblk(B, 64 * AFF_K)), dim3(64), 0, st, B, status, Pj, out);
  return hipGetLastError();
}

hipError_t launch_sig_vm(hipStream_t st, size_t B, const int* gstat, int* status, const int* dstat,
                         const G1P* apk_aff, const G2A* sig, const uint64_t* rsc, G1P* rPj, G1A* rP) {
  if (!B) return hipSuccess;
  hipError_t e = launch_sig_lane(st, B, gstat, status, dstat, apk_aff, sig, rsc, rPj);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_g1_affine_b, dim3(nblk(B, 64 * AFF_K)), dim3(64), 0, st, B, status, rPj, rP);
  return hipGetLastError();
}

}  // namespace bls
