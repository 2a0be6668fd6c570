// Host-side launchers for the gfx950 kernels in bls_kernels.hip.
#pragma once
#include "bls_ops.h"

namespace bls {

hipError_t launch_key_validate(hipStream_t st, const uint8_t* pks, size_t n, G1A* out, int* ok);
hipError_t launch_sig_validate(hipStream_t st, const uint8_t* sigs, size_t n, G2A* out, int* ok);
hipError_t launch_g1_sum_aff(hipStream_t st, const G1A* in, const int* ok, size_t n, G1J* tmp, G1J* out);
hipError_t launch_g2_sum_aff(hipStream_t st, const G2A* in, const int* ok, size_t n, G2J* tmp, G2J* out);
hipError_t launch_g1_compress(hipStream_t st, const G1J* in, uint8_t* out48, int* is_inf);
hipError_t launch_g2_compress(hipStream_t st, const G2J* in, uint8_t* out96);
hipError_t launch_percall_pairs(hipStream_t st, const G1A* keys, const int* key_ok, size_t n, const G1J* apk_sum,
                                const int* sig_ok, G1A* P, int* live, Fp* pz = nullptr);
hipError_t launch_hash_many(hipStream_t st, const uint8_t* msgs, const uint64_t* offs, size_t n, const uint8_t* dst, uint32_t dst_len, G2A* out);
hipError_t launch_sign_many(hipStream_t st, const uint8_t* sks, const uint8_t* msgs, const uint64_t* offs, size_t n, uint8_t* out, int* ok);
hipError_t launch_sk_to_pk_many(hipStream_t st, const uint8_t* sks, size_t n, uint8_t* out, int* ok);
hipError_t launch_fav_gather(hipStream_t st, const uint32_t* idx, const uint64_t* offs, size_t B, const RegKey* reg, uint32_t reg_n, G1P* apk, int* status);
// the affine gather (bls_gather_aff.hip) for batches of >= 1,024 aggregates: scratch of fav_gather_aff_words(B) u32,
// redo[B] (1 = recompute with launch_fav_gather_redo, the complete-formula kernel on the flagged aggregates only)
size_t fav_gather_aff_words(size_t B);
hipError_t launch_fav_gather_aff(hipStream_t st, const uint32_t* idx, const uint64_t* offs, size_t B,
                                 const RegKey* reg, uint32_t reg_n, G1P* apk, int* status, uint32_t* scr, int* redo);
hipError_t launch_fav_gather_redo(hipStream_t st, const uint32_t* idx, const uint64_t* offs, size_t B,
                                  const RegKey* reg, uint32_t reg_n, G1P* apk, int* status, const int* redo);
// registry entries from k_key_validate output (+ the host validity mask)
hipError_t launch_reg_pack(hipStream_t st, const G1A* a, const int* ok, size_t n, RegKey* reg, uint8_t* valid);
hipError_t launch_av_items(hipStream_t st, size_t B, const uint64_t* io, const int* pk_ok, const int* sig_ok, const G2A* sig, const uint64_t* rsc, int* status, G1A* P2, G2A* Q2);
hipError_t launch_av_pairs(hipStream_t st, size_t total, const uint32_t* pair_item, const int* status, const uint64_t* rsc, const G1A* pk, const G2A* H, G1A* P2, G2A* Q2);
// out[b] = product of in[io[b] + b .. io[b + 1] + b] (the AggregateVerify batch's per-item segments)
hipError_t launch_fp12_seg_prod(hipStream_t st, const Fp12* in, const uint64_t* io, size_t B, Fp12* out);
// SHA-256 of 64-byte nodes (bls_ssz.hip): signing roots and SSZ merkleization
hipError_t launch_sha256_pairs(hipStream_t st, const uint8_t* left, const uint8_t* right, size_t rstride, size_t n,
                               uint8_t* out);
hipError_t launch_merkleize(hipStream_t st, uint8_t* a, uint8_t* b, size_t n, int depth, uint8_t* zero, uint8_t** root);
// KZG: checked G1 decode (identity allowed), per-point scalar products for multi_exp
hipError_t launch_g1_decode_checked(hipStream_t st, const uint8_t* in48, size_t n, G1A* out, int* ok);
hipError_t launch_g1_scale(hipStream_t st, const G1A* P, const uint8_t* k32, size_t n, G1A* out, int* live);
hipError_t launch_verdicts(hipStream_t st, const int* status, const uint8_t* bad, size_t B, uint8_t* out);
hipError_t launch_status_to_u8(hipStream_t st, const int* status, size_t B, uint8_t* out);
hipError_t launch_fp12_to_bytes(hipStream_t st, const Fp12* f, uint8_t* out);
hipError_t launch_fp12_from_bytes(hipStream_t st, const uint8_t* in, size_t n, Fp12* f);
hipError_t launch_g2_compress_aff(hipStream_t st, const G2A* in, uint8_t* out96);
hipError_t launch_registry_generate(hipStream_t st, uint64_t first, size_t n, G1J* tmpJ, RegKey* reg, uint8_t* out48);
hipError_t launch_miller_wave(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, Fp12* f);
constexpr int HCF = 24;  // hash_to_G2 staging: Fd slots per item (bls_fav_kernels.hip, bls_chain_lane.hip)
// one lane per item (bls_chain_lane.hip)
// gstat: gather status (read-only: the MSM reads it concurrently on another stream); status: written
hipError_t launch_sig_lane(hipStream_t st, size_t B, const int* gstat, int* status, const int* dstat, const G1P* apk,
                           const G2A* sig, const uint64_t* rsc, G1P* rPj);
// hf: h2c_scratch_fd(B) Fd slots of staging between the hash_to_G2 phases
size_t h2c_scratch_fd(size_t B);
hipError_t launch_h2c(hipStream_t st, size_t B, const uint8_t* msgs32, const int* status, Fd* hf, G2A* H, int* flag);
// hash_to_G2 (POP DST) of B messages of any length, msgs[offs[i] .. offs[i+1]); same phases as launch_h2c
hipError_t launch_h2c_msgs(hipStream_t st, size_t B, const uint8_t* msgs, const uint64_t* offs, Fd* hf, G2A* H,
                           int* flag);
// exceptional h2c items (flag set: an isogeny denominator vanished) recomputed by one workgroup; offs == nullptr
// for 32-byte messages.  Not part of launch_h2c / launch_h2c_msgs: the caller picks its stream (bls_capi.hip).
hipError_t launch_h2c_fallback(hipStream_t st, size_t B, const uint8_t* msgs, const uint64_t* offs, const int* flag,
                               G2A* H);
hipError_t launch_sig_decode(hipStream_t st, size_t B, const uint8_t* msgs32, const uint8_t* sigs96, const uint8_t* seed32, G2A* sig, uint64_t* rsc, int* dstat);
// rPj: B projective scratch points (r_i apk_i before the affine conversion)
hipError_t launch_sig_vm(hipStream_t st, size_t B, const int* gstat, int* status, const int* dstat, const G1P* apk_aff,
                         const G2A* sig, const uint64_t* rsc, G1P* rPj, G1A* rP);
size_t msm_scratch_u32(size_t B);
size_t msm_scratch_fd();
// the 64 bit-sums U_b of S = sum_i r_i sigma_i = sum_b 2^b U_b as Miller pairs (-2^b G1, U_b) at P[0 .. 64),
// Q[0 .. 64), ok[0 .. 64) = 1; comb: the bisection's -G1 comb (neg_g1_comb_entries() entries)
constexpr int MSM_UPAIRS = 64;
hipError_t launch_msm_upairs(hipStream_t st, size_t B, const int* status, const int* status2, const uint64_t* rsc,
                             const G2A* sig, uint32_t* scr, Fd* pts, const G1A* comb, G1A* P, G2A* Q, int* ok);
// the same Miller values in two kernels (G2 lines, then f); L: miller_lines_u32(n) words of scratch
constexpr int MILLER_NLINES = 68;  // 63 doublings + 5 additions (|x| = 0xd201000000010000)
// Miller line records (k_miller_lines2 -> k_miller_acc4q): three Fp2 -- (l0, E ZZ, z3 ZZ) for a doubling, (l0, r,
// z3) for an addition -- as 14-digit bound-typed values (bls_fqb.h FqB<ML_LV, ML_LD>: value < ML_LV p, digits <=
// ML_LD), word w of line k of pair i at L[(k * ML_WORDS + w) * n + i]
constexpr int ML_WORDS = 84;
constexpr uint64_t ML_LV = 4096, ML_LD = 0x20000000ull + 64;
size_t miller_lines_ld(size_t n);  // the records' leading dimension (>= n, a multiple of 32 pairs)
size_t miller_lines_u32(size_t n);
hipError_t launch_miller_lines(hipStream_t st, const G2A* Q, size_t n, uint32_t* L);
// four lanes per f, G = 1 or 2 pairs per f (bls_miller_pair.hip); writes ceil(n / G) values; ld >= n: the
// line records' leading dimension (the n of the launch_miller_lines that wrote them)
hipError_t launch_miller_acc4(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, const uint32_t* L,
                              size_t ld, Fp12* f, int G);
// the same with four pairs per f and each round's four lines multiplied together before they meet f
// (k_miller_acc4l); writes ceil(n / 4) values
hipError_t launch_miller_acc4l(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, const uint32_t* L,
                               size_t ld, Fp12* f);
// one pair per f on eight lanes (k_miller_acc8, the latency form for small batches); writes n values
hipError_t launch_miller_acc8(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, const uint32_t* L,
                              size_t ld, Fp12* f);
// the whole Miller loop of n pairs in one kernel (k_miller_fused: the G2 side and the f accumulation in the same
// workgroup, line records in LDS); G = 1 or 2 pairs per f; writes ceil(n / G) values (conjugated, x < 0)
hipError_t launch_miller_fused(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, Fp12* f, int G);
hipError_t launch_final_check_wave(hipStream_t st, const Fp12* f, int n, int* out);
// one bisection-tree level: node b is checked (res[b] = FE(node[b]) == 1, ++*nchecks) when parent is null or
// parent[b / pdiv] == 0, else res[b] = 1 (bls_fe.hip k_fe_check_gated)
hipError_t launch_final_check_gated(hipStream_t st, const Fp12* node, size_t n, const int* parent, uint32_t pdiv,
                                    int* res, uint32_t* nchecks);
// the same on the six-wave kernel (k_fe_wide)
hipError_t launch_fe_wide_gated(hipStream_t st, const Fp12* node, size_t n, const int* parent, uint32_t pdiv, int* res,
                                uint32_t* nchecks);
// out[b] = prod_{i in [b chunk, (b + 1) chunk) and < n} a[i] b[i]
hipError_t launch_fp12_chunk_prod2(hipStream_t st, const Fp12* a, const Fp12* b, size_t n, int chunk, Fp12* out);
// bisection fallback (bls_bisect.hip): the -G1 comb table (neg_g1_comb_entries() G1A), -r_i G1 in affine (tmp: B
// projective scratch points), verdicts from the leaf results
size_t neg_g1_comb_entries();
hipError_t launch_neg_g1_comb_table(hipStream_t st, G1A* tab);
hipError_t launch_neg_rg1(hipStream_t st, size_t B, const int* status, const uint64_t* rsc, const G1A* tab, G1P* tmp,
                          G1A* out);
hipError_t launch_verdicts_res(hipStream_t st, const int* status, const int* res, size_t B, uint8_t* out);
// projective -> affine with one inversion per 8 items (k_g1_affine_b); status-0 items -> identity
hipError_t launch_g1_affine(hipStream_t st, size_t B, const int* status, const G1P* Pj, G1A* out);
// nsel independent checks: out[b] = (FE(f[sel[b]]) == 1)
hipError_t launch_final_check_sel(hipStream_t st, const Fp12* f, const uint32_t* sel, size_t nsel, int* out);
hipError_t launch_fp12_chunk_prod(hipStream_t st, const Fp12* in, size_t n, int chunk, Fp12* out);
hipError_t launch_fp12_prod_vm(hipStream_t st, const Fp12* in, size_t n, Fp12* tmp, Fp12* out);
// out[b] = prod in[b chunk .. (b + 1) chunk) with the final exponentiation's lane-parallel product (bls_fe.hip)
hipError_t launch_fp12_chunk_prod_fe(hipStream_t st, const Fp12* in, size_t n, int chunk, Fp12* out);
hipError_t launch_fp12_chunk_prod2_fe(hipStream_t st, const Fp12* a, const Fp12* b, size_t n, int chunk, Fp12* out);
hipError_t launch_fp12_seg_prod_fe(hipStream_t st, const Fp12* in, const uint64_t* io, size_t B, Fp12* out);

// curve objects (bls_points.hip): group 1 = G1 (48-B encodings, G1A), 2 = G2 (96-B, G2A)
hipError_t launch_pt_decode(hipStream_t st, int group, const uint8_t* in, size_t n, int subgroup, void* out, int* ok);
// op 0: a + b, op 1: [k32] a; *ok = 0 if an encoding is invalid
hipError_t launch_pt_binop(hipStream_t st, int group, const uint8_t* a, const uint8_t* b, const uint8_t* k32, int op,
                           uint8_t* out, int* ok);
size_t pt_msm_scratch_bytes(int group, size_t n);
hipError_t launch_pt_msm(hipStream_t st, int group, const void* P, const uint8_t* k32, size_t n, void* tmp,
                         uint8_t* out);
hipError_t launch_gt_final_exp(hipStream_t st, const Fp12* f, uint8_t* out576);
hipError_t launch_gt_mul(hipStream_t st, const uint8_t* a, const uint8_t* b, uint8_t* out);

// wavefront-cooperative arithmetic (bls_wide.hip)
hipError_t launch_wide_selftest(hipStream_t st, size_t nw, const uint8_t* be48, int* bad);
// hash_to_G2 with one wave per message (msgs 32 B apart when offs is null); flag[i] = 1: recompute on the fallback;
// Hz: H in Jacobian coordinates (Z in Hz, 1 for flagged items) instead of affine
hipError_t launch_h2c_wide(hipStream_t st, size_t B, const uint8_t* msgs, const uint64_t* offs, G2A* H, int* flag,
                           Fp2* Hz = nullptr);
hipError_t launch_h2c_wide_dbg(hipStream_t st, const uint8_t* msg32, Fp* out);
// signature decode + subgroup check with one wave per signature (k_sig_validate semantics)
hipError_t launch_sig_validate_wide(hipStream_t st, const uint8_t* sigs, size_t n, G2A* out, int* ok);
// the whole Miller loop of npairs <= 2 pairs on one workgroup (line waves + six f waves): out = f (tower Fp12);
// ok0 / ok1 (nullable): pair 0 / 1 runs with constant lines unless *okp; qz (nullable): the pairs' Q are Jacobian
// (X, Y in Q, Z in qz; the f differs from the affine Q's by an Fp2 factor: the same final exponentiation)
// pz (nullable): the pairs' P are Jacobian (X, Y in P, Z in pz; the lines scaled by Z^3, an Fp factor)
hipError_t launch_miller_wide(hipStream_t st, const G1A* P, const G2A* Q, const int* ok0, const int* ok1, int npairs,
                              Fp12* out, const Fp2* qz = nullptr, const Fp* pz = nullptr);
// n pairs on miller_wide_nf(n) = ceil(n / 2) workgroups of the per-call kernel: out[0 .. miller_wide_nf(n)) (ok per
// pair, or nullptr)
size_t miller_wide_nf(size_t n);
hipError_t launch_miller_wide_n(hipStream_t st, const G1A* P, const G2A* Q, const int* ok, size_t n, Fp12* out,
                                const Fp2* qz = nullptr);
// final-exponentiation check of the product of f[0 .. n): easy part lane-parallel, hard part on six waves (F2)
hipError_t launch_fe_wide(hipStream_t st, const Fp12* f, int n, int* out, uint64_t* ts = nullptr);  // ts: stage clocks (tests)
// KeyValidate with two keys per wave (k_key_validate semantics)
hipError_t launch_key_validate_wide(hipStream_t st, const uint8_t* pks, size_t n, G1A* out, int* ok);
// the checked G1 decode (identity accepted, k_pt_decode semantics) on the wide KeyValidate kernel
hipError_t launch_g1_decode_checked_wide(hipStream_t st, const uint8_t* in48, size_t n, G1A* out, int* ok);

}  // namespace bls
