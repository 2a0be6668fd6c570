/*
 * libblsmi355x -- MI355X (gfx950) BLS12-381 signature-verification backend.
 *
 * C ABI: plain pointers and sizes, caller-owned contiguous buffers, no torch
 * or HIP types.  It replaces the arithmetic the reference reaches through
 * ``eth2spec.utils.bls`` (reference ``tests/core/pyspec/eth2spec/utils/bls.py``,
 * written ``E/utils/bls.py`` below), i.e. the milagro_bls_binding /
 * py_ecc entry points bound at E/utils/bls.py:1-32,57-68.
 *
 * Return convention:
 *    1  valid / success
 *    0  invalid input (decode, subgroup, infinity, empty-list rejection,
 *       failed verification)
 *   <0  internal or device error (BLS_E_*); bls_last_error() describes it.
 * The Python shim maps a negative code to an exception everywhere, and 0 to
 * an exception exactly where the reference raises (Aggregate, AggregatePKs,
 * Sign, SkToPk), to False elsewhere.
 *
 * Threading: one context per process/device; calls on a context are
 * serialised by an internal mutex.  All device memory and streams are owned
 * by the context.  Every compute entry point runs on the GPU; there is no
 * CPU fallback (a missing/failed device is an error).
 */
#ifndef BLSMI355X_H
#define BLSMI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BLS_E_DEVICE (-1)  /* HIP runtime / kernel failure */
#define BLS_E_ARG (-2)     /* bad argument (NULL pointer, size overflow) */
#define BLS_E_NOREG (-3)   /* indexed call without a loaded registry */

typedef struct bls_ctx bls_ctx;

/* FAV batch slots of one context (bls_fav_job_*): the first BLS_FAV_JOBS_INIT (env, default 10) get streams
 * (BLS_JOB_STREAMS per job, default 2). */
#define BLS_FAV_JOBS 16

/* Context on HIP device `device` (ordinal).  Returns 0 or BLS_E_*. */
int bls_ctx_create(int device, bls_ctx** out);
void bls_ctx_destroy(bls_ctx* ctx);
const char* bls_last_error(bls_ctx* ctx);
/* Device name / CU count for reports; returns 0 or BLS_E_*. */
int bls_device_info(bls_ctx* ctx, char* name, size_t name_len, int* cu_count);

/* ---- drop-in per-call API (one call = one reference wrapper call) ---- */

/* Verify  <- E/utils/bls.py:141-151 (milagro Verify / py_ecc Verify). */
int bls_verify(bls_ctx* ctx, const uint8_t* pk48, const uint8_t* msg, size_t msg_len, const uint8_t* sig96);

/* FastAggregateVerify  <- E/utils/bls.py:167-177.  n == 0 -> 0. */
int bls_fast_aggregate_verify(bls_ctx* ctx, const uint8_t* pks48, size_t n, const uint8_t* msg, size_t msg_len,
                              const uint8_t* sig96);

/* AggregateVerify  <- E/utils/bls.py:154-164.  msgs is the concatenation of
 * the n messages, msg_lens[i] their lengths.  n == 0 -> 0. */
int bls_aggregate_verify(bls_ctx* ctx, const uint8_t* pks48, size_t n, const uint8_t* msgs, const size_t* msg_lens,
                         const uint8_t* sig96);

/* Aggregate  <- E/utils/bls.py:180-184.  1 and out96 on success; 0 on empty
 * list or an undecodable / non-G2 signature (the reference raises). */
int bls_aggregate(bls_ctx* ctx, const uint8_t* sigs96, size_t n, uint8_t* out96);

/* _AggregatePKs  <- E/utils/bls.py:202-213 (eth_aggregate_pubkeys,
 * specs/altair/bls.md:36-52).  0 on empty list or any key failing
 * KeyValidate (the reference raises). */
int bls_aggregate_pks(bls_ctx* ctx, const uint8_t* pks48, size_t n, uint8_t* out48);

/* KeyValidate  <- E/utils/bls.py:395-397. */
int bls_key_validate(bls_ctx* ctx, const uint8_t* pk48);

/* Sign / SkToPk  <- E/utils/bls.py:187-194,216-221; sk is 32 bytes
 * big-endian, 0 < sk < r (else 0). */
int bls_sign(bls_ctx* ctx, const uint8_t* sk32, const uint8_t* msg, size_t msg_len, uint8_t* out96);
int bls_sk_to_pk(bls_ctx* ctx, const uint8_t* sk32, uint8_t* out48);

/* hash_to_G2 (RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_) with caller DST,
 * compressed output.  The POP DST is the spec's (beacon-chain.md:692). */
int bls_hash_to_g2(bls_ctx* ctx, const uint8_t* msg, size_t msg_len, const uint8_t* dst, size_t dst_len,
                   uint8_t* out96);

/* ---- batch API (throughput path) -------------------- */

/* Decode + KeyValidate n compressed pubkeys into the HBM-resident affine
 * registry (replacing any previous one).  out_valid[i] = 1/0 (may be NULL).
 * Returns 1 or BLS_E_*. */
int bls_registry_load(bls_ctx* ctx, const uint8_t* pks48, size_t n, uint8_t* out_valid);
size_t bls_registry_size(bls_ctx* ctx);
/* Generation of the registry table: bumped whenever bls_registry_load or
 * bls_registry_generate replaces it (appends keep it).  A host-side
 * pubkey -> index map is valid only for the generation it was built on. */
uint64_t bls_registry_generation(bls_ctx* ctx);

/* B FastAggregateVerify calls over registry indices: item b uses
 * idx[offsets[b] .. offsets[b+1]) (offsets has B+1 entries), message
 * msgs32[32 b ..], signature sigs96[96 b ..].  out[b] = 1/0.  One random-
 * linear-combination pairing check for the whole batch; on failure a
 * bisection (16-ary product tree, batched final exponentiations) isolates the
 * invalid items.  Returns 1 or BLS_E_*. */
int bls_fav_batch_indexed(bls_ctx* ctx, const uint32_t* idx, const uint64_t* offsets, size_t B, const uint8_t* msgs32,
                          const uint8_t* sigs96, uint8_t* out);

/* B independent Verify calls with registry indices (gossip firehose): the
 * same RLC batch check + bisection as bls_fav_batch_indexed with one key per
 * item.  Returns 1 or BLS_E_*. */
int bls_verify_batch_indexed(bls_ctx* ctx, const uint32_t* idx, size_t B, const uint8_t* msgs32,
                             const uint8_t* sigs96, uint8_t* out);

/* B AggregateVerify calls  <- E/utils/bls.py:154-164 (one call per item).
 * Item b owns the pairs item_offs[b] .. item_offs[b+1] (item_offs has B+1
 * entries, total = item_offs[B]): pubkeys pks48[48 t ..], messages
 * msgs[msg_offs[t] .. msg_offs[t+1]) (msg_offs has total+1 entries, any
 * lengths), and signature sigs96[96 b ..].  out[b] = 1/0 with the per-call
 * semantics of bls_aggregate_verify (empty item, invalid key or signature ->
 * 0).  One random-linear-combination pairing check over all items; when it
 * fails every item is checked on its own (batched final exponentiations).
 * Returns 1 or BLS_E_*. */
int bls_aggregate_verify_batch(bls_ctx* ctx, const uint8_t* pks48, const uint8_t* msgs, const uint64_t* msg_offs,
                               const uint64_t* item_offs, size_t B, const uint8_t* sigs96, uint8_t* out);

/* Append n compressed keys to the HBM registry (deposits: new validator
 * indices reg_n .. reg_n + n), decoding + KeyValidate on the device like
 * bls_registry_load; out_valid as there.  Existing entries keep their
 * indices.  <- specs/phase0/beacon-chain.md:2037-2062 (add_validator_to_registry),
 * specs/electra/beacon-chain.md:1577-1588.  Returns 1 or BLS_E_*. */
int bls_registry_append(bls_ctx* ctx, const uint8_t* pks48, size_t n, uint8_t* out_valid);

/* ---- signing roots and SSZ merkleization ------ */
/* out32[i] = SHA-256(object_roots32[32 i ..] || domains32[domain_stride i ..]):
 * compute_signing_root  <- specs/phase0/beacon-chain.md:953-962 (SigningData
 * :317-320).  domain_stride 0 = one domain for all, 32 = one per item.
 * Returns 1 or BLS_E_*. */
int bls_signing_roots(bls_ctx* ctx, const uint8_t* object_roots32, const uint8_t* domains32, size_t domain_stride,
                      size_t n, uint8_t* out32);
/* SSZ merkleize(chunks, limit): n 32-byte chunks, tree of 2^depth leaves
 * (depth >= ceil(log2 n); missing leaves are zero chunks).  n = 0 gives the
 * zero-subtree root of that depth.  Returns 1 or BLS_E_*. */
int bls_merkleize(bls_ctx* ctx, const uint8_t* chunks32, size_t n, int depth, uint8_t* root32);

/* ---- KZG pieces ---------------------------------- */
/* pairing_check  <- E/utils/bls.py pairing_check (used by
 * specs/deneb/polynomial-commitments.md:284,407,451): 1 iff
 * prod_i e(P_i, Q_i) == 1 for compressed P_i (48 B, identity allowed) and
 * Q_i (96 B, identity allowed); both subgroup-checked.  0 if the product is
 * not 1 or any encoding is invalid.  Returns 1 / 0 / BLS_E_*. */
int bls_pairing_check(bls_ctx* ctx, const uint8_t* g1s48, const uint8_t* g2s96, size_t n);
/* multi_exp / g1_lincomb  <- E/utils/bls.py multi_exp
 * (specs/deneb/polynomial-commitments.md g1_lincomb): out48 = compressed
 * sum_i [k_i] P_i, scalars as 32-byte big-endian integers.  1 on success, 0
 * if a point encoding is invalid (the reference raises).  Returns 1 / 0 /
 * BLS_E_*. */
int bls_g1_multi_exp(bls_ctx* ctx, const uint8_t* g1s48, const uint8_t* scalars32, size_t n, uint8_t* out48);

/* ---- curve objects  <- E/utils/bls.py:224-392 ---------------------------
 * The arkworks G1Point / G2Point / GT operations of the reference's
 * fastest_bls helpers: add (:239-246), multiply (:249-259), multi_exp
 * (:262-296), neg (:299-306), bytes48_to_G1 / bytes96_to_G2 (unchecked decode,
 * :367-392), G1_to_bytes48 / G2_to_bytes96 (:345-364), pairing_check
 * (:224-236).  group: 1 = G1 (48-byte compressed), 2 = G2 (96-byte).  The
 * identity encoding is a valid point.  Return 1 on success, 0 if an encoding
 * is invalid (the reference raises), BLS_E_* on errors. */
/* out_ok[i] (may be NULL) = 1 iff in[i] decodes (and, with subgroup_check, lies
 * in G1 / G2); returns 1 iff all do. */
int bls_point_decode(bls_ctx* ctx, int group, const uint8_t* in, size_t n, int subgroup_check, uint8_t* out_ok);
int bls_point_add(bls_ctx* ctx, int group, const uint8_t* a, const uint8_t* b, uint8_t* out);
/* [k] P, k a 32-byte big-endian integer (the reference reduces scalars mod r first) */
int bls_point_mul(bls_ctx* ctx, int group, const uint8_t* p, const uint8_t* k32, uint8_t* out);
int bls_point_neg(bls_ctx* ctx, int group, const uint8_t* p, uint8_t* out);
/* sum_i [k_i] P_i.  n == 0 -> 0 (the reference raises, E/utils/bls.py:270-271).
 * subgroup_check 0 = multiexp_unchecked (:280-282). */
int bls_multi_exp(bls_ctx* ctx, int group, const uint8_t* pts, const uint8_t* scalars32, size_t n, int subgroup_check,
                  uint8_t* out);
/* GT.multi_pairing: prod_i e(P_i, Q_i) after the final exponentiation, as 576
 * bytes (six Fp2 coefficients c0..c5 of the w-basis, each c0||c1 big-endian;
 * GT one = byte 47 set).  n == 0 gives one. */
int bls_multi_pairing(bls_ctx* ctx, const uint8_t* g1s48, const uint8_t* g2s96, size_t n, int subgroup_check,
                      uint8_t* out576);
int bls_gt_mul(bls_ctx* ctx, const uint8_t* a576, const uint8_t* b576, uint8_t* out576);
/* pairing_check over curve objects (arkworks GT.multi_pairing(...) == GT.one(),
 * :229): subgroup_check 0 skips the subgroup checks of bls_pairing_check. */
int bls_pairing_check_ex(bls_ctx* ctx, const uint8_t* g1s48, const uint8_t* g2s96, size_t n, int subgroup_check);

/* Fallback statistics of the last batch finished on this context: the number
 * of final-exponentiation checks and bisection rounds (tree levels) it ran
 * (both 0 when the whole-batch check passed; waits for that batch's
 * verdicts).  Returns 0 or BLS_E_*. */
int bls_last_fallback_stats(bls_ctx* ctx, uint64_t* fe_checks, uint64_t* rounds);

/* Synthetic registry for benchmarks: pk_i = (first_sk + i) * G1 written
 * straight into the HBM registry (all valid); compressed keys are copied
 * to out_pks48 when non-NULL.  Returns 1 or BLS_E_*. */
int bls_registry_generate(bls_ctx* ctx, uint64_t first_sk, size_t n, uint8_t* out_pks48);

/* Synthetic-data helpers (used by bench.py and tests to make inputs). */
int bls_sign_batch(bls_ctx* ctx, const uint8_t* sks32, const uint8_t* msgs32, size_t B, uint8_t* out96);
int bls_sk_to_pk_batch(bls_ctx* ctx, const uint8_t* sks32, size_t B, uint8_t* out48);

/* ---- device-resident variants (inputs already in HBM) ----------------- */
void* bls_dev_alloc(bls_ctx* ctx, size_t bytes);
int bls_dev_free(bls_ctx* ctx, void* dptr);
int bls_h2d(bls_ctx* ctx, void* dst, const void* src, size_t bytes);
/* bls_d2h and bls_sync first wait for every job stream of the context (verdicts
 * of pipelined jobs are written asynchronously, see bls_fav_job_finish_dev). */
int bls_d2h(bls_ctx* ctx, void* dst, const void* src, size_t bytes);
int bls_sync(bls_ctx* ctx);

/* Phase 1 of a (possibly multi-GPU) FAV batch on device pointers: per-item
 * checks and this shard's Miller-loop product, written to partial576 (host,
 * 576 bytes: the 6 w-basis Fp2 coefficients, each c0||c1 big-endian).
 * seed32 keys the RLC scalars.  Per-item state stays in the context. */
int bls_fav_batch_partial_dev(bls_ctx* ctx, const uint32_t* d_idx, const uint64_t* d_offsets, size_t B,
                              const uint8_t* d_msgs32, const uint8_t* d_sigs96, const uint8_t* seed32,
                              uint8_t* partial576);
/* Final exponentiation of the product of n partials == 1 ?  1 / 0. */
int bls_partials_check(bls_ctx* ctx, const uint8_t* partials576, size_t n);
/* Phase 2: write verdicts for the batch prepared by the last
 * bls_fav_batch_partial_dev call on this context.  batch_ok = result of
 * bls_partials_check; when 0 this shard is bisected (its own product is
 * re-checked first, so a bad shard elsewhere leaves these verdicts intact). */
int bls_fav_batch_finish_dev(bls_ctx* ctx, int batch_ok, uint8_t* d_out);

/* ---- pipelined FAV batches (device-resident inputs) --------------------
 * The three phases above, split per job so that up to BLS_FAV_JOBS batches
 * are in flight on one context: while job k's Miller product is gathered
 * (RCCL) and final-exponentiated, job k+1's kernels already run on the job's
 * own streams.  A job must be finished before it is submitted again; each
 * job keeps its own per-item state for its finish/bisection.  Same meaning,
 * return codes and verdicts as bls_fav_batch_partial_dev / bls_partials_check
 * / bls_fav_batch_finish_dev (those are job 0, submitted and waited at once).
 *   submit:  enqueue the batch, return at once (1 or BLS_E_*)
 *   partial: wait for the job's 576-byte Miller product
 *   check:   final exponentiation of the product of n partials: 1 / 0
 *   finish:  verdicts into d_out, enqueued on the job's stream without a host
 *            wait -- a failing batch's bisection runs there on the device (no
 *            host round trip per round) while the host checks the next job;
 *            bls_d2h / bls_sync wait for it */
int bls_fav_job_submit_dev(bls_ctx* ctx, int job, const uint32_t* d_idx, const uint64_t* d_offsets, size_t B,
                           const uint8_t* d_msgs32, const uint8_t* d_sigs96, const uint8_t* seed32);
int bls_fav_job_partial(bls_ctx* ctx, int job, uint8_t* partial576);
int bls_fav_job_check(bls_ctx* ctx, int job, const uint8_t* partials576, size_t n);
/* check_own: the final exponentiation of the job's own product alone, which
 * submit already enqueued on the job's stream (the single-GPU check: no host
 * round trip of the partial; with a communicator it runs on demand): 1 / 0.
 * A finish after a failed multi-shard check uses the same verdict -- a job
 * whose own product passes keeps every per-item status, one whose own product
 * fails bisects below its root.  Another batch prepared on the job since its
 * submit (the host-buffer calls use job 0) voids that verdict: check_own is
 * then BLS_E_ARG and a failing finish bisects from the root. */
int bls_fav_job_check_own(bls_ctx* ctx, int job);
int bls_fav_job_finish_dev(bls_ctx* ctx, int job, int batch_ok, uint8_t* d_out);

/* ---- multi-GPU exchange over RCCL ----------------------
 * One communicator per context.  bls_comm_unique_id runs on one rank; its 128
 * bytes reach the other ranks out of band (bench.py: the torchrun TCP store).
 * With a communicator on the context, bls_fav_job_submit_dev itself enqueues
 * the exchange behind the job's Miller product: the 576-byte partial is
 * all-gathered on the device (ncclAllGather over xGMI, on the context's one
 * comm stream, so the collectives run in submission order -- every rank
 * submits the same jobs in the same order) and the job's stream multiplies
 * the world partials inside the final-exponentiation kernel.  No host step
 * sits between a job's product and its verdict; bls_fav_job_check_comm only
 * waits for that verdict (1 / 0).  The job's own check is then not enqueued:
 * a failing verdict is localised by bls_fav_job_finish_dev(..., 0, ...) on
 * every rank, which checks its own partial first, so only the bad shard
 * bisects.  A rank with an empty shard submits B = 0 (its partial is the
 * identity) and still joins every all-gather; B = 0 without a communicator is
 * BLS_E_ARG.  A submit that fails after the communicator exists aborts it
 * (below), so peers never wait for this rank's collective. */
int bls_comm_unique_id(uint8_t* out128);
int bls_comm_init(bls_ctx* ctx, const uint8_t* uid128, int rank, int world);
int bls_comm_destroy(bls_ctx* ctx);
int bls_fav_job_check_comm(bls_ctx* ctx, int job);
/* Abort the communicator (ncclCommAbort): peers blocked in a collective with
 * this rank fail instead of hanging.  The library calls it itself when
 * bls_fav_job_submit_dev or bls_fav_job_check_comm fails after the communicator exists; a host that
 * leaves the exchange on its own error (bench.py, dist.py) calls it before
 * exiting.  No-op without a communicator. */
int bls_comm_abort(bls_ctx* ctx);

/* ---- tracing: hipEvent time per kernel of the FAV path ------------------ */
int bls_profile_enable(bls_ctx* ctx, int on);  /* also resets the totals */
/* Fills up to max entries of total_ms / counts; returns the entry count. */
int bls_profile_read(bls_ctx* ctx, double* total_ms, uint64_t* counts, int max);
const char* bls_profile_name(int i);

/* ---- RLC seed entropy (host only, no device needed) ----------------------
 * bls_host_seed fills 32 bytes from the entropy source (/dev/urandom) and
 * returns 0, or BLS_E_DEVICE (seed zeroed) when fewer than 32 bytes can be
 * read: every batch call that draws an RLC seed then fails closed with
 * BLS_E_DEVICE instead of using a predictable seed.  bls_set_entropy_source
 * redirects the source (process-wide) and exists for tests. */
int bls_host_seed(uint8_t* seed32);
int bls_set_entropy_source(const char* path);

/* ---- test hooks (tests/ only; no reference counterpart) -------------------
 * bls_test_force_h2c_fallback: items i < n with mask[i] != 0 of every later
 * hash_to_G2 (batch, per-call, AggregateVerify) take the reference-path
 * fallback kernel as if the lane kernels had flagged them; n = 0 clears.
 * Refused (BLS_E_ARG) unless the environment has BLSMI355X_TEST_HOOKS=1, so a
 * production process cannot reroute its hashes by accident.
 * bls_test_hash_to_g2_batch: hash_to_G2 (DST POP) of n 32-byte messages through
 * the FAV batch's kernels and fallback routing, compressed into out96. */
int bls_test_force_h2c_fallback(bls_ctx* ctx, const uint8_t* mask, size_t n);
int bls_test_hash_to_g2_batch(bls_ctx* ctx, const uint8_t* msgs32, size_t n, uint8_t* out96);
/* bls_test_miller_forms: the product of n pairings (48-B G1 / 96-B G2 encodings, no subgroup checks) through each
 * Miller-loop form of the batch path, final-exponentiated: out576 holds 8 x 576 bytes -- split lines +
 * accumulation (G = 2), fused (G = 2), fused (G = 1), split (G = 4), the wave-program kernel, split (G = 8),
 * split (G = 4, each step's lines multiplied together first), split (G = 1 on eight lanes per f).
 * 1, or 0 on an invalid encoding. */
int bls_test_miller_forms(bls_ctx* ctx, const uint8_t* g1s48, const uint8_t* g2s96, size_t n, uint8_t* out576);
/* the same through the one-wave-per-message kernel of the per-call path */
int bls_test_hash_to_g2_wide(bls_ctx* ctx, const uint8_t* msgs32, size_t n, uint8_t* out96);
/* intermediate stages of the one-wave hash of one 32-byte message (debugging) */
int bls_test_h2c_wide_stages(bls_ctx* ctx, const uint8_t* msg32, uint8_t* out);
/* bls_test_final_check: the final-exponentiation check (FE(f_0 .. f_{n-1}) == 1) of n <= 64 raw Fp12 values
 * (576 bytes each: 12 little-endian Montgomery Fp in tower order) on the six-wave kernel (wide != 0) or the
 * one-wave lane kernel; *out = 1 / 0.  wide == 2: also the six-wave kernel's stage clocks (wall_clock64, 100 MHz)
 * as 8 uint64 at out + 2 (out then needs room for 18 int32). */
int bls_test_final_check(bls_ctx* ctx, const uint8_t* f576, size_t n, int wide, int32_t* out);

/* bls_test_wide_selftest: nw waves compare the wavefront-cooperative products
 * (bls_wide.h) with the lane form on four inputs each (48-byte big-endian
 * integers < p); bad[w] = bitmask of differing forms, 0 when all agree. */
int bls_test_wide_selftest(bls_ctx* ctx, const uint8_t* in48, size_t nw, int32_t* bad);

#ifdef __cplusplus
}
#endif
#endif /* BLSMI355X_H */
