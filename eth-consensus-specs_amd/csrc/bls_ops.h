// Per-item BLS operations shared by the batch kernels (bls_kernels.hip):
// key validation, signature decode + subgroup check, and the pairing-product
// check.  Semantics follow the reference wrappers (E/utils/bls.py:141-221,
// 395-397) with milagro/py_ecc decode rules; any decode or subgroup failure
// yields "invalid" (0), never an exception, exactly like the reference's
// Verify/FastAggregateVerify/AggregateVerify try/except -> False mapping.
#pragma once
#include "bls_h2c.h"
#include "bls_pairing.h"

namespace bls {

// KeyValidate (py_ecc, E/utils/bls.py:395-397): decodes, not infinity, in G1.
BLS_HDNI int key_validate(G1A& out, const uint8_t* pk48) {
  int st = g1_decompress(out, pk48);
  if (st != DEC_OK) return 0;
  if (!g1_in_subgroup(jac_from_aff(out))) return 0;
  return 1;
}

// Signature decode + G2 subgroup check; the identity encoding is accepted.
BLS_HDNI int sig_validate(G2A& out, const uint8_t* sig96) {
  int st = g2_decompress(out, sig96);
  if (st == DEC_INFINITY) return 1;
  if (st != DEC_OK) return 0;
  if (!g2_in_subgroup(jac_from_aff(out))) return 0;
  return 1;
}

BLS_HD G1A g1_neg_generator() {
  G1A g = g1_generator();
  g.y = fp_neg(g.y);
  return g;
}

// e(P1, Q1) * e(P2, Q2) == 1
BLS_HDNI bool pairing_check2(const G1A& p1, const G2A& q1, const G1A& p2, const G2A& q2) {
  Fp12 f = fp12_mul(miller_loop(p1, q1), miller_loop(p2, q2));
  return fp12_is_one(final_exponentiation(f));
}

// CoreVerify with an already validated (non-identity) public key point.
BLS_HDNI int core_verify_point(const G1A& pk, const uint8_t* msg, uint32_t msg_len, const uint8_t* dst,
                             uint32_t dst_len, const uint8_t* sig96) {
  G2A s;
  if (!sig_validate(s, sig96)) return 0;
  G2A h = jac_to_aff(hash_to_g2(msg, msg_len, dst, dst_len));
  return pairing_check2(pk, h, g1_neg_generator(), s) ? 1 : 0;
}

}  // namespace bls
