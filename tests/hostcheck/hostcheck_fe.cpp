// TEST HARNESS ONLY: host build of the lane-parallel final exponentiation (bls_fe.h): the 64 lanes of every
// phase run in a loop (FeHost) over the same phase tables the kernel uses, with the digit-form column / value
// checks of bls_fq.h compiled in.  A translation unit of its own so it compiles beside the others.
#define BLS_FQ_CHECK 1
#define BLS_HD __host__ __device__ inline
#include "bls_ops.h"
#include "bls_fe.h"
#include <string.h>
using namespace bls;

static Fp in_fp(const uint8_t* b) { return fp_to_mont(raw_from_be48(b)); }
static void out_fp(uint8_t* b, const Fp& a) { raw_to_be48(fp_from_mont(a), b); }

// f: n Fp12 values, 12 canonical big-endian Fp each in tower order (c0.c0.c0, c0.c0.c1, c0.c1.c0, ...);
// out = FE(prod f)^3 in the same layout; returns 1 iff it is one
extern "C" int hc_fe_check(const uint8_t* f, int n, uint8_t* out) {
  static FeSlot s[FE_NSLOT];
  memset(s, 0, sizeof s);
  fe_load_consts(s, 0, 1);
  FeHost ex;
  ex.s = s;
  for (int i = 0; i < n; i++) {
    for (int j = 0; j < 12; j++) fe_st(s, 12 * (i ? 1 : 0) + j, fq_unpack(in_fp(f + 576 * i + 48 * j)));
    if (i) ex.mul(0, 1, 0);
  }
  fe_schedule(ex);
  int one = 1;
  for (int j = 0; j < 12; j++) {
    const Fp v = fq_pack(fe_ld(s, 12 + j));
    out_fp(out + 48 * j, v);
    one = one && (j == 0 ? fp_is_one(v) : fp_is_zero(v));
  }
  return one;
}
