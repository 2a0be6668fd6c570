// Field / point storage types for the MI355X BLS12-381 backend.
//
// Fp is one 381-bit residue in Montgomery form (R = 2^406) stored as 12 x
// 32-bit little-endian limbs (48 B, 16-B aligned for b128 LDS/global access);
// multiplication unpacks it to 14 radix-2^29 digits (bls_fp.h).  Every arithmetic routine is __host__ __device__
// so the same source is unit-tested on the host (tests/hostcheck) and run in
// the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef BLS_HD  // the host test harness's digit-form unit (tests/hostcheck/hostcheck_fq.cpp) predefines it without
                // the forced inlining: its checked products inlined everywhere took ~15 min to compile
#define BLS_HD __host__ __device__ __forceinline__
#endif
#define BLS_HDNI __host__ __device__ inline __attribute__((noinline))

namespace bls {

struct alignas(16) Fp {
  uint32_t l[12];
};
// VM slot form of an Fp value (bls_vm.h): 14 radix-2^29 digits + 2 zero pad
// words, canonical residue in Montgomery form, in an 80-B slot.  The VM reads
// a slot as four ds_read_b128 (d[0..15]); d[16..19] only space the slots.  With
// 64-B slots, slot s began at bank group (4 s) mod 16 of a ds_read_b128, so
// the 16 lanes of a group met in 4 groups (rocprofv3: 41-82 % of the VM
// kernels' LDS cycles were bank conflicts); at 80 B it is (5 s) mod 16.
struct alignas(16) Fd {
  uint32_t d[20];
};
// Lane-kernel form of an Fp value (bls_fq.h): 14 digits of radix 2^29, the
// same Montgomery radix R = 2^406, redundant (digits may exceed 2^29 and the
// value p) -- additions and subtractions are digit-wise with no carry chain.
struct Fq {
  uint32_t d[14];
};
struct Fq2 {
  Fq c0, c1;
};
struct Fq6 {
  Fq2 c0, c1, c2;
};
struct Fp2 {
  Fp c0, c1;  // c0 + c1 * i,  i^2 = -1
};
struct Fp6 {
  Fp2 c0, c1, c2;  // c0 + c1 v + c2 v^2,  v^3 = xi = 1 + i
};
struct Fp12 {
  Fp6 c0, c1;  // c0 + c1 w,  w^2 = v
};
// HBM registry entry: affine (x, y) of one key in Montgomery form, 96 B of
// data in a 128-B record, 128-B aligned (hipMalloc is 256-B aligned), so a
// random key read is exactly one 128-B line: with 96-B records half of them
// straddled two lines, and the gather moved ~192 B per key (profiles/r03*_pmc_fetch.md).
// Bit 31 of x.l[11] lies above the 381-bit residue and holds the KeyValidate
// verdict (REG_VALID), so no side array is read.
struct alignas(128) RegKey {
  Fp x, y;
  uint32_t pad[8];
};
constexpr uint32_t REG_VALID = 0x80000000u;

}  // namespace bls
