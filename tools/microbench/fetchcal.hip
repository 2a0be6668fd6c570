// FETCH_SIZE calibration for 4-byte-per-lane loads (MI355X_MICROARCH.md: the counter reads exactly 1/2 of the
// bytes of 16-B/lane streaming reads; other widths are uncalibrated).  Two kernels with known byte counts:
//   k_stream4   every word of a 1 GiB buffer once, 4 B per lane, coalesced (past the 256 MiB Infinity Cache)
//   k_acc_like  (ld = n, then ld padded to 32 pairs) the line-record reads of k_miller_acc4q<2> (bls_miller_pair.hip ld_line) for n pairs: 68 lines x
//               84 words per pair, word w of line k of pair i at L[(84 k + w) n + i]; lane 4 grp + 2 h + q reads l0
//               (28 words, the same for the group's four lanes) and its 14 words of c for pairs 2 grp, 2 grp + 1
// Run under rocprofv3 --pmc FETCH_SIZE; the expected bytes are printed.  Build:
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/fetchcal.hip -o tools/microbench/fetchcal
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void __launch_bounds__(256) k_stream4(const uint32_t* in, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= in[i];
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void __launch_bounds__(64) k_acc_like(const uint32_t* L, size_t n, size_t ld, uint32_t* out) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t grp = t >> 2;
  const bool h = (t & 2) != 0, q = (t & 1) != 0;
  if (grp * 2 >= n) return;
  uint32_t acc = 0;
  for (int k = 0; k < 68; ++k)
    for (int g = 0; g < 2; ++g) {
      const size_t p = grp * 2 + g < n ? grp * 2 + g : n - 1;
      const uint32_t* Li = L + (size_t)k * 84 * ld + p;
#pragma unroll
      for (int j = 0; j < 28; ++j) acc += Li[(size_t)j * ld];
      const int w0 = (h ? 56 : 28) + (q ? 14 : 0);
#pragma unroll
      for (int j = 0; j < 14; ++j) acc ^= Li[(size_t)(w0 + j) * ld];
    }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const size_t nw = (size_t)1 << 28;  // 1 GiB
  const size_t npair = 10064;          // a C2 batch (10,000 items + 64 MSM pairs)
  const size_t ldp = (npair + 31) & ~(size_t)31;  // bls_miller_lane.hip miller_lines_ld
  const size_t nl = (size_t)68 * 84 * ldp;
  uint32_t *a, *l, *o;
  if (hipMalloc(&a, nw * 4) || hipMalloc(&l, nl * 4) || hipMalloc(&o, 64)) return 1;
  hipMemset(a, 1, nw * 4);
  hipMemset(l, 1, nl * 4);
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(k_stream4, dim3(8192), dim3(256), 0, 0, a, nw, o);
    // a 1 GiB sweep between the record reads evicts them from the Infinity Cache
    hipLaunchKernelGGL(k_acc_like, dim3((unsigned)((npair / 2 * 4 + 63) / 64)), dim3(64), 0, 0, l, npair, npair, o);
    hipLaunchKernelGGL(k_stream4, dim3(8192), dim3(256), 0, 0, a, nw, o);
    hipLaunchKernelGGL(k_acc_like, dim3((unsigned)((npair / 2 * 4 + 63) / 64)), dim3(64), 0, 0, l, npair, ldp, o);
  }
  if (hipDeviceSynchronize()) return 1;
  printf("k_stream4 expected %zu bytes; k_acc_like expected %zu bytes (84 words x 4 B x 68 lines x %zu pairs), "
         "ld = n then ld = %zu\n",
         nw * 4, (size_t)68 * 84 * 4 * npair, npair, ldp);
  return 0;
}
