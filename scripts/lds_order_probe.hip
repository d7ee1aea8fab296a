// Diagnostic: does ds_add_rtn_u32 return values in lane order when several
// lanes of one wave hit the same LDS word?  Compares against the ballot-match
// rank for random digit patterns (dense, sparse, partial exec).  Not product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../tinyhipradixsort_amd/csrc/thrs_kernels.hpp"
using namespace thrs_dev;

__global__ void probe(unsigned long long* bad, unsigned long long* total, int iters, int mode) {
  __shared__ uint32_t cnt[4][256];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned long long b = 0, t = 0;
  uint64_t x = (blockIdx.x * 256ull + threadIdx.x) * 0x9E3779B97F4A7C15ull + 12345;
  for (int it = 0; it < iters; ++it) {
    for (int i = lane; i < 256; i += 64) cnt[w][i] = 0;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 29;
    uint32_t d = (uint32_t)(x >> 24) & 0xFF;
    if (mode == 1) d &= 0x3;            // heavy conflicts
    if (mode == 2) d = (it & 1) ? 7 : d & 0x1F;
    bool active = (mode == 3) ? ((x >> 60) != 0) : true;
    if (active) {
      uint32_t mlo, mhi;
      match_digit(d, mlo, mhi);
      const uint32_t want = __builtin_amdgcn_mbcnt_hi(mhi, __builtin_amdgcn_mbcnt_lo(mlo, 0u));
      const uint32_t got = __hip_atomic_fetch_add(&cnt[w][d], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      b += (got != want);
      t += 1;
    }
  }
  atomicAdd(bad, b);
  atomicAdd(total, t);
}

int main() {
  unsigned long long *d, h[2];
  hipMalloc(&d, 16);
  for (int mode = 0; mode < 4; ++mode) {
    hipMemset(d, 0, 16);
    hipLaunchKernelGGL(probe, dim3(4096), dim3(256), 0, 0, d, d + 1, 256, mode);
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    std::printf("mode %d: lanes %llu  out-of-lane-order %llu\n", mode, h[1], h[0]);
  }
  return 0;
}
