// scatter_probe.hip -- achievable HBM rate of a radix pass's memory pattern
// without any sort work (experiment support for DESIGN.md s3; not product code).
//
// n u32 keys; a "tile" of T keys is read coalesced (like thrs_pass) and
// written as B = 256 runs of T/256 consecutive keys, run r of tile t going to
// region r (n/256 keys) at offset t*T/256: exactly the write pattern of one
// LSD pass over uniformly distributed digits.  Also timed: a plain contiguous
// copy.  Reports GB/s counting read + written bytes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

// THREADS threads, KPT keys per thread; tile = THREADS*KPT keys
template <int THREADS, int KPT>
__global__ __launch_bounds__(THREADS) void scatter_runs(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       uint32_t n) {
  extern __shared__ uint32_t dummy_lds[];  // occupancy control only
  if (n == 0) dummy_lds[threadIdx.x] = 0;
  constexpr uint32_t T = THREADS * KPT, RUN = T / 256;
  const uint32_t tile = blockIdx.x;
  const uint32_t regionKeys = n / 256;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t k[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) k[j] = in[(uint64_t)tile * T + w * 64 * KPT + j * 64 + lane];
  // write: item i of the tile (i = j*THREADS + tid, like the stage write-out)
  // goes to run i / RUN at position i % RUN
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint32_t i = j * THREADS + threadIdx.x;
    const uint32_t r = i / RUN, p = i % RUN;
    out[(uint64_t)r * regionKeys + (uint64_t)tile * RUN + p] = k[j] + 1;
  }
}

// Same, but every run starts at a per-(tile, run) offset that is NOT line
// aligned (shift in [0,64) keys, as random digit counts produce): runs
// straddle 128-B lines whose other part belongs to a neighbouring tile.
// POLICY: 0 plain store, 1 nt, 2 sc1 (write-through), 3 sc0 sc1
template <int THREADS, int KPT, int POLICY>
__global__ __launch_bounds__(THREADS) void scatter_runs_misaligned(const uint32_t* __restrict__ in,
                                                                  uint32_t* __restrict__ out, uint32_t n) {
  constexpr uint32_t T = THREADS * KPT, RUN = T / 256;
  const uint32_t tile = blockIdx.x;
  const uint32_t regionKeys = n / 256;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t k[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) k[j] = in[(uint64_t)tile * T + w * 64 * KPT + j * 64 + lane];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint32_t i = j * THREADS + threadIdx.x;
    const uint32_t r = i / RUN, p = i % RUN;
    const uint32_t shift = (tile * 2654435761u + r * 40503u) >> 26;  // 0..63
    uint64_t pos = (uint64_t)r * regionKeys + (uint64_t)tile * RUN + shift + p;
    if (pos >= n) pos = n - 1;
    uint32_t* a = out + pos;
    const uint32_t v = k[j] + 1;
    if constexpr (POLICY == 0) *a = v;
    if constexpr (POLICY == 1) __builtin_nontemporal_store(v, a);
    if constexpr (POLICY == 2) __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (POLICY == 3) __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <int THREADS, int KPT, int POLICY>
double time_misaligned(const uint32_t* in, uint32_t* out, uint32_t n, int reps) {
  constexpr uint32_t T = THREADS * KPT;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((scatter_runs_misaligned<THREADS, KPT, POLICY>), dim3(n / T), dim3(THREADS), 0, 0, in, out, n);
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((scatter_runs_misaligned<THREADS, KPT, POLICY>), dim3(n / T), dim3(THREADS), 0, 0, in, out, n);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

__global__ void copy4(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

template <int THREADS, int KPT>
double time_scatter(const uint32_t* in, uint32_t* out, uint32_t n, int reps, size_t lds = 0) {
  constexpr uint32_t T = THREADS * KPT;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  if (lds > 65536)
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(scatter_runs<THREADS, KPT>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL((scatter_runs<THREADS, KPT>), dim3(n / T), dim3(THREADS), lds, 0, in, out, n);
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((scatter_runs<THREADS, KPT>), dim3(n / T), dim3(THREADS), lds, 0, in, out, n);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main() {
  const uint32_t n = 1u << 30;
  uint32_t *in, *out;
  CK(hipMalloc(&in, (size_t)n * 4));
  CK(hipMalloc(&out, (size_t)n * 4));
  CK(hipMemset(in, 1, (size_t)n * 4));
  const double bytes = 2.0 * n * 4;
  const int reps = 10;
  auto rep = [&](const char* name, double ms) {
    printf("{\"case\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, bytes / ms / 1e6);
    fflush(stdout);
  };
  rep("run32_tile8K_256thr", time_scatter<256, 32>(in, out, n, reps));
  rep("run64_tile16K_512thr", time_scatter<512, 32>(in, out, n, reps));
  rep("run64_tile16K_1024thr", time_scatter<1024, 16>(in, out, n, reps));
  rep("run64_tile16K_512thr_lds73K(2WG/CU)", time_scatter<512, 32>(in, out, n, reps, 73 * 1024));
  rep("run64_tile16K_512thr_lds50K(3WG/CU)", time_scatter<512, 32>(in, out, n, reps, 50 * 1024));
  rep("run64_tile16K_512thr_lds150K(1WG/CU)", time_scatter<512, 32>(in, out, n, reps, 150 * 1024));
  rep("misaligned_run64_tile16K_plain", time_misaligned<512, 32, 0>(in, out, n, reps));
  rep("misaligned_run64_tile16K_nt", time_misaligned<512, 32, 1>(in, out, n, reps));
  rep("misaligned_run64_tile16K_sc1", time_misaligned<512, 32, 2>(in, out, n, reps));
  rep("misaligned_run64_tile16K_sys", time_misaligned<512, 32, 3>(in, out, n, reps));
  rep("misaligned_run128_tile32K_plain", time_misaligned<1024, 32, 0>(in, out, n, reps));
  rep("misaligned_run256_tile64K_plain", time_misaligned<1024, 64, 0>(in, out, n, reps));
  rep("run128_tile32K_1024thr", time_scatter<1024, 32>(in, out, n, reps));
  rep("run256_tile64K_1024thr", time_scatter<1024, 64>(in, out, n, reps));
  {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t n4 = (size_t)n / 4;
    for (int grid : {1024, 2048, 8192}) {
      hipLaunchKernelGGL(copy4, dim3(grid), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, n4);
      CK(hipEventRecord(e0, 0));
      for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(copy4, dim3(grid), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, n4);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      char nm[64];
      snprintf(nm, sizeof nm, "copy_uint4_grid%d", grid);
      rep(nm, ms / reps);
    }
  }
  return 0;
}
