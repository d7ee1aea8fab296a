// rp_probe.hip -- memory-pattern floor of a top-digit pass when each
// workgroup owns a contiguous RANGE of tiles and walks it in order
// (range-persistent, no look-back), against the XCD-contiguous one-tile-per-
// workgroup placement the segmented passes use today.  (experiment support,
// not product code)
//
// Digits of n random keys -> per-(tile, digit) counts and exact global write
// offsets (host, like one LSD pass).  Tiles are written exactly as a pass
// writes them: item i of a tile's sorted order to off[tile][digit(i)] + i -
// localStart[digit(i)] by consecutive threads.  Codecs (bytes per key):
//   0 keys   u32 in, u32 out                       (8)
//   1 split  u32 in, u16 + u8 planes out           (7: the bucket path's pass A)
//   2 planes u16 + u8 planes in, u16 out           (5: its pass B)
// Maps:
//   xcd   one tile per workgroup, XCD x gets a contiguous tile range
//   rp    PROBE_R persistent workgroups, workgroup g walks tiles
//         [g nT / R, (g+1) nT / R) in order
//   rpf   rp with the next tile's loads issued before the current write-out
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

#ifndef PROBE_THREADS
#define PROBE_THREADS 1024
#endif
#ifndef PROBE_KPT
#define PROBE_KPT 32
#endif
#ifndef PROBE_R
#define PROBE_R 256
#endif
#ifndef PROBE_LDS
#define PROBE_LDS (96 * 1024)  // dynamic LDS per workgroup (occupancy as the real pass)
#endif
constexpr int THREADS = PROBE_THREADS, KPT = PROBE_KPT;
constexpr uint32_t T = THREADS * KPT;

template <int CODEC>
__device__ __forceinline__ void load(const void* in, const uint8_t* inHi, uint64_t base, uint32_t (&k)[KPT]) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t b = base + (uint64_t)w * 64 * KPT + lane;
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    if constexpr (CODEC == 2)
      k[j] = ((uint32_t)inHi[b + j * 64] << 16) | reinterpret_cast<const uint16_t*>(in)[b + j * 64];
    else
      k[j] = reinterpret_cast<const uint32_t*>(in)[b + j * 64];
  }
}

template <int CODEC>
__device__ __forceinline__ void write_tile(void* out, uint8_t* outHi, const uint32_t (&k)[KPT], const uint32_t* s_off,
                                           const uint32_t* s_ls) {
  const uint32_t tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint32_t i = j * THREADS + tid;
    uint32_t lo = 0, hi = 256;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const uint32_t mid = (lo + hi) >> 1;
      if (s_ls[mid] <= i) lo = mid;
      else hi = mid;
    }
    const uint32_t dst = s_off[lo] + (i - s_ls[lo]);
    const uint32_t v = k[j] + 1;
    if constexpr (CODEC == 0) {
      reinterpret_cast<uint32_t*>(out)[dst] = v;
    } else if constexpr (CODEC == 1) {
      reinterpret_cast<uint16_t*>(out)[dst] = (uint16_t)v;
      outHi[dst] = (uint8_t)(v >> 24);
    } else {
      reinterpret_cast<uint16_t*>(out)[dst] = (uint16_t)v;
    }
  }
}

__device__ __forceinline__ void load_tables(const uint32_t* off, const uint16_t* ls, uint32_t tile, uint32_t* s_off,
                                            uint32_t* s_ls) {
  const uint32_t tid = threadIdx.x;
  if (tid < 256) {
    s_off[tid] = off[(uint64_t)tile * 256 + tid];
    s_ls[tid] = ls[(uint64_t)tile * 256 + tid];
  }
  if (tid == 0) s_ls[256] = T;
}

// MAP 0 = xcd (one tile per workgroup), 1 = rp, 2 = rpf
template <int MAP, int CODEC>
__global__ __launch_bounds__(THREADS) void probe(const void* __restrict__ in, const uint8_t* __restrict__ inHi,
                                                 void* __restrict__ out, uint8_t* __restrict__ outHi,
                                                 const uint32_t* __restrict__ off, const uint16_t* __restrict__ ls,
                                                 uint32_t nT) {
  extern __shared__ uint32_t dyn[];
  uint32_t* s_off = dyn;
  uint32_t* s_ls = dyn + 256;
  const uint32_t b = blockIdx.x;
  uint32_t k[KPT];
  if constexpr (MAP == 0) {
    const uint32_t tile = (b % 8) * (nT / 8) + b / 8;
    load_tables(off, ls, tile, s_off, s_ls);
    load<CODEC>(in, inHi, (uint64_t)tile * T, k);
    __syncthreads();
    write_tile<CODEC>(out, outHi, k, s_off, s_ls);
  } else {
    const uint32_t t0 = (uint32_t)((uint64_t)b * nT / gridDim.x), t1 = (uint32_t)((uint64_t)(b + 1) * nT / gridDim.x);
    if (t0 >= t1) return;
    load<CODEC>(in, inHi, (uint64_t)t0 * T, k);
    for (uint32_t t = t0; t < t1; ++t) {
      __syncthreads();
      load_tables(off, ls, t, s_off, s_ls);
      __syncthreads();
      if constexpr (MAP == 2) {
        uint32_t kn[KPT];
        if (t + 1 < t1) load<CODEC>(in, inHi, (uint64_t)(t + 1) * T, kn);
        write_tile<CODEC>(out, outHi, k, s_off, s_ls);
#pragma unroll
        for (int j = 0; j < KPT; ++j) k[j] = kn[j];
      } else {
        write_tile<CODEC>(out, outHi, k, s_off, s_ls);
        if (t + 1 < t1) load<CODEC>(in, inHi, (uint64_t)(t + 1) * T, k);
      }
    }
  }
}

template <int MAP, int CODEC>
double run(const void* in, const uint8_t* inHi, void* out, uint8_t* outHi, const uint32_t* off, const uint16_t* ls,
           uint32_t nT, uint32_t grid, int reps) {
  auto kern = probe<MAP, CODEC>;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, PROBE_LDS));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(THREADS), PROBE_LDS, 0, in, inHi, out, outHi, off, ls, nT);
  CK(hipGetLastError());
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(kern, dim3(grid), dim3(THREADS), PROBE_LDS, 0, in, inHi, out, outHi, off, ls, nT);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main() {
  const uint32_t n = 1u << 30, nT = n / T;
  std::vector<uint32_t> cnt((size_t)nT * 256, 0);
  uint64_t x = 0;
  for (uint32_t t = 0; t < nT; ++t)
    for (uint32_t i = 0; i < T; i += 8) {
      x += 0x9E3779B97F4A7C15ull;
      uint64_t z = x;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      for (int q = 0; q < 8; ++q) cnt[(size_t)t * 256 + ((z >> (8 * q)) & 255)]++;
    }
  std::vector<uint64_t> run_(256, 0);
  {
    std::vector<uint64_t> tot(256, 0);
    for (uint32_t t = 0; t < nT; ++t)
      for (int d = 0; d < 256; ++d) tot[d] += cnt[(size_t)t * 256 + d];
    for (int d = 1; d < 256; ++d) run_[d] = run_[d - 1] + tot[d - 1];
  }
  std::vector<uint32_t> off((size_t)nT * 256);
  std::vector<uint16_t> ls((size_t)nT * 256);
  for (uint32_t t = 0; t < nT; ++t) {
    uint32_t l = 0;
    for (int d = 0; d < 256; ++d) {
      off[(size_t)t * 256 + d] = (uint32_t)run_[d];
      ls[(size_t)t * 256 + d] = (uint16_t)l;
      run_[d] += cnt[(size_t)t * 256 + d];
      l += cnt[(size_t)t * 256 + d];
    }
  }
  void *in, *out;
  uint8_t *inHi, *outHi;
  uint32_t* doff;
  uint16_t* dls;
  CK(hipMalloc(&in, (size_t)n * 4));
  CK(hipMalloc(&out, (size_t)n * 4));
  CK(hipMalloc(&inHi, (size_t)n));
  CK(hipMalloc(&outHi, (size_t)n));
  CK(hipMalloc(&doff, off.size() * 4));
  CK(hipMalloc(&dls, ls.size() * 2));
  CK(hipMemset(in, 1, (size_t)n * 4));
  CK(hipMemset(inHi, 1, (size_t)n));
  CK(hipMemcpy(doff, off.data(), off.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dls, ls.data(), ls.size() * 2, hipMemcpyHostToDevice));
  printf("{\"tile\": %u, \"R\": %d, \"lds\": %d}\n", T, PROBE_R, PROBE_LDS);
  const double bpk[3] = {8, 7, 5};
  for (int rep = 0; rep < 2; ++rep) {
    double r[3][3];
    r[0][0] = run<0, 0>(in, inHi, out, outHi, doff, dls, nT, nT, 5);
    r[0][1] = run<1, 0>(in, inHi, out, outHi, doff, dls, nT, PROBE_R, 5);
    r[0][2] = run<2, 0>(in, inHi, out, outHi, doff, dls, nT, PROBE_R, 5);
    r[1][0] = run<0, 1>(in, inHi, out, outHi, doff, dls, nT, nT, 5);
    r[1][1] = run<1, 1>(in, inHi, out, outHi, doff, dls, nT, PROBE_R, 5);
    r[1][2] = run<2, 1>(in, inHi, out, outHi, doff, dls, nT, PROBE_R, 5);
    r[2][0] = run<0, 2>(in, inHi, out, outHi, doff, dls, nT, nT, 5);
    r[2][1] = run<1, 2>(in, inHi, out, outHi, doff, dls, nT, PROBE_R, 5);
    r[2][2] = run<2, 2>(in, inHi, out, outHi, doff, dls, nT, PROBE_R, 5);
    const char* cn[3] = {"keys", "split", "planes"};
    const char* mn[3] = {"xcd", "rp", "rpf"};
    for (int c = 0; c < 3; ++c)
      for (int m = 0; m < 3; ++m)
        printf("{\"codec\": \"%s\", \"map\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", cn[c], mn[m], r[c][m],
               bpk[c] * n / r[c][m] / 1e6);
    fflush(stdout);
  }
  return 0;
}
