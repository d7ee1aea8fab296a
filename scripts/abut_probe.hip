// abut_probe.hip -- does XCD placement of consecutive tiles change the cost of
// a radix pass's partial-line writes?  (experiment support, not product code)
//
// Digits of n random keys -> per-(tile, digit) counts and exact global write
// offsets (host, like one LSD pass).  Each workgroup takes one tile: loads its
// keys (coalesced), and writes item i of the tile's sorted order to
// off[tile][digit(i)] + i - localStart[digit(i)], so runs of neighbouring
// tiles abut exactly as in thrs_pass.  Two tile placements:
//   rr     tile = blockIdx.x          (hardware round-robins blockIdx over the
//          8 XCDs: consecutive tiles land on different XCDs / L2s)
//   xcd    tile = (b % 8) * (nT / 8) + b / 8   (XCD x gets a contiguous range:
//          consecutive tiles share an L2, so a line split between two tiles'
//          runs is merged in L2 before write-back)
// Reports GB/s over read + written bytes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <type_traits>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

// geometry / element size (-D): PROBE_THREADS x PROBE_KPT keys per tile,
// PROBE_ELEM-byte elements (2: the u16 planes of the bucket path's passes)
#ifndef PROBE_THREADS
#define PROBE_THREADS 512
#endif
#ifndef PROBE_KPT
#define PROBE_KPT 32
#endif
#ifndef PROBE_ELEM
#define PROBE_ELEM 4
#endif
constexpr int THREADS = PROBE_THREADS, KPT = PROBE_KPT;
constexpr uint32_t T = THREADS * KPT;
using E = std::conditional<PROBE_ELEM == 2, uint16_t, uint32_t>::type;

template <int MAP>
__global__ __launch_bounds__(THREADS) void abut(const E* __restrict__ in, E* __restrict__ out,
                                                const uint32_t* __restrict__ off, const uint16_t* __restrict__ lstart,
                                                uint32_t nT) {
  __shared__ uint32_t s_off[256];
  __shared__ uint32_t s_ls[257];  // (T itself may not fit 16 bits)
  const uint32_t b = blockIdx.x;
  // MAP 0: round-robin; 1: one contiguous range per XCD; B>1: blocks of B
  // consecutive tiles per XCD, blocks round-robin over XCDs (thrs_pass_xb)
  uint32_t tile;
  if constexpr (MAP == 0) tile = b;
  else if constexpr (MAP == 1) tile = (b % 8) * (nT / 8) + b / 8;
  else tile = ((b / 8) / MAP * 8 + (b % 8)) * MAP + (b / 8) % MAP;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid < 256) {
    s_off[tid] = off[(uint64_t)tile * 256 + tid];
    s_ls[tid] = lstart[(uint64_t)tile * 256 + tid];
  }
  if (tid == 0) s_ls[256] = T;
  E k[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) k[j] = in[(uint64_t)tile * T + w * 64 * KPT + j * 64 + lane];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint32_t i = j * THREADS + tid;
    // digit of sorted position i: binary search over the local starts
    uint32_t lo = 0, hi = 256;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const uint32_t mid = (lo + hi) >> 1;
      if (s_ls[mid] <= i) lo = mid; else hi = mid;
    }
    out[s_off[lo] + (i - s_ls[lo])] = (E)(k[j] + 1);
  }
}

template <int MAP>
double run(const E* in, E* out, const uint32_t* off, const uint16_t* ls, uint32_t nT, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(abut<MAP>, dim3(nT), dim3(THREADS), 0, 0, in, out, off, ls, nT);
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(abut<MAP>, dim3(nT), dim3(THREADS), 0, 0, in, out, off, ls, nT);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main() {
  const uint32_t n = 1u << 30, nT = n / T;
  // per-tile digit counts of uniformly random digits (splitmix64)
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
  std::vector<uint64_t> tot(256, 0);
  for (uint32_t t = 0; t < nT; ++t)
    for (int d = 0; d < 256; ++d) tot[d] += cnt[(size_t)t * 256 + d];
  std::vector<uint64_t> base(256, 0);
  for (int d = 1; d < 256; ++d) base[d] = base[d - 1] + tot[d - 1];
  std::vector<uint32_t> off((size_t)nT * 256);
  std::vector<uint16_t> ls((size_t)nT * 256);
  std::vector<uint64_t> run_(base);
  for (uint32_t t = 0; t < nT; ++t) {
    uint32_t l = 0;
    for (int d = 0; d < 256; ++d) {
      off[(size_t)t * 256 + d] = (uint32_t)run_[d];
      ls[(size_t)t * 256 + d] = (uint16_t)l;
      run_[d] += cnt[(size_t)t * 256 + d];
      l += cnt[(size_t)t * 256 + d];
    }
  }
  E *in, *out;
  uint32_t* doff;
  uint16_t* dls;
  CK(hipMalloc(&in, (size_t)n * sizeof(E)));
  CK(hipMalloc(&out, (size_t)n * sizeof(E)));
  CK(hipMalloc(&doff, off.size() * 4));
  CK(hipMalloc(&dls, ls.size() * 2));
  CK(hipMemset(in, 1, (size_t)n * sizeof(E)));
  CK(hipMemcpy(doff, off.data(), off.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dls, ls.data(), ls.size() * 2, hipMemcpyHostToDevice));
  const double bytes = 2.0 * n * sizeof(E);
  printf("{\"tile\": %u, \"elem\": %d}\n", T, (int)sizeof(E));
  for (int rep = 0; rep < 2; ++rep) {
    const double r[5] = {run<0>(in, out, doff, dls, nT, 10), run<1>(in, out, doff, dls, nT, 10),
                         run<4>(in, out, doff, dls, nT, 10), run<8>(in, out, doff, dls, nT, 10),
                         run<32>(in, out, doff, dls, nT, 10)};
    const char* nm[5] = {"rr", "xcd_contiguous", "xcd_blocks4", "xcd_blocks8", "xcd_blocks32"};
    for (int i = 0; i < 5; ++i) printf("{\"map\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", nm[i], r[i], bytes / r[i] / 1e6);
    fflush(stdout);
  }
  return 0;
}
