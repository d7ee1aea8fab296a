// thrs_testutil.hip -- libthrs_testutil.so: GPU-side input generators and
// size-independent property checkers for tests and bench.py.  NOT part of
// the sort path; the sort never calls into it.
//
// Generators reproduce the reference's inputs bit-exactly: splitmix64 with
// state 0 (unittest.cpp:24-35) is counter-based, so draw i (1-based) is
// mix(0x9e3779b97f4a7c15 * i), and randomizeValues (unittest.cpp:96-116)
// masks it per key type.  Checkers let tests verify a 2^30-key sort without a
// CPU copy: sortedness of getKeyBits^ORDER_MASK, a multiset fingerprint, and
// for pairs whose values are the input index: gather consistency + stability.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "thrs/thrs_capi.h"
#include "thrs_kernels.hpp"

using namespace thrs_dev;

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t draw(uint64_t state, uint64_t i1) { return mix64(state + 0x9e3779b97f4a7c15ull * i1); }

__global__ void k_fill(int keyType, void* out, uint64_t n, uint64_t start, uint64_t state) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = draw(state, start + i + 1);
    switch (keyType) {
      case THRS_KEY_U32: ((uint32_t*)out)[i] = (uint32_t)r; break;
      case THRS_KEY_F32: ((uint32_t*)out)[i] = (uint32_t)(r & 0xFF7FFFFFull); break;
      case THRS_KEY_U64: ((uint64_t*)out)[i] = r; break;
      case THRS_KEY_F64: ((uint64_t*)out)[i] = r & 0xFFEFFFFFFFFFFFFFull; break;
      default: break;
    }
  }
}

// raw key whose getKeyBits image is y (inverse of KeyTraits::bits)
__device__ __forceinline__ uint64_t unbits(int keyType, uint64_t y) {
  switch (keyType) {
    case THRS_KEY_F32: return (y & 0x80000000ull) ? (y ^ 0x80000000ull) : (~y & 0xFFFFFFFFull);
    case THRS_KEY_F64: return (y >> 63) ? (y ^ 0x8000000000000000ull) : ~y;
    default: return y;
  }
}

// Non-uniform key distributions (bench.py workloads c2_*, low-entropy tests):
//   1 sorted   image of key i in [floor(i*2^W/n), floor((i+1)*2^W/n)): a
//              stratified sorted uniform sample (the digit runs of sorting
//              uniform keys, which is what a sort of already-sorted data sees)
//   2 reverse  the same, descending
//   3 extreme  all zero except key n/3 = 1 and key 2n/3 = 42
//              (SortKeys.extremeCase, unittest.cpp:191-225)
//   4 fewuniq  16 distinct uniform keys, chosen per key by the stream
__global__ void k_fill_dist(int keyType, void* out, uint64_t n, uint64_t start, uint64_t state, int dist) {
  const bool k32 = keyType == THRS_KEY_U32 || keyType == THRS_KEY_F32;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = draw(state, start + i + 1);
    uint64_t raw = 0;
    if (dist == 1 || dist == 2) {
      const uint64_t j = dist == 1 ? i : n - 1 - i;
      uint64_t y;
      if (k32) {
        const uint64_t lo = (j << 32) / n, hi = ((j + 1) << 32) / n;
        y = lo + (hi > lo ? r % (hi - lo) : 0);
      } else {
        const uint64_t step = ~0ull / n;
        y = j * step + (step ? r % step : 0);
      }
      raw = unbits(keyType, y);
    } else if (dist == 3) {
      raw = i == n / 3 ? 1 : (i == 2 * n / 3 ? 42 : 0);
    } else if (dist == 4) {
      raw = draw(state, 1000003ull + (r & 15));
      if (keyType == THRS_KEY_F32) raw &= 0xFF7FFFFFull;
      if (keyType == THRS_KEY_F64) raw &= 0xFFEFFFFFFFFFFFFFull;
    } else {
      raw = keyType == THRS_KEY_F32 ? (r & 0xFF7FFFFFull) : keyType == THRS_KEY_F64 ? (r & 0xFFEFFFFFFFFFFFFFull) : r;
    }
    if (k32) ((uint32_t*)out)[i] = (uint32_t)raw;
    else ((uint64_t*)out)[i] = raw;
  }
}

// values = input index (sequentialValues / ValueType(i), unittest.cpp:118-125, 394-397);
// u128 = {i, i} as in K64V128 (unittest.cpp:471-481).
__global__ void k_iota(int valueBytes, void* out, uint64_t n, uint64_t start) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t v = start + i;
    if (valueBytes == 4) ((uint32_t*)out)[i] = (uint32_t)v;
    else if (valueBytes == 8) ((uint64_t*)out)[i] = v;
    else { ((uint64_t*)out)[2 * i] = v; ((uint64_t*)out)[2 * i + 1] = v; }
  }
}

__device__ __forceinline__ uint64_t tkey(int keyType, const void* keys, uint64_t i, int desc) {
  switch (keyType) {
    case THRS_KEY_U32: return KeyTraits<0>::bits(((const uint32_t*)keys)[i]) ^ (desc ? 0xFFFFFFFFull : 0ull);
    case THRS_KEY_U64: return KeyTraits<1>::bits(((const uint64_t*)keys)[i]) ^ (desc ? ~0ull : 0ull);
    case THRS_KEY_F32: return KeyTraits<2>::bits(((const uint32_t*)keys)[i]) ^ (desc ? 0xFFFFFFFFull : 0ull);
    default: return KeyTraits<3>::bits(((const uint64_t*)keys)[i]) ^ (desc ? ~0ull : 0ull);
  }
}
__device__ __forceinline__ uint64_t rawkey(int keyType, const void* keys, uint64_t i) {
  return (keyType == THRS_KEY_U32 || keyType == THRS_KEY_F32) ? ((const uint32_t*)keys)[i] : ((const uint64_t*)keys)[i];
}
// window [start,end) of the transformed key, as compared by an LSD sort of
// those digits: bits at or past the key width read as zero.
__device__ __forceinline__ uint64_t window(uint64_t t, int width, int s, int e) {
  if (s >= width) return 0;
  const int hi = e < width ? e : width;
  const int len = hi - s;
  const uint64_t m = len >= 64 ? ~0ull : ((1ull << len) - 1);
  return (t >> s) & m;
}

// out[0] += #i with window(key[i]) > window(key[i+1])
__global__ void k_sorted(int keyType, int desc, const void* keys, uint64_t n, int s, int e, unsigned long long* out) {
  const int width = (keyType == THRS_KEY_U32 || keyType == THRS_KEY_F32) ? 32 : 64;
  unsigned long long bad = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += (uint64_t)gridDim.x * blockDim.x)
    bad += window(tkey(keyType, keys, i, desc), width, s, e) > window(tkey(keyType, keys, i + 1, desc), width, s, e);
  if (bad) atomicAdd(out, bad);
}

// multiset fingerprint of raw key bits: out[0] += sum mix(k), out[1] ^= xor mix(k ^ c)
__global__ void k_fingerprint(int keyType, const void* keys, uint64_t n, unsigned long long* out) {
  unsigned long long s = 0, x = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = rawkey(keyType, keys, i);
    s += mix64(k);
    x ^= mix64(k ^ 0x5bd1e9955bd1e995ull);
  }
  atomicAdd(&out[0], s);
  atomicXor(&out[1], x);
}

// Pairs whose values were the input index: for every output slot i,
//  out[0] += keysOut[i] != keysIn[idx[i]]                       (gather consistency)
//  out[1] += window equal with neighbour but idx not increasing  (stability)
//  out[2] += sum of idx, out[3] ^= xor of mix(idx)               (permutation fingerprint)
//  out[4] += u128 halves disagree
__global__ void k_pairs(int keyType, int desc, int valueBytes, const void* keysIn, const void* keysOut,
                        const void* vals, uint64_t n, int s, int e, unsigned long long* out) {
  const int width = (keyType == THRS_KEY_U32 || keyType == THRS_KEY_F32) ? 32 : 64;
  unsigned long long bad = 0, unstable = 0, sum = 0, x = 0, halves = 0;
  auto idx = [&](uint64_t i) -> uint64_t {
    if (valueBytes == 4) return ((const uint32_t*)vals)[i];
    if (valueBytes == 8) return ((const uint64_t*)vals)[i];
    return ((const uint64_t*)vals)[2 * i];
  };
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t v = idx(i);
    if (valueBytes == 16) halves += ((const uint64_t*)vals)[2 * i + 1] != v;
    bad += (v >= n) || (rawkey(keyType, keysOut, i) != rawkey(keyType, keysIn, v));
    sum += v;
    x ^= mix64(v);
    if (i + 1 < n) {
      const uint64_t a = window(tkey(keyType, keysOut, i, desc), width, s, e);
      const uint64_t b = window(tkey(keyType, keysOut, i + 1, desc), width, s, e);
      unstable += (a == b) && !(idx(i + 1) > v);
    }
  }
  if (bad) atomicAdd(&out[0], bad);
  if (unstable) atomicAdd(&out[1], unstable);
  atomicAdd(&out[2], sum);
  atomicXor(&out[3], x);
  if (halves) atomicAdd(&out[4], halves);
}

// Calibration copies for rocprofv3 byte counters (FETCH_SIZE/WRITE_SIZE are
// only calibrated for 16-B streaming accesses on gfx950): known byte counts at
// 4-B and 16-B per lane.
__global__ void k_copy_u32(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}
__global__ void k_copy_u128(uint4* __restrict__ dst, const uint4* __restrict__ src, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// The rank's lane-order property under PARTIAL exec masks (thrs_probe_lds_order
// checks fully active waves only, which is all the product kernels issue:
// their rank loops run whole waves, padding items included).  Same digit
// patterns, with 4 lane subsets active: odd lanes, lanes < 40, a random mask,
// lanes not divisible by 3.  *bad counts disagreeing active lanes.
__global__ __launch_bounds__(256) void k_probe_partial(uint32_t* bad, int iters) {
  __shared__ uint32_t cnt[4][kBins];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t b = 0;
  uint64_t x = (blockIdx.x * 256ull + threadIdx.x + 1) * 0x9E3779B97F4A7C15ull;
  for (int it = 0; it < iters; ++it) {
    for (uint32_t i = lane; i < (uint32_t)kBins; i += 64) cnt[w][i] = (uint32_t)it;
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    uint32_t d = (uint32_t)(x >> 24) & 0xFFu;
    const int mode = it & 3, pm = (it >> 2) & 3;
    if (mode == 1) d &= 0x3u;
    if (mode == 2) d = 0x5Au;
    if (mode == 3) d &= 0x1Fu;
    const bool act = pm == 0 ? (lane & 1u) != 0 : pm == 1 ? lane < 40u : pm == 2 ? ((x >> 40) & 1u) != 0 : (lane % 3u) != 0;
    if (act) {
      uint32_t mlo, mhi;
      match_digit(d, mlo, mhi);
      const uint64_t ex = __ballot(1);  // inactive lanes read as digit 0 in the ballots: mask them out
      mlo &= (uint32_t)ex;
      mhi &= (uint32_t)(ex >> 32);
      const uint32_t want = (uint32_t)it + __builtin_amdgcn_mbcnt_hi(mhi, __builtin_amdgcn_mbcnt_lo(mlo, 0u));
      const uint32_t got = __hip_atomic_fetch_add(&cnt[w][d], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      b += got != want;
    }
  }
  if (b) atomicAdd(bad, b);
}

inline int grid_for(uint64_t n) {
  uint64_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  return g ? (int)g : 1;
}
inline int ok(hipError_t e) { return e == hipSuccess ? THRS_SUCCESS : THRS_ERROR_HIP; }

}  // namespace

#define THRS_API __attribute__((visibility("default")))
extern "C" {

THRS_API int thrsu_fill_keys(int keyType, void* out, uint64_t n, uint64_t start, uint64_t state, hipStream_t stream) {
  if (!n) return THRS_SUCCESS;
  hipLaunchKernelGGL(k_fill, dim3(grid_for(n)), dim3(256), 0, stream, keyType, out, n, start, state);
  return ok(hipGetLastError());
}

THRS_API int thrsu_fill_dist(int keyType, void* out, uint64_t n, uint64_t start, uint64_t state, int dist,
                             hipStream_t stream) {
  if (!n) return THRS_SUCCESS;
  if (dist < 0 || dist > 4) return THRS_ERROR_INVALID_VALUE;
  hipLaunchKernelGGL(k_fill_dist, dim3(grid_for(n)), dim3(256), 0, stream, keyType, out, n, start, state, dist);
  return ok(hipGetLastError());
}

THRS_API int thrsu_iota(int valueBytes, void* out, uint64_t n, uint64_t start, hipStream_t stream) {
  if (!n) return THRS_SUCCESS;
  hipLaunchKernelGGL(k_iota, dim3(grid_for(n)), dim3(256), 0, stream, valueBytes, out, n, start);
  return ok(hipGetLastError());
}

THRS_API int thrsu_copy(void* dst, const void* src, uint64_t bytes, int width16, hipStream_t stream) {
  if (width16)
    hipLaunchKernelGGL(k_copy_u128, dim3(4096), dim3(256), 0, stream, (uint4*)dst, (const uint4*)src, bytes / 16);
  else
    hipLaunchKernelGGL(k_copy_u32, dim3(4096), dim3(256), 0, stream, (uint32_t*)dst, (const uint32_t*)src, bytes / 4);
  return ok(hipGetLastError());
}

// result[0] = number of out-of-order neighbours (synchronising)
THRS_API int thrsu_check_sorted(int keyType, int desc, const void* keys, uint64_t n, int startBits, int endBits,
                       unsigned long long* result, hipStream_t stream) {
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, 8) != hipSuccess) return THRS_ERROR_HIP;
  (void)hipMemsetAsync(d, 0, 8, stream);
  if (n > 1) hipLaunchKernelGGL(k_sorted, dim3(grid_for(n)), dim3(256), 0, stream, keyType, desc, keys, n, startBits, endBits, d);
  (void)hipMemcpyAsync(result, d, 8, hipMemcpyDeviceToHost, stream);
  int rc = ok(hipStreamSynchronize(stream));
  (void)hipFree(d);
  return rc;
}

THRS_API int thrsu_fingerprint(int keyType, const void* keys, uint64_t n, unsigned long long* result2, hipStream_t stream) {
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, 16) != hipSuccess) return THRS_ERROR_HIP;
  (void)hipMemsetAsync(d, 0, 16, stream);
  if (n) hipLaunchKernelGGL(k_fingerprint, dim3(grid_for(n)), dim3(256), 0, stream, keyType, keys, n, d);
  (void)hipMemcpyAsync(result2, d, 16, hipMemcpyDeviceToHost, stream);
  int rc = ok(hipStreamSynchronize(stream));
  (void)hipFree(d);
  return rc;
}

THRS_API int thrsu_check_pairs(int keyType, int desc, int valueBytes, const void* keysIn, const void* keysOut, const void* vals,
                      uint64_t n, int startBits, int endBits, unsigned long long* result5, hipStream_t stream) {
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, 40) != hipSuccess) return THRS_ERROR_HIP;
  (void)hipMemsetAsync(d, 0, 40, stream);
  if (n)
    hipLaunchKernelGGL(k_pairs, dim3(grid_for(n)), dim3(256), 0, stream, keyType, desc, valueBytes, keysIn, keysOut,
                       vals, n, startBits, endBits, d);
  (void)hipMemcpyAsync(result5, d, 40, hipMemcpyDeviceToHost, stream);
  int rc = ok(hipStreamSynchronize(stream));
  (void)hipFree(d);
  return rc;
}

// disagreeing lanes of the partial-mask lane-order probe (synchronising)
THRS_API int thrsu_probe_lds_order_partial(int iters, unsigned int* bad) {
  uint32_t* d = nullptr;
  if (hipMalloc(&d, 4) != hipSuccess) return THRS_ERROR_HIP;
  (void)hipMemset(d, 0, 4);
  hipLaunchKernelGGL(k_probe_partial, dim3(256), dim3(256), 0, 0, d, iters);
  int rc = ok(hipGetLastError());
  if (rc == THRS_SUCCESS) rc = ok(hipMemcpy(bad, d, 4, hipMemcpyDeviceToHost));
  (void)hipFree(d);
  return rc;
}

}  // extern "C"
