// thrs_kernels.hpp -- gfx950 (CDNA4, wave64) LSD radix sort kernels.
//
// Replaces the reference's hipRTC string kernels (tinyhipradixsort.hpp:46-476,
// == kernel.cu) with an ahead-of-time-compiled Onesweep-style design:
//
//   thrs_hist   one read of the keys builds the 256-bin digit histogram of
//               EVERY pass at once (digit histograms are order-invariant, so
//               pass p+1 never has to re-read keys to count; the reference
//               re-counts per pass in blockCount, kernel.cu:73-103).
//   thrs_scan   exclusive scan of each pass's 256 global counts -> digit bases.
//   thrs_pass   one launch per 8-bit digit: load a tile, stable rank in
//               registers (wave64 ballot match + per-wave LDS counters),
//               decoupled look-back over per-(tile,digit) status words for the
//               global offset (dynamic tile ids, so no dispatch-order
//               assumption -- the reference's g_iterator CAS chain,
//               kernel.cu:165-182, relies on in-order dispatch), LDS-staged
//               tile in sorted order, coalesced write-out.  Keys and values are
//               read once and written once per pass (the reference re-reads
//               keys in blockCount and re-gathers them in reorder).
//
// Everything is integer arithmetic on the key's bit image; floats go through
// getKeyBits (kernel.cu:46-69) restated on bits, so denormals are never
// flushed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace thrs_dev {

constexpr int kRadixBits = 8;
constexpr int kBins = 256;
constexpr int kThreads = 256;  // 4 waves of 64
constexpr int kWaves = kThreads / 64;

// ---------------------------------------------------------------- key traits
// getKeyBits (kernel.cu:46-61 / fpKey.hpp:15-38) as bit operations.
template <int KT> struct KeyTraits;
template <> struct KeyTraits<0> {  // U32
  using U = uint32_t;
  __device__ static inline U bits(U x) { return x; }
};
template <> struct KeyTraits<1> {  // U64
  using U = uint64_t;
  __device__ static inline U bits(U x) { return x; }
};
template <> struct KeyTraits<2> {  // F32: -0 -> +0 (on bits), then sign flip
  using U = uint32_t;
  __device__ static inline U bits(U b) {
    b = (b & 0x7FFFFFFFu) ? b : 0u;
    return b ^ ((uint32_t)((int32_t)b >> 31) | 0x80000000u);
  }
};
template <> struct KeyTraits<3> {  // F64
  using U = uint64_t;
  __device__ static inline U bits(U b) {
    b = (b & 0x7FFFFFFFFFFFFFFFull) ? b : 0ull;
    return b ^ ((uint64_t)((int64_t)b >> 63) | 0x8000000000000000ull);
  }
};

// value payloads: 4, 8 or 16 bytes moved as opaque words
template <int VB> struct ValueWord;
template <> struct ValueWord<4> { using T = uint32_t; };
template <> struct ValueWord<8> { using T = uint64_t; };
template <> struct ValueWord<16> { using T = uint4; };
template <> struct ValueWord<0> { using T = uint32_t; };  // unused

// ------------------------------------------------------------ status words
// One word per (tile, digit).  0 = not yet published.
//   32-bit form (n < 2^31): aggregate = count+1 (bit31 clear, nonzero);
//                           inclusive prefix = 0x80000000 | prefix.
//   64-bit form:            aggregate = 1<<62 | count; prefix = 1<<63 | prefix.
template <typename ST> struct Status;
template <> struct Status<uint32_t> {
  __device__ static inline uint32_t agg(uint32_t c) { return c + 1u; }
  __device__ static inline uint32_t pre(uint32_t p) { return 0x80000000u | p; }
  __device__ static inline bool is_pre(uint32_t w) { return (w & 0x80000000u) != 0; }
  __device__ static inline uint32_t val(uint32_t w) { return is_pre(w) ? (w & 0x7FFFFFFFu) : (w - 1u); }
};
template <> struct Status<uint64_t> {
  __device__ static inline uint64_t agg(uint32_t c) { return (1ull << 62) | c; }
  __device__ static inline uint64_t pre(uint32_t p) { return (1ull << 63) | p; }
  __device__ static inline bool is_pre(uint64_t w) { return (w >> 63) != 0; }
  __device__ static inline uint32_t val(uint64_t w) { return (uint32_t)w; }
};

template <typename T>
__device__ __forceinline__ void store_agent(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T load_agent(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------ wave helpers
__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// Peers of this lane's 8-bit digit in the wave: 8 ballots, each folded into
// the 64-bit mask with one v_bitop3 per half (gfx950).
__device__ __forceinline__ void match_digit(uint32_t d, uint32_t& mlo, uint32_t& mhi) {
  mlo = ~0u;
  mhi = ~0u;
#pragma unroll
  for (int b = 0; b < kRadixBits; ++b) {
    const int t = __builtin_amdgcn_sbfe((int)d, b, 1);  // 0 or -1
    const uint64_t bb = __ballot(t != 0);
    mlo &= ~((uint32_t)bb ^ (uint32_t)t);
    mhi &= ~((uint32_t)(bb >> 32) ^ (uint32_t)t);
  }
}

// Inclusive scan over the 64 lanes of a wave.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, uint32_t lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    uint32_t y = __shfl_up(x, off, 64);
    if (lane >= (uint32_t)off) x += y;
  }
  return x;
}

// Exclusive scan of one value per thread over a 256-thread block.
// s_w: 4 words of LDS scratch.  Leaves *total = block sum.  Two barriers.
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* s_w, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan(v, lane);
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  const uint32_t w0 = s_w[0], w1 = s_w[1], w2 = s_w[2], w3 = s_w[3];
  uint32_t pre = (w > 0 ? w0 : 0u) + (w > 1 ? w1 : 0u) + (w > 2 ? w2 : 0u);
  *total = w0 + w1 + w2 + w3;
  __syncthreads();
  return pre + inc - v;
}

// ================================================================ histogram
// Histograms of up to NP_MAX digits of every key in one read.
//   hist[p*256 + d] += #keys with digit d at bit startBits + 8p.
// LDS: per-wave private copies [wave][p][256] to spread LDS atomics; merged
// with one device-scope atomic per (p, bin) per workgroup.
template <int KT>
__global__ __launch_bounds__(kThreads) void thrs_hist(const typename KeyTraits<KT>::U* __restrict__ keys,
                                                      uint32_t n, typename KeyTraits<KT>::U orderMask,
                                                      int startBits, int nPass, int vec, uint32_t* __restrict__ hist) {
  using U = typename KeyTraits<KT>::U;
  constexpr int NP_MAX = sizeof(U);
  extern __shared__ __attribute__((aligned(16))) uint32_t s_hist[];  // [kWaves][NP_MAX][256]
  const uint32_t tid = threadIdx.x, w = tid >> 6;
  for (uint32_t i = tid; i < (uint32_t)(kWaves * NP_MAX * kBins); i += kThreads) s_hist[i] = 0;
  __syncthreads();
  uint32_t* my = s_hist + w * NP_MAX * kBins;

  auto count = [&](U k) {
    const U b = KeyTraits<KT>::bits(k) ^ orderMask;
#pragma unroll
    for (int p = 0; p < NP_MAX; ++p) {
      if (p < nPass) {
        const uint32_t d = (uint32_t)(b >> (startBits + 8 * p)) & 0xFFu;
        atomicAdd(&my[p * kBins + d], 1u);
      }
    }
  };

  const uint64_t gstride = (uint64_t)gridDim.x * kThreads;
  const uint64_t gtid = (uint64_t)blockIdx.x * kThreads + tid;
  uint64_t tailStart = 0;
  if (vec) {  // 16-byte loads; keys base is 16-B aligned (checked on host)
    constexpr int PER = 16 / sizeof(U);
    const uint64_t nv = n / PER;
    const uint4* kv = reinterpret_cast<const uint4*>(keys);
    for (uint64_t i = gtid; i < nv; i += gstride) {
      uint4 q = kv[i];
      if constexpr (sizeof(U) == 4) {
        count(q.x); count(q.y); count(q.z); count(q.w);
      } else {
        count(((uint64_t)q.y << 32) | q.x);
        count(((uint64_t)q.w << 32) | q.z);
      }
    }
    tailStart = nv * PER;
  }
  for (uint64_t i = tailStart + gtid; i < n; i += gstride) count(keys[i]);
  __syncthreads();
  for (uint32_t i = tid; i < (uint32_t)(nPass * kBins); i += kThreads) {
    uint32_t s = 0;
#pragma unroll
    for (int ww = 0; ww < kWaves; ++ww) s += s_hist[ww * NP_MAX * kBins + i];
    if (s) atomicAdd(&hist[i], s);
  }
}

// exclusive scan of each pass's histogram -> global digit bases
__global__ __launch_bounds__(kThreads) void thrs_scan(const uint32_t* __restrict__ hist, uint32_t* __restrict__ base,
                                                      int nPass) {
  __shared__ uint32_t s_w[4];
  for (int p = 0; p < nPass; ++p) {
    uint32_t total;
    const uint32_t v = hist[p * kBins + threadIdx.x];
    base[p * kBins + threadIdx.x] = block_excl_scan256(v, s_w, &total);
  }
}

// ================================================================ one pass
// Tile = 256 threads x KPT keys.  Wave w owns the contiguous chunk
// [w*64*KPT, (w+1)*64*KPT) of the tile; item j of that chunk is 64
// consecutive keys, one per lane, so (wave, item, lane) order is input order
// and ranking item by item is stable.
//
// LDS (dynamic, 16-B aligned):
//   stage_k [T]   keys in tile-sorted order
//   stage_v [T]   values in tile-sorted order (pairs only)
//   s_cnt   [4][256]  per-wave running digit counts -> per-wave offsets
//   s_gofs  [256]     global dst of sorted slot 0 for digit d = base + excl - localStart
//   s_misc  [8]       tile id, scan scratch
template <int KT, int VB, int KPT, typename ST>
__global__ __launch_bounds__(kThreads) void thrs_pass(
    const typename KeyTraits<KT>::U* __restrict__ keysIn, typename KeyTraits<KT>::U* __restrict__ keysOut,
    const typename ValueWord<VB>::T* __restrict__ valsIn, typename ValueWord<VB>::T* __restrict__ valsOut,
    uint32_t n, typename KeyTraits<KT>::U orderMask, int shift, const uint32_t* __restrict__ digitBase,
    ST* __restrict__ status, ST* __restrict__ statusNext, uint32_t* __restrict__ tileCounter,
    uint32_t* __restrict__ errFlag) {
  using U = typename KeyTraits<KT>::U;
  using VW = typename ValueWord<VB>::T;
  constexpr uint32_t T = kThreads * KPT;
  constexpr uint32_t CHUNK = 64 * KPT;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  U* stage_k = reinterpret_cast<U*>(smem);
  VW* stage_v = reinterpret_cast<VW*>(smem + T * sizeof(U));
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(smem + T * sizeof(U) + (VB ? T * VB : 0));
  uint32_t* s_gofs = s_cnt + kWaves * kBins;
  uint32_t* s_misc = s_gofs + kBins;

  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;

  if (tid == 0) s_misc[0] = atomicAdd(tileCounter, 1u);
#pragma unroll
  for (int i = 0; i < kWaves; ++i) s_cnt[i * kBins + tid] = 0;
  __syncthreads();
  const uint32_t tile = s_misc[0];
  const uint64_t tileBase = (uint64_t)tile * T;
  const uint32_t valid = (uint32_t)min((uint64_t)T, (uint64_t)n - tileBase);
  const uint64_t chunkBase = tileBase + w * CHUNK;

  // ---- load keys (striped per wave: item j = 64 consecutive keys)
  U k[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint32_t local = w * CHUNK + j * 64 + lane;
    k[j] = (local < valid) ? keysIn[chunkBase + j * 64 + lane] : (U)0;
  }
  const uint32_t myBase = digitBase[tid];  // global base of digit `tid` (used after look-back)

  // ---- stable rank inside the wave chunk
  uint32_t pk[KPT];  // (rank << 8) | digit
  uint32_t* cnt = s_cnt + w * kBins;
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint32_t local = w * CHUNK + j * 64 + lane;
    uint32_t d = (uint32_t)((KeyTraits<KT>::bits(k[j]) ^ orderMask) >> shift) & 0xFFu;
    d = (local < valid) ? d : 0xFFu;  // padding ranks after every real key
    uint32_t mlo, mhi;
    match_digit(d, mlo, mhi);
    const uint32_t c = cnt[d];
    const uint32_t r = c + __builtin_amdgcn_mbcnt_hi(mhi, __builtin_amdgcn_mbcnt_lo(mlo, 0u));
    cnt[d] = c + __builtin_popcount(mlo) + __builtin_popcount(mhi);
    pk[j] = (r << 8) | d;
  }
  __syncthreads();

  // ---- per digit (thread tid == digit d): tile count, per-wave offsets
  const uint32_t d = tid;
  const uint32_t c0 = s_cnt[0 * kBins + d], c1 = s_cnt[1 * kBins + d];
  const uint32_t c2 = s_cnt[2 * kBins + d], c3 = s_cnt[3 * kBins + d];
  const uint32_t tot = c0 + c1 + c2 + c3;
  const uint32_t realTot = (d == 255u) ? tot - (T - valid) : tot;
  ST* myStatus = status + (uint64_t)tile * kBins + d;
  if (tile != 0) store_agent(myStatus, Status<ST>::agg(realTot));
  else store_agent(myStatus, Status<ST>::pre(realTot));

  uint32_t blockTotal;
  const uint32_t localStart = block_excl_scan256(tot, s_misc + 4, &blockTotal);
  s_cnt[0 * kBins + d] = localStart;
  s_cnt[1 * kBins + d] = localStart + c0;
  s_cnt[2 * kBins + d] = localStart + c0 + c1;
  s_cnt[3 * kBins + d] = localStart + c0 + c1 + c2;

  // ---- decoupled look-back for digit d
  uint32_t excl = 0;
  if (tile != 0) {
    int64_t j = (int64_t)tile - 1;
    uint32_t spins = 0;
    while (true) {
      const ST s = load_agent(status + (uint64_t)j * kBins + d);
      if (s == 0) {
        if (++spins > (1u << 24)) {  // bounded spin: never hang the GPU
          atomicOr(errFlag, 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      excl += Status<ST>::val(s);
      if (Status<ST>::is_pre(s)) break;
      --j;
    }
    store_agent(myStatus, Status<ST>::pre(excl + realTot));
  }
  s_gofs[d] = myBase + excl - localStart;
  if (statusNext) statusNext[(uint64_t)tile * kBins + d] = 0;  // ready for the next pass
  __syncthreads();

  // ---- scatter into the LDS tile in sorted order
  const uint32_t* offs = s_cnt + w * kBins;
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint32_t dd = pk[j] & 0xFFu;
    const uint32_t p = offs[dd] + (pk[j] >> 8);
    stage_k[p] = k[j];
    pk[j] = p;
  }
  if constexpr (VB != 0) {
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      const uint32_t local = w * CHUNK + j * 64 + lane;
      VW v;
      if (local < valid) v = valsIn[chunkBase + j * 64 + lane];
      else v = VW{};
      stage_v[pk[j]] = v;
    }
  }
  __syncthreads();

  // ---- coalesced write-out: sorted slot i -> s_gofs[digit] + i
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint32_t i = j * kThreads + tid;
    if (i < valid) {
      const U key = stage_k[i];
      const uint32_t dd = (uint32_t)((KeyTraits<KT>::bits(key) ^ orderMask) >> shift) & 0xFFu;
      const uint32_t dst = s_gofs[dd] + i;
      keysOut[dst] = key;
      if constexpr (VB != 0) valsOut[dst] = stage_v[i];
    }
  }
}

}  // namespace thrs_dev
