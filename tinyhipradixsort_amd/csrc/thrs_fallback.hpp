// thrs_fallback.hpp -- the bucket path's per-bucket fallback (gfx950).
//
// A BIG chunk is a bucket (the window's top 16 bits) holding more keys than
// its local sort's capacity -- skewed or low-cardinality input.  After the two
// top-digit passes every bucket is one contiguous range, so a big chunk can
// be sorted on its own: the plan lists the big chunks (bigB), the local sort
// skips them, and only they take device-wide stable LSD passes on the
// window's low digits -- each big chunk one segment with its own digit bases
// and look-back chain, exactly as the reference's pass loop
// (tinyhipradixsort.hpp:862-930) restricted to that range.  All launches are
// gated on meta[kMetaFallback] (written by the plan): no host
// synchronisation, and ~5 us per launch when nothing overflowed.
//
//   (plan)          the plan's last workgroup (thrs_plan_rows; thrs_big_plan
//                   after thrs_plan's multi-bucket chunks): prefix of the big
//                   chunks' sizes (bigPos, positions in the concatenation of
//                   the big chunks) and of their tile counts (bigTile); their
//                   digit counts zeroed as they are listed; the fallback's
//                   look-back tables zeroed by thrs_big_hist
//   thrs_big_hist   persistent: counts every low digit of every
//                   big chunk (bigHist[chunk][pass][256]); the last workgroup
//                   decides per low pass whether it RUNS -- a pass whose
//                   digit is one value in every big chunk is the identity
//                   (16 distinct keys: both low passes; counted as they
//                   happen: the count add that completes a bin to its
//                   chunk's size marks that chunk single) -- and the parity
//                   (which buffer holds the big chunks) of each running pass
//   thrs_pass_big   one launch per low digit: persistent, ticket tile claims
//                   over the concatenated big chunks' tiles (monotone tickets:
//                   a walk waits only on earlier tiles of its own chunk, held
//                   by running workgroups); the flat per-tile look-back (a
//                   chunk may be shorter than a look-back group), on tables of
//                   its own (rows: the n/TILE tiles + one partial tile per big
//                   chunk); ping-pong between the caller's buffer and the
//                   temporary buffer at the same positions
//   thrs_big_copy   an odd number of running passes leaves the big chunks in
//                   the temporary buffer: copied back
#pragma once
#include "thrs_hybrid.hpp"

namespace thrs_dev {
namespace {

constexpr int kBigPlanThreads = 1024;

// concatenated big-chunk position x -> the big chunk holding it (bigPos[M] =
// total): largest i with bigPos[i] <= x
__device__ __forceinline__ uint32_t big_find(const uint32_t* __restrict__ pos, uint32_t M, uint32_t x) {
  uint32_t lo = 0, hi = M;  // invariant: pos[lo] <= x < pos[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pos[mid] <= x) lo = mid;
    else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(kBigPlanThreads) void thrs_big_plan(
    const uint32_t* __restrict__ chunkOff, uint32_t* __restrict__ meta, const uint32_t* __restrict__ bigB,
    uint32_t* __restrict__ bigPos, uint32_t* __restrict__ bigTile, uint32_t tileKeys, uint4* __restrict__ bigHist,
    int nLow, uint4* __restrict__ tables, uint64_t tableWords) {
  if (meta[kMetaFallback] == 0) return;
  __shared__ uint32_t s_w[2][kBigPlanThreads / 64];
  const uint32_t M = meta[kMetaBigCount];
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t gstride = (uint64_t)gridDim.x * kBigPlanThreads, g0 = (uint64_t)blockIdx.x * kBigPlanThreads + tid;
  // zero the big chunks' digit counts (thrs_big_hist adds into them) and
  // the fallback's look-back tables
  const uint64_t histWords = (uint64_t)M * nLow * kBins / 4;
  for (uint64_t i = g0; i < histWords; i += gstride) bigHist[i] = make_uint4(0, 0, 0, 0);
  for (uint64_t i = g0; i < tableWords; i += gstride) tables[i] = make_uint4(0, 0, 0, 0);
  if (blockIdx.x != 0) return;
  const uint32_t per = (M + kBigPlanThreads - 1) / kBigPlanThreads;
  const uint32_t i0 = min(M, tid * per), i1 = min(M, i0 + per);
  auto size_of = [&](uint32_t i) { return chunkOff[bigB[i] + 1] - chunkOff[bigB[i]]; };
  auto tiles_of = [&](uint32_t sz) { return (sz + tileKeys - 1) / tileKeys; };
  uint32_t ks = 0, ts = 0;
  for (uint32_t i = i0; i < i1; ++i) {
    const uint32_t sz = size_of(i);
    ks += sz;
    ts += tiles_of(sz);
  }
  const uint32_t ik = wave_incl_scan(ks, lane), it = wave_incl_scan(ts, lane);
  if (lane == 63) {
    s_w[0][w] = ik;
    s_w[1][w] = it;
  }
  __syncthreads();
  uint32_t pk = ik - ks, pt = it - ts;
  for (uint32_t ww = 0; ww < w; ++ww) {
    pk += s_w[0][ww];
    pt += s_w[1][ww];
  }
  for (uint32_t i = i0; i < i1; ++i) {
    const uint32_t sz = size_of(i);
    bigPos[i] = pk;
    bigTile[i] = pt;
    pk += sz;
    pt += tiles_of(sz);
  }
  if (tid == kBigPlanThreads - 1) {
    bigPos[M] = pk;
    bigTile[M] = pt;
  }
}

// LDS digit counts of the low passes: [pass][256][kBigCopies]
constexpr int kBigCopies = 8;
constexpr int kBigUnroll = 8;
constexpr int kBigMaxLow = 6;  // 8-byte keys: 8 digits - the two top ones
constexpr size_t kBigHistLds = (size_t)kBigMaxLow * kBins * kBigCopies * 4;

template <int KT>
__global__ __launch_bounds__(kHistThreads) void thrs_big_hist(
    const typename KeyTraits<KT>::U* __restrict__ keys, KeyMap<typename KeyTraits<KT>::U> kmh, int startBits, int nLow,
    const uint32_t* __restrict__ chunkOff, uint32_t* __restrict__ meta, const uint32_t* __restrict__ bigB,
    const uint32_t* __restrict__ bigPos, uint32_t* __restrict__ bigHist, const SqueezeWords* __restrict__ sq,
    uint4* __restrict__ tables, uint64_t tableWords) {
  using U = typename KeyTraits<KT>::U;
  if (meta[kMetaFallback] == 0) return;
  {  // (plan_rows paths) the fallback passes' look-back tables: read from the first pass on
    const uint64_t gstride = (uint64_t)gridDim.x * kHistThreads, g0 = (uint64_t)blockIdx.x * kHistThreads + threadIdx.x;
    if (tables)
      for (uint64_t i = g0; i < tableWords; i += gstride) tables[i] = make_uint4(0, 0, 0, 0);
  }
  extern __shared__ __attribute__((aligned(16))) uint32_t s_h[];  // [nLow][256][kBigCopies]
  __shared__ uint32_t s_last;
  const uint32_t tid = threadIdx.x, G = gridDim.x;
  const uint32_t words = (uint32_t)nLow * kBins * kBigCopies;
  for (uint32_t i = tid; i < words; i += kHistThreads) s_h[i] = 0;
  __syncthreads();
  const uint32_t M = meta[kMetaBigCount], total = bigPos[M];
  const uint32_t len = (total + G - 1) / G;
  const uint32_t lo = min(total, blockIdx.x * len), hi = min(total, lo + len);
  uint32_t* my = s_h + (tid % kBigCopies);
  if (lo < hi) with_map<KT>(kmh, sq, [&](auto km) __attribute__((always_inline)) {
    for (uint32_t c = big_find(bigPos, M, lo); c < M && bigPos[c] < hi; ++c) {
      const uint32_t p0 = bigPos[c], a = max(lo, p0), b = min(hi, bigPos[c + 1]);
      const uint32_t start = chunkOff[bigB[c]], size = bigPos[c + 1] - p0;
      const U* src = keys + start;  // chunk position x - p0
      auto count = [&](U raw) {
        const U img = kimg<KT>(km, raw);
        for (int p = 0; p < nLow; ++p) {
          const uint32_t d = (uint32_t)(img >> (startBits + 8 * p)) & 0xFFu;
          __hip_atomic_fetch_add(&my[(p * kBins + d) * kBigCopies], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      };
      // kBigUnroll loads in flight per thread (one at a time leaves the
      // workgroup latency-bound: ~1/3 of the read bandwidth)
      uint32_t x = a + tid;
      for (; x + (kBigUnroll - 1) * kHistThreads < b; x += kBigUnroll * kHistThreads) {
        U r[kBigUnroll];
#pragma unroll
        for (int u = 0; u < kBigUnroll; ++u) r[u] = src[x - p0 + u * kHistThreads];
#pragma unroll
        for (int u = 0; u < kBigUnroll; ++u) count(r[u]);
      }
      for (; x < b; x += kHistThreads) count(src[x - p0]);
      __syncthreads();
      for (uint32_t i = tid; i < (uint32_t)nLow * kBins; i += kHistThreads) {
        uint32_t sum = 0;
#pragma unroll
        for (int k = 0; k < kBigCopies; ++k) {
          sum += s_h[i * kBigCopies + k];
          s_h[i * kBigCopies + k] = 0;
        }
        // the add that completes a bin to the chunk's size finds the chunk
        // single-valued on that digit (one such add per chunk and pass)
        if (sum && atomicAdd(&bigHist[(uint64_t)c * nLow * kBins + i], sum) + sum == size)
          atomicAdd(&meta[kMetaBigSingle + i / kBins], 1u);
      }
      __syncthreads();
    }
  });
  // the last workgroup to finish plans the low passes
  __threadfence();
  if (tid == 0) s_last = atomicAdd(&meta[kMetaBigDone], 1u) == G - 1;
  __syncthreads();
  if (!s_last || tid != 0) return;
  __threadfence();
  // pass p runs unless its digit is a single value in every big chunk
  {
    uint32_t par = 0;
    for (int p = 0; p < nLow; ++p) {
      const uint32_t run = load_agent(&meta[kMetaBigSingle + p]) < M;
      meta[kMetaBigPass + p] = run | (par << 1);
      par ^= run;
    }
    meta[kMetaBigCopy] = par;
  }
}

// One low pass over the big chunks.  src / dst by the pass's parity: the big
// chunks start in keys (parity 0) and move to tmpKeys, back, ...; look-back
// table = parity (the running passes alternate tables, and each clears its
// successor's rows as it goes, as the LSD passes do).
template <int KT, int VB, typename ST, bool ATOMIC_RANK>
__global__ __launch_bounds__((PassGeom<sizeof(typename KeyTraits<KT>::U), VB>::THREADS))
__attribute__((amdgpu_waves_per_eu(PassGeom<sizeof(typename KeyTraits<KT>::U), VB>::WPE))) void thrs_pass_big(
    typename KeyTraits<KT>::U* __restrict__ keys, typename KeyTraits<KT>::U* __restrict__ tmpKeys,
    typename ValueWord<VB>::T* __restrict__ vals, typename ValueWord<VB>::T* __restrict__ tmpVals,
    KeyMap<typename KeyTraits<KT>::U> km, int shift, int p, int nLow, const uint32_t* __restrict__ chunkOff,
    uint32_t* __restrict__ meta, const uint32_t* __restrict__ bigB, const uint32_t* __restrict__ bigPos,
    const uint32_t* __restrict__ bigTile, const uint32_t* __restrict__ bigHist, ST* __restrict__ status0,
    ST* __restrict__ status1, uint32_t* __restrict__ errFlag, const SqueezeWords* __restrict__ sq) {
  using U = typename KeyTraits<KT>::U;
  using VW = typename ValueWord<VB>::T;
  using G = PassGeom<sizeof(U), VB>;
  constexpr uint32_t T = G::TILE;
  if (meta[kMetaFallback] == 0) return;
  const uint32_t info = meta[kMetaBigPass + p];
  if ((info & 1u) == 0) return;  // the identity for every big chunk
  const bool par = (info >> 1) & 1u;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(smem + G::STAGE * (sizeof(U) + VB));
  uint32_t* s_misc = s_cnt + (G::WAVES + 1) * kBins;
  __shared__ uint32_t s_w[4];
  const U* kin = par ? tmpKeys : keys;
  U* kout = par ? keys : tmpKeys;
  const VW* vin = par ? tmpVals : vals;
  VW* vout = par ? vals : tmpVals;
  ST* status = par ? status1 : status0;
  ST* statusNext = p + 1 < nLow ? (par ? status0 : status1) : nullptr;
  const uint32_t M = meta[kMetaBigCount], nTiles = bigTile[M];
  const uint32_t tid = threadIdx.x;
  with_map<KT>(km, sq, [&](auto kmx) __attribute__((always_inline)) {
  U k[G::KPT];
  VW v[VB ? G::KPT : 1];
  for (;;) {
    if (tid == 0) s_misc[8] = atomicAdd(&meta[kMetaBigTicket + p], 1u);
    for (uint32_t i = tid; i < (uint32_t)(G::WAVES * kBins); i += G::THREADS) s_cnt[i] = 0;
    lds_barrier();
    const uint32_t tile = s_misc[8];
    if (tile >= nTiles) break;
    const uint32_t c = big_find(bigTile, M, tile);
    const uint32_t chain = bigTile[c], size = bigPos[c + 1] - bigPos[c], t = tile - chain;
    const uint32_t start = chunkOff[bigB[c]];
    const uint64_t keyStart = (uint64_t)start + (uint64_t)t * T;
    const uint32_t valid = min(T, size - t * T);
    // digit d's base in this chunk: start + keys of the chunk with a smaller digit
    uint32_t myBase = 0;
    if (tid < kBins) {
      const uint32_t lane = tid & 63, w = tid >> 6;
      const uint32_t x = bigHist[(uint64_t)c * nLow * kBins + (uint64_t)p * kBins + tid];
      const uint32_t inc = wave_incl_scan(x, lane);
      if (lane == 63) s_w[w] = inc;
      lds_barrier();
      myBase = start + inc - x + (w > 0 ? s_w[0] : 0u) + (w > 1 ? s_w[1] : 0u) + (w > 2 ? s_w[2] : 0u);
    } else {
      lds_barrier();
    }
    GroupTables<ST> g{};  // (flat look-back: no group tables)
    g.nTiles = chain + (size + T - 1) / T;
    load_tile<KT, VB>(kin, vin, keyStart, valid, k, v);
    pass_tile<KT, VB, ST, ATOMIC_RANK, NoMid, kCodecKeys, false>(kin, kout, vin, vout, keyStart, valid, kmx, shift,
                                                                myBase, start + size, status, statusNext, errFlag, tile, chain, g,
                                                                smem, nullptr, k, v, NoMid{});
    lds_barrier();  // stage, s_gofs, s_misc and s_w are reused by the next tile
  }
  });
}

// An odd number of running low passes left the big chunks in the temporary
// buffer: copy them back (values too).  The last launch of every bucket-path
// sort, so it also publishes the sort's error word to the sticky word (the
// LSD path's thrs_err_publish), whether or not it has anything to copy.
template <typename U, typename VW>
__global__ __launch_bounds__(256) void thrs_big_copy(U* __restrict__ keys, const U* __restrict__ tmpKeys,
                                                     VW* __restrict__ vals, const VW* __restrict__ tmpVals,
                                                     const uint32_t* __restrict__ chunkOff,
                                                     const uint32_t* __restrict__ meta,
                                                     const uint32_t* __restrict__ bigB,
                                                     const uint32_t* __restrict__ bigPos,
                                                     const uint32_t* __restrict__ err, uint32_t* __restrict__ sticky) {
  if (sticky && blockIdx.x == 0 && threadIdx.x == 0) {
    const uint32_t e = *err;
    if (e) __hip_atomic_fetch_or(sticky, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (meta[kMetaFallback] == 0 || meta[kMetaBigCopy] == 0) return;
  const uint32_t M = meta[kMetaBigCount], total = bigPos[M];
  const uint32_t G = gridDim.x, len = (total + G - 1) / G;
  const uint32_t lo = min(total, blockIdx.x * len), hi = min(total, lo + len);
  if (lo >= hi) return;
  for (uint32_t c = big_find(bigPos, M, lo); c < M && bigPos[c] < hi; ++c) {
    const uint32_t p0 = bigPos[c], a = max(lo, p0), b = min(hi, bigPos[c + 1]);
    const uint64_t start = chunkOff[bigB[c]];
    for (uint32_t x = a + threadIdx.x; x < b; x += blockDim.x) {
      const uint64_t i = start + (x - p0);
      keys[i] = tmpKeys[i];
      if (vals) vals[i] = tmpVals[i];
    }
  }
}

}  // namespace
}  // namespace thrs_dev
