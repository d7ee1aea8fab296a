// thrs_hybrid.hpp -- the 3-HBM-pass path for 4-byte keys (gfx950).
//
// The reference sorts by P full passes over HBM (tinyhipradixsort.hpp:862-930),
// each reading and writing every key.  Here, when the window has P >= 3
// digits, only the window's TOP two digits get device-wide passes:
//
//   thrs_hist_joint  one read of the keys: histogram of the 16-bit BUCKET
//                    (the top two digits) + the low digits' histograms
//   thrs_plan        one workgroup: bucket offsets (exclusive scan), the two
//                    top digits' bases (column / row sums of the bucket
//                    histogram), CHUNKS of whole consecutive buckets that fit
//                    one workgroup's LDS, and the fallback flag
//   thrs_pass x2     the usual onesweep passes for digits P-2 and P-1 (stable
//                    LSD): the keys end up grouped by bucket in bucket order
//   thrs_local       one workgroup per chunk: load the chunk (<= kLocCap
//                    keys) into registers, sort it by the P-2 low digits in
//                    LDS (stable LSD rounds, same rank as the pass kernel),
//                    write it back in place -- coalesced, whole lines.
//
// HBM traffic: 1 (histogram read) + 2 x 2 (passes) + 2 (local) = 7 N*K vs
// 1 + 2P = 9 N*K for P = 4, and the local write-out has none of the partial-
// line read-modify-writes a digit scatter pays.
//
// Stability / exactness: the two passes are stable, so within a bucket keys
// keep their input order; the local LSD rounds are stable; so the result is
// THE stable sort by the window bits -- bit-identical to P LSD passes.
//
// Per-bucket fallback: a bucket larger than its local sort's capacity (skewed
// or low-cardinality input) cannot be sorted in one workgroup.  The plan lists
// such BIG chunks and sets meta[kMetaFallback]; the local sorts skip them and
// only they get device-wide LSD passes on their low digits, each big chunk
// its own segment (thrs_fallback.hpp; gated launches, no host
// synchronisation).  The other buckets keep the local sort.
#pragma once
#include "thrs_kernels.hpp"

namespace thrs_dev {
// (internal linkage: every translation unit of libthrs.so gets its own copy
// of the kernels it launches)
namespace {

constexpr uint32_t kBuckets = 65536;  // 16-bit bucket = the window's top two digits
// meta[kMetaMode]: 0 = local path (no bucket above the local capacity);
// 1 = some big chunks (the per-bucket fallback, thrs_fallback.hpp); 2 = ONE
// bucket holds every key, so both top digits are constant and their passes
// are identities (skipped); 3 = as 0, but the top-digit passes move whole
// keys, not the image planes (f32 keys-only with planes: -0 and +0 share one
// image, so the planes lose the zeros' signs; up to kZeroLogCap zero keys the
// zero log restores them, past that a -0 key means mode 3).
// meta[kMetaBigCount]: big chunks listed in bigB.
// The fallback's own words follow (thrs_fallback.hpp).
enum {
  kMetaChunks = 0,
  kMetaFallback = 1,
  kMetaMode = 3,
  kMetaBigCount = 4,
  kMetaBigDone = 5,  // thrs_big_hist workgroups finished (last one plans the passes)
  kMetaBigCopy = 6,  // 1: an odd number of low passes ran -- big chunks end in the temp buffer
  kMetaBigPass = 8,  // [8]: per low pass p, bit 0 = runs (not the identity for every big chunk), bit 1 = parity
  kMetaBigTicket = 16,  // [8]: per low pass p, its tile ticket
  kMetaBigSingle = 24,  // [6]: per low pass p, big chunks whose digit p is one value
  // the squeeze (float keys, thrs_plan_rows; KeyMap<U, true>):
  kMetaRehist = 32,     // 1: the squeeze is on -- histogram and plan again under it
  kMetaPlanDone = 33,   // thrs_plan_rows workgroups finished (the last one decides)
  kMetaOr1 = 34,        // [2]: per image half, OR of the non-empty buckets' indices
  kMetaOr0 = 36,        // [2]: per image half, OR of their complements (16 bits)
  kMetaBigHalf = 38,    // [2]: per image half, buckets above the local capacity
  kMetaPlanDone2 = 40,  // the squeezed plan's finished workgroups
  kMetaSqViol = 41,     // a key broke the sampled squeeze (its dropped bit differs): histogram again, plain
  kMetaNegZero = 42,    // f32: some key is -0 (thrs_hist_joint)
  kMetaZeroCount = 43,  // f32: keys that are +-0 (their first kZeroLogCap positions in the zero log)
  kMetaSqO1 = 44,       // [2]: the sample's per-half OR of bucket indices (thrs_squeeze_sample)
  kMetaSqO0 = 46,       // [2]: ... and of their complements
  kMetaSqCnt = 30,      // [2]: ... and its keys per half
  kMetaSqDone = 62,     // the sample's finished workgroups (the last one decides)
  kMetaSqueeze = 48,    // SqueezeWords (14 words, to 61)
};
static_assert(kMetaSqueeze * 4 + sizeof(SqueezeWords) <= 256, "meta is 64 words");
// gate masks of the gated launches: bit v set = run when the gate word is v
constexpr uint32_t kGateMode0 = 1u << 0, kGateMode1 = 1u << 1, kGateMode2 = 1u << 2,
                   kGateMode3 = 1u << 3;  // on meta[kMetaMode]
// f32 zero log (thrs_hist_joint -> thrs_local16): input position | sign << 31
// of the first kZeroLogCap keys that are +0 or -0
constexpr uint32_t kZeroLogCap = 1024;

// ------------------------------------------------------------ joint histogram
// LDS: bucket counts as 15-bit fields, two per word (bits 0-14 | guard 15 |
// 16-30 | guard 31): 128 KiB for 65536 buckets.  The add that carries a field
// into its guard bit clears the guard again and moves 32768 to the global
// count; with at most 32768 increments per barrier epoch (thrs_hist_joint) no
// carry can reach the neighbouring field, so any skew is counted exactly.
// (The two top digits' histograms are the row and column sums of this one:
// thrs_plan.)
constexpr int kHjUnroll = 4;  // bucket histogram: 16-byte loads in flight per lane
constexpr uint32_t kJointWords = kBuckets / 2;
// Carries (32768 keys of one bucket) are logged in LDS and flushed once per
// distinct bucket at the end: a constant input would otherwise send every
// workgroup's carries to ONE global word (~32K same-address atomics at C2).
// A workgroup of len keys carries at most len / 32768 times (128 at C2);
// past kCarryLog entries carries go straight to global memory.
constexpr uint32_t kCarryLog = 1024;
// s_joint[kJointWords] | s_d2[256] (the range's second-digit counts) | s_log[kCarryLog] | s_logN
constexpr size_t kJointLds = (size_t)kJointWords * 4 + kBins * 4 + kCarryLog * 4 + 16;

// Workgroup i of the bucket histogram reads the contiguous key range
// [i*len, (i+1)*len) (len a multiple of 4: 16-byte loads stay aligned), and
// workgroups [ceil(sG/8), ceil((s+1)G/8)) make up position segment s of the
// segmented second-digit pass: their second-digit counts are segment s's.
__device__ __forceinline__ uint64_t hj_len(uint32_t n, uint32_t G) {
  return (((uint64_t)n + G - 1) / G + 3) & ~3ull;
}
__device__ __forceinline__ uint32_t hj_seg_pos(uint32_t n, uint32_t G, uint32_t s) {
  const uint64_t first = ((uint64_t)s * G + kSegs - 1) / kSegs;
  return (uint32_t)min((uint64_t)n, first * hj_len(n, G));
}

// The zero log's rare path (f32, thrs_hist_joint): the +-0 keys among the
// 4 * un words kv[i + u * gstride] (u < un, below nv), with their positions
// and signs.  Not inlined: its registers must not count against the
// histogram's loop (128 VGPRs).
__device__ __attribute__((noinline)) void hist_log_zeros(const uint4* __restrict__ kv, uint64_t i, uint64_t gstride,
                                                         uint64_t nv, int un, uint32_t* __restrict__ meta,
                                                         uint32_t* __restrict__ zeroLog) {
  for (int u = 0; u < un; ++u) {
    const uint64_t v = i + u * gstride;
    if (v >= nv) continue;
    const uint4 x = kv[v];
    const uint32_t w4[4] = {x.x, x.y, x.z, x.w};
    for (int c = 0; c < 4; ++c) {
      const uint32_t k = w4[c];
      const uint64_t pos = 4 * v + c;
      if ((k & 0x7FFFFFFFu) != 0) continue;
      const bool neg = k != 0;
      if (neg) atomicOr(&meta[kMetaNegZero], 1u);
      if (pos >> 31) {  // (a position past 2^31 does not fit the log's 31 bits: the log counts as full)
        atomicMax(&meta[kMetaZeroCount], kZeroLogCap + 1);
        continue;
      }
      const uint32_t slot = atomicAdd(&meta[kMetaZeroCount], 1u);
      if (slot < kZeroLogCap) zeroLog[slot] = (uint32_t)pos | (neg ? 0x80000000u : 0u);
    }
  }
}

// segRows (thrs_partition_pass): segHist gets the position segments' counts of
// the bucket's TOP byte (its row) instead of its low byte, and joint may be
// null (no bucket totals: nothing is flushed).
// Float keys (the squeeze, KeyMap<U, true>): the map is sq's when sq->on.
// First histogram (SECOND = false): sq = the sample's guess
// (thrs_squeeze_sample); every key of a squeezed half is checked to carry the
// dropped bit's value, and a key that does not raises meta[kMetaSqViol] (the
// plan then takes the histogram again under the plain map).  SECOND = true:
// the second histogram, only when meta[kMetaRehist] is set, under the map
// the plan chose (meta's SqueezeWords, on or off).
template <int KT, bool SECOND = false>
__global__ __launch_bounds__(kHistThreads) void thrs_hist_joint(const typename KeyTraits<KT>::U* __restrict__ keys,
                                                                uint32_t n, KeyMap<typename KeyTraits<KT>::U> kmh,
                                                                int bucketShift, int vec,
                                                                uint32_t* __restrict__ joint,
                                                                uint32_t* __restrict__ segHist /* [8][256] */,
                                                                uint32_t* __restrict__ rowHist /* [256] */,
                                                                ZeroRanges tables, uint32_t* __restrict__ meta,
                                                                const SqueezeWords* __restrict__ sq,
                                                                uint32_t* __restrict__ zeroLog,
                                                                uint32_t* __restrict__ partial, int segRows) {
  using U = typename KeyTraits<KT>::U;
  if constexpr (SECOND) {
    if (meta[kMetaRehist] == 0) return;
  }
  extern __shared__ __attribute__((aligned(16))) uint32_t s_joint[];
  uint32_t* s_d2 = s_joint + kJointWords;
  uint32_t* s_log = s_d2 + kBins;
  uint32_t* s_logN = s_log + kCarryLog;
  const uint32_t tid = threadIdx.x;
  {  // the top-digit passes' look-back tables (first read after this kernel):
     // their zero stores ride along with this read-bound kernel
    const uint64_t g = (uint64_t)blockIdx.x * kHistThreads + tid, stride = (uint64_t)gridDim.x * kHistThreads;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      uint4* p = reinterpret_cast<uint4*>(tables.ptr[r]);
      for (uint64_t i = g; i < tables.words[r]; i += stride) p[i] = make_uint4(0, 0, 0, 0);
    }
  }
  for (uint32_t i = tid; i < kJointWords + kBins; i += kHistThreads) s_joint[i] = 0;
  if (tid == 0) *s_logN = 0;
  __syncthreads();
  with_map<KT>(kmh, sq, [&](auto km) __attribute__((always_inline)) {
  // (a squeezed first histogram: does every key carry its half's dropped bit?)
  constexpr bool kCheck = !SECOND && !std::is_same<decltype(km), KeyMap<U>>::value;
  U viol = 0;
  const uint64_t len = hj_len(n, gridDim.x);
  const uint64_t lo = min((uint64_t)n, (uint64_t)blockIdx.x * len), hi = min((uint64_t)n, lo + len);
  uint32_t* segH = segHist + (blockIdx.x * kSegs / gridDim.x) * kBins;

  const uint32_t lane = tid & 63;
  // f32 (first histogram, zeroLog set: the image planes): keys that are +0
  // or -0 share one image, so the planes lose their signs.  Each wave notes
  // (a ballot, scalar registers) whether an iteration met any; only then are
  // that iteration's keys read again and the zeros logged with their
  // positions (zero_log), and a -0 flagged.
  constexpr bool kZeros = KT == 2 && !SECOND;
  uint64_t zany = 0;
  bool zfull = false;  // (this thread saw the log full: only the -0 flag from then on)
  auto log_zero = [&](U k, uint64_t pos) {
    if ((k & (U)0x7FFFFFFFu) != 0) return;
    const bool neg = k != 0;
    if (neg) atomicOr(&meta[kMetaNegZero], 1u);
    if (zfull) return;
    if (pos >> 31) {  // (a position past 2^31 does not fit the log's 31 bits: the log counts as full)
      atomicMax(&meta[kMetaZeroCount], kZeroLogCap + 1);
      zfull = true;
      return;
    }
    const uint32_t slot = atomicAdd(&meta[kMetaZeroCount], 1u);
    if (slot < kZeroLogCap) zeroLog[slot] = (uint32_t)pos | (neg ? 0x80000000u : 0u);
    else zfull = true;
  };
  auto bucket_of = [&](U k) -> uint32_t {
    if constexpr (kZeros) zany |= __ballot((k & (U)0x7FFFFFFFu) == 0);
    if constexpr (kCheck) {
      const U y0 = ((KeyTraits<KT>::bits(k) ^ km.mask) - km.lo) << km.sh;  // the plain image
      const bool h = (y0 >> (8 * sizeof(U) - 1)) != 0;
      const U sbit = (h ? km.loM[1] : km.loM[0]) + 1u;  // the dropped bit (0 in an unsqueezed half)
      const U hm = h ? km.hiM[1] : km.hiM[0];
      viol |= (y0 & sbit & ~hm) ^ (h ? km.cst[1] : km.cst[0]);
    }
    return (uint32_t)(kimg<KT>(km, k) >> bucketShift) & 0xFFFFu;
  };
  // Adds are wave-aggregated as in wave_count_items (sorted input would
  // otherwise make every add a 64-way same-address conflict): a wave whose 16
  // elements all fall in one bucket adds 1024 from lane 0; elements whose
  // bucket is uniform over the wave add 64 from lane 0; the rest add 1 per lane.
  auto add = [&](uint32_t b, uint32_t inc) -> uint32_t {
    return __hip_atomic_fetch_add(&s_joint[b >> 1], inc << ((b & 1u) << 4), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  // The add that carried the field from below 0x8000 to 0x8000 or above
  // (guard bit set) takes 0x8000 back out and credits it globally.
  auto check = [&](uint32_t b, uint32_t old, uint32_t inc) {
    const uint32_t sh = (b & 1u) << 4;
    const uint32_t f = (old >> sh) & 0xFFFFu;
    if (inc && f < 0x8000u && f + inc >= 0x8000u) {
      __hip_atomic_fetch_sub(&s_joint[b >> 1], 0x8000u << sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const uint32_t slot = __hip_atomic_fetch_add(s_logN, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (slot < kCarryLog) {
        s_log[slot] = b;
      } else {
        if (joint) atomicAdd(&joint[b], 0x8000u);
        atomicAdd(&segH[segRows ? b >> 8 : b & 255u], 0x8000u);
        atomicAdd(&rowHist[b >> 8], 0x8000u);
      }
    }
  };
  // Exactness bound: between two workgroup barriers the workgroup adds at
  // most kEpoch <= 32768 increments, and every carry of the epoch has been
  // taken out (lgkmcnt(0)) before its barrier.  So an epoch starts with every
  // field below 0x8000 and ends at most at 0x7FFF + 0x8000 = 0xFFFF: no carry
  // ever reaches the neighbouring field, whatever the skew or the wave
  // scheduling.  Iteration counts are uniform over the workgroup (lanes past
  // the range are masked), so every wave meets every barrier.
#ifndef THRS_HJ_EPOCH
#define THRS_HJ_EPOCH 16384  // <= 32768 (exactness bound below); 16384 measured 1% faster
#endif
  constexpr uint32_t kEpoch = THRS_HJ_EPOCH;
  constexpr uint64_t gstride = kHistThreads;  // the workgroup's own range
  uint64_t tailStart = lo;
  if (vec) {  // 16-byte loads, UN in flight per lane (keys base 16-B aligned, checked on host)
    constexpr int PER = 16 / sizeof(U);
    // (the squeeze check's extra registers: three 16-byte loads in flight,
    // not four, or the 128-VGPR budget spills ~35 registers -- 4x slower)
#ifndef THRS_HJ_CHECK_UN
#define THRS_HJ_CHECK_UN 3
#endif
    constexpr int UN = kCheck ? THRS_HJ_CHECK_UN : kHjUnroll;
#ifndef THRS_HJ_CHECK_EPOCH
#define THRS_HJ_CHECK_EPOCH THRS_HJ_EPOCH
#endif
    constexpr uint32_t ITERS_PER_EPOCH = (kCheck ? (uint32_t)THRS_HJ_CHECK_EPOCH : kEpoch) / (kHistThreads * UN * PER);
    static_assert((kCheck ? (uint32_t)THRS_HJ_CHECK_EPOCH : kEpoch) <= 32768u, "exactness bound");
    static_assert(ITERS_PER_EPOCH >= 1, "one iteration must fit an epoch");
    const uint64_t v0 = lo / PER, nv = hi / PER;   // lo is a multiple of 4 (hj_len)
    const uint4* kv = reinterpret_cast<const uint4*>(keys);
    const uint64_t nIter = nv > v0 ? (nv - v0 + UN * gstride - 1) / (UN * gstride) : 0;
    // software pipelined: iteration it+1's loads are issued before iteration
    // it's LDS adds, so every wave keeps UN loads in flight while it counts.
    // Loads past the range read the range's last word (clamped, unconditional:
    // a lane-conditional load would make the compiler wait for all of them).
    // (the thread index re-pinned every iteration: no lane-dependent address
    // is hoisted out of the loop into a long-lived register)
    uint32_t tidv = tid;
    auto load_iter = [&](uint64_t it, uint4 (&q)[UN]) {
      const uint64_t i = v0 + it * UN * gstride + tidv;
#pragma unroll
      for (int u = 0; u < UN; ++u) q[u] = kv[min(i + u * gstride, nv - 1)];
    };
    uint4 qn[UN];
    if (nIter) load_iter(0, qn);
    for (uint64_t it = 0; it < nIter; ++it) {
      pin(tidv);
      const uint64_t i = v0 + it * UN * gstride + tidv;
      uint4 q[UN];
#pragma unroll
      for (int u = 0; u < UN; ++u) q[u] = qn[u];
      load_iter(min(it + 1, nIter - 1), qn);
      uint32_t b[UN * PER], o[UN * PER] = {}, inc[UN * PER];
#pragma unroll
      for (int u = 0; u < UN; ++u) {
        if constexpr (sizeof(U) == 4) {
          b[u * 4 + 0] = bucket_of(q[u].x);
          b[u * 4 + 1] = bucket_of(q[u].y);
          b[u * 4 + 2] = bucket_of(q[u].z);
          b[u * 4 + 3] = bucket_of(q[u].w);
        } else {
          b[u * 2 + 0] = bucket_of(((uint64_t)q[u].y << 32) | q[u].x);
          b[u * 2 + 1] = bucket_of(((uint64_t)q[u].w << 32) | q[u].z);
        }
      }
      constexpr int E = UN * PER;
      if constexpr (kZeros) {
        if (zany && zeroLog) hist_log_zeros(kv, i, gstride, nv, UN, meta, zeroLog);  // (rare) read again
        zany = 0;
      }
      if (v0 + (it + 1) * UN * gstride <= nv) {  // every element of every lane is in the range
        uint32_t b0;
        const uint32_t mode = wave_mode<E>([&](int e) { return b[e]; }, E, b0);
        if (mode == kAllUniform) {
          if (lane == 0) check(b0, add(b0, 64u * E), 64u * E);
        } else if (mode == kMixed) {
#pragma unroll
          for (int e = 0; e < E; ++e) o[e] = add(b[e], 1u);
#pragma unroll
          for (int e = 0; e < E; ++e) check(b[e], o[e], 1u);
        } else {
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const bool uni = wave_uniform(b[e]);
            inc[e] = uni ? (lane == 0 ? 64u : 0u) : 1u;
            if (inc[e]) o[e] = add(b[e], inc[e]);
          }
#pragma unroll
          for (int e = 0; e < E; ++e) check(b[e], o[e], inc[e]);
        }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          inc[e] = (i + (e / PER) * gstride < nv) ? 1u : 0u;
          if (inc[e]) o[e] = add(b[e], 1u);
        }
#pragma unroll
        for (int e = 0; e < E; ++e) check(b[e], o[e], inc[e]);
      }
      if ((it + 1) % ITERS_PER_EPOCH == 0) lds_barrier();
    }
    tailStart = max(lo, nv * PER);
  }
  {  // scalar keys (unaligned base, and the < PER keys past the last 16-B word)
    const uint64_t nIter = hi > tailStart ? (hi - tailStart + gstride - 1) / gstride : 0;
    constexpr uint32_t ITERS_PER_EPOCH = kEpoch / kHistThreads;
    for (uint64_t it = 0; it < nIter; ++it) {
      const uint64_t i = tailStart + it * gstride + tid;
      if (i < hi) {
        const U k = keys[i];
        const uint32_t b = bucket_of(k);
        check(b, add(b, 1u), 1u);
        if constexpr (kZeros) {
          if (zeroLog) log_zero(k, i);
        }
      }
      if ((it + 1) % ITERS_PER_EPOCH == 0) lds_barrier();
    }
  }
  __syncthreads();
  // logged carries: the first log entry of each bucket flushes all of them
  const uint32_t nLog = min(*s_logN, kCarryLog);
  for (uint32_t t = tid; t < nLog; t += kHistThreads) {
    const uint32_t b = s_log[t];
    uint32_t mult = 0;
    bool first = true;
    for (uint32_t u = 0; u < nLog; ++u) {
      const uint32_t x = s_log[u];
      mult += x == b;
      first = first && !(x == b && u < t);
    }
    if (first) {
      if (joint) atomicAdd(&joint[b], mult * 0x8000u);
      atomicAdd(&segH[segRows ? b >> 8 : b & 255u], mult * 0x8000u);
      atomicAdd(&rowHist[b >> 8], mult * 0x8000u);
    }
  }
  // the flush.  partial (the temporary buffer's keyOut region, free until the
  // first pass): the workgroup's 128 KiB of packed counts as plain 16-byte
  // stores, summed by thrs_hist_reduce -- 65536 x 256 global atomics (64 MB
  // of memory-side adds at ~1.3 TB/s) cost 45-78 us at the end of the kernel
  // (docs/EXPERIMENTS.md row 113).  Otherwise (keyOut too small: n < 2^16)
  // one 64-bit add per LDS word (its two buckets are neighbours in joint, and
  // no bucket's total reaches 2^32: no carry crosses them).
  if (partial) {
    uint4* pv = reinterpret_cast<uint4*>(partial + (uint64_t)blockIdx.x * kJointWords);
    const uint4* sv = reinterpret_cast<const uint4*>(s_joint);
    for (uint32_t i = tid; i < kJointWords / 4; i += kHistThreads) pv[i] = sv[i];
  } else if (joint) {
    for (uint32_t wi = tid; wi < kJointWords; wi += kHistThreads) {
      const uint32_t x = s_joint[wi];
      if (x)
        atomicAdd(reinterpret_cast<unsigned long long*>(joint) + wi,
                  (unsigned long long)(x & 0xFFFFu) | ((unsigned long long)(x >> 16) << 32));
    }
  }
  // the range's second-digit counts (column sums; lanes d, d+1 share a word)
  static_assert(kHistThreads == 4 * kBins, "four top-digit quarters per second digit");
  if (!segRows) {
    const uint32_t d = tid & (kBins - 1), top0 = (tid >> 8) * 64;
    uint32_t c = 0;
#pragma unroll 8
    for (uint32_t t = top0; t < top0 + 64; ++t) {
      const uint32_t b = t * kBins + d;
      c += (s_joint[b >> 1] >> ((b & 1u) << 4)) & 0xFFFFu;
    }
    __hip_atomic_fetch_add(&s_d2[d], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  // the range's top-digit counts (row sums: thread 4r+q sums words [128r +
  // 32q, +32), two fields each, every field < 0x8000 after the last epoch)
  {
    const uint32_t r = tid >> 2, q = tid & 3u;
    uint32_t c = 0;
#pragma unroll 8
    for (uint32_t i = 0; i < 32; ++i) {
      const uint32_t x = s_joint[128 * r + 32 * q + i];
      c += (x & 0xFFFFu) + (x >> 16);
    }
    c += __shfl_xor(c, 1);
    c += __shfl_xor(c, 2);
    if (q == 0 && c) {
      atomicAdd(&rowHist[r], c);
      if (segRows) atomicAdd(&segH[r], c);
    }
  }
  __syncthreads();
  if (!segRows && tid < kBins && s_d2[tid]) atomicAdd(&segH[tid], s_d2[tid]);
  if constexpr (kCheck) {
    if (__ballot(viol != 0)) {
      if (lane == 0) atomicOr(&meta[kMetaSqViol], 1u);
    }
  }
  });
}

// ----------------------------------------------------- the sampled squeeze
// Float keys over the whole key (before the first bucket histogram; one
// 256-thread workgroup): kSqSample keys (32 evenly spaced runs) give, per
// image half, the bucket bits that all of them share.  In a half whose keys
// would overflow the local sort -- its share of n over the 2^(15 - constant
// bits) buckets it can reach, mean + 4.5 sigma above the capacity -- the highest such bit is
// dropped (KeyMap<U, true>), so the FIRST histogram already counts the
// squeezed buckets: the reference's own float generator (the lowest exponent
// bit cleared, unittest.cpp:103/108) needs one read of the keys, not two.
// A sample can miss a key that breaks the guess: the histogram checks every
// key (meta[kMetaSqViol]) and the plan then histograms again, plainly.
constexpr int kSqSampleThreads = 256;
constexpr uint32_t kSqSample = 8192;  // keys sampled (kSqSample / 256 runs of 256)
// One workgroup per run (kSqBlocks = 32 runs of 256 consecutive keys, evenly
// spaced): the runs' address translations and loads proceed on 32 CUs at
// once (one workgroup loading all 32 took ~17 us); partial ORs and counts go
// to meta (zeroed with it), the last workgroup decides.
constexpr uint32_t kSqBlocks = kSqSample / kSqSampleThreads;
template <int KT>
__global__ __launch_bounds__(kSqSampleThreads) void thrs_squeeze_sample(const typename KeyTraits<KT>::U* __restrict__ keys,
                                                                        uint32_t n, KeyMap<typename KeyTraits<KT>::U> km,
                                                                        uint32_t cap, SqueezeWords* __restrict__ out,
                                                                        uint32_t* __restrict__ meta) {
  using U = typename KeyTraits<KT>::U;
  constexpr int W = 8 * (int)sizeof(U);
  __shared__ uint32_t s_o1[2], s_o0[2], s_cnt[2], s_last;
  const uint32_t t = threadIdx.x, j = blockIdx.x;
  if (t < 2) s_o1[t] = s_o0[t] = s_cnt[t] = 0;
  __syncthreads();
  {
    const uint64_t i = (uint64_t)j * n / kSqBlocks + t;
    const uint32_t b = (uint32_t)(kimg<KT>(km, keys[min(i, (uint64_t)n - 1)]) >> (W - 16)) & 0xFFFFu;
    const int h = b >> 15;
    atomicOr(&s_o1[h], b);
    atomicOr(&s_o0[h], ~b & 0xFFFFu);
    atomicAdd(&s_cnt[h], 1u);
  }
  __syncthreads();
  if (t < 2 && s_cnt[t]) {
    atomicOr(&meta[kMetaSqO1 + t], s_o1[t]);
    atomicOr(&meta[kMetaSqO0 + t], s_o0[t]);
    atomicAdd(&meta[kMetaSqCnt + t], s_cnt[t]);
  }
  __syncthreads();  // (both threads' contributions before thread 0's arrival)
  if (t == 0) {
    __threadfence();
    s_last = atomicAdd(&meta[kMetaSqDone], 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (t != 0 || !s_last) return;
  __threadfence();
  for (int h = 0; h < 2; ++h) {
    s_o1[h] = load_agent(&meta[kMetaSqO1 + h]);
    s_o0[h] = load_agent(&meta[kMetaSqO0 + h]);
    s_cnt[h] = load_agent(&meta[kMetaSqCnt + h]);
  }
  const uint32_t total = s_cnt[0] + s_cnt[1];
  bool any = false;
  uint64_t hiM[2], loM[2], cst[2];
  for (int h = 0; h < 2; ++h) {
    hiM[h] = ~0ull;
    loM[h] = 0;
    cst[h] = 0;
    const uint32_t cm = ~(s_o1[h] & s_o0[h]) & 0x7FFFu;  // bucket bits every sampled key of the half shares
    if (!s_cnt[h] || !cm) continue;
    // keys of this half per bucket it can reach: squeeze only if the fullest
    // such bucket (mean + 4.5 sigma) would overflow the local sort
    const double load = (double)n * s_cnt[h] / total / (double)(1u << (15 - __builtin_popcount(cm)));
    if (1.02 * load + 4.5 * sqrt(load) <= (double)cap) continue;
    const int bb = 31 - __builtin_clz(cm);
    const int b = bb + W - 16;
    hiM[h] = ~((2ull << b) - 1ull);
    loM[h] = (1ull << b) - 1ull;
    cst[h] = (uint64_t)((s_o1[h] >> bb) & 1u) << b;
    any = true;
  }
  for (int h = 0; h < 2; ++h) {
    out->hiM[h] = hiM[h];
    out->loM[h] = loM[h];
    out->cst[h] = cst[h];
  }
  out->pad = 0;
  out->on = any ? 1u : 0u;
}

// ------------------------------------------------------- partition plan
// thrs_partition_pass (the multi-GPU bucket exchange's first step, one stable
// pass by one digit): after thrs_hist_joint in segRows mode (the bucket's top
// byte = the pass's digit, per position segment), one 256-thread workgroup
// turns the digit totals into bases and the 256 counts the caller gets, and
// the position segments into the segmented pass's tables (as thrs_plan_rows
// does for the second-digit pass): segBase[s][d] = base(d) + (keys of digit d
// in earlier segments), segment positions, first tile ids, tickets.
__global__ __launch_bounds__(kBins) void thrs_partition_plan(const uint32_t* __restrict__ rowHist,
                                                             const uint32_t* __restrict__ segHist, uint32_t n,
                                                             uint32_t histGrid, uint32_t tileKeys,
                                                             uint32_t* __restrict__ counts,
                                                             uint32_t* __restrict__ segInfo,
                                                             uint32_t* __restrict__ segBase) {
  __shared__ uint32_t s_w[4];
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t tot = rowHist[t];
  const uint32_t inc = wave_incl_scan(tot, lane);
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  uint32_t b = inc - tot;
  for (uint32_t ww = 0; ww < w; ++ww) b += s_w[ww];
  counts[t] = tot;
#pragma unroll
  for (int sg = 0; sg < kSegs; ++sg) {
    segBase[sg * kBins + t] = b;
    b += segHist[sg * kBins + t];
  }
  if (t == 0) {
    uint32_t tiles = 0;
    segInfo[kSegAlignWord] = 0;
    segInfo[kSegVecWord] = 0;
    for (int sg = 0; sg <= kSegs; ++sg) {
      const uint32_t pos = sg < kSegs ? hj_seg_pos(n, histGrid, (uint32_t)sg) : n;
      segInfo[sg] = pos;
      segInfo[kSegs + 1 + sg] = tiles;
      if (sg < kSegs) {
        const uint32_t next = sg + 1 < kSegs ? hj_seg_pos(n, histGrid, (uint32_t)sg + 1) : n;
        const uint32_t nT = seg_tiles(pos, next, tileKeys, false);
        tiles += (nT + kGroup - 1) / kGroup * kGroup;
        segInfo[64 + sg] = 0;  // ticket (own cache line)
      }
    }
  }
}

// ------------------------------------------------------------- plan, rows
// Single-bucket chunks (pairs, thrs_local16, 8-byte keys): chunk c is bucket
// c, so the plan needs no chunk-counting sweep and splits by top digit: one
// workgroup per row r (the 256 buckets of top digit r).  The top-digit totals
// come from thrs_hist_joint (rowHist), the second digit's from the position
// segments' counts (segHistA), so no workgroup waits on another.
//   chunkOff[256r + t] = base(r) + (keys of row r's buckets before t)
//   segBase[s][r]      = base(r) + (keys of row r in columns < 32s)
//   fallback / mode    raised atomically (meta is zeroed with the histogram)
// Workgroup 0 also writes the second digit's bases, both passes' segment
// tables and the chunk count.
constexpr int kPlanRowThreads = 256;
// The squeeze decision (float keys, sqMode 1), by the last workgroup to
// finish: in each image half that holds big buckets, the highest bucket bit
// below the half bit that every non-empty bucket of the half shares (from the
// OR of the indices and of their complements) is dropped (KeyMap<U, true>);
// if any half gets one, the squeeze goes on and the histogram and the plan
// are taken again under it (meta[kMetaRehist]; the flags raised by this plan
// are cleared for the second one).  Only when some bucket would take the
// per-bucket fallback (mode 1): an in-capacity plan is kept as it is.
__device__ __forceinline__ void plan_squeeze(uint32_t* __restrict__ meta, int keyBits,
                                             const SqueezeWords* __restrict__ sample) {
  SqueezeWords* sq = reinterpret_cast<SqueezeWords*>(meta + kMetaSqueeze);
  if (sample && sample->on) {
    // the first histogram ran under the sample's squeeze: keep it (every later
    // launch reads meta's copy) -- unless a key broke it: histogram again
    // under the plain map
    if (load_agent(&meta[kMetaSqViol]) == 0u) {
      *sq = *sample;
    } else {
      meta[kMetaRehist] = 1;
      meta[kMetaMode] = 0;
      meta[kMetaFallback] = 0;
      meta[kMetaBigCount] = 0;
    }
    return;
  }
  if (load_agent(&meta[kMetaMode]) != 1u) return;
  uint64_t hiM[2], loM[2], cst[2];
  bool any = false;
  for (int h = 0; h < 2; ++h) {
    const uint32_t o1 = load_agent(&meta[kMetaOr1 + h]), o0 = load_agent(&meta[kMetaOr0 + h]);
    const uint32_t big = load_agent(&meta[kMetaBigHalf + h]);
    const uint32_t cm = ~(o1 & o0) & 0x7FFFu;  // constant bucket bits below the half bit
    hiM[h] = ~0ull;
    loM[h] = 0;
    cst[h] = 0;
    if (big && (o1 | o0) && cm) {
      const int bb = 31 - __builtin_clz(cm);
      const int b = bb + keyBits - 16;  // its image bit
      hiM[h] = ~((2ull << b) - 1ull);
      loM[h] = (1ull << b) - 1ull;
      cst[h] = (uint64_t)((o1 >> bb) & 1u) << b;
      any = true;
    }
  }
  if (!any) return;
  for (int h = 0; h < 2; ++h) {
    sq->hiM[h] = hiM[h];
    sq->loM[h] = loM[h];
    sq->cst[h] = cst[h];
  }
  sq->on = 1;
  meta[kMetaRehist] = 1;
  meta[kMetaMode] = 0;
  meta[kMetaFallback] = 0;
  meta[kMetaBigCount] = 0;
}

// The per-bucket fallback's plan (thrs_fallback.hpp), by the plan's last
// workgroup (256 threads): prefixes of the big chunks' sizes (bigPos: their
// positions in the concatenation of the big chunks) and tile counts (bigTile).
// Every listed entry is checked first: a bucket id past the histogram, or a
// bucket that is not above the capacity, can only come from a plan-ordering
// bug; it must never address past a table (the fallback indexes chunkOff by
// these ids), so the fallback is switched off (no big chunk listed) and the
// sort reports THRS_ERROR_DEVICE_CHECK through its error word.
// (inject: fault-injection builds only -- a stale first entry, see
// thrs_debug_inject)
__device__ __forceinline__ void plan_big_prefix(const uint32_t* __restrict__ joint, uint32_t* __restrict__ meta,
                                                uint32_t* __restrict__ bigB, uint32_t* __restrict__ bigPos,
                                                uint32_t* __restrict__ bigTile, uint32_t tileKeys, uint32_t cap,
                                                uint32_t (*s_w)[4], uint32_t* __restrict__ errFlag, int inject) {
  const uint32_t M = load_agent(&meta[kMetaBigCount]);
  if (M == 0) return;
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (inject && t == 0) bigB[0] = 0xFFFFFFF0u;
  __syncthreads();
  const uint32_t per = (M + kPlanRowThreads - 1) / kPlanRowThreads;
  const uint32_t i0 = min(M, t * per), i1 = min(M, i0 + per);
  bool bad = false;
  for (uint32_t i = i0; i < i1; ++i) {
    const uint32_t b = bigB[i];
    bad = bad || b >= kBuckets || joint[b] <= cap;
  }
  if (__syncthreads_or(bad)) {
    if (t == 0) {
      atomicOr(errFlag, kErrRunClamped);
      meta[kMetaBigCount] = 0;
      meta[kMetaFallback] = 0;
    }
    return;
  }
  auto tiles_of = [&](uint32_t sz) { return (sz + tileKeys - 1) / tileKeys; };
  uint32_t ks = 0, ts = 0;
  auto size_of = [&](uint32_t i) { return joint[bigB[i]]; };
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
  if (t == kPlanRowThreads - 1) {
    bigPos[M] = pk;
    bigTile[M] = pt;
  }
}

// The bucket histogram's workgroup partials (thrs_hist_joint with partial):
// G x 32768 words, each two 15-bit counts (buckets 2w, 2w + 1).  Workgroup r
// owns buckets [256r, 256r + 256) = words [128r, 128r + 128): thread t sums
// 16-byte column t & 31 over the partials g = t >> 5, + 32, ... (8 loads in
// flight at G = 256), the 32 phases meet in LDS, and bucket 256r + t adds its
// total to joint (which holds the workgroups' logged carries already).
constexpr int kHistReduceThreads = 1024;
__global__ __launch_bounds__(kHistReduceThreads) void thrs_hist_reduce(const uint32_t* __restrict__ partial,
                                                                        uint32_t G, uint32_t* __restrict__ joint) {
  __shared__ uint32_t s_sum[32][kBins + 1];
  const uint32_t t = threadIdx.x, q = t & 31u, p = t >> 5, r = blockIdx.x;
  const uint4* pv = reinterpret_cast<const uint4*>(partial) + (uint64_t)r * 32 + q;
  uint32_t f[8] = {};
#pragma unroll 8
  for (uint32_t g = p; g < G; g += 32) {
    const uint4 x = pv[(uint64_t)g * (kJointWords / 4)];
    f[0] += x.x & 0xFFFFu;
    f[1] += x.x >> 16;
    f[2] += x.y & 0xFFFFu;
    f[3] += x.y >> 16;
    f[4] += x.z & 0xFFFFu;
    f[5] += x.z >> 16;
    f[6] += x.w & 0xFFFFu;
    f[7] += x.w >> 16;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) s_sum[p][8 * q + i] = f[i];
  __syncthreads();
  if (t < kBins) {
    uint32_t tot = 0;
#pragma unroll 8
    for (int i = 0; i < 32; ++i) tot += s_sum[i][t];
    joint[kBins * r + t] += tot;
  }
}

// sqMode: 0 = plain plan; 1 = float keys, first plan (gathers the bucket
// occupancy per image half and decides the squeeze, plan_squeeze); 2 = the
// plan of the squeezed histogram (runs only if the squeeze went on).  The
// last workgroup to finish also plans the per-bucket fallback (the big
// chunks' prefixes); the thread that lists a big chunk zeroes its low-digit
// counts (bigHist, nLow x 256 words).
__global__ __launch_bounds__(kPlanRowThreads) void thrs_plan_rows(
    const uint32_t* __restrict__ joint, const uint32_t* __restrict__ rowHist, const uint32_t* __restrict__ segHistA,
    uint32_t n, uint32_t cap, uint32_t* __restrict__ baseTop /* [2][256]: second, top */,
    uint32_t* __restrict__ chunkOff, uint32_t* __restrict__ chunkB0, uint32_t* __restrict__ meta,
    uint32_t* __restrict__ segInfo, uint32_t* __restrict__ segBase, uint32_t tileKeys, uint32_t histGrid,
    uint32_t* __restrict__ segInfoA, uint32_t* __restrict__ segBaseA, uint32_t* __restrict__ bigB, int sqMode,
    int keyBits, uint32_t* __restrict__ bigPos, uint32_t* __restrict__ bigTile, uint4* __restrict__ bigHist,
    int nLow, const SqueezeWords* __restrict__ sample, int planes /* 0 none, 1 keys only, 2 with values */,
    uint32_t* __restrict__ errFlag, int inject) {
  if (sqMode == 2 && meta[kMetaRehist] == 0) return;
  __shared__ uint32_t s_w[2][4], s_base, s_b2[kBins], s_sq[3], s_last;
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6, r = blockIdx.x;
  const uint32_t x = joint[kBins * r + t];
  // 256-thread exclusive scan (4 waves)
  auto scan256 = [&](uint32_t v, int slot, uint32_t* total) -> uint32_t {
    const uint32_t inc = wave_incl_scan(v, lane);
    if (lane == 63) s_w[slot][w] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t x = s_w[slot][i];
      pre += (i < (int)w) ? x : 0u;
      tot += x;
    }
    if (total) *total = tot;
    return pre + inc - v;
  };
  // base(r): exclusive scan of the top-digit totals
  const uint32_t rowTot = rowHist[t];
  const uint32_t rowEx = scan256(rowTot, 0, nullptr);
  if (t == r) s_base = rowEx;
  const uint32_t pre = scan256(x, 1, nullptr);  // (its barrier also publishes s_base)
  const uint32_t base = s_base;
  chunkOff[kBins * r + t] = base + pre;
  chunkB0[kBins * r + t] = kBins * r + t;
  if ((t & 31u) == 0) segBase[(t >> 5) * kBins + r] = base + pre;  // segment s = columns [32s, 32s+32)
  if (t == 0) baseTop[kBins + r] = base;
  if (x > cap) {  // a bucket above the chunk capacity: a big chunk; all n keys in one bucket: mode 2
    atomicOr(&meta[kMetaFallback], 1u);
    atomicMax(&meta[kMetaMode], x == n ? 2u : 1u);
    const uint32_t slot = atomicAdd(&meta[kMetaBigCount], 1u);
    bigB[slot] = kBins * r + t;
    uint4* h = bigHist + (uint64_t)slot * nLow * kBins / 4;
    for (int i = 0; i < nLow * (int)kBins / 4; ++i) h[i] = make_uint4(0, 0, 0, 0);
  }
  if (sqMode == 1) {  // occupancy of this row's image half (for the squeeze decision)
    if (t == 0) s_sq[0] = s_sq[1] = s_sq[2] = 0;
    __syncthreads();
    const uint32_t b = kBins * r + t;
    if (x) {
      atomicOr(&s_sq[0], b);
      atomicOr(&s_sq[1], ~b & 0xFFFFu);
    }
    if (x > cap) atomicAdd(&s_sq[2], 1u);
    __syncthreads();
    if (t == 0) {
      // (128 workgroups per half OR into the same two words: an atomic only
      // where it adds bits -- same-address device atomics serialise, ~5 us
      // over the launch when every workgroup issues them)
      const uint32_t h = r >> 7;
      const uint32_t o1 = load_agent(&meta[kMetaOr1 + h]), o0 = load_agent(&meta[kMetaOr0 + h]);
      if (s_sq[0] & ~o1) atomicOr(&meta[kMetaOr1 + h], s_sq[0]);
      if (s_sq[1] & ~o0) atomicOr(&meta[kMetaOr0 + h], s_sq[1]);
      if (s_sq[2]) atomicAdd(&meta[kMetaBigHalf + h], s_sq[2]);
    }
  }
  // the last workgroup: the squeeze decision (sqMode 1), then -- unless the
  // squeeze went on and a second plan follows -- the fallback's prefixes.
  // (The barrier orders every thread's big-chunk entry, bigB[slot], before
  // thread 0's release and arrival: the last workgroup reads them all.)
  __syncthreads();
  if (t == 0) {
    __threadfence();
    s_last = atomicAdd(&meta[sqMode == 2 ? kMetaPlanDone2 : kMetaPlanDone], 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (s_last) {
    __threadfence();
    if (sqMode == 1 && t == 0) plan_squeeze(meta, keyBits, sample);
    __syncthreads();
    if (!(sqMode == 1 && load_agent(&meta[kMetaRehist]) != 0u)) {
      plan_big_prefix(joint, meta, bigB, bigPos, bigTile, tileKeys, cap, s_w, errFlag, inject);
      // f32 with a -0 key: whole keys through the top-digit passes (mode 3)
      // (more zeros than the zero log holds: thrs_local16 / thrs_local_pairs
      // could not restore the -0 signs from the planes)
      if (t == 0 && planes && load_agent(&meta[kMetaNegZero]) != 0u &&
          load_agent(&meta[kMetaZeroCount]) > kZeroLogCap && load_agent(&meta[kMetaMode]) == 0u)
        meta[kMetaMode] = 3;
    }
    __syncthreads();  // s_w is reused below
  }
  if (r != 0) return;
  // second digit: totals over the position segments -> bases, segment bases
  uint32_t tot2 = 0;
#pragma unroll
  for (int sg = 0; sg < kSegs; ++sg) tot2 += segHistA[sg * kBins + t];
  __syncthreads();  // s_w reuse
  const uint32_t b2 = scan256(tot2, 0, nullptr);
  baseTop[t] = b2;
  s_b2[t] = b2;
  uint32_t sa = b2;
#pragma unroll
  for (int sg = 0; sg < kSegs; ++sg) {
    segBaseA[sg * kBins + t] = sa;
    sa += segHistA[sg * kBins + t];
  }
  __syncthreads();
  // segment positions, first tile ids (multiples of kGroup), tickets: thread 0
  // for the top-digit pass (second-digit ranges), thread 64 for the
  // second-digit pass (position ranges) -- as thrs_plan
  if (t == 0 || t == 64) {
    const bool top = t == 0;
    uint32_t* info = top ? segInfo : segInfoA;
    auto pos_of = [&](int sg) -> uint32_t {
      if (sg >= kSegs) return n;
      return top ? s_b2[32 * sg] : hj_seg_pos(n, histGrid, (uint32_t)sg);
    };
    uint32_t tiles = 0;
    // the top-digit pass's tiles are aligned when it reads the key planes
    // without values (their vector loads, thrs_pass_seg_body; planes == 2,
    // pairs, take none); other codecs count tiles from the segment start
    // (aligned tiles measured slower, docs/EXPERIMENTS.md row 85)
    const bool align = top && planes == 1;
    info[kSegAlignWord] = align ? 1u : 0u;
    info[kSegVecWord] = 0;  // vector-load tiles of the top-digit pass (diagnostics)
    for (int sg = 0; sg <= kSegs; ++sg) {
      const uint32_t pos = pos_of(sg);
      info[sg] = pos;
      info[kSegs + 1 + sg] = tiles;
      if (sg < kSegs) {
        const uint32_t nT = seg_tiles(pos, pos_of(sg + 1), tileKeys, align);
        tiles += (nT + kGroup - 1) / kGroup * kGroup;
        info[64 + sg] = 0;  // ticket (own cache line)
      }
    }
  }
  if (t == 128) {
    chunkOff[kBuckets] = n;
    chunkB0[kBuckets] = kBuckets;
    meta[kMetaChunks] = kBuckets;
  }
}

// ------------------------------------------------------------------- plan
// One workgroup of 1024 threads; thread t owns buckets [64t, 64t+64).
// Chunks: bucket b opens a new chunk iff b % 256 == 0 (a chunk never leaves
// one top digit, so the bucket is (top digit, second digit) and the second
// digit minus the chunk's first is < 256), or the chunk's T-window changes
// (floor(off/T) differs from the previous bucket's), or b or b-1 holds more
// than T keys.  All buckets of a multi-bucket chunk start inside one T-window
// and hold <= T keys, so a chunk holds < 2T <= cap keys unless it is a single
// bucket; a single bucket above cap sets the fallback flag.  T = 2^logT.
// logT < 0 (single mode: u32 keys-only at n > 2^29, pairs, 8-byte keys):
// chunk c is bucket c, empty or not, so no sweep counts the chunks.
constexpr int kPlanThreads = 1024;
__device__ __forceinline__ uint32_t block_excl_scan1024(uint32_t v, uint32_t* s_w, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan(v, lane);
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kPlanThreads / 64; ++i) {
    const uint32_t x = s_w[i];
    pre += (i < (int)w) ? x : 0u;
    tot += x;
  }
  *total = tot;
  __syncthreads();
  return pre + inc - v;
}

__global__ __launch_bounds__(kPlanThreads) void thrs_plan(const uint32_t* __restrict__ joint, uint32_t n,
                                                          uint32_t* __restrict__ baseTop /* [2][256]: second, top */,
                                                          uint32_t* __restrict__ chunkOff,
                                                          uint32_t* __restrict__ chunkB0, uint32_t* __restrict__ meta,
                                                          uint32_t cap, int logT, uint32_t* __restrict__ segInfo,
                                                          uint32_t* __restrict__ segBase, uint32_t tileKeys,
                                                          const uint32_t* __restrict__ segHistA, uint32_t histGrid,
                                                          uint32_t* __restrict__ segInfoA,
                                                          uint32_t* __restrict__ segBaseA, uint32_t* __restrict__ bigB) {
  // Wave w owns buckets [4096w, 4096w + 4096); in step i (0..63) lane l holds
  // bucket 4096w + 64i + l, so every load and every chunk-table store is
  // lane-consecutive; prefixes in bucket order come from wave scans.
  constexpr int WAVES = kPlanThreads / 64, STEPS = (int)kBuckets / kPlanThreads;  // 16, 64
  __shared__ uint32_t s_col[WAVES][kBins], s_row[kBins], s_wsum[WAVES], s_wopen[WAVES], s_wlast[WAVES], s_flag, s_one,
      s_nbig;
  // top-digit histogram of every second-digit segment [32s, 32s+32) (the
  // segmented top-digit pass, thrs_pass_seg) and the second digit's bases
  __shared__ uint32_t s_seg[kSegs][kBins], s_b2[kBins];
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t* src = joint + w * (64 * STEPS) + lane;
  if (tid == 0) {
    s_flag = 0;
    s_one = 0;
    s_nbig = 0;
  }
  __syncthreads();  // before any wave can set them (a wave may finish sweep 1 before wave 0 starts)
  // logT < 0: single-bucket chunks (every non-empty bucket, and every bucket
  // after one, opens a chunk); else T = 2^logT (a shift, not a division)
  const bool single = logT < 0;
  const int lt = single ? 0 : logT;
  const uint32_t T = 1u << lt;
  auto opens = [&](uint32_t b, uint32_t off, uint32_t sz, uint32_t prevSz) -> bool {
    if (single) return true;  // chunk c = bucket c (empty chunks exit at once)
    return (b & 255u) == 0 || (off >> lt) != ((off - prevSz) >> lt) || sz > T || prevSz > T;
  };

  // sweep 1: wave totals, the fallback test, row (top digit) and column
  // (second digit) sums.  Bucket 4096w + 64i + l: row 16w + i/4, column 64(i%4) + l.
  uint32_t tot = 0, col[4] = {0, 0, 0, 0};
  bool big = false, one = false;
#pragma unroll 8
  for (int q4 = 0; q4 < STEPS / 4; ++q4) {
    uint32_t rs = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t x = src[64 * (4 * q4 + q)];
      big |= x > cap;
      one |= x == n;
      col[q] += x;
      rs += x;
      // bucket (top 16w + q4, second 64q + l): segment 2q + l/32, one half-wave each
      const uint32_t sc = wave_incl_scan(x, lane);
      const uint32_t h0 = (uint32_t)__builtin_amdgcn_readlane((int)sc, 31), h1 = lane63(sc) - h0;
      if (lane == 0) {
        s_seg[2 * q][16 * w + q4] = h0;
        s_seg[2 * q + 1][16 * w + q4] = h1;
      }
    }
    tot += rs;
    // row 16w + q4: sum over the wave
    rs = lane63(wave_incl_scan(rs, lane));
    if (lane == 0) s_row[16 * w + q4] = rs;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) s_col[w][64 * q + lane] = col[q];
  tot = lane63(wave_incl_scan(tot, lane));
  if (lane == 0) s_wsum[w] = tot;
  if (lane == 63) s_wlast[w] = src[64 * (STEPS - 1)];
  if (big) s_flag = 1;
  if (one) s_one = 1;
  __syncthreads();
  uint32_t wbase = 0;
  for (uint32_t ww = 0; ww < w; ++ww) wbase += s_wsum[ww];
  const uint32_t prevLast0 = w ? s_wlast[w - 1] : 0u;  // bucket before this wave's first

  // digit bases of the two top digits: [0] second digit (column sums), [1] top digit (row sums)
  if (tid < kBins) {
    uint32_t cs = 0;
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) cs += s_col[ww][tid];
    s_col[0][tid] = cs;  // (each thread reads and rewrites its own column only)
  }
  __syncthreads();
  {
    __shared__ uint32_t s_wt[2][4];
    const uint32_t x0 = tid < kBins ? s_col[0][tid] : 0u, x1 = tid < kBins ? s_row[tid] : 0u;
    const uint32_t i0 = wave_incl_scan(x0, lane), i1 = wave_incl_scan(x1, lane);
    if (tid < kBins && lane == 63) {
      s_wt[0][w] = i0;
      s_wt[1][w] = i1;
    }
    __syncthreads();
    if (tid < kBins) {
      uint32_t p0 = 0, p1 = 0;
      for (uint32_t ww = 0; ww < w; ++ww) {
        p0 += s_wt[0][ww];
        p1 += s_wt[1][ww];
      }
      baseTop[tid] = p0 + i0 - x0;
      baseTop[kBins + tid] = p1 + i1 - x1;
      s_b2[tid] = p0 + i0 - x0;
      // segment bases of the second digit (position segments: thrs_hist_joint's ranges)
      uint32_t sa = p0 + i0 - x0;
      for (int sg = 0; sg < kSegs; ++sg) {
        segBaseA[sg * kBins + tid] = sa;
        sa += segHistA[sg * kBins + tid];
      }
      // segment bases of the top digit: base + the top digit's keys in earlier segments
      uint32_t sb = p1 + i1 - x1;
      for (int sg = 0; sg < kSegs; ++sg) {
        segBase[sg * kBins + tid] = sb;
        sb += s_seg[sg][tid];
      }
    }
  }
  __syncthreads();
  // segment positions, first tile ids (multiples of kGroup), tickets: thread 0
  // for the top-digit pass (second-digit ranges), thread 64 for the
  // second-digit pass (position ranges)
  if (tid == 0 || tid == 64) {
    const bool top = tid == 0;
    constexpr int planes = 0;  // the 32-bit local sort's passes move keys
    uint32_t* info = top ? segInfo : segInfoA;
    auto pos_of = [&](int sg) -> uint32_t {
      if (sg >= kSegs) return n;
      return top ? s_b2[32 * sg] : hj_seg_pos(n, histGrid, (uint32_t)sg);
    };
    uint32_t tiles = 0;
    // the top-digit pass's tiles are aligned when it reads the key planes
    // without values (their vector loads, thrs_pass_seg_body; planes == 2,
    // pairs, take none); other codecs count tiles from the segment start
    // (aligned tiles measured slower, docs/EXPERIMENTS.md row 85)
    const bool align = top && planes == 1;
    info[kSegAlignWord] = align ? 1u : 0u;
    info[kSegVecWord] = 0;  // vector-load tiles of the top-digit pass (diagnostics)
    for (int sg = 0; sg <= kSegs; ++sg) {
      const uint32_t pos = pos_of(sg);
      info[sg] = pos;
      info[kSegs + 1 + sg] = tiles;
      if (sg < kSegs) {
        const uint32_t nT = seg_tiles(pos, pos_of(sg + 1), tileKeys, align);
        tiles += (nT + kGroup - 1) / kGroup * kGroup;
        info[64 + sg] = 0;  // ticket (own cache line)
      }
    }
  }

  // sweeps 2 and 3: absolute offsets in bucket order, chunk-opening flags;
  // sweep 2 counts the wave's chunks, sweep 3 writes them
  auto sweep = [&](bool write, uint32_t cbase) -> uint32_t {
    uint32_t run = wbase, prevTop = prevLast0, nOpen = 0;
    constexpr int BATCH = 16;  // loads of a batch in flight together (L2 hits, ~1 us each otherwise)
    for (int i0 = 0; i0 < STEPS; i0 += BATCH) {
    uint32_t xb[BATCH];
#pragma unroll
    for (int q = 0; q < BATCH; ++q) xb[q] = src[64 * (i0 + q)];
#pragma unroll
    for (int q = 0; q < BATCH; ++q) {
      const int i = i0 + q;
      const uint32_t x = xb[q];
      const uint32_t inc = wave_incl_scan(x, lane);
      const uint32_t off = run + inc - x;
      const uint32_t prev = wave_prev_lane(x, prevTop);
      const uint32_t b = w * (64 * STEPS) + 64 * i + lane;
      const bool o = opens(b, off, x, prev);
      const uint64_t m = __ballot(o);
      if (write && o) {
        const uint32_t c = cbase + nOpen + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        chunkOff[c] = off;
        chunkB0[c] = b;
        // a bucket above cap is a chunk of its own (it opens one, and so does
        // the bucket after it): a big chunk for the per-bucket fallback
        if (x > cap) bigB[atomicAdd(&s_nbig, 1u)] = c;
      }
      nOpen += (uint32_t)__builtin_popcountll(m);
      run += lane63(inc);
      prevTop = lane63(x);
    }
    }
    return nOpen;
  };
  uint32_t cbase = w * (64 * STEPS), nChunks = kBuckets;  // single: every bucket is a chunk
  if (!single) {
    const uint32_t myOpen = sweep(false, 0);
    if (lane == 0) s_wopen[w] = myOpen;
    __syncthreads();
    cbase = 0;
    nChunks = 0;
    for (int ww = 0; ww < WAVES; ++ww) {
      cbase += ((uint32_t)ww < w) ? s_wopen[ww] : 0u;
      nChunks += s_wopen[ww];
    }
  }
  sweep(true, cbase);
  __syncthreads();  // every big chunk appended
  if (tid == kPlanThreads - 1) {
    chunkOff[nChunks] = n;
    chunkB0[nChunks] = kBuckets;
    meta[kMetaChunks] = nChunks;
    meta[kMetaFallback] = s_flag;
    meta[kMetaMode] = s_flag ? (s_one ? 2u : 1u) : 0u;
    meta[kMetaBigCount] = s_nbig;
  }
}

// ------------------------------------------------------------- local sort
// One workgroup per chunk (a persistent form with next-chunk prefetch was
// slower: docs/EXPERIMENTS.md).  Per chunk: KPT keys per lane in registers (item j of lane l of wave w =
// chunk position w*64*KPT + j*64 + l, the order the stable rank walks -- as
// in pass_tile).  Each round: per-wave digit counts (LDS atomics) -> one wave
// scans the 256 digits and turns the counts into per-wave running offsets ->
// rank (lane-ordered ds_add_rtn, or the ballot match) -> scatter into the LDS
// stage -> reload in stage order.  Rounds 0..nLow-1 sort by the window's low
// digits; a chunk of several buckets takes one more round on (second digit -
// chunk's first), which orders its buckets.  The stage then holds the sorted
// chunk: written back in place, each wave storing 256 contiguous bytes per
// instruction.
//
// Positions past the chunk hold a PADDING key whose digit is 255 in every
// round: padding sorts after every real key (same digit, later position), so
// real keys take slots [0, size) and no per-item predicate is needed between
// the load and the final store.
#ifndef THRS_LOC_CFG
#define THRS_LOC_CFG 8, 36  // waves, keys per lane of the large geometry: 2 workgroups per CU
#endif
constexpr int kLocCfg[2] = {THRS_LOC_CFG};
// Local-sort geometry: WAVES waves x KPT keys per lane = CAP slots per chunk.
//   LocBig   8 x 36 = 18432 keys, 2 WGs / CU (72 KiB stage + 8 KiB counters):
//            buckets of 2^30-key sorts (~16K keys)
//   LocSmall 4 x 36 = 9216 keys, 4 WGs / CU (36 KiB + 4 KiB): buckets of
//            2^27..2^29-key sorts, where a large chunk's fixed cost dominates
template <int W, int K, int WPE_ = 4> struct LocG {
  static constexpr int WAVES = W, KPT = K, THREADS = 64 * W, WPE = WPE_;
  static constexpr uint32_t CAP = (uint32_t)THREADS * K;
  template <typename U> static constexpr size_t lds() { return (size_t)CAP * sizeof(U) + (size_t)W * kBins * 4; }
};
using LocBig = LocG<kLocCfg[0], kLocCfg[1]>;
using LocSmall = LocG<4, 36>;
// u32 pairs up to 3 x 2^26 keys: 4096-key chunks, 8 WGs per CU (as Loc16Tiny,
// docs/EXPERIMENTS.md row 115)
using LocTiny = LocG<4, 16, 6>;
constexpr int kLocWaves = LocBig::WAVES, kLocThreads = LocBig::THREADS, kLocKpt = LocBig::KPT;
constexpr uint32_t kLocCap = LocBig::CAP;  // 18432 keys
// chunking windows T = 2^logT (<= CAP/2): uniform buckets of the size range a
// geometry serves never merge (a merged chunk's bucket round has few distinct
// digits, i.e. same-address atomics)
constexpr int kLocLogT = 12, kLocSmallLogT = 11;
template <typename U> constexpr size_t local_lds_bytes() { return LocBig::lds<U>(); }


struct LocChunk {
  uint32_t start, size, b0;
  int rounds;
};

template <int KT>
__device__ __forceinline__ LocChunk loc_chunk(uint32_t c, int nLow, const uint32_t* __restrict__ chunkOff,
                                              const uint32_t* __restrict__ chunkB0) {
  LocChunk ch;
  ch.start = chunkOff[c];
  ch.size = chunkOff[c + 1] - ch.start;  // <= kLocCap (else the fallback flag is set)
  const uint32_t bA = chunkB0[c], bB = chunkB0[c + 1];
  ch.b0 = bA & 0xFFu;
  ch.rounds = nLow + ((bB - bA > 1u) ? 1 : 0);
  return ch;
}

// padding image: ones in every low digit, (b0 - 1) in the second digit (its
// multi-round digit is 255), zero elsewhere -- bits 24..31 are never a local
// digit and stay 0, so the image is never 0x7FFFFFFF (the one unbits32 miss).
// (thrs_local sorts the keys themselves, so it runs only without a key range:
// the padding must be a key.)
template <int KT>
__device__ __forceinline__ uint32_t loc_pad(uint32_t b0, int nLow, int startBits, uint32_t orderMask) {
  const uint32_t padT = (((1u << (8 * nLow)) - 1u) << startBits) | (((b0 - 1u) & 0xFFu) << (startBits + 8 * nLow));
  return unbits32<KT>(padT ^ orderMask);
}

// A wave's KPT coalesced loads of its run of a chunk, all issued before any
// is waited for.  A load under a lane condition is waited for before the next
// one issues, so there is none.  The wave-uniform `avail` = the chunk's keys
// from the wave's first slot on: a whole run loads plainly (one base address,
// immediate offsets); the chunk's partial run clamps every index into the
// chunk (repeats of its last key: no extra HBM traffic); a wave past the
// chunk's end loads nothing.  Callers select per lane (r[j] is garbage for
// slots past the chunk).
// (R: the register type, e.g. u16 plane entries loaded into u32 registers)
template <int KPT, typename R, typename T>
__device__ __forceinline__ void load_run(R (&r)[KPT], const T* __restrict__ chunk, uint32_t myOff, uint32_t size,
                                         int32_t avail) {
  if (avail <= 0) return;
  if (avail >= 64 * KPT) {
    const T* p = chunk + myOff;
#pragma unroll
    for (int j = 0; j < KPT; ++j) r[j] = (R)p[j * 64];
  } else {
    const uint32_t last = size - 1;
#pragma unroll
    for (int j = 0; j < KPT; ++j) r[j] = (R)chunk[min(myOff + (uint32_t)(j * 64), last)];
  }
}

template <int KT, typename LG>
__device__ __forceinline__ void loc_load(typename KeyTraits<KT>::U (&k)[LG::KPT],
                                         const typename KeyTraits<KT>::U* __restrict__ keys, const LocChunk& ch,
                                         uint32_t pad) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int32_t lim = (int32_t)ch.size - (int32_t)(w * 64 * LG::KPT + lane);
  pin(reinterpret_cast<uint32_t&>(lim));
  if (ch.size == 0) {
#pragma unroll
    for (int j = 0; j < LG::KPT; ++j) k[j] = pad;
    return;
  }
  load_run<LG::KPT>(k, keys + ch.start, w * 64 * LG::KPT + lane, ch.size,
                    __builtin_amdgcn_readfirstlane((int32_t)ch.size - (int32_t)(w * 64 * LG::KPT)));
#pragma unroll
  for (int j = 0; j < LG::KPT; ++j) k[j] = (j * 64 < lim) ? k[j] : pad;
}

// THRS_STAMPS builds: per chunk, s_memrealtime (100 MHz) at 0 entry, 1 keys
// loaded, 2 round 0 done, 3 round 1 done, 4 write-out issued, 5 stores
// drained; slot 6 = HW_ID (CU / SE), 7 = XCC id (thread 0 of the workgroup).
constexpr int kLocStampSlots = 8;
__device__ __forceinline__ void loc_stamp(uint64_t* st, int i) {
#ifdef THRS_STAMPS
  if (st && threadIdx.x == 0) st[i] = __builtin_amdgcn_s_memrealtime();
#else
  (void)st;
  (void)i;
#endif
}

// The LDS rounds of one chunk: on return (after a barrier) the stage holds
// the chunk's items in sorted order; returns the number of rounds run.
template <int KT, bool ATOMIC_RANK, typename LG>
__device__ __forceinline__ int loc_rounds(typename KeyTraits<KT>::U (&k)[LG::KPT], const LocChunk& ch,
                                          KeyMap<typename KeyTraits<KT>::U> km, int startBits, int nLow,
                                          unsigned char* smem, uint64_t* st) {
  using U = typename KeyTraits<KT>::U;
  constexpr int KPT = LG::KPT;
  constexpr uint32_t CHUNK = 64 * KPT;
  U* stage = reinterpret_cast<U*>(smem);
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(smem + (size_t)LG::CAP * sizeof(U));  // [waves][256]
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint32_t* cnt = s_cnt + w * kBins;
  U* stw = stage + w * CHUNK + lane;
  // items wholly past the chunk (j*64 >= limw: padding in every lane) take no
  // part in any round: they rank after every real key, so skipping them
  // changes no real key's slot (scalar test: limw is wave-uniform)
  const int32_t limw = __builtin_amdgcn_readfirstlane((int32_t)ch.size - (int32_t)(w * CHUNK));
  const int nItems = limw <= 0 ? 0 : min(KPT, (limw + 63) >> 6);  // items j with j*64 < limw
  const int roundsRun = ch.rounds;
  for (int r = 0; r < roundsRun; ++r) {
    const int shift = r < nLow ? startBits + 8 * r : startBits + 8 * nLow;
    const uint32_t sub = r < nLow ? 0u : ch.b0;
    auto digit_of = [&](U key) -> uint32_t {
      return ((uint32_t)(kimg<KT>(km, key) >> shift) - sub) & 0xFFu;
    };
#pragma unroll
    for (int i = 0; i < kBins / 64; ++i) cnt[i * 64 + lane] = 0;
    // (no wave aggregation here: these kernels sit at their VGPR limit, and
    // the inputs that make a local round's digits wave-uniform -- constant
    // low bytes -- are rare; sorted input is not among them)
    // whole waves (nItems == KPT) run without per-item tests: a scalar branch
    // around an LDS atomic or read makes the compiler wait for every earlier
    // one (thrs_local16)
    const bool wfull = nItems == KPT;
    if (wfull) {
#pragma unroll
      for (int j = 0; j < KPT; ++j)
        __hip_atomic_fetch_add(&cnt[digit_of(k[j])], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
#pragma unroll
      for (int j = 0; j < KPT; ++j)
        if (j < nItems) __hip_atomic_fetch_add(&cnt[digit_of(k[j])], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    lds_barrier();
    {  // threads d < 256: digit d's total over the waves -> block exclusive scan
       // (wave totals through stage words: the stage is free between the
       // reload and the scatter) -> per-wave running offsets
      uint32_t* s_wt = reinterpret_cast<uint32_t*>(stage);
      uint32_t c[LG::WAVES], tot = 0, inc = 0;
      if (tid < kBins) {
#pragma unroll
        for (int ww = 0; ww < LG::WAVES; ++ww) {
          c[ww] = s_cnt[ww * kBins + tid];
          tot += c[ww];
        }
        inc = wave_incl_scan(tot, lane);
        if (lane == 63) s_wt[w] = inc;
      }
      lds_barrier();
      if (tid < kBins) {
        const uint32_t w0 = s_wt[0], w1 = s_wt[1], w2 = s_wt[2];
        uint32_t run = inc - tot + (w > 0 ? w0 : 0u) + (w > 1 ? w1 : 0u) + (w > 2 ? w2 : 0u);
#pragma unroll
        for (int ww = 0; ww < LG::WAVES; ++ww) {
          s_cnt[ww * kBins + tid] = run;
          run += c[ww];
        }
      }
    }
    lds_barrier();
    // rank + scatter (every lane of every item: the rank's wave is fully
    // active).  Ranks are taken in batches of RB items -- their atomics issue
    // back to back and return together -- then the batch is scattered: a
    // scatter write right after each rank would wait for that rank's round
    // trip (the compiler cannot reorder LDS accesses that may alias).
#ifndef THRS_LOC_RB
#define THRS_LOC_RB 12
#endif
    constexpr int RB = THRS_LOC_RB;
    auto rank_scatter = [&](auto fullc) __attribute__((always_inline)) {
      constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
      for (int j0 = 0; j0 < KPT; j0 += RB) {
        uint32_t sl[RB];
#pragma unroll
        for (int jj = 0; jj < RB; ++jj) {
          const int j = j0 + jj;
          if (j < KPT && (FULL || j < nItems)) sl[jj] = wave_rank<ATOMIC_RANK>(cnt, digit_of(k[j]), lane, false);
        }
#pragma unroll
        for (int jj = 0; jj < RB; ++jj)
          if (j0 + jj < KPT && (FULL || j0 + jj < nItems)) stage[sl[jj]] = k[j0 + jj];
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if (wfull) rank_scatter(std::true_type{});
    else rank_scatter(std::false_type{});
    lds_barrier();
    loc_stamp(st, 2 + (r & 1));
    if (r + 1 < roundsRun) {
      if (limw >= (int32_t)CHUNK) {
#pragma unroll
        for (int j = 0; j < KPT; ++j) k[j] = stw[j * 64];
      } else {
#pragma unroll
        for (int j = 0; j < KPT; ++j)
          if (j * 64 < limw) k[j] = stw[j * 64];
      }
    }
  }
  return roundsRun;
}

template <int KT, bool ATOMIC_RANK, typename LG>
__device__ __forceinline__ void loc_sort_chunk(typename KeyTraits<KT>::U (&k)[LG::KPT],
                                               typename KeyTraits<KT>::U* __restrict__ keys, const LocChunk& ch,
                                               KeyMap<typename KeyTraits<KT>::U> km, int startBits, int nLow,
                                               unsigned char* smem, uint64_t* st = nullptr) {
  using U = typename KeyTraits<KT>::U;
  constexpr int KPT = LG::KPT;
  constexpr uint32_t CHUNK = 64 * KPT;
  const int roundsRun = loc_rounds<KT, ATOMIC_RANK, LG>(k, ch, km, startBits, nLow, smem, st);
  const U* stage = reinterpret_cast<const U*>(smem);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const U* stw = stage + w * CHUNK + lane;
  int32_t lim = (int32_t)ch.size - (int32_t)(w * CHUNK + lane);
  pin(reinterpret_cast<uint32_t&>(lim));
  U* src = keys + ch.start + w * CHUNK + lane;
  if (roundsRun == 0) {
#pragma unroll
    for (int j = 0; j < KPT; ++j)
      if (j * 64 < lim) src[j * 64] = k[j];
    return;
  }
  U o[KPT];  // stage reads first, then the lane-conditional stores (see thrs_local16)
#pragma unroll
  for (int j = 0; j < KPT; ++j) o[j] = stw[j * 64];
#pragma unroll
  for (int j = 0; j < KPT; ++j)
    if (j * 64 < lim) src[j * 64] = o[j];
#ifdef THRS_STAMPS
  loc_stamp(st, 4);
  if (st) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    loc_stamp(st, 5);
  }
#endif
}

template <int KT, bool ATOMIC_RANK, typename LG>
__global__ __launch_bounds__(LG::THREADS) void thrs_local(typename KeyTraits<KT>::U* __restrict__ keys,
                                                          KeyMap<typename KeyTraits<KT>::U> km, int startBits,
                                                          int nLow, const uint32_t* __restrict__ chunkOff,
                                                          const uint32_t* __restrict__ chunkB0,
                                                          uint32_t* __restrict__ meta, uint64_t* __restrict__ stamps) {
  using U = typename KeyTraits<KT>::U;
  static_assert(sizeof(U) == 4, "the local sort is for 4-byte keys");
  const uint32_t nChunks = meta[kMetaChunks];
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t c = blockIdx.x;
  if (c >= nChunks) return;
  uint64_t* st = stamps ? stamps + (uint64_t)c * kLocStampSlots : nullptr;
  loc_stamp(st, 0);
  const LocChunk ch = loc_chunk<KT>(c, nLow, chunkOff, chunkB0);
  if (ch.size == 0 || ch.size > LG::CAP) return;  // big chunk: the per-bucket fallback sorts it
  U k[LG::KPT];
  loc_load<KT, LG>(k, keys, ch, loc_pad<KT>(ch.b0, nLow, startBits, (uint32_t)km.mask));
#ifdef THRS_STAMPS
  if (st) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    loc_stamp(st, 1);
    if (threadIdx.x == 0) {
      uint32_t hw;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      st[6] = hw;
      st[7] = xcc_id();
    }
  }
#endif
  loc_sort_chunk<KT, ATOMIC_RANK, LG>(k, keys, ch, km, startBits, nLow, smem, st);
}

// ------------------------------------------------- local sort, 16-bit items
// u32 keys without values over the whole key (startBits 0, 32 bits), single-
// bucket chunks (thrs_plan single mode): every key of a chunk is
// (bucket << 16 | low16) in image space, so only its low 16 bits take part:
// the LDS stage holds 2-byte items (36 KiB for 18432 keys instead of 72) and
// registers hold two items each -- three workgroups per CU instead of two.
// The rounds are those of loc_rounds (count, scan, lane-ordered rank,
// scatter, reload) on 16-bit items; the keys are rebuilt on the way out.
// u32 only: f32 keys' +0 and -0 share one image.
// The stage is padded by one word (two items) per 64 items: item slot s lives
// at (s / 64) * 66 + s % 64.  Structured inputs scatter with regular strides
// (sorted keys: a wave's 64 slots ~288 apart, all on 2 of the 32 store banks);
// the pad spreads them.  A wave's 64 consecutive slots stay contiguous.
// The first round (the low byte) need not be stable: equal 16-bit items are
// indistinguishable, and only the second round must keep the first's order.
// It counts and ranks into ONE workgroup-wide table of TC copies of the 256
// digit counters, copy = lane % TC, as 16-bit halves (digits 2i and 2i+1
// share word i * TC + copy; copy_table_scan).  The second round keeps the
// per-wave counters and the lane-ordered rank (stable).  The table shares
// the counters' LDS: 128 x TC words (TC = 8: 4 KiB, within every geometry's
// per-wave counters).  Measured (docs/EXPERIMENTS.md row 120): local16 C2
// 1.741 -> 1.660 ms, C4 0.446 -> 0.410, ref160m 0.317 -> 0.300; TC = 4 and
// TC = 16 (16 KiB: a workgroup fewer per CU at 9216-key chunks) are slower.
#ifndef THRS_LOC16_TC
#define THRS_LOC16_TC 8
#endif
template <int W, int K, int WPE_ = 6, int LB_ = K, int TC_ = THRS_LOC16_TC> struct Loc16G {
  static constexpr int WAVES = W, KPT = K, THREADS = 64 * W, NP = (K + 1) / 2, WPE = WPE_, LB = LB_, TC = TC_;
  static constexpr uint32_t CAP = (uint32_t)THREADS * K;
  static_assert(TC == 0 || (CAP < 65536 && (TC & (TC - 1)) == 0 && TC % 4 == 0 && TC <= 64),
                "16-bit table halves; whole uint4 rows");
  static constexpr uint32_t ROW = 66;                                // u16 slots per 64 items
  static constexpr size_t STAGE_BYTES = (size_t)(CAP / 64) * ROW * 2;
  static constexpr size_t CNT_BYTES = (size_t)W * kBins * 4 > (size_t)(kBins / 2) * TC * 4
                                          ? (size_t)W * kBins * 4
                                          : (size_t)(kBins / 2) * TC * 4;
  static constexpr size_t LDS = STAGE_BYTES + CNT_BYTES;
  __device__ static uint32_t at(uint32_t s) { return (s >> 6) * ROW + (s & 63u); }
};
using Loc16 = Loc16G<8, 36>;
// n <= 2^29: 9216-key chunks (uniform buckets of <= 8K keys), 6 WGs per CU
#ifndef THRS_L16S_CFG
#define THRS_L16S_CFG 4, 36, 6, 36
#endif
using Loc16Small = Loc16G<THRS_L16S_CFG>;
// u32 keys-only up to 3 x 2^26 keys (uniform buckets of <= 3072 keys): 4096-
// key chunks, 8 WGs per CU.  A chunk's items spread over all four waves
// (~10 per lane at 160M keys instead of 36 in wave 0 and ~2 in wave 1 of a
// 9216-key chunk): the rounds' critical path is 2-3x shorter
// (docs/EXPERIMENTS.md row 112)
#ifndef THRS_L16T_CFG
#define THRS_L16T_CFG 4, 16, 8, 16
#endif
using Loc16Tiny = Loc16G<THRS_L16T_CFG>;
static_assert(Loc16::CAP == LocBig::CAP, "same chunk capacity as the 32-bit geometry (thrs_plan's cap)");
// Wide chunks for u32 keys-only sorts above 2^30 + 2^26, whose uniform
// buckets (n / 65536 keys) outgrow Loc16's 18432 slots: 34816 keys (8 waves x
// 68 items, 79.8 KiB of LDS: two workgroups per CU, which overlap their
// rounds; up to ~2^31 + 2^25, where the largest of 65536 uniform buckets is
// ~4.5 sigma below the capacity)
#ifndef THRS_WIDE_K
#define THRS_WIDE_K 68
#endif
#ifndef THRS_WIDE_W
#define THRS_WIDE_W 8
#endif
using Loc16Wide = Loc16G<THRS_WIDE_W, THRS_WIDE_K, 4, THRS_WIDE_K / 2>;

// f32 keys, the chunk holding the zero image Z (at most one per sort): its
// sorted 16-bit items are in the stage; the keys with image Z are +0 or -0,
// occupy the output slots [s0, s0 + z) (s0 = the chunk's items below Z) and
// keep their input order there (stable).  The input keys (still in place)
// give each zero its rank among the zeros and its sign, as bits in the
// counters' LDS (free after the rounds); the write-out takes the zeros' bit
// patterns from there and rebuilds every other key.
template <typename LG, typename KM>
__device__ __attribute__((noinline)) void loc16_write_zero_chunk(uint32_t* __restrict__ keys, KM km,
                                                                 uint32_t start, uint32_t size, uint32_t hiBits,
                                                                 unsigned char* smem) {
  constexpr int KPT = LG::KPT;
  constexpr uint32_t CHUNK = 64 * KPT;
  static_assert(LG::CAP / 32 + LG::WAVES + 1 <= (uint32_t)LG::WAVES * kBins, "sign bits fit the counters' LDS");
  const uint16_t* stage = reinterpret_cast<const uint16_t*>(smem);
  uint32_t* negBits = reinterpret_cast<uint32_t*>(smem + LG::STAGE_BYTES);  // [CAP / 32]
  uint32_t* s_wz = negBits + LG::CAP / 32;                                   // [WAVES]: zeros per wave
  uint32_t* s_s0 = s_wz + LG::WAVES;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t zlo = kimg<2>(km, 0u) & 0xFFFFu;
  for (uint32_t i = tid; i < LG::CAP / 32 + LG::WAVES + 1; i += LG::THREADS) negBits[i] = 0;
  lds_barrier();
  const uint32_t* src = keys + start + w * CHUNK + lane;
  const int32_t lim = (int32_t)size - (int32_t)(w * CHUNK + lane);
  uint32_t nz = 0, below = 0;
  for (int j = 0; j < KPT; ++j) {  // input position w*CHUNK + 64j + lane: the stable order
    const bool in = j * 64 < lim;
    const uint32_t raw = in ? src[j * 64] : 1u;
    below += (in && (kimg<2>(km, raw) & 0xFFFFu) < zlo) ? 1u : 0u;
    nz += (uint32_t)__builtin_popcountll(__ballot(in && (raw & 0x7FFFFFFFu) == 0));
  }
  if (lane == 0) s_wz[w] = nz;
  atomicAdd(s_s0, below);
  lds_barrier();
  uint32_t q = 0;
  for (uint32_t ww = 0; ww < w; ++ww) q += s_wz[ww];
  for (int j = 0; j < KPT; ++j) {
    const bool in = j * 64 < lim;
    const uint32_t raw = in ? src[j * 64] : 1u;
    const uint64_t m = __ballot(in && (raw & 0x7FFFFFFFu) == 0);
    const uint32_t r = q + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (in && raw == 0x80000000u) atomicOr(&negBits[r >> 5], 1u << (r & 31));
    q += (uint32_t)__builtin_popcountll(m);
  }
  lds_barrier();
  uint32_t z = 0;
  for (int ww = 0; ww < LG::WAVES; ++ww) z += s_wz[ww];
  const uint32_t s0 = *s_s0;
  const uint16_t* stw = stage + w * KPT * LG::ROW + lane;
  uint32_t* dst = keys + start + w * CHUNK + lane;
  for (int j = 0; j < KPT; ++j) {
    if (j * 64 < lim) {
      const uint32_t slot = w * CHUNK + 64 * j + lane, r = slot - s0;
      dst[j * 64] = r < z ? (((negBits[r >> 5] >> (r & 31)) & 1u) ? 0x80000000u : 0u)
                          : kinv<2>(km, hiBits | (uint32_t)stw[j * LG::ROW]);
    }
  }
}

// The same chunk when the keys came as image planes (mode 0) and a -0 was
// seen (at most kZeroLogCap zeros, thrs_plan_rows): the zeros' signs come from
// the zero log (input positions, any order).  A -0's rank among the zeros is
// the number of logged zeros at smaller positions (their stable order).
template <typename LG, typename KM>
__device__ __attribute__((noinline)) void loc16_write_zero_log(uint32_t* __restrict__ keys, KM km, uint32_t start,
                                                               uint32_t size, uint32_t hiBits, unsigned char* smem,
                                                               const uint32_t* __restrict__ zlog, uint32_t z) {
  constexpr int KPT = LG::KPT;
  constexpr uint32_t CHUNK = 64 * KPT;
  static_assert(kZeroLogCap / 32 + 1 <= (uint32_t)LG::WAVES * kBins, "sign bits fit the counters' LDS");
  const uint16_t* stage = reinterpret_cast<const uint16_t*>(smem);
  uint32_t* negBits = reinterpret_cast<uint32_t*>(smem + LG::STAGE_BYTES);  // [kZeroLogCap / 32]
  uint32_t* s_s0 = negBits + kZeroLogCap / 32;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t zlo = kimg<2>(km, 0u) & 0xFFFFu;
  for (uint32_t i = tid; i < kZeroLogCap / 32 + 1; i += LG::THREADS) negBits[i] = 0;
  lds_barrier();
  const uint16_t* stw = stage + w * KPT * LG::ROW + lane;
  const int32_t lim = (int32_t)size - (int32_t)(w * CHUNK + lane);
  uint32_t below = 0;  // sorted items below the zeros' item: the run's start s0
  for (int j = 0; j < KPT; ++j)
    if (j * 64 < lim) below += (uint32_t)stw[j * LG::ROW] < zlo ? 1u : 0u;
  atomicAdd(s_s0, below);
  for (uint32_t e = tid; e < z; e += LG::THREADS) {
    const uint32_t x = zlog[e];
    if (x >> 31) {
      const uint32_t p = x & 0x7FFFFFFFu;
      uint32_t r = 0;
      for (uint32_t f = 0; f < z; ++f) r += (zlog[f] & 0x7FFFFFFFu) < p ? 1u : 0u;
      atomicOr(&negBits[r >> 5], 1u << (r & 31));
    }
  }
  lds_barrier();
  const uint32_t s0 = *s_s0;
  uint32_t* dst = keys + start + w * CHUNK + lane;
  for (int j = 0; j < KPT; ++j) {
    if (j * 64 < lim) {
      const uint32_t r = w * CHUNK + 64 * j + lane - s0;
      dst[j * 64] = r < z ? (((negBits[r >> 5] >> (r & 31)) & 1u) ? 0x80000000u : 0u)
                          : kinv<2>(km, hiBits | (uint32_t)stw[j * LG::ROW]);
    }
  }
}

// The copy table of a non-stable first round (Loc16G::TC, thrs_local_kv):
// 256 digits x TC copies of their counters as 16-bit halves, word
// (d >> 1) * TC + copy, copy = lane % TC.  After the count, one exclusive
// scan in (digit, copy) order turns every counter into its copy's first slot;
// a returning add then hands each item its slot.  Every thread calls it (two
// barriers inside; the count's barrier is the caller's, before).
// thrs_local16 / thrs_local_kv: no half reaches 65536 (CAP < 65536).
template <int TC>
__device__ __forceinline__ void copy_table_scan(uint32_t* __restrict__ tbl, unsigned char* smem, uint32_t tid,
                                                uint32_t lane, uint32_t w) {
  // exclusive scan in (digit, copy) order: thread t < 128 owns digits 2t
  // (low halves) and 2t + 1 (high halves) of row t; the rows' totals are
  // scanned over the first two waves (stage words carry wave 0's total).
  // The row is read twice (sums, then prefixes + bases) so that no row stays
  // in registers across the barrier.
  uint32_t* s_wt = reinterpret_cast<uint32_t*>(smem);
  uint32_t t0 = 0, t1 = 0, tot = 0, inc = 0;
  uint4* row = reinterpret_cast<uint4*>(tbl + (tid & (kBins / 2 - 1)) * TC);
  if (tid < kBins / 2) {
#pragma unroll
    for (int q = 0; q < TC / 4; ++q) {
      const uint4 x = row[q];
      const uint32_t s4 = x.x + x.y + x.z + x.w;  // (four 16-bit halves each: no carry, every half < CAP)
      t0 += s4 & 0xFFFFu;
      t1 += s4 >> 16;
    }
    tot = t0 + t1;
    inc = wave_incl_scan(tot, lane);
    if (lane == 63 && w == 0) s_wt[0] = inc;
  }
  lds_barrier();
  if (tid < kBins / 2) {
    const uint32_t b0 = inc - tot + (w == 1 ? s_wt[0] : 0u), b1 = b0 + t0;  // digit 2t's base, digit 2t+1's
    uint32_t run = b0 | (b1 << 16);  // (every half stays below CAP < 65536: no carry between halves)
#pragma unroll
    for (int q = 0; q < TC / 4; ++q) {
      const uint4 x = row[q];
      uint4 y;
      y.x = run;
      run += x.x;
      y.y = run;
      run += x.y;
      y.z = run;
      run += x.z;
      y.w = run;
      run += x.w;
      row[q] = y;
    }
  }
  lds_barrier();
}
__device__ __forceinline__ uint32_t* copy_cell(uint32_t* tbl, uint32_t d, uint32_t cp, int tc) {
  return &tbl[(d >> 1) * (uint32_t)tc + cp];
}
__device__ __forceinline__ uint32_t copy_inc(uint32_t d) { return 1u << ((d & 1u) << 4); }

// thrs_local16's first round (the items' low byte) from the copy table
// (Loc16G::TC): count, scan, rank and scatter into the stage.  Every thread
// of the workgroup calls it; on return the stage holds the chunk's items
// ordered by their low byte (equal low bytes in no particular order) and a
// barrier is due before the stage is read.
template <typename LG>
__device__ __forceinline__ void local16_table_round(const uint32_t (&it)[LG::NP], uint32_t* __restrict__ tbl,
                                                    uint16_t* __restrict__ stage, unsigned char* smem, int nItems,
                                                    uint32_t lane, uint32_t tid, uint32_t w) {
  constexpr int KPT = LG::KPT, TC = LG::TC;
  constexpr uint32_t WORDS = (kBins / 2) * TC;
  auto digit_of = [&](int j) -> uint32_t { return (it[j >> 1] >> ((j & 1) * 16)) & 0xFFu; };
  const uint32_t cp = lane & (uint32_t)(TC - 1);
  for (uint32_t i = tid; i < WORDS / 4; i += LG::THREADS) reinterpret_cast<uint4*>(tbl)[i] = make_uint4(0, 0, 0, 0);
  lds_barrier();
  auto cell = [&](uint32_t d) -> uint32_t* { return &tbl[(d >> 1) * TC + cp]; };
  auto inc_of = [](uint32_t d) -> uint32_t { return 1u << ((d & 1u) << 4); };
  // (whole waves without per-item tests: see the second round's count)
  if (nItems == KPT) {
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      const uint32_t d = digit_of(j);
      __hip_atomic_fetch_add(cell(d), inc_of(d), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  } else {
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      const uint32_t d = digit_of(j);
      if (j < nItems) __hip_atomic_fetch_add(cell(d), inc_of(d), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  lds_barrier();
  copy_table_scan<TC>(tbl, smem, tid, lane, w);
  // rank (the returned half is the slot) + scatter, RB atomics in flight
  constexpr int RB = THRS_LOC_RB;
  auto rank_scatter = [&](auto fullc) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
    for (int j0 = 0; j0 < KPT; j0 += RB) {
      uint32_t sl[RB];
#pragma unroll
      for (int jj = 0; jj < RB; ++jj) {
        const int j = j0 + jj;
        if (j < KPT && (FULL || j < nItems)) {
          const uint32_t d = digit_of(j);
          sl[jj] = (__hip_atomic_fetch_add(cell(d), inc_of(d), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >>
                    ((d & 1u) << 4)) & 0xFFFFu;
        }
      }
#pragma unroll
      for (int jj = 0; jj < RB; ++jj) {
        const int j = j0 + jj;
        if (j < KPT && (FULL || j < nItems)) stage[LG::at(sl[jj])] = (uint16_t)((it[j >> 1] >> ((j & 1) * 16)) & 0xFFFFu);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  if (nItems == KPT) rank_scatter(std::true_type{});
  else rank_scatter(std::false_type{});
}

// One chunk of thrs_local16 under the key map km: the plain map, or the
// squeeze fixed to the chunk's image half (KeyMapHalf).  A device function on
// a plain branch, not a with_map lambda: the closure and the two-half map
// spilled the f32 kernel at its 80-VGPR budget (docs/EXPERIMENTS.md row 96).
template <int KT, bool ATOMIC_RANK, typename LG, typename KM>
__device__ __forceinline__ void local16_chunk(uint32_t* __restrict__ keys, KM km, uint32_t c, uint32_t start,
                                              uint32_t size, const uint32_t* __restrict__ chunkB0,
                                              const uint32_t* __restrict__ meta, const uint16_t* __restrict__ lo,
                                              const uint32_t* __restrict__ zeroLog) {
  constexpr int KPT = LG::KPT, NP = LG::NP;
  constexpr uint32_t CHUNK = 64 * KPT;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t hiBits = chunkB0[c] << 16;  // the bucket: the image's top 16 bits
  uint16_t* stage = reinterpret_cast<uint16_t*>(smem);
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(smem + LG::STAGE_BYTES);  // [waves][256]
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint32_t* cnt = s_cnt + w * kBins;
  const uint16_t* stw = stage + w * KPT * LG::ROW + lane;  // item j of this lane: stw[j * ROW]
  int32_t lim = (int32_t)size - (int32_t)(w * CHUNK + lane);
  pin(reinterpret_cast<uint32_t&>(lim));
  const int32_t limw = __builtin_amdgcn_readfirstlane((int32_t)size - (int32_t)(w * CHUNK));
  const int nItems = limw <= 0 ? 0 : min(KPT, (limw + 63) >> 6);  // items j with j*64 < limw
  uint32_t* src = keys + start + w * CHUNK + lane;

  // items: low 16 bits of the image, two per register; padding 0xFFFF ranks
  // after every real item (stable: it sits at the chunk's end)
  // (loads: load_run)
  // lo != nullptr: the top-digit passes wrote the image's low 16 bits to the
  // u16 plane lo (kCodecPlanes) -- unless both were skipped (mode 2: one
  // bucket holds every key), which leaves the keys in place
  uint32_t it[NP];
  // (in batches of LB items: a wide geometry's raw loads would not fit the
  // register budget at once)
  constexpr int LB = LG::LB;
  static_assert(KPT % LB == 0 && LB % 2 == 0, "load batches hold whole item pairs");
  if (lo && meta[kMetaMode] == 0) {
#pragma unroll
    for (int h = 0; h < KPT; h += LB) {
      uint16_t raw[LB];
      load_run<LB>(raw, lo + start, w * CHUNK + h * 64 + lane, size, limw - h * 64);
#pragma unroll
      for (int jj = 0; jj < LB; jj += 2) {
        const int j = h + jj;
        const uint32_t a = (j * 64 < lim) ? (uint32_t)raw[jj] : 0xFFFFu;
        const uint32_t b = (j + 1 < KPT && (j + 1) * 64 < lim) ? (uint32_t)raw[jj + 1] : 0xFFFFu;
        it[j >> 1] = a | (b << 16);
      }
    }
  } else {
#pragma unroll
    for (int h = 0; h < KPT; h += LB) {
      uint32_t raw[LB];
      load_run<LB>(raw, keys + start, w * CHUNK + h * 64 + lane, size, limw - h * 64);
#pragma unroll
      for (int jj = 0; jj < LB; jj += 2) {
        const int j = h + jj;
        const uint32_t a = (j * 64 < lim) ? (kimg<KT>(km, raw[jj]) & 0xFFFFu) : 0xFFFFu;
        const uint32_t b =
            (j + 1 < KPT && (j + 1) * 64 < lim) ? (kimg<KT>(km, raw[jj + 1]) & 0xFFFFu) : 0xFFFFu;
        it[j >> 1] = a | (b << 16);
      }
    }
  }
  auto item = [&](int j) -> uint32_t { return (it[j >> 1] >> ((j & 1) * 16)) & 0xFFFFu; };

  constexpr int TC = LG::TC;
  if constexpr (TC > 0) {  // the first round from the copy table (Loc16G): not stable, fewer bank conflicts
    local16_table_round<LG>(it, s_cnt, stage, smem, nItems, lane, tid, w);
    lds_barrier();
    if (limw >= (int32_t)CHUNK) {
#pragma unroll
      for (int j = 0; j < KPT; j += 2) {
        const uint32_t a = stw[j * LG::ROW];
        const uint32_t b = (j + 1 < KPT) ? (uint32_t)stw[(j + 1) * LG::ROW] : 0xFFFFu;
        it[j >> 1] = a | (b << 16);
      }
    } else {
#pragma unroll
      for (int j = 0; j < KPT; j += 2) {
        const uint32_t a = (j * 64 < limw) ? (uint32_t)stw[j * LG::ROW] : 0xFFFFu;
        const uint32_t b = (j + 1 < KPT && (j + 1) * 64 < limw) ? (uint32_t)stw[(j + 1) * LG::ROW] : 0xFFFFu;
        it[j >> 1] = a | (b << 16);
      }
    }
  }
  for (int r = TC > 0 ? 1 : 0; r < 2; ++r) {
    const int shift = 8 * r;
    auto digit_of = [&](int j) -> uint32_t { return (it[j >> 1] >> ((j & 1) * 16 + shift)) & 0xFFu; };
#pragma unroll
    for (int i = 0; i < kBins / 64; ++i) cnt[i * 64 + lane] = 0;
    // A wave whose KPT items all lie in the chunk (every wave but the chunk's
    // last) runs the loops below without per-item tests: a scalar branch
    // around an LDS atomic makes the compiler wait for every earlier one, so
    // the batched rank atomics would be issued one round trip apart.
    const bool wfull = nItems == KPT;
    if (wfull) {
#pragma unroll
      for (int j = 0; j < KPT; ++j)
        __hip_atomic_fetch_add(&cnt[digit_of(j)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
#pragma unroll
      for (int j = 0; j < KPT; ++j)
        if (j < nItems) __hip_atomic_fetch_add(&cnt[digit_of(j)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    lds_barrier();
    {  // digit totals over the waves -> block exclusive scan -> per-wave running offsets
      uint32_t* s_wt = reinterpret_cast<uint32_t*>(smem);  // stage words: free until the scatter
      uint32_t cw[LG::WAVES], tot = 0, inc = 0;
      if (tid < kBins) {
#pragma unroll
        for (int ww = 0; ww < LG::WAVES; ++ww) {
          cw[ww] = s_cnt[ww * kBins + tid];
          tot += cw[ww];
        }
        inc = wave_incl_scan(tot, lane);
        if (lane == 63) s_wt[w] = inc;
      }
      lds_barrier();
      if (tid < kBins) {
        const uint32_t w0 = s_wt[0], w1 = s_wt[1], w2 = s_wt[2];
        uint32_t run = inc - tot + (w > 0 ? w0 : 0u) + (w > 1 ? w1 : 0u) + (w > 2 ? w2 : 0u);
#pragma unroll
        for (int ww = 0; ww < LG::WAVES; ++ww) {
          s_cnt[ww * kBins + tid] = run;
          run += cw[ww];
        }
      }
    }
    lds_barrier();
    constexpr int RB = THRS_LOC_RB;
    auto rank_scatter = [&](auto fullc) __attribute__((always_inline)) {
      constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
      for (int j0 = 0; j0 < KPT; j0 += RB) {
        uint32_t sl[RB];
#pragma unroll
        for (int jj = 0; jj < RB; ++jj) {
          const int j = j0 + jj;
          if (j < KPT && (FULL || j < nItems)) sl[jj] = wave_rank<ATOMIC_RANK>(cnt, digit_of(j), lane, false);
        }
#pragma unroll
        for (int jj = 0; jj < RB; ++jj)
          if (j0 + jj < KPT && (FULL || j0 + jj < nItems)) stage[LG::at(sl[jj])] = (uint16_t)item(j0 + jj);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if (wfull) rank_scatter(std::true_type{});
    else rank_scatter(std::false_type{});
    lds_barrier();
    if (r == 0) {
      if (limw >= (int32_t)CHUNK) {  // the wave's whole run is in the chunk: plain reads
#pragma unroll
        for (int j = 0; j < KPT; j += 2) {
          const uint32_t a = stw[j * LG::ROW];
          const uint32_t b = (j + 1 < KPT) ? (uint32_t)stw[(j + 1) * LG::ROW] : 0xFFFFu;
          it[j >> 1] = a | (b << 16);
        }
      } else {
#pragma unroll
        for (int j = 0; j < KPT; j += 2) {
          const uint32_t a = (j * 64 < limw) ? (uint32_t)stw[j * LG::ROW] : 0xFFFFu;
          const uint32_t b = (j + 1 < KPT && (j + 1) * 64 < limw) ? (uint32_t)stw[(j + 1) * LG::ROW] : 0xFFFFu;
          it[j >> 1] = a | (b << 16);
        }
      }
    }
  }
  if constexpr (KT == 2) {
    // f32: +0 and -0 share one image Z, so the chunk of Z's bucket takes its
    // zeros' bit patterns from the input, in input order (their stable order)
    // -- unless the keys came as planes (mode 0): then the signs of up to
    // kZeroLogCap zeros are in the zero log (none -0: every zero is +0, as
    // kinv rebuilds it)
    if ((kimg<2>(km, 0u) >> 16) == chunkB0[c]) {
      if (!(lo && meta[kMetaMode] == 0)) {
        loc16_write_zero_chunk<LG>(keys, km, start, size, hiBits, smem);
        return;
      }
      if (zeroLog && meta[kMetaNegZero]) {
        loc16_write_zero_log<LG>(keys, km, start, size, hiBits, smem, zeroLog, meta[kMetaZeroCount]);
        return;
      }
    }
  }
  // every stage read first (in bounds for all lanes), then the lane-conditional
  // stores: a read inside the condition would be waited for one at a time.
  // f32 without a key range: the inverse map on one chunk is linear in the
  // item -- key = k0 ^ item (k0 = the key of item 0), or k0 ^ (item >> 1) in
  // a squeezed half (its items keep bit 0 clear; the bits below the dropped
  // one move down by one): one or two operations per key instead of the
  // float transform and the squeeze.  (u32: the general inverse, already one
  // to three operations, in a loop of its own -- a lambda costs registers.)
  if constexpr (KT != 2) {
#pragma unroll
    for (int h = 0; h < KPT; h += LB) {
      uint32_t o[LB];
#pragma unroll
      for (int jj = 0; jj < LB; ++jj) o[jj] = stw[(h + jj) * LG::ROW];
#pragma unroll
      for (int jj = 0; jj < LB; ++jj)
        if ((h + jj) * 64 < lim) src[(h + jj) * 64] = kinv<KT>(km, hiBits | o[jj]);
    }
  } else {
    auto write_all = [&](auto mode) __attribute__((always_inline)) {
      constexpr int MODE = decltype(mode)::value;  // 0: general, 1: k0 ^ item, 2: k0 ^ (item >> 1)
      const uint32_t k0 = kinv<KT>(km, hiBits);
#pragma unroll
      for (int h = 0; h < KPT; h += LB) {
        uint32_t o[LB];
#pragma unroll
        for (int jj = 0; jj < LB; ++jj) o[jj] = stw[(h + jj) * LG::ROW];
#pragma unroll
        for (int jj = 0; jj < LB; ++jj)
          if ((h + jj) * 64 < lim)
            src[(h + jj) * 64] = MODE == 0 ? kinv<KT>(km, hiBits | o[jj]) : MODE == 1 ? k0 ^ o[jj] : k0 ^ (o[jj] >> 1);
      }
    };
    bool sqh = false;
    if constexpr (!std::is_same<KM, KeyMap<uint32_t>>::value) sqh = km.lm != 0u;
    if (km.sh != 0u || km.lo != 0u) write_all(std::integral_constant<int, 0>{});
    else if (sqh) write_all(std::integral_constant<int, 2>{});
    else write_all(std::integral_constant<int, 1>{});
  }
}

template <int KT, bool ATOMIC_RANK, typename LG>
__global__ __launch_bounds__(LG::THREADS) __attribute__((amdgpu_waves_per_eu(LG::WPE))) void thrs_local16(uint32_t* __restrict__ keys, KeyMap<uint32_t> kmh,
                                                            const uint32_t* __restrict__ chunkOff,
                                                            const uint32_t* __restrict__ chunkB0,
                                                            const uint32_t* __restrict__ meta,
                                                            const uint16_t* __restrict__ lo,
                                                            const SqueezeWords* __restrict__ sq,
                                                            const uint32_t* __restrict__ zeroLog) {
  const uint32_t c = blockIdx.x;
  if (c >= meta[kMetaChunks]) return;
  const uint32_t start = chunkOff[c], size = chunkOff[c + 1] - start;
  if (size == 0 || size > LG::CAP) return;  // big chunk: the per-bucket fallback sorts it
  if constexpr (kSqueezable<KT>) {
    if (sq && sq->on) {
      const int h = (int)(chunkB0[c] >> 15);  // the chunk's image half
      local16_chunk<KT, ATOMIC_RANK, LG>(keys, half_map(kmh, sq, h), c, start, size, chunkB0, meta, lo, zeroLog);
      return;
    }
  }
  local16_chunk<KT, ATOMIC_RANK, LG>(keys, kmh, c, start, size, chunkB0, meta, lo, zeroLog);
}

// ------------------------------------------- local sort, counting (keys only)
// The same chunks as thrs_local16 (u32 keys without values over the whole key,
// single-bucket chunks), sorted by COUNTING instead of two LSD rounds: without
// values, equal 16-bit items are indistinguishable, so a chunk's sorted order
// is fully described by how often each of the 65536 item values occurs.
// Per chunk (one 1024-thread workgroup per CU, persistent):
//   1. count   one no-return LDS add per key into 65536 16-bit counters (two
//              per word, 128 KiB; a chunk holds <= 18432 keys, so no field
//              overflows); a wave whose 64 items are equal adds 64 once
//   2. scan    thread t owns counter words [32t, 32t + 32) (values 64t ..
//              64t + 63): a running sum in registers, one block scan of the
//              thread totals; every word is zeroed as it is read.  Words are
//              rotated within their 32-word row (cnt_at) so that the 64 lanes
//              reading "their j-th word" hit distinct banks
//   3. marks   for each present value v with output offset o: stage[o] = v
//              (the stage is the first 36 KiB of the zeroed counters)
//   4. fill    an inclusive MAX scan over the stage fills the runs of equal
//              items (values ascend with the position, unmarked slots are 0);
//              the keys are rebuilt from the bucket and written coalesced
// LDS work is ~4 counter words per key instead of two rounds of count / scan
// / rank / scatter; the next chunk's items are loaded during this one (its
// offsets one chunk earlier still).  Every global load and store is
// unconditional (clamped loads; a lane past the chunk stores the chunk's last
// key again, which the max scan carries there, or -- empty chunk -- writes
// the sink), so the compiler's vmcnt waits count exactly and the prefetch
// stays in flight.
struct LocCount {
  static constexpr int THREADS = 1024, WAVES = 16, ITEMS = 18;
  static constexpr uint32_t CAP = (uint32_t)THREADS * ITEMS;     // 18432
  static constexpr uint32_t WORDS = kBuckets / 2;                // counters: two 16-bit fields per word
  static constexpr int ROWW = (int)(WORDS / THREADS);            // 32 words per thread
  static constexpr uint32_t WAVE_SLOTS = CAP / WAVES;            // 1152 stage slots per wave in step 4
  static constexpr size_t LDS = (size_t)WORDS * 4;               // 128 KiB
  __device__ static uint32_t cnt_at(uint32_t word) {             // rotate within the 32-word row
    return (word & ~31u) | ((word + (word >> 5)) & 31u);
  }
};
static_assert(LocCount::CAP == Loc16::CAP, "same chunk capacity as thrs_local16 (thrs_plan's cap)");
static_assert(LocCount::CAP / 2 <= LocCount::WORDS, "the stage fits in the counter words");
static_assert(LocCount::ROWW == 32, "cnt_at rotates 32-word rows");

__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppRowShr | 1, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppRowShr | 2, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppRowShr | 4, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppRowShr | 8, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppRowBcast15, 0xa, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppRowBcast31, 0xc, 0xf, false));
  return x;
}

// PLANE: items from the u16 plane `lo` (the key-planes codecs), else the low
// 16 bits of the keys' images in place.  sink: >= 64 * ITEMS words of scratch
// nobody reads (the bucket histogram, consumed by thrs_plan before this launch).
template <bool PLANE>
__global__ __launch_bounds__(LocCount::THREADS) void thrs_local_count16(
    uint32_t* __restrict__ keys, uint32_t n, KeyMap<uint32_t> km, const uint32_t* __restrict__ chunkOff,
    const uint32_t* __restrict__ chunkB0, const uint32_t* __restrict__ meta, const uint16_t* __restrict__ lo,
    uint32_t* __restrict__ sink) {
  using LC = LocCount;
  constexpr int IT = LC::ITEMS, RW = LC::ROWW;
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  const uint32_t nChunks = meta[kMetaChunks];
  // the planes exist in mode 0 only (mode 1, big chunks: the top passes
  // carried full keys)
  const bool plane = PLANE && meta[kMetaMode] == 0;
  if (blockIdx.x >= nChunks) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* cnt = reinterpret_cast<uint32_t*>(smem);
  uint16_t* stage = reinterpret_cast<uint16_t*>(smem);
  __shared__ uint32_t s_wsum[LC::WAVES], s_wmax[LC::WAVES];
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t G = gridDim.x;

  for (uint32_t i = tid; i < LC::WORDS / 4; i += LC::THREADS)
    reinterpret_cast<uint4*>(cnt)[i] = make_uint4(0, 0, 0, 0);
  lds_barrier();  // every counter zero before the first chunk's adds

  // item k of thread tid = chunk position 1024k + tid (64 consecutive per wave)
  // (indices built from loop-variant bases: per-item constants hoisted out of
  // the chunk loop would pin 18 registers each)
  // Raw loads only: whether item k exists is decided where it is used.
  // Addresses are a scalar chunk base plus a 32-bit byte offset (one VGPR).
  auto load_items = [&](uint32_t (&nx)[IT], uint32_t st, uint32_t sz) __attribute__((always_inline)) {
    const uint32_t last = sz ? sz - 1 : 0u;
    const size_t b = sz ? st : 0u;  // an empty chunk may start at n: read key 0 instead
    const char* base = plane ? reinterpret_cast<const char*>(lo + b) : reinterpret_cast<const char*>(keys + b);
    uint32_t r0 = tid;
    pin(r0);
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const uint32_t off = min(r0 + (uint32_t)k * LC::THREADS, last) * (plane ? 2u : 4u);
      if (plane) nx[k] = *reinterpret_cast<const uint16_t*>(base + off);
      else nx[k] = *reinterpret_cast<const uint32_t*>(base + off);
    }
  };
  // Two register sets, A and B, in turn: chunk i is counted from one while
  // chunk i+1 loads into the other (a single set would be copied at the loop
  // latch, which waits for the loads -- and the stores issued after them).
  uint32_t A[IT], B[IT];
  uint32_t c = blockIdx.x;
  uint32_t nStart = chunkOff[c], nSize = chunkOff[c + 1] - nStart, nHi = chunkB0[c];
  load_items(A, nStart, nSize);
  uint32_t c2 = min(c + G, nChunks - 1);
  uint32_t mStart = chunkOff[c2], mEnd = chunkOff[c2 + 1], mHi = chunkB0[c2];

  auto body = [&](uint32_t (&it)[IT], uint32_t (&nx)[IT]) __attribute__((always_inline)) {
    // a big chunk (the per-bucket fallback sorts it) takes the empty-chunk branch
    const uint32_t start = nStart, size = nSize > LC::CAP ? 0u : nSize, hiBits = nHi << 16;
    // the next chunk's items in flight during this one (clamped: always a
    // valid load); the one after that: its offsets
    nStart = mStart;
    nSize = mEnd - mStart;
    nHi = mHi;
    load_items(nx, nStart, nSize);
    c2 = min(c + 2 * G, nChunks - 1);
    mStart = chunkOff[c2];
    mEnd = chunkOff[c2 + 1];
    mHi = chunkB0[c2];

    if (size != 0) {
      // 1. count
      uint32_t rc = tid;
      pin(rc);
#pragma unroll
      for (int k = 0; k < IT; ++k) {
        const uint32_t v = rc + (uint32_t)k * LC::THREADS < size ? (plane ? it[k] : kimg<0>(km, it[k]) & 0xFFFFu) : NONE;
        const bool uni = __all(__builtin_amdgcn_readfirstlane(v) == v);
        const uint32_t add = uni ? (lane == 0 ? 64u : 0u) : 1u;
        if (v != NONE && add != 0)
          __hip_atomic_fetch_add(&cnt[LC::cnt_at(v >> 1)], add << ((v & 1u) * 16), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      lds_barrier();
      // 2. scan: this thread's 32 words in value order, zeroed as read
      uint32_t cw[RW], run = 0;
      uint32_t rt = tid;
      pin(rt);  // opaque per chunk: the 32 word addresses are not hoisted out of the chunk loop
#pragma unroll
      for (int j = 0; j < RW; ++j) {
        const uint32_t a = rt * RW + ((uint32_t)j + rt) % RW;  // cnt_at(32 tid + j)
        cw[j] = cnt[a];
        cnt[a] = 0;
      }
#pragma unroll
      for (int j = 0; j < RW; ++j) run += (cw[j] & 0xFFFFu) + (cw[j] >> 16);
      for (int j = 0; j < RW; ++j) pin(cw[j]);  // else the fields are split into 64 registers (spills)
      const uint32_t inc = wave_incl_scan(run, lane);
      if (lane == 63) s_wsum[w] = inc;
      lds_barrier();
      uint32_t o = inc - run;
#pragma unroll
      for (int ww = 0; ww < LC::WAVES - 1; ++ww) o += ww < (int)w ? s_wsum[ww] : 0u;
      // 3. marks
#pragma unroll
      for (int j = 0; j < RW; ++j) {
        const uint32_t a = cw[j] & 0xFFFFu, b = cw[j] >> 16, v0 = 2 * (rt * RW + j);
        if (a) stage[o] = (uint16_t)v0;
        o += a;
        if (b) stage[o] = (uint16_t)(v0 + 1);
        o += b;
      }
      lds_barrier();
      // 4a. read this wave's stage slots, their max, zero them for the next chunk
      const uint16_t* sw = stage + w * LC::WAVE_SLOTS + lane;
      uint32_t y[IT], m = 0;
#pragma unroll
      for (int k = 0; k < IT; ++k) {
        y[k] = sw[64 * k];
        m = max(m, y[k]);
      }
      m = lane63(wave_incl_max(m));
      if (lane == 0) s_wmax[w] = m;
      uint32_t* zw = cnt + w * (LC::WAVE_SLOTS / 2) + lane;
#pragma unroll
      for (int j = 0; j < (int)(LC::WAVE_SLOTS / 128); ++j) zw[64 * j] = 0;
      lds_barrier();
      // 4b. max scan and write-out (every store unconditional, see above)
      uint32_t carry = 0;
#pragma unroll
      for (int ww = 0; ww < LC::WAVES - 1; ++ww) carry = max(carry, ww < (int)w ? s_wmax[ww] : 0u);
      char* const dbase = reinterpret_cast<char*>(keys + start);
      uint32_t d0 = w * LC::WAVE_SLOTS + lane;
      pin(d0);
#pragma unroll
      for (int k = 0; k < IT; ++k) {
        const uint32_t x = max(wave_incl_max(y[k]), carry);
        carry = lane63(x);
        *reinterpret_cast<uint32_t*>(dbase + min(d0 + 64u * k, size - 1) * 4u) = kinv_int(km, hiBits | x);
      }
    } else {
      // empty chunk: as many (dummy) stores as a full one, so the vmcnt
      // waits on the prefetched items are the same on both paths
#pragma unroll
      for (int k = 0; k < IT; ++k) sink[64 * k + lane] = k;
    }
  };
  for (;;) {
    body(A, B);
    c += G;
    if (c >= nChunks) break;
    body(B, A);
    c += G;
    if (c >= nChunks) break;
  }
}

// ------------------------------------------------------ local sort, pairs
// sortPairs with u32 / f32 keys and 4-byte values over the whole key (startBits 0,
// 32 bits): chunks are single buckets (thrs_plan single mode), so a key is
// (bucket << 16 | low16) in image space and needs only its low 16 bits plus
// its chunk position to be carried: item = low16 << 16 | position (positions
// < 18432 < 2^16).  The rounds sort the items by their top 16 bits, exactly
// as the keys-only rounds (stable, lane-ordered rank); then the keys are
// rebuilt from the bucket and written, and the values are permuted through
// the same LDS stage by the carried positions.  f32 keys (+0 and -0 share one
// image, so they cannot be rebuilt bit-exactly) are permuted the same way.
// thrs_local_pairs' items: low 16 image bits << 16 | chunk position.  (A
// function, not a with_map lambda: the closure costs registers.)
// plane: it[] holds the u16 plane's entries (the images' low 16 bits) already
template <int KT, int KPT, typename KM>
__device__ __forceinline__ void pairs_items(uint32_t (&it)[KPT], KM km, uint32_t myOff, int32_t lim, bool plane = false) {
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint32_t pos = myOff + j * 64;
    const uint32_t lo16 = plane ? it[j] : (uint32_t)kimg<KT>(km, it[j]);
    it[j] = (j * 64 < lim) ? ((lo16 << 16) | pos) : 0xFFFF0000u;  // padding: digits 255
  }
}

// f32 pairs from the key planes (mode 0) after a -0 was seen: the chunk of
// +0's image takes its zeros' signs from the zero log, by loc16_write_zero_log's
// rule (a zero's rank among the zeros = logged zeros at smaller input
// positions: their stable order).  stage: the chunk's sorted items (image low
// 16 bits << 16 | position); leaves the signs in negBits[kZeroLogCap / 32] and
// returns the zeros' first slot.  Every thread of the workgroup calls it.
template <typename LG>
__device__ __forceinline__ uint32_t pairs_zero_signs(const uint32_t* stage, uint32_t size, uint32_t zlo,
                                                               uint32_t* negBits, const uint32_t* __restrict__ zlog,
                                                               uint32_t z) {
  constexpr uint32_t CHUNK = 64 * LG::KPT;
  static_assert(kZeroLogCap / 32 + 1 <= (uint32_t)LG::WAVES * kBins, "sign bits fit the counters' LDS");
  uint32_t* s_s0 = negBits + kZeroLogCap / 32;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (uint32_t i = tid; i < kZeroLogCap / 32 + 1; i += LG::THREADS) negBits[i] = 0;
  lds_barrier();
  uint32_t below = 0;  // sorted items below the zeros' item: the run's start
  for (int j = 0; j < LG::KPT; ++j) {
    const uint32_t slot = w * CHUNK + 64 * j + lane;
    if (slot < size) below += (stage[slot] >> 16) < zlo ? 1u : 0u;
  }
  atomicAdd(s_s0, below);
  for (uint32_t e = tid; e < z; e += LG::THREADS) {
    const uint32_t x = zlog[e];
    if (x >> 31) {
      const uint32_t p = x & 0x7FFFFFFFu;
      uint32_t r = 0;
      for (uint32_t f = 0; f < z; ++f) r += (zlog[f] & 0x7FFFFFFFu) < p ? 1u : 0u;
      atomicOr(&negBits[r >> 5], 1u << (r & 31));
    }
  }
  lds_barrier();
  return *s_s0;
}

template <int KT, bool ATOMIC_RANK, typename LG>
__global__ __launch_bounds__(LG::THREADS) __attribute__((amdgpu_waves_per_eu(LG::WPE))) void thrs_local_pairs(
    uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, KeyMap<uint32_t> km,
    const uint32_t* __restrict__ chunkOff, const uint32_t* __restrict__ chunkB0, const uint32_t* __restrict__ meta,
    const SqueezeWords* __restrict__ sq, const uint32_t* __restrict__ zeroFlag, const uint16_t* __restrict__ lo,
    const uint32_t* __restrict__ zeroLog) {
  constexpr int KPT = LG::KPT;
  constexpr uint32_t CHUNK = 64 * KPT;
  const uint32_t c = blockIdx.x;
  const uint32_t nChunks = meta[kMetaChunks];
  if (c >= nChunks) return;
  LocChunk ch;
  ch.start = chunkOff[c];
  ch.size = chunkOff[c + 1] - ch.start;
  if (ch.size == 0 || ch.size > LG::CAP) return;  // big chunk: the per-bucket fallback sorts it
  ch.b0 = 0;
  ch.rounds = 2;  // single-bucket chunk: the two low digits of the key = the item's top 16 bits
  const uint32_t hiImg = chunkB0[c] << 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int32_t lim = (int32_t)ch.size - (int32_t)(w * CHUNK + lane);
  pin(reinterpret_cast<uint32_t&>(lim));
  uint32_t* ksrc = keys + ch.start + w * CHUNK + lane;
  uint32_t* vsrc = vals + ch.start + w * CHUNK + lane;
  // loads unconditional and clamped into the chunk (see loc_load)
  const uint32_t myOff = w * CHUNK + lane;
  const int32_t avail = __builtin_amdgcn_readfirstlane((int32_t)ch.size - (int32_t)(w * CHUNK));
  uint32_t it[KPT];
  // lo != nullptr: the top-digit passes wrote the images' low 16 bits to the
  // u16 plane lo (kCodecPlanes) -- unless they ran on whole keys (mode 1, big
  // chunks; mode 3, f32 with a -0 among more zeros than the zero log holds)
  // or not at all (mode 2), which leaves the keys
  const bool plane = lo && meta[kMetaMode] == 0;
  if (plane) load_run<KPT>(it, lo + ch.start, myOff, ch.size, avail);
  else load_run<KPT>(it, keys + ch.start, myOff, ch.size, avail);
  if constexpr (kSqueezable<KT>) {
    // (the squeeze, f32 keys: only the items' images depend on it; the
    // plane holds squeezed images already)
    if (!plane && sq && sq->on) pairs_items<KT, KPT>(it, half_map(km, sq, (int)(hiImg >> 31)), myOff, lim);
    else pairs_items<KT, KPT>(it, km, myOff, lim, plane);
  } else {
    pairs_items<KT, KPT>(it, km, myOff, lim, plane);
  }
  loc_rounds<0, ATOMIC_RANK, LG>(it, ch, KeyMap<uint32_t>{0u, 0u, 0u}, 16, 2, smem, nullptr);
  pin(reinterpret_cast<uint32_t&>(lim));
  // values of this thread's positions (the item registers are free again;
  // loading them with the keys would spill: EXPERIMENTS row 31)
  load_run<KPT>(it, vals + ch.start, myOff, ch.size, avail);
  uint32_t* stage = reinterpret_cast<uint32_t*>(smem);
  const uint32_t* stw = stage + w * CHUNK + lane;
  // f32 keys: rebuilt from the bucket and the items, like u32 keys, unless
  // whole keys crossed the passes and the input holds a -0 (thrs_hist_joint's
  // flag; +0 and -0 share one image): then they travel by position like the
  // values.  From the planes (mode 0) they are always rebuilt, and the chunk
  // of +0's image takes the zeros' signs from the zero log (at most
  // kZeroLogCap zeros: thrs_plan_rows takes mode 3 above that).  The chunk's
  // image half fixes the squeeze's masks (scalars).
  const bool negZero = KT == 2 && zeroFlag && load_agent(zeroFlag) != 0u;
  const bool f32Rebuild = KT == 2 && zeroFlag && (plane || !negZero);
  uint32_t hm2 = ~0u, lm2 = 0u, cs2 = 0u;
  bool zfix = false;
  uint32_t zlo = 0, zs0 = 0;
  const uint32_t* negBits = stage + LG::CAP;  // (the rounds' counters: free now)
  if constexpr (KT == 2) {
    const bool sqOn = sq && sq->on;
    if (sqOn) {
      const int hh = (int)(hiImg >> 31);
      hm2 = (uint32_t)sq->hiM[hh];
      lm2 = (uint32_t)sq->loM[hh];
      cs2 = (uint32_t)sq->cst[hh];
    }
    if (plane && negZero && zeroLog) {
      const uint32_t zimg = sqOn ? (uint32_t)kimg<2>(half_map(km, sq, (int)(hiImg >> 31)), 0u) : kimg<2>(km, 0u);
      if ((zimg >> 16) == (hiImg >> 16)) {  // (uniform over the workgroup)
        zfix = true;
        zlo = zimg & 0xFFFFu;
        zs0 = pairs_zero_signs<LG>(stage, ch.size, zlo, stage + LG::CAP, zeroLog,
                                   min(meta[kMetaZeroCount], kZeroLogCap));
      }
    }
  }
  auto f32_key = [&](uint32_t y) -> uint32_t {
    y = (y & hm2) | ((y >> 1) & lm2) | cs2;
    return unbits32<2>(((y >> km.sh) + km.lo) ^ km.mask);
  };
  uint32_t id[(KPT + 1) / 2];  // carried positions, two 16-bit halves per register
#pragma unroll
  for (int j = 0; j < (KPT + 1) / 2; ++j) id[j] = 0;
  // sorted items read in batches (reads unconditional, stores lane-conditional)
  constexpr int BR = 12;
#pragma unroll
  for (int j0 = 0; j0 < KPT; j0 += BR) {
    uint32_t o[BR];
#pragma unroll
    for (int jj = 0; jj < BR; ++jj)
      if (j0 + jj < KPT) o[jj] = stw[(j0 + jj) * 64];
#pragma unroll
    for (int jj = 0; jj < BR; ++jj) {
      const int j = j0 + jj;
      if (j < KPT) {
        id[j / 2] |= (j * 64 < lim ? (o[jj] & 0xFFFFu) : 0u) << (16 * (j & 1));
        if (KT == 0 && j * 64 < lim) ksrc[j * 64] = kinv_int(km, hiImg | (o[jj] >> 16));
        if (KT == 2 && f32Rebuild && j * 64 < lim) {
          uint32_t key = f32_key(hiImg | (o[jj] >> 16));
          if (zfix && (o[jj] >> 16) == zlo) {
            const uint32_t r = w * CHUNK + 64 * j + lane - zs0;
            key = ((negBits[r >> 5] >> (r & 31)) & 1u) ? 0x80000000u : 0u;
          }
          ksrc[j * 64] = key;
        }
      }
    }
  }
  lds_barrier();  // every sorted item has been read: the stage takes the values
#pragma unroll
  for (int j = 0; j < KPT; ++j)
    if (j * 64 < lim) stage[w * CHUNK + j * 64 + lane] = it[j];
  lds_barrier();
#pragma unroll
  for (int j0 = 0; j0 < KPT; j0 += BR) {
    uint32_t o[BR];
#pragma unroll
    for (int jj = 0; jj < BR; ++jj)
      if (j0 + jj < KPT) o[jj] = stage[(id[(j0 + jj) / 2] >> (16 * ((j0 + jj) & 1))) & 0xFFFFu];
#pragma unroll
    for (int jj = 0; jj < BR; ++jj)
      if (j0 + jj < KPT && (j0 + jj) * 64 < lim) vsrc[(j0 + jj) * 64] = o[jj];
  }
  if (KT == 2 && !f32Rebuild) {
    // f32 keys travel by position like the values (+0 and -0 share one image)
    load_run<KPT>(it, keys + ch.start, myOff, ch.size, avail);
    lds_barrier();  // every value read from the stage
#pragma unroll
    for (int j = 0; j < KPT; ++j)
      if (j * 64 < lim) stage[w * CHUNK + j * 64 + lane] = it[j];
    lds_barrier();
#pragma unroll
    for (int j0 = 0; j0 < KPT; j0 += BR) {
      uint32_t o[BR];
#pragma unroll
      for (int jj = 0; jj < BR; ++jj)
        if (j0 + jj < KPT) o[jj] = stage[(id[(j0 + jj) / 2] >> (16 * ((j0 + jj) & 1))) & 0xFFFFu];
#pragma unroll
      for (int jj = 0; jj < BR; ++jj)
        if (j0 + jj < KPT && (j0 + jj) * 64 < lim) ksrc[(j0 + jj) * 64] = o[jj];
    }
  }
}

// ------------------------------------ local sort, carried positions (wide)
// Full-window sorts whose keys or values cannot take the 16-bit or 32-bit
// item kernels above: 8-byte keys (u64 / f64) with no, 4-, 8- or 16-byte
// values, and 4-byte keys (u32 / f32) with 8- or 16-byte values.  Chunks are
// single buckets (the top 16 bits of the image).  Item = the image's bits
// below the bucket << 16 | chunk position (positions < 17408 < 2^16): 32-bit
// items and two in-LDS rounds for 4-byte keys, 64-bit items and six rounds
// for 8-byte keys -- stable count / scan / lane-ordered rank / scatter /
// reload as loc_rounds.  The carried position then permutes, through the
// LDS stage, what cannot be rebuilt from the item: the values, and float
// keys (+0 and -0 share one image).  u32 / u64 keys are rebuilt from the
// bucket and the item.  16-byte values are loaded and stored whole (one
// 16-B access per lane, full lines) and pass the 8-byte stage in two halves.
// Geometries (W waves x 17 items, 8 bytes of LDS stage per slot + W x 1 KiB
// of per-wave counters; 17 items per lane in every one, so the same 128-VGPR
// budget at four waves per SIMD):
//   LocKV   16 x 17 = 17408 slots, 152 KiB, one workgroup per CU: buckets of
//           2^30-key sorts (~16K keys)
//   LocKVM   8 x 17 =  8704 slots,  76 KiB, two per CU: up to 2^29 keys
//   LocKVS   4 x 17 =  4352 slots,  38 KiB, four per CU: up to 3 x 2^26 keys
// (the per-chunk fixed cost -- barriers, scans, counter zeroing -- is what a
// bucket far below its chunk's capacity pays, and one workgroup per CU
// exposes every barrier: docs/EXPERIMENTS.md row 130)
// (8 waves x 34 items, 248 VGPRs at two waves per SIMD: u64 keys 5.76 vs
// 5.00 ms, C5 shape 7.82 vs 7.29 -- docs/EXPERIMENTS.md row 116)
template <int W> struct LocKVG {
  static constexpr int WAVES = W, KPT = 17, THREADS = 64 * WAVES, WPE = 4;
  static constexpr uint32_t CAP = (uint32_t)THREADS * KPT;
  static constexpr size_t LDS = (size_t)CAP * 8 + (size_t)WAVES * kBins * 4;
  static_assert(W >= 4, "the scans take the first 256 threads");
};
using LocKV = LocKVG<16>;
using LocKVM = LocKVG<8>;
using LocKVS = LocKVG<4>;
static_assert(LocKV::CAP < 65536, "positions are carried in 16 bits");
constexpr int kTieScan = 32;  // thrs_local_kv: longest tie run the fix-up walks

// One stable LDS round of thrs_local_kv on the item bits [shift, shift + 8)
// of it[] (32- or 64-bit items): count (per-wave counters), scan, lane-ordered
// rank, scatter into st (sorted order).  Items past nItems of the wave are
// not there; the counters sit after the 64-bit stage.
template <bool ATOMIC_RANK, typename LK, typename Item>
__device__ __forceinline__ void kv_round(Item (&it)[LK::KPT], Item* st, int shift, unsigned char* smem, int nItems) {
  constexpr int KPT = LK::KPT, W = LK::WAVES;
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(smem + (size_t)LK::CAP * 8);  // [W][256]
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint32_t* cnt = s_cnt + w * kBins;
  const bool wfull = nItems == KPT;  // whole wave: no per-item tests (see loc_rounds)
  auto digit_of = [&](int j) -> uint32_t { return (uint32_t)(it[j] >> shift) & 0xFFu; };
#pragma unroll
  for (int i = 0; i < kBins / 64; ++i) cnt[i * 64 + lane] = 0;
  if (wfull) {
#pragma unroll
    for (int j = 0; j < KPT; ++j)
      __hip_atomic_fetch_add(&cnt[digit_of(j)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
#pragma unroll
    for (int j = 0; j < KPT; ++j)
      if (j < nItems) __hip_atomic_fetch_add(&cnt[digit_of(j)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  lds_barrier();
  {  // digit totals over the waves -> block exclusive scan -> per-wave running offsets
    uint32_t* s_wt = reinterpret_cast<uint32_t*>(smem);  // stage words: reloaded into registers before each round
    uint32_t cw[W], tot = 0, inc = 0;
    if (tid < kBins) {
#pragma unroll
      for (int ww = 0; ww < W; ++ww) {
        cw[ww] = s_cnt[ww * kBins + tid];
        tot += cw[ww];
      }
      inc = wave_incl_scan(tot, lane);
      if (lane == 63) s_wt[w] = inc;
    }
    lds_barrier();
    if (tid < kBins) {
      const uint32_t w0 = s_wt[0], w1 = s_wt[1], w2 = s_wt[2];
      uint32_t run = inc - tot + (w > 0 ? w0 : 0u) + (w > 1 ? w1 : 0u) + (w > 2 ? w2 : 0u);
#pragma unroll
      for (int ww = 0; ww < W; ++ww) {
        s_cnt[ww * kBins + tid] = run;
        run += cw[ww];
      }
    }
  }
  lds_barrier();
  constexpr int RB = 9;
  auto rank_scatter = [&](auto fullc) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
    for (int j0 = 0; j0 < KPT; j0 += RB) {
      uint32_t sl[RB];
#pragma unroll
      for (int jj = 0; jj < RB; ++jj) {
        const int j = j0 + jj;
        if (j < KPT && (FULL || j < nItems)) sl[jj] = wave_rank<ATOMIC_RANK>(cnt, digit_of(j), lane, false);
      }
#pragma unroll
      for (int jj = 0; jj < RB; ++jj)
        if (j0 + jj < KPT && (FULL || j0 + jj < nItems)) st[sl[jj]] = it[j0 + jj];
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  if (wfull) rank_scatter(std::true_type{});
  else rank_scatter(std::false_type{});
  lds_barrier();
}

// thrs_local_kv, 8-byte keys, a tie run longer than kTieScan: from the
// 32-bit items sorted by the 16 bits below the bucket (stage st) and the
// image's low 32 bits (low[position]), back to input order as 64-bit items
// (the image's low 48 bits << 16 | position) in the same LDS seen as one
// 64-bit stage, then six rounds; leaves the sorted items in that stage.  A
// call (not inlined): the caller's live registers (prefetched values) are
// saved around it instead of squeezing the six rounds.
template <bool ATOMIC_RANK, typename LK>
__device__ __noinline__ void kv8_six_rounds(unsigned char* smem, uint32_t size) {
  constexpr int KPT = LK::KPT;
  constexpr uint32_t CHUNK = 64 * KPT;
  const uint32_t* st = reinterpret_cast<const uint32_t*>(smem);
  const uint32_t* low = st + LK::CAP;
  uint64_t* st64 = reinterpret_cast<uint64_t*>(smem);
  const uint32_t lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t myOff = w * CHUNK + lane;
  const int32_t lim = (int32_t)size - (int32_t)myOff;
  const int32_t limw = __builtin_amdgcn_readfirstlane((int32_t)size - (int32_t)(w * CHUNK));
  const int nItems = limw <= 0 ? 0 : min(KPT, (limw + 63) >> 6);
  uint64_t it[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint32_t v = st[myOff + j * 64];
    it[j] = ((uint64_t)(v >> 16) << 48) | ((uint64_t)low[v & 0xFFFFu] << 16) | (v & 0xFFFFu);
  }
  lds_barrier();
#pragma unroll
  for (int j = 0; j < KPT; ++j)  // back to the input order (the position field)
    if (myOff + 64 * j < size) st64[(uint32_t)(it[j] & 0xFFFFu)] = it[j];
  lds_barrier();
#pragma unroll
  for (int j = 0; j < KPT; ++j)
    if (j < nItems) it[j] = (j * 64 < lim) ? st64[myOff + j * 64] : ~(uint64_t)0xFFFF;
  for (int r = 0; r < 6; ++r) {
    kv_round<ATOMIC_RANK, LK>(it, st64, 16 + 8 * r, smem, nItems);
    if (r < 5) {
#pragma unroll
      for (int j = 0; j < KPT; ++j)
        if (j < nItems) it[j] = st64[myOff + j * 64];
    }
  }
}

// One chunk of thrs_local_kv under the key map km (plain, or the squeeze).
// A device function, not a lambda handed to with_map: the closure cost the
// 8-byte-key kernel 12 spilled VGPRs (C5 shape local sort 9.6 -> 11.1 ms).
template <int KT, int VB, bool ATOMIC_RANK, typename LK, typename KM>
__device__ __forceinline__ void local_kv_chunk(typename KeyTraits<KT>::U* __restrict__ keys,
                                               typename ValueWord<VB>::T* __restrict__ vals, KM km, uint32_t c,
                                               uint32_t start, uint32_t size, const uint32_t* __restrict__ chunkB0,
                                               uint64_t* stp) {
  using U = typename KeyTraits<KT>::U;
  constexpr int KB = (int)sizeof(U);
  using Item = typename std::conditional<KB == 4, uint32_t, uint64_t>::type;
  constexpr int KPT = LK::KPT;
  constexpr uint32_t CHUNK = 64 * KPT;
  // Float keys are rebuilt from their images like integer keys, except in
  // the chunk holding +0's image: -0 shares it, so that chunk's keys travel
  // by position (permuted through the stage).  (All float chunks permuted
  // their keys -- a second, unprefetched load -- until row 114.)
  bool permKeys = false;
  if constexpr (KT == 2 || KT == 3)
    permKeys = (uint32_t)(kimg<KT>(km, (typename KeyTraits<KT>::U)0) >> (8 * sizeof(typename KeyTraits<KT>::U) - 16)) ==
               chunkB0[c];
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const U hiImg = (U)chunkB0[c] << (8 * KB - 16);  // the bucket: the image's top 16 bits
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t myOff = w * CHUNK + lane;
  int32_t lim = (int32_t)size - (int32_t)myOff;
  pin(reinterpret_cast<uint32_t&>(lim));
  const int32_t limw = __builtin_amdgcn_readfirstlane((int32_t)size - (int32_t)(w * CHUNK));
  const int nItems = limw <= 0 ? 0 : min(KPT, (limw + 63) >> 6);  // items j with j*64 < limw

  const bool wfull = nItems == KPT;  // whole wave: no per-item tests (see loc_rounds)
  auto round = [&](auto& it, auto* st, int shift) __attribute__((always_inline)) {
    kv_round<ATOMIC_RANK, LK>(it, st, shift, smem, nItems);
  };
  auto reload = [&](auto& it, const auto* st) __attribute__((always_inline)) {  // this lane's slots (past the chunk: padding)
    if (wfull) {
#pragma unroll
      for (int j = 0; j < KPT; ++j) it[j] = st[myOff + j * 64];
    } else {
#pragma unroll
      for (int j = 0; j < KPT; ++j)
        if (j < nItems) it[j] = st[myOff + j * 64];
    }
  };
  // 4- / 8-byte values with integer keys: loaded now, used after the sort
  // (the loads land while the workgroup works in LDS)
  // (f64 keys with 8-byte values: the prefetched values spill ~25 VGPRs at
  // the 128-VGPR cap, so those load theirs after the sort)
  constexpr bool PREFETCH = (VB == 4 || VB == 8) && !(KT == 3 && VB == 8);
  using VW = typename ValueWord<VB>::T;
  VW xv[PREFETCH ? KPT : 1];
  // the sorted chunk, per output slot myOff + 64j: the image below the
  // bucket, and the input position
  Item img[KPT];
  uint32_t pos[(KPT + 1) / 2];
  if constexpr (KB == 4) {
    // items: the image's low 16 bits << 16 | position; padding (past the
    // chunk) sorts last (stable: it sits at the end)
    uint32_t it[KPT];
    {
      U raw[KPT];
      load_run<KPT>(raw, keys + start, myOff, size, limw);
      if constexpr (PREFETCH) load_run<KPT>(xv, vals + start, myOff, size, limw);
#pragma unroll
      for (int j = 0; j < KPT; ++j)
        it[j] = (j * 64 < lim) ? ((uint32_t)kimg<KT>(km, raw[j]) << 16) | (myOff + j * 64) : 0xFFFF0000u;
    }
    uint32_t* st = reinterpret_cast<uint32_t*>(smem);
    round(it, st, 16);
    reload(it, st);
    round(it, st, 24);
#pragma unroll
    for (int j = 0; j < KPT; ++j) it[j] = st[myOff + j * 64];
#pragma unroll
    for (int j = 0; j < KPT; ++j) img[j] = it[j] >> 16;
#pragma unroll
    for (int j = 0; j < (KPT + 1) / 2; ++j) pos[j] = 0;
#pragma unroll
    for (int j = 0; j < KPT; ++j) pos[j / 2] |= (it[j] & 0xFFFFu) << (16 * (j & 1));
  } else {
    // 8-byte keys.  Items are 32-bit: the 16 image bits below the bucket
    // (bits 32..47) << 16 | position; the image's low 32 bits wait in LDS
    // (low[position]).  Two rounds sort by those 16 bits; then each run of
    // items sharing them (random keys: ~1 item in 4 is in one, mostly pairs)
    // is insertion-sorted in place by its first slot's thread on (low bits,
    // position): stable.  Runs are disjoint, and a thread reading a
    // neighbouring run mid-sort still sees that run's 16 bits.  A run longer
    // than kTieScan makes the workgroup restore the input order and take six
    // rounds on 64-bit items (the image's low 48 bits << 16 | position), in
    // the same LDS seen as one 64-bit stage.
    uint32_t* st = reinterpret_cast<uint32_t*>(smem);
    uint32_t* low = st + LK::CAP;
    uint64_t* st64 = reinterpret_cast<uint64_t*>(smem);
    __shared__ uint32_t s_over;
    if (tid == 0) s_over = 0;  // (the rounds' barriers order this before any set)
    uint32_t it[KPT];
    {
      U raw[KPT];
      load_run<KPT>(raw, keys + start, myOff, size, limw);
      if constexpr (PREFETCH) load_run<KPT>(xv, vals + start, myOff, size, limw);
#pragma unroll
      for (int j = 0; j < KPT; ++j) {
        const uint64_t im = kimg<KT>(km, raw[j]);
        const uint32_t p = myOff + j * 64;
        if (j * 64 < lim) low[p] = (uint32_t)im;
        it[j] = (j * 64 < lim) ? ((uint32_t)(im >> 32) << 16) | p : 0xFFFF0000u | p;
      }
    }
    loc_stamp(stp, 1);
    round(it, st, 16);
    reload(it, st);
    round(it, st, 24);
    loc_stamp(stp, 2);
    auto pre_of = [&](uint32_t slot) -> uint32_t { return st[slot] >> 16; };
    auto key_of = [&](uint32_t v) -> uint64_t { return ((uint64_t)low[v & 0xFFFFu] << 16) | (v & 0xFFFFu); };
    bool over = false;
    // The runs' first slots among this lane's slots (neighbours read FB
    // slots at a time: independent loads, one wait) as a bit mask; then
    // each lane walks its own runs (random keys: ~1.7 per lane, a few lanes
    // with 5-6).  A run of up to four items -- all but ~1 run in 10^4 -- is
    // sorted by a four-input network in registers (items past the run rank
    // last), a longer one insertion-sorted.  (Per-slot predicated code for
    // the runs cost ~7000 instructions per wave -- the fix-up was issue-bound
    // at 13 us per chunk; docs/EXPERIMENTS.md row 111.)
    auto sort_run = [&](uint32_t h, uint32_t pre) __attribute__((always_inline)) {
      uint32_t e = h + 5;  // (h .. h + 4 are in the run)
      while (e < size && e - h <= (uint32_t)kTieScan && pre_of(e) == pre) ++e;
      if (e - h > (uint32_t)kTieScan) {
        over = true;
        return;
      }
      for (uint32_t i = h + 1; i < e; ++i) {
        const uint32_t x = st[i];
        const uint64_t kx = key_of(x);
        uint32_t j = i;
        for (; j > h && key_of(st[j - 1]) > kx; --j) st[j] = st[j - 1];
        st[j] = x;
      }
    };
    auto cx = [](uint64_t& x, uint64_t& y) __attribute__((always_inline)) {
      const uint64_t lo = x < y ? x : y, hi = x < y ? y : x;
      x = lo;
      y = hi;
    };
    static_assert(LK::KPT <= 64, "one mask bit per slot of the lane");
    uint64_t fm = 0;
    constexpr int FB = 6;
#pragma unroll
    for (int j0 = 0; j0 < KPT; j0 += FB) {
      uint32_t c[FB], pv[FB], n1[FB];
#pragma unroll
      for (int jj = 0; jj < FB; ++jj) {
        if (j0 + jj < KPT) {  // (st[s + 1] <= st[CAP]: the low words, in the LDS)
          const uint32_t s = myOff + 64 * (j0 + jj);
          c[jj] = st[s];
          pv[jj] = st[s == 0 ? 0u : s - 1];
          n1[jj] = st[s + 1];
        }
      }
#pragma unroll
      for (int jj = 0; jj < FB; ++jj) {
        if (j0 + jj < KPT) {
          const uint32_t s = myOff + 64 * (j0 + jj), pre = c[jj] >> 16;
          const bool f = s + 1 < size && (n1[jj] >> 16) == pre && (s == 0 || (pv[jj] >> 16) != pre);
          fm |= (f ? 1ull : 0ull) << (j0 + jj);
        }
      }
    }
    auto fix_run = [&](uint32_t h) __attribute__((always_inline)) {
      // (h + 1 < size <= CAP: h + 4 <= CAP + 2, in the LDS)
      const uint32_t w0 = st[h], w1 = st[h + 1], w2 = st[h + 2], w3 = st[h + 3], w4 = st[h + 4];
      const uint32_t pre = w0 >> 16;
      const bool m2 = h + 2 < size && (w2 >> 16) == pre;
      const bool m3 = m2 && h + 3 < size && (w3 >> 16) == pre;
      if (m3 && h + 4 < size && (w4 >> 16) == pre) {
        sort_run(h, pre);
        return;
      }
      constexpr uint32_t PMAX = LK::CAP - 1;  // (a slot past the run may hold anything)
      const uint32_t l0 = low[w0 & 0xFFFFu], l1 = low[w1 & 0xFFFFu];
      const uint32_t l2 = low[min(w2 & 0xFFFFu, PMAX)], l3 = low[min(w3 & 0xFFFFu, PMAX)];
      uint64_t k0 = ((uint64_t)l0 << 16) | (w0 & 0xFFFFu), k1 = ((uint64_t)l1 << 16) | (w1 & 0xFFFFu);
      uint64_t k2 = m2 ? ((uint64_t)l2 << 16) | (w2 & 0xFFFFu) : ~(uint64_t)0;
      uint64_t k3 = m3 ? ((uint64_t)l3 << 16) | (w3 & 0xFFFFu) : ~(uint64_t)0;
      cx(k0, k1);
      cx(k2, k3);
      cx(k0, k2);
      cx(k1, k3);
      cx(k1, k2);
      const uint32_t hi = w0 & 0xFFFF0000u;
      st[h] = hi | (uint32_t)(k0 & 0xFFFFu);
      st[h + 1] = hi | (uint32_t)(k1 & 0xFFFFu);
      if (m2) st[h + 2] = hi | (uint32_t)(k2 & 0xFFFFu);
      if (m3) st[h + 3] = hi | (uint32_t)(k3 & 0xFFFFu);
    };
    {
      // the wave's runs listed in its (now free) counter words, then taken
      // one per lane: ~2 passes instead of the busiest lane's ~6 runs
      uint32_t* list = reinterpret_cast<uint32_t*>(smem + (size_t)LK::CAP * 8) + w * kBins;
      const uint32_t cnt = (uint32_t)__builtin_popcountll(fm);
      const uint32_t incl = wave_incl_scan(cnt, lane);
      const uint32_t R = min(lane63(incl), (uint32_t)kBins);
      uint32_t k = incl - cnt;
      uint64_t f = fm;
      while (f && k < (uint32_t)kBins) {
        const uint32_t j = (uint32_t)__builtin_ctzll(f);
        f &= f - 1;
        list[k++] = myOff + 64u * j;
        fm &= ~(1ull << j);
      }
      for (uint32_t i = lane; i < R; i += 64) fix_run(list[i]);
    }
    while (fm) {  // (more runs than list words: the rest by their own lane)
      const uint32_t h = myOff + 64u * (uint32_t)__builtin_ctzll(fm);
      fm &= fm - 1;
      fix_run(h);
    }
    if (over) s_over = 1;  // (every writer stores 1)
    lds_barrier();
    loc_stamp(stp, 3);
    if (s_over == 0) {
#pragma unroll
      for (int j = 0; j < KPT; ++j) it[j] = st[myOff + j * 64];
#pragma unroll
      for (int j = 0; j < KPT; ++j) img[j] = ((uint64_t)(it[j] >> 16) << 32) | low[it[j] & 0xFFFFu];
#pragma unroll
      for (int j = 0; j < (KPT + 1) / 2; ++j) pos[j] = 0;
#pragma unroll
      for (int j = 0; j < KPT; ++j) pos[j / 2] |= (it[j] & 0xFFFFu) << (16 * (j & 1));
    } else {
      kv8_six_rounds<ATOMIC_RANK, LK>(smem, size);  // (a call: its registers are its own)
#pragma unroll
      for (int j = 0; j < KPT; ++j) {
        const uint64_t v = st64[myOff + j * 64];
        img[j] = v >> 16;
      }
#pragma unroll
      for (int j = 0; j < (KPT + 1) / 2; ++j) pos[j] = 0;
#pragma unroll
      for (int j = 0; j < KPT; ++j) pos[j / 2] |= (uint32_t)(st64[myOff + j * 64] & 0xFFFFu) << (16 * (j & 1));
    }
  }
  loc_stamp(stp, 4);
  U* kdst = keys + start + myOff;
  if (!permKeys) {
#pragma unroll
    for (int j = 0; j < KPT; ++j)
      if (j * 64 < lim) kdst[j * 64] = kinv_key<KT>(km, (U)(hiImg | (U)img[j]));  // rebuilt from the image
  }
  loc_stamp(stp, 5);
  // carried positions: two 16-bit halves per register
  auto pos_of = [&](int j) -> uint32_t { return (pos[j / 2] >> (16 * (j & 1))) & 0xFFFFu; };
  // out[j] = in[pos_of(j)] through the stage, for T of 4 or 8 bytes
  auto permute = [&](auto* arr, auto pre) {
    using T = typename std::remove_pointer<decltype(arr)>::type;
    T* st = reinterpret_cast<T*>(smem);
    T x[KPT];
    if constexpr (std::is_same<decltype(pre), std::nullptr_t>::value) load_run<KPT>(x, arr + start, myOff, size, limw);
    else {
#pragma unroll
      for (int j = 0; j < KPT; ++j) x[j] = pre[j];
    }
    lds_barrier();  // every stage read of the previous step is done
#pragma unroll
    for (int j = 0; j < KPT; ++j)
      if (j < nItems) st[myOff + j * 64] = x[j];
    lds_barrier();
#pragma unroll
    for (int j = 0; j < KPT; ++j) x[j] = st[pos_of(j)];
#pragma unroll
    for (int j = 0; j < KPT; ++j)
      if (j * 64 < lim) arr[start + myOff + j * 64] = x[j];
  };
  if (permKeys) permute(keys, nullptr);
  if constexpr (PREFETCH) permute(vals, xv);
  else if constexpr (VB == 4 || VB == 8) permute(vals, nullptr);
  if constexpr (VB == 16) {
    // whole 16-byte values in registers; the halves pass the stage in turn
    uint4 x[KPT];
    load_run<KPT>(x, reinterpret_cast<const uint4*>(vals) + start, myOff, size, limw);
    uint64_t* st = reinterpret_cast<uint64_t*>(smem);
    uint64_t o[KPT];
    lds_barrier();
#pragma unroll
    for (int j = 0; j < KPT; ++j)
      if (j < nItems) st[myOff + j * 64] = ((uint64_t)x[j].y << 32) | x[j].x;
    lds_barrier();
#pragma unroll
    for (int j = 0; j < KPT; ++j) o[j] = st[pos_of(j)];
    lds_barrier();
#pragma unroll
    for (int j = 0; j < KPT; ++j)
      if (j < nItems) st[myOff + j * 64] = ((uint64_t)x[j].w << 32) | x[j].z;
    lds_barrier();
    uint4* vdst = reinterpret_cast<uint4*>(vals) + start + myOff;
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      const uint64_t h = st[pos_of(j)];
      if (j * 64 < lim) vdst[j * 64] = make_uint4((uint32_t)o[j], (uint32_t)(o[j] >> 32), (uint32_t)h, (uint32_t)(h >> 32));
    }
  }
#ifdef THRS_STAMPS
  if (stp) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    loc_stamp(stp, 6);
    if (threadIdx.x == 0) {
      uint32_t hw;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      stp[7] = hw;
    }
  }
#endif
}

template <int KT, int VB, bool ATOMIC_RANK, typename LK = LocKV>
__global__ __launch_bounds__(LK::THREADS) __attribute__((amdgpu_waves_per_eu(LK::WPE))) void thrs_local_kv(
    typename KeyTraits<KT>::U* __restrict__ keys,
                                                                typename ValueWord<VB>::T* __restrict__ vals,
                                                                KeyMap<typename KeyTraits<KT>::U> kmh,
                                                                const uint32_t* __restrict__ chunkOff,
                                                                const uint32_t* __restrict__ chunkB0,
                                                                const uint32_t* __restrict__ meta,
                                                                const SqueezeWords* __restrict__ sq,
                                                                uint64_t* __restrict__ stamps) {
  using U = typename KeyTraits<KT>::U;
  constexpr int KB = (int)sizeof(U);
  static_assert(KB == 8 || VB >= 8, "4-byte keys with 0 / 4-byte values: thrs_local16 / thrs_local / thrs_local_pairs");
  const uint32_t c = blockIdx.x;
  if (c >= meta[kMetaChunks]) return;
  const uint32_t start = chunkOff[c], size = chunkOff[c + 1] - start;
  if (size == 0 || size > LK::CAP) return;  // big chunk: the per-bucket fallback sorts it
  uint64_t* st = stamps ? stamps + (uint64_t)c * kLocStampSlots : nullptr;
  loc_stamp(st, 0);
  if constexpr (kSqueezable<KT>) {
    if (sq && sq->on) {  // (the squeeze fixed to the chunk's image half: fewer scalars, as thrs_local16)
      const int h = (int)(chunkB0[c] >> 15);
      local_kv_chunk<KT, VB, ATOMIC_RANK, LK>(keys, vals, half_map(kmh, sq, h), c, start, size, chunkB0, st);
      return;
    }
  }
  local_kv_chunk<KT, VB, ATOMIC_RANK, LK>(keys, vals, kmh, c, start, size, chunkB0, st);
}

}  // namespace
}  // namespace thrs_dev
