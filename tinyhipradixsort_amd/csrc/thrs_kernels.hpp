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

#include <type_traits>

namespace thrs_dev {
// (internal linkage: every translation unit of libthrs.so gets its own copy
// of the kernels it launches)
namespace {

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

// The image a sort orders by: getKeyBits (above) XOR the descending mask
// (kernel.cu:18-24), optionally restated on a range the caller promises
// (thrs_options.keyRange -- the multi-GPU finish, where a rank's keys lie in a
// known [lo, hi]):  img(k) = ((getKeyBits(k) ^ mask) - lo) << sh, sh = the
// leading zero bits of hi - lo.  On the range it is monotone and one-to-one,
// so sorting by img is sorting by the key, and the range's keys fill the
// whole image width (the bucket path's 16-bit buckets stay balanced).
// Without a range lo = sh = 0.
//
// SQ = true adds a SQUEEZE chosen on the device from the data (float keys on
// the bucket path, thrs_plan_rows): in each half of the image space (top
// image bit h) one bit b that every key of that half has at the same value
// (cst[h]) is dropped and the bits below it move up by one:
//   img' = (img & hiM[h]) | ((img & loM[h]) << 1),  hiM = ~(2^(b+1) - 1),
//   loM = 2^b - 1  (identity: hiM = ~0, loM = 0).
// Monotone and one-to-one on the keys of that half (the dropped bit is the
// same for all of them) and the top bit stays, so the order is unchanged; the
// 16-bit buckets then take one more varying bit.  The reference's own float
// generator clears the lowest exponent bit of every key (unittest.cpp:103,
// 108), which is such a bit: without the squeeze half the buckets are empty.
// (kernel-argument structs: every field has a default initialiser and there
// is no implicit padding, so a struct the host fills field by field never
// carries indeterminate bytes; tests/cpp/struct_init.cpp checks both)
template <typename U, bool SQ = false> struct KeyMap {
  U mask = 0;
  U lo = 0;
  uint32_t sh = 0;
  uint32_t pad = 0;
};
template <typename U> struct KeyMap<U, true> {
  U mask = 0;
  U lo = 0;
  uint32_t sh = 0;
  uint32_t pad = 0;
  U hiM[2] = {}, loM[2] = {}, cst[2] = {};
};
// the squeeze as thrs_plan_rows (or the sample, thrs_squeeze_sample) writes
// it: on, and per half the masks and the dropped bit's value (cst)
struct SqueezeWords {
  uint32_t on = 0, pad = 0;
  uint64_t hiM[2] = {}, loM[2] = {}, cst[2] = {};
};
template <int KT> constexpr bool kSqueezable = KT == 2 || KT == 3;  // float keys
template <typename U> __device__ __forceinline__ KeyMap<U, true> with_squeeze(const KeyMap<U>& m,
                                                                              const SqueezeWords* s) {
  KeyMap<U, true> r;
  r.mask = m.mask;
  r.lo = m.lo;
  r.sh = m.sh;
  for (int h = 0; h < 2; ++h) {
    r.hiM[h] = (U)s->hiM[h];
    r.loM[h] = (U)s->loM[h];
    r.cst[h] = (U)s->cst[h];
  }
  return r;
}
// body(km) with the host's map, or with the device-chosen squeeze when
// thrs_plan_rows switched it on (float keys only: compiled out otherwise)
template <int KT, typename F>
__device__ __forceinline__ void with_map(const KeyMap<typename KeyTraits<KT>::U>& km, const SqueezeWords* sq,
                                         F&& body) {
  if constexpr (kSqueezable<KT>) {
    if (sq && sq->on) {
      body(with_squeeze(km, sq));
      return;
    }
  }
  body(km);
}
template <int KT, bool SQ>
__device__ __forceinline__ typename KeyTraits<KT>::U kimg(const KeyMap<typename KeyTraits<KT>::U, SQ>& m,
                                                          typename KeyTraits<KT>::U k) {
  using U = typename KeyTraits<KT>::U;
  U y = ((KeyTraits<KT>::bits(k) ^ m.mask) - m.lo) << m.sh;
  if constexpr (SQ) {
    const bool h = (y >> (8 * sizeof(U) - 1)) != 0;
    y = (y & (h ? m.hiM[1] : m.hiM[0])) | ((y & (h ? m.loM[1] : m.loM[0])) << 1);
  }
  return y;
}
// the key whose image is y (u32 / u64: getKeyBits is the identity)
template <typename U, bool SQ> __device__ __forceinline__ U kinv_int(const KeyMap<U, SQ>& m, U y) {
  if constexpr (SQ) {
    const bool h = (y >> (8 * sizeof(U) - 1)) != 0;
    y = (y & (h ? m.hiM[1] : m.hiM[0])) | ((y >> 1) & (h ? m.loM[1] : m.loM[0])) | (h ? m.cst[1] : m.cst[0]);
  }
  return ((y >> m.sh) + m.lo) ^ m.mask;
}
// The squeeze fixed to ONE image half (a local sort's chunk lies in one
// half: its bucket holds the half bit): scalars instead of per-key selects
// between the halves' masks, and fewer of them (the 80-VGPR local sort
// spilled with the two-half map's scalars, docs/EXPERIMENTS.md row 96).
template <typename U> struct KeyMapHalf {
  U mask;
  U lo;
  uint32_t sh;
  U hm, lm, cs;  // the half's hiM, loM, cst
};
template <typename U> __device__ __forceinline__ KeyMapHalf<U> half_map(const KeyMap<U>& m, const SqueezeWords* s, int h) {
  KeyMapHalf<U> r;
  r.mask = m.mask;
  r.lo = m.lo;
  r.sh = m.sh;
  r.hm = (U)(h ? s->hiM[1] : s->hiM[0]);
  r.lm = (U)(h ? s->loM[1] : s->loM[0]);
  r.cs = (U)(h ? s->cst[1] : s->cst[0]);
  return r;
}
template <int KT>
__device__ __forceinline__ typename KeyTraits<KT>::U kimg(const KeyMapHalf<typename KeyTraits<KT>::U>& m,
                                                          typename KeyTraits<KT>::U k) {
  using U = typename KeyTraits<KT>::U;
  const U y = ((KeyTraits<KT>::bits(k) ^ m.mask) - m.lo) << m.sh;
  return (y & m.hm) | ((y & m.lm) << 1);
}
template <typename U> __device__ __forceinline__ U kinv_int(const KeyMapHalf<U>& m, U y) {
  y = (y & m.hm) | ((y >> 1) & m.lm) | m.cs;
  return ((y >> m.sh) + m.lo) ^ m.mask;
}
// raw 4-byte key whose getKeyBits image is y (inverse of KeyTraits::bits, for
// images that do not come from -0: -0 and +0 have one image, this gives +0)
template <int KT> __device__ __forceinline__ uint32_t unbits32(uint32_t y) {
  if constexpr (KT == 2) return (y & 0x80000000u) ? (y ^ 0x80000000u) : ~y;
  else return y;
}
// the 4-byte key whose image (under m) is y
template <int KT, bool SQ> __device__ __forceinline__ uint32_t kinv(const KeyMap<uint32_t, SQ>& m, uint32_t y) {
  return unbits32<KT>(kinv_int(m, y));
}
template <int KT> __device__ __forceinline__ uint32_t kinv(const KeyMapHalf<uint32_t>& m, uint32_t y) {
  return unbits32<KT>(kinv_int(m, y));
}

// raw 8-byte key whose getKeyBits image is y (f64: as unbits32)
template <int KT> __device__ __forceinline__ uint64_t unbits64(uint64_t y) {
  if constexpr (KT == 3) return (y >> 63) ? (y ^ 0x8000000000000000ull) : ~y;
  else return y;
}
// the key of any type whose image (under m: KeyMap or KeyMapHalf) is y
template <int KT, typename M, typename U> __device__ __forceinline__ U kinv_key(const M& m, U y) {
  if constexpr (sizeof(U) == 4) return unbits32<KT>(kinv_int(m, y));
  else return unbits64<KT>(kinv_int(m, y));
}

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

// Opaque redefinition of a register value: computations that depend on x
// cannot be hoisted above this point (the compiler otherwise precomputes every
// item's digit and LDS address up front and spills).
__device__ __forceinline__ void pin(uint32_t& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(uint64_t& x) { asm volatile("" : "+v"(x)); }

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

// ---- wave-aggregated LDS counting and ranking.  Conflicting lanes of one
// LDS atomic are serviced one per cycle: when all 64 lanes of a wave carry the
// same digit (sorted, reverse-sorted and constant inputs do this on most
// items) a per-lane atomic costs 64 cycles of the CU's LDS pipe.  A wave
// classifies its N items once (wave_mode, scalar result):
//   kAllUniform  every item of every lane has the digit d0: one atomic of
//                64*N for the whole wave, slots base + 64j + lane;
//   kSomeUniform its first or last item is uniform (a wave straddling a digit
//                boundary of sorted input): each item is tested (one ballot)
//                and a uniform one takes one atomic of 64 from lane 0;
//   kMixed       random input: one atomic per lane and item, no extra test.
// Every lane of the wave is active in all of these.
enum : uint32_t { kMixed = 0, kSomeUniform = 1, kAllUniform = 2 };

__device__ __forceinline__ bool wave_uniform(uint32_t d) {
  const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d);
  return __ballot(d == d0) == ~0ull;
}
// items j in [0, nItems) (wave-uniform, >= 1) take part; d0 = item 0's digit in lane 0
template <int N, typename F>
__device__ __forceinline__ uint32_t wave_mode(F digit, int nItems, uint32_t& d0) {
  d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)digit(0));
  uint32_t diff = 0;
#pragma unroll
  for (int j = 0; j < N; ++j)
    if (j < nItems) diff |= digit(j) ^ d0;
  if (__ballot(diff != 0) == 0) return kAllUniform;
  bool some = wave_uniform(digit(0));
#pragma unroll
  for (int j = 1; j < N; ++j)
    if (j == nItems - 1) some = some || wave_uniform(digit(j));
  return some ? kSomeUniform : kMixed;
}

// true iff digit(j) is the same for every j < N in every lane; d0 = that digit
template <int N, typename F>
__device__ __forceinline__ bool wave_all_uniform(F digit, uint32_t& d0) {
  d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)digit(0));
  uint32_t diff = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) diff |= digit(j) ^ d0;
  return __ballot(diff != 0) == 0;
}

// cnt[d] += 1 for every lane; uni: d is the same in every lane
__device__ __forceinline__ void wave_count(uint32_t* cnt, uint32_t d, uint32_t lane, bool uni) {
  if (uni) {
    if (lane == 0) __hip_atomic_fetch_add(&cnt[d], 64u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
    __hip_atomic_fetch_add(&cnt[d], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}
// count items j in [0, nItems) of every lane, by mode
template <int N, typename F>
__device__ __forceinline__ void wave_count_items(uint32_t* cnt, uint32_t mode, uint32_t d0, uint32_t lane, F digit,
                                                 int nItems) {
  if (mode == kAllUniform) {
    if (lane == 0)
      __hip_atomic_fetch_add(&cnt[d0], 64u * (uint32_t)nItems, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else if (mode == kSomeUniform) {
#pragma unroll
    for (int j = 0; j < N; ++j)
      if (j < nItems) wave_count(cnt, digit(j), lane, wave_uniform(digit(j)));
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j)
      if (j < nItems) __hip_atomic_fetch_add(&cnt[digit(j)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// Stable rank of this lane's item among the wave's items with the same digit,
// added to (and advancing) the wave's running counter cnt[d]: the returned
// slot.  ATOMIC_RANK: one ds_add_rtn_u32 per lane, whose conflicting lanes
// return in lane order on gfx950 (probed per device, thrs_probe_lds_order);
// otherwise the 8-ballot match.  uni: slot = base + lane.
template <bool ATOMIC_RANK>
__device__ __forceinline__ uint32_t wave_rank(uint32_t* cnt, uint32_t d, uint32_t lane, bool uni) {
  if (uni) {
    uint32_t old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(&cnt[d], 64u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return (uint32_t)__builtin_amdgcn_readlane((int)old, 0) + lane;
  }
  if constexpr (ATOMIC_RANK) {
    return __hip_atomic_fetch_add(&cnt[d], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
    uint32_t mlo, mhi;
    match_digit(d, mlo, mhi);
    const uint32_t c = cnt[d];
    const uint32_t slot = __builtin_amdgcn_mbcnt_hi(mhi, __builtin_amdgcn_mbcnt_lo(mlo, c));
    cnt[d] = __builtin_popcount(mhi) + __builtin_popcount(mlo) + c;
    return slot;
  }
}
// kAllUniform: the wave's N items take slots base .. base + 64N (one atomic)
__device__ __forceinline__ uint32_t wave_rank_all(uint32_t* cnt, uint32_t d0, uint32_t lane, uint32_t items) {
  uint32_t old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(&cnt[d0], 64u * items, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return (uint32_t)__builtin_amdgcn_readlane((int)old, 0);
}

// Inclusive scan over the 64 lanes of a wave, in DPP (no LDS round trips:
// __shfl_up compiles to ds_bpermute, ~100+ cycles each): row_shr 1, 2, 4, 8
// scan each row of 16 lanes, then row_bcast:15 / row_bcast:31 carry rows
// 0 -> 1, 2 -> 3 and {0,1} -> {2,3}.  Lanes outside a DPP source keep 0.
constexpr int kDppRowShr = 0x110, kDppRowBcast15 = 0x142, kDppRowBcast31 = 0x143, kDppWaveShr1 = 0x138;
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, uint32_t lane) {
  (void)lane;
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppRowShr | 1, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppRowShr | 2, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppRowShr | 4, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppRowShr | 8, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppRowBcast15, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppRowBcast31, 0xc, 0xf, false);
  return x;
}
// value of the previous lane (lane 0: `first`), in DPP
__device__ __forceinline__ uint32_t wave_prev_lane(uint32_t x, uint32_t first) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)first, (int)x, kDppWaveShr1, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t lane63(uint32_t x) { return (uint32_t)__builtin_amdgcn_readlane((int)x, 63); }

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
// LDS layout [p][d][COPIES]: lane l always adds into copy (l % COPIES), so for
// COPIES = 32 the bank of every ds_add_u32 is l % 32 -- conflict-free whatever
// the digits are (random digits into one shared 256-bin table collide ~3-4 way
// per 32-lane half).  128 KiB of LDS -> one 1024-thread workgroup per CU (64 KiB of loads in flight);
// 64-bit keys (8 digits) use 16 copies.  Copies are summed once per workgroup
// and merged with one device-scope atomic per (p, bin).
constexpr int kHistThreads = 1024;
#ifndef THRS_HIST_COPIES
#define THRS_HIST_COPIES 32  // LDS copies per bin for 4-byte keys (8-byte keys: half)
#endif
#ifndef THRS_HIST_UNROLL
#define THRS_HIST_UNROLL 4   // 16-B loads in flight per lane
#endif
#ifndef THRS_HIST_GRID_MULT
#define THRS_HIST_GRID_MULT 1  // workgroups per CU
#endif
template <int KB> constexpr int hist_copies() { return KB == 4 ? THRS_HIST_COPIES : THRS_HIST_COPIES / 2; }
template <int KT>
__global__ __launch_bounds__(kHistThreads) void thrs_hist(const typename KeyTraits<KT>::U* __restrict__ keys,
                                                          uint32_t n, KeyMap<typename KeyTraits<KT>::U> km,
                                                          int startBits, int nPass, int vec,
                                                          uint32_t* __restrict__ hist) {
  using U = typename KeyTraits<KT>::U;
  constexpr int NP_MAX = sizeof(U);
  constexpr int COPIES = hist_copies<(int)sizeof(U)>();
  extern __shared__ __attribute__((aligned(16))) uint32_t s_hist[];  // [nPass][256][COPIES]
  const uint32_t tid = threadIdx.x;
  const uint32_t words = (uint32_t)nPass * kBins * COPIES;
  for (uint32_t i = tid; i < words; i += kHistThreads) s_hist[i] = 0;
  __syncthreads();
  uint32_t* my = s_hist + (tid % COPIES);

  auto count = [&](U k) {
    const U b = kimg<KT>(km, k);
#pragma unroll
    for (int p = 0; p < NP_MAX; ++p) {
      if (p < nPass) {
        const uint32_t d = (uint32_t)(b >> (startBits + 8 * p)) & 0xFFu;
        __hip_atomic_fetch_add(&my[(p * kBins + d) * COPIES], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  };

  const uint64_t gstride = (uint64_t)gridDim.x * kHistThreads;
  const uint64_t gtid = (uint64_t)blockIdx.x * kHistThreads + tid;
  uint64_t tailStart = 0;
  if (vec) {  // 16-byte loads, 4 in flight per lane; keys base is 16-B aligned (checked on host)
    constexpr int PER = 16 / sizeof(U);
    const uint64_t nv = n / PER;
    const uint4* kv = reinterpret_cast<const uint4*>(keys);
    uint64_t i = gtid;
    constexpr int UN = THRS_HIST_UNROLL;
    for (; i + (UN - 1) * gstride < nv; i += UN * gstride) {
      uint4 q[UN];
#pragma unroll
      for (int u = 0; u < UN; ++u) q[u] = kv[i + u * gstride];
#pragma unroll
      for (int u = 0; u < UN; ++u) {
        if constexpr (sizeof(U) == 4) {
          count(q[u].x); count(q[u].y); count(q[u].z); count(q[u].w);
        } else {
          count(((uint64_t)q[u].y << 32) | q[u].x);
          count(((uint64_t)q[u].w << 32) | q[u].z);
        }
      }
    }
    for (; i < nv; i += gstride) {
      const uint4 q = kv[i];
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
  for (uint32_t i = tid; i < (uint32_t)(nPass * kBins); i += kHistThreads) {
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < COPIES; ++c) s += s_hist[i * COPIES + ((c + i) % COPIES)];  // rotate: conflict-free reads
    if (s) atomicAdd(&hist[i], s);
  }
}

// Digit histograms of the keys matching a prefix, for up to
// kMaxHistTargets key ranges at once (multi-GPU split refinement: one launch
// per level for every boundary still being refined,
// tinyhipradixsort_amd/dist.py): counts[y][d] += #keys of range y whose
// transformed key t has (t & mask[y]) == value[y] and digit d at bit `shift`.
// blockIdx.y = the range.  One read, any alignment; LDS bins in 32
// bank-private copies (conflict-free whatever the skew), merged with one
// device atomic per bin and workgroup.
constexpr int kMaxHistTargets = 16;
struct HistTargets {
  uint64_t off[kMaxHistTargets] = {};
  uint64_t mask[kMaxHistTargets] = {};
  uint64_t value[kMaxHistTargets] = {};
  uint32_t n[kMaxHistTargets] = {};
};
template <typename U>
__global__ __launch_bounds__(kHistThreads) void thrs_digit_hist(const U* __restrict__ keys, HistTargets tg,
                                                                int keyType, U orderMask, int shift,
                                                                uint32_t* __restrict__ counts) {
  __shared__ uint32_t s_h[kBins * 32];
  const uint32_t tid = threadIdx.x, y = blockIdx.y;
  const U* kk = keys + tg.off[y];
  const uint32_t n = tg.n[y];
  const U prefixMask = (U)tg.mask[y], prefixValue = (U)tg.value[y];
  for (uint32_t i = tid; i < kBins * 32; i += kHistThreads) s_h[i] = 0;
  __syncthreads();
  uint32_t* my = s_h + (tid & 31);
  for (uint64_t i = (uint64_t)blockIdx.x * kHistThreads + tid; i < n; i += (uint64_t)gridDim.x * kHistThreads) {
    const U k = kk[i];
    U t;
    if constexpr (sizeof(U) == 4) t = (keyType == 2 ? KeyTraits<2>::bits(k) : k) ^ orderMask;
    else t = (keyType == 3 ? KeyTraits<3>::bits(k) : k) ^ orderMask;
    if ((t & prefixMask) == prefixValue)
      __hip_atomic_fetch_add(&my[(uint32_t)((t >> shift) & 0xFFu) * 32], 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  uint32_t* out = counts + (uint64_t)y * kBins;
  for (uint32_t b = tid; b < (uint32_t)kBins; b += kHistThreads) {
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) c += s_h[b * 32 + ((j + b) & 31)];
    if (c) atomicAdd(&out[b], c);
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
// Workgroup-local barrier that does NOT drain vector memory: every hand-off
// between the waves of a workgroup in thrs_pass goes through LDS, so only
// lgkmcnt must be zero.  (__syncthreads() also waits for vmcnt(0), which would
// park the workgroup on the in-flight look-back load and status store.)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Bound on the polls of a look-back or tile-claim wait (each poll sleeps ~64
// clocks): hitting it sets the sort's error word (thrs_capi.h "Device-side
// failures") instead of hanging the GPU.  -DTHRS_SPIN_MAX=0 builds the
// fault-injection library of the error-path tests (libthrs_spin0.so).
#ifndef THRS_SPIN_MAX
#define THRS_SPIN_MAX (1u << 22)
#endif
constexpr uint32_t kSpinMax = THRS_SPIN_MAX;

// Look-back window: predecessors read per round trip.
#ifndef THRS_LOOK_WINDOW
#define THRS_LOOK_WINDOW 8
#endif
constexpr int kLookWindow = THRS_LOOK_WINDOW;
// Two-level look-back (THRS_GROUP = tiles per group, 0 = flat per-tile chain).
// Every tile adds its digit counts to its group's aggregate row with one
// fire-and-forget atomic per digit; the word also counts arrivals, so a reader
// knows when the aggregate is complete:  ga = count | arrivals << 20.
// The last tile of a group publishes the group's inclusive prefix (gp).  A
// walker sums the rows of its own group's earlier tiles, then walks GROUP
// rows (kGroupWindow per round trip): a group prefix ends the walk, a complete
// aggregate skips THRS_GROUP tiles at once.  The walk depth in rows falls by
// about THRS_GROUP (docs/EXPERIMENTS.md).
#ifndef THRS_GROUP
#define THRS_GROUP 16
#endif
#ifndef THRS_GROUP_WINDOW
#define THRS_GROUP_WINDOW 8
#endif
constexpr int kGroup = THRS_GROUP;
constexpr int kStampSlots = 24;  // THRS_STAMPS diagnostics: u64 slots per tile
#ifdef THRS_STAMPS
constexpr uint32_t kStampLds = kStampSlots * 8;
#else
constexpr uint32_t kStampLds = 0;
#endif
constexpr int kGroupWindow = THRS_GROUP_WINDOW;
#ifndef THRS_TILE_WINDOW
#define THRS_TILE_WINDOW 8
#endif
constexpr int kTileWindow = THRS_TILE_WINDOW;  // own-group tile rows per round trip
constexpr uint32_t kArrival = 1u << 20;
// error word bits (the sort's temp buffer): a look-back / claim spin gave up;
// a run reserved past the output end was clamped
constexpr uint32_t kErrSpin = 1u, kErrRunClamped = 2u;
template <typename ST> struct GroupTables {
  uint32_t* ga = nullptr;  // [nGroups][256] count | arrivals << 20   (this pass)
  ST* gp = nullptr;        // [nGroups][256] Status<ST>::pre(inclusive prefix)
  uint32_t* gaNext = nullptr;  // next pass's tables, cleared by each group's last tile
  ST* gpNext = nullptr;
  uint32_t nTiles = 0;  // end of this tile's chain (tile ids)
  uint32_t gmin = 0;  // first group of this tile's chain (segmented passes)
};

#ifndef THRS_RANK_PIPE
#define THRS_RANK_PIPE 2  // pass rank: LDS atomics in flight per wave
#endif
#ifndef THRS_WO_BATCH
#define THRS_WO_BATCH 8
#endif

// Tile configuration per (key bytes, value bytes).  A tile is what one
// workgroup holds in REGISTERS (THREADS x KPT keys) and publishes one status
// row for; it is written out through an LDS stage of STAGE keys in ROUNDS
// rounds.  Large tiles keep the look-back short: its depth is about
// (tiles completed per us) x (cross-XCD visibility latency, ~1-2 us under load)
// and every step reads one 1 KiB status row.
#ifndef THRS_K4V0_CFG
#define THRS_K4V0_CFG 16, 32, 1, 4
#endif
template <int KB, int VB> struct PassCfg;
template <> struct PassCfg<4, 0> {
  static constexpr int CFG[4] = {THRS_K4V0_CFG};  // waves, keys/thread, rounds, min waves per SIMD
  static constexpr int WAVES = CFG[0], KPT = CFG[1], ROUNDS = CFG[2], WPE = CFG[3];
};
#ifndef THRS_K4V4_CFG
#define THRS_K4V4_CFG 16, 16, 1, 4
#endif
#ifndef THRS_K4V8_CFG
#define THRS_K4V8_CFG 16, 16, 4, 4
#endif
#ifndef THRS_K4V16_CFG
#define THRS_K4V16_CFG 16, 8, 2, 4
#endif
#ifndef THRS_K8V0_CFG
#define THRS_K8V0_CFG 16, 16, 1, 4
#endif
#ifndef THRS_K8V4_CFG
#define THRS_K8V4_CFG 16, 16, 4, 4
#endif
#ifndef THRS_K8V8_CFG
#define THRS_K8V8_CFG 16, 16, 2, 4
#endif
#ifndef THRS_K8V16_CFG
#define THRS_K8V16_CFG 16, 8, 2, 4
#endif
#define THRS_PASS_CFG(KB_, VB_, MACRO)                                           \
  template <> struct PassCfg<KB_, VB_> {                                          \
    static constexpr int CFG[4] = {MACRO};                                        \
    static constexpr int WAVES = CFG[0], KPT = CFG[1], ROUNDS = CFG[2], WPE = CFG[3]; \
  };
THRS_PASS_CFG(4, 4, THRS_K4V4_CFG)
THRS_PASS_CFG(4, 8, THRS_K4V8_CFG)
THRS_PASS_CFG(4, 16, THRS_K4V16_CFG)
THRS_PASS_CFG(8, 0, THRS_K8V0_CFG)
THRS_PASS_CFG(8, 4, THRS_K8V4_CFG)
THRS_PASS_CFG(8, 8, THRS_K8V8_CFG)
THRS_PASS_CFG(8, 16, THRS_K8V16_CFG)
#undef THRS_PASS_CFG

template <int KB, int VB> struct PassGeom {
  static constexpr int WAVES = PassCfg<KB, VB>::WAVES, KPT = PassCfg<KB, VB>::KPT, ROUNDS = PassCfg<KB, VB>::ROUNDS;
  static constexpr int WPE = PassCfg<KB, VB>::WPE;
  static constexpr int THREADS = 64 * WAVES;
  static constexpr uint32_t TILE = (uint32_t)THREADS * KPT;
  static constexpr uint32_t STAGE = TILE / ROUNDS;
  // stage | s_cnt[WAVES][256] | s_gofs[256] | s_misc[16] | stamps
  static constexpr uint32_t LDS_BYTES = STAGE * (KB + VB) + (WAVES + 1) * kBins * 4 + 16 * 4 + kStampLds;
  static_assert(TILE <= 65536, "slots are kept as 16-bit halves");
  static_assert(kGroup == 0 || (uint64_t)kGroup * TILE < kArrival, "group counts must fit below the arrival bits");
  static_assert((STAGE & (STAGE - 1)) == 0 && STAGE % THREADS == 0, "stage must be a power of two");
};

// Phases (threads tid < 256 double as "digit d = tid" in the per-digit steps):
//   A  tile id, load keys (+values) into registers
//   B  per-wave digit histogram (LDS atomics) -> tile counts; publish the
//      tile aggregate; local exclusive scan -> per-wave running offsets
//   C  rank item by item (wave64 ballot match + per-wave running counters):
//      every key gets its final slot in the tile's sorted order
//   D  decoupled look-back (window of kLookWindow rows per round trip)
//      -> global offset of digit d
//   E  ROUNDS x { scatter keys whose slot falls in this round into the LDS
//      stage, coalesced write-out of the stage }
__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x;
}

// Output start of a tile's digit-d run of cnt keys, base + total, clamped so
// the run ends by outEnd.  Only a look-back that gave up (error word set:
// the sort's bytes are garbage and the caller is told) or stale tables after
// one can put a run past the end; it is still never written out of bounds.
// A clamp that changed the run is reported (kErrRunClamped): the caller sees
// THRS_ERROR_DEVICE_CHECK unless a spin that gave up explains it.
__device__ __forceinline__ uint32_t clamp_run(uint32_t base, uint32_t total, uint32_t cnt, uint32_t outEnd,
                                              uint32_t* __restrict__ errFlag) {
  const uint64_t pos = (uint64_t)base + total;
  const uint64_t hi = outEnd >= cnt ? (uint64_t)(outEnd - cnt) : 0u;
  if (pos > hi) atomicOr(errFlag, kErrRunClamped);
  return (uint32_t)(pos < hi ? pos : hi);
}

// Two-level look-back for digit d of one tile (THRS_GROUP > 0).  issue()
// sends one round of status loads (this group's earlier tile rows + a window
// of group rows); finish() consumes rounds until the walk ends, writes the
// digit's global write offset to s_gofs[d] and, from the group's last tile,
// publishes the group's inclusive prefix.
template <typename ST>
struct GroupWalk {
  const ST* status;
  const GroupTables<ST>* grp;
  uint32_t tile, d, g, gstart, gend;
  uint32_t inGroup = 0, excl = 0, spins = 0, rounds = 0;
  uint32_t jt;        // next earlier tile of this group to add (ascending)
  int32_t jg;         // next earlier group to add (descending); -1 = done
  int32_t found = -1; // group whose prefix ended the walk (diagnostics)
  ST wt[kTileWindow];
  ST wp[kGroupWindow];
  uint32_t wa[kGroupWindow];

  __device__ __forceinline__ GroupWalk(const ST* st, const GroupTables<ST>& gt, uint32_t t, uint32_t dd)
      : status(st), grp(&gt), tile(t), d(dd) {
    g = t / kGroup;
    gstart = g * kGroup;
    gend = min(gstart + (uint32_t)kGroup, gt.nTiles);
    jt = gstart;
    jg = (int32_t)g - 1;
  }
  __device__ __forceinline__ bool walking() const { return jt < tile || jg >= (int32_t)grp->gmin; }
  __device__ __forceinline__ void issue() {
#pragma unroll
    for (int q = 0; q < kTileWindow; ++q)
      wt[q] = (jt + q < tile) ? load_agent(status + (uint64_t)(jt + q) * kBins + d) : (ST)0;
#pragma unroll
    for (int q = 0; q < kGroupWindow; ++q) {
      const bool in = jg - q >= (int32_t)grp->gmin;
      wp[q] = in ? load_agent(grp->gp + (uint64_t)(jg - q) * kBins + d) : (ST)0;
      wa[q] = in ? load_agent(grp->ga + (uint64_t)(jg - q) * kBins + d) : 0u;
    }
    ++rounds;
  }
  // consume the issued round; true if something was not published yet
  __device__ __forceinline__ bool consume() {
    bool stall = false;
#pragma unroll
    for (int q = 0; q < kTileWindow; ++q) {
      if (!stall && jt < tile) {
        if (wt[q] == 0) stall = true;
        else {
          inGroup += Status<ST>::val(wt[q]);
          ++jt;
        }
      }
    }
    bool gstop = false;
#pragma unroll
    for (int q = 0; q < kGroupWindow; ++q) {
      if (!gstop && jg >= (int32_t)grp->gmin) {
        if (wp[q] != 0) {  // inclusive prefix of group jg: done
          excl += Status<ST>::val(wp[q]);
          found = jg;
          jg = (int32_t)grp->gmin - 1;
        } else {
          const uint32_t members = min((uint32_t)kGroup, grp->nTiles - (uint32_t)jg * kGroup);
          if ((wa[q] >> 20) == members) {
            excl += wa[q] & (kArrival - 1);
            --jg;
          } else {
            gstop = true;
            stall = true;
          }
        }
      }
    }
    return stall;
  }
  __device__ __forceinline__ void finish(uint32_t realTot, uint32_t myBase, uint32_t outEnd, uint32_t localStart,
                                         uint32_t* s_gofs, uint32_t* s_misc, uint32_t* errFlag,
                                         uint64_t* __restrict__ stamps) {
#ifdef THRS_STAMPS
    // slot 16: walk (re)starts here, 17: first window consumed, 18: walk done (digit 0's thread)
    const bool st0 = stamps && d == 0;
    uint64_t* s_stamp = reinterpret_cast<uint64_t*>(s_misc + 16);
    if (st0) s_stamp[16] = __builtin_amdgcn_s_memrealtime();
#else
    (void)stamps;
#endif
    while (walking()) {
      issue();
      const bool stall = consume();
#ifdef THRS_STAMPS
      if (st0 && rounds == 1) {
        uint32_t dep = inGroup + excl;
        pin(dep);
        s_stamp[17] = __builtin_amdgcn_s_memrealtime() + (uint64_t)(dep == 0xFFFFFFFFu);
      }
#endif
      if (stall && walking()) {
        if (++spins > kSpinMax) {  // bounded spin: never hang the GPU
          atomicOr(errFlag, kErrSpin);
          break;
        }
#if THRS_WALK_BACKOFF
        // experiment: poll less often once a walk has waited a few rounds
        // (every poll re-reads a window of status words from memory)
        if (spins > THRS_WALK_BACKOFF) __builtin_amdgcn_s_sleep(8);
        else
#endif
        __builtin_amdgcn_s_sleep(1);
      }
    }
    const uint32_t total = excl + inGroup;
#ifdef THRS_STAMPS
    if (stamps && (d & 63) == 0) {  // slots 8..11: walk end of waves 0..3
      uint32_t dep = total;
      pin(dep);
      const uint64_t tnow = __builtin_amdgcn_s_memrealtime();
      s_stamp[8 + (d >> 6)] = tnow + (uint64_t)(dep == 0xFFFFFFFFu);
    }
    if ((d & 63) == 0) {  // one lane per wave: a divergent atomicMax would compile to a 64-step loop
      atomicMax(&s_misc[1], rounds);
      atomicMax(&s_misc[2], spins);
      atomicMax(&s_misc[3], (uint32_t)(tile - gstart) + (uint32_t)((int32_t)g - 1 - found) * kGroup);
    }
#else
    (void)s_misc;
#endif
    s_gofs[d] = clamp_run(myBase, total, realTot, outEnd, errFlag) - localStart;
    if (tile == gend - 1) {
      store_agent(grp->gp + (uint64_t)g * kBins + d, Status<ST>::pre(total + realTot));
    }
  }
};

// Everything one workgroup does for one tile (phases A-E below).
//   tile        global tile index (rows of the status table, key range)
//   chainStart  first tile of this tile's look-back chain: tile == chainStart
//               publishes its prefix directly
//   myBase      (thread d < 256) global output base of digit d for the chain
// Returns after the tile's last store is issued.
// Load one tile's keys (and values) into registers: item j of lane l of wave
// w is key w*64*KPT + j*64 + l of the tile (blocked by wave, striped by lane),
// which is the order the stable rank walks.  Keys past n read as 0.
// keyStart / valid: the tile's first key and key count (tile * TILE and
// min(TILE, n - tile * TILE) except in segmented passes).
// Key codecs of the pass kernels.  The bucket path for u32 / f32 keys without
// values (thrs_hybrid.hpp, thrs_local16) and for u32 / f32 keys with 4-byte
// values (thrs_local_pairs; the values travel as they are) carries only what the
// next step reads, in two planes instead of the 4-byte keys:
//   kCodecKeys    keys in, keys out
//   kCodecSplit   keys in; out: the image's low 16 bits to the u16 plane
//                 (keysOut) and its top byte to the u8 plane (hiPlane) -- the
//                 second digit (bits 16-23), which this pass sorts by, is
//                 implied by the output position
//   kCodecPlanes  in: the two planes, as k' = top byte << 16 | low 16 bits (the
//                 pass's digit at shift 16, identity map); out: the low 16 bits
//                 to a u16 plane -- the local sort rebuilds the top 16 bits
//                 from its chunk's bucket
// 7 + 5 bytes per key instead of 8 + 8 for the two top-digit passes, 6
// instead of 8 for the local sort.
enum { kCodecKeys = 0, kCodecSplit = 1, kCodecPlanes = 2 };

template <int KT, int VB, int CODEC = kCodecKeys>
__device__ __forceinline__ void load_tile(const typename KeyTraits<KT>::U* __restrict__ keysIn,
                                          const typename ValueWord<VB>::T* __restrict__ valsIn, uint64_t keyStart,
                                          uint32_t valid,
                                          typename KeyTraits<KT>::U (&k)[PassGeom<sizeof(typename KeyTraits<KT>::U), VB>::KPT],
                                          typename ValueWord<VB>::T (&v)[VB ? PassGeom<sizeof(typename KeyTraits<KT>::U), VB>::KPT : 1],
                                          const uint8_t* __restrict__ hiIn = nullptr, bool vec = false) {
  using U = typename KeyTraits<KT>::U;
  using VW = typename ValueWord<VB>::T;
  using G = PassGeom<sizeof(U), VB>;
  constexpr int KPT = G::KPT;
  constexpr uint32_t T = G::TILE, CHUNK = 64 * KPT;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t chunkBase = keyStart + w * CHUNK;
  int32_t lim = (int32_t)valid - (int32_t)(w * CHUNK + lane);  // item j is real iff j*64 < lim
  pin(reinterpret_cast<uint32_t&>(lim));
  // the values (pairs): issued after the keys, before anything waits on them
  auto load_vals = [&]() __attribute__((always_inline)) {
    if constexpr (VB != 0) {
#pragma unroll
      for (int j = 0; j < KPT; ++j) v[j] = (valid == T || j * 64 < lim) ? valsIn[chunkBase + j * 64 + lane] : VW{};
    }
  };
  if constexpr (CODEC == kCodecPlanes) {
    static_assert(sizeof(U) == 4 && (VB == 0 || VB == 4), "planes: u32 keys, no values or 4-byte values");
    const uint16_t* lo = reinterpret_cast<const uint16_t*>(keysIn);
    if constexpr (KPT % 4 == 0) {
      // vec (a whole tile, keyStart a multiple of 4, inside ONE second-digit
      // region -- thrs_pass_seg_body): four consecutive keys per lane and
      // load, item 4q + c of lane l = key 256q + 4l + c of the wave's run: an
      // 8-byte load of the u16 plane and a dword of the u8 plane, no lane
      // permutes (a third of the loads, none of the ds_bpermutes).  The rank
      // then walks the keys out of their input order, which changes nothing
      // a keys-only sort can see: every key of the tile lands in the same
      // bucket run, and the order inside a bucket is the local sort's
      // (docs/EXPERIMENTS.md row 107).
      if (vec) {  // (keys only: thrs_pass_seg_body)
        const uint2* lq = reinterpret_cast<const uint2*>(lo + chunkBase) + lane;
        const uint32_t* hq = reinterpret_cast<const uint32_t*>(hiIn + chunkBase) + lane;
        uint2 l2[KPT / 4];
        uint32_t h4[KPT / 4];
#pragma unroll
        for (int q = 0; q < KPT / 4; ++q) {
          l2[q] = lq[q * 64];
          h4[q] = hq[q * 64];
        }
#pragma unroll
        for (int q = 0; q < KPT / 4; ++q) {
          k[4 * q] = (U)(((h4[q] & 0xFFu) << 16) | (l2[q].x & 0xFFFFu));
          k[4 * q + 1] = (U)((((h4[q] >> 8) & 0xFFu) << 16) | (l2[q].x >> 16));
          k[4 * q + 2] = (U)((((h4[q] >> 16) & 0xFFu) << 16) | (l2[q].y & 0xFFFFu));
          k[4 * q + 3] = (U)(((h4[q] >> 24) << 16) | (l2[q].y >> 16));
        }
        return;
      }
    }
#ifndef THRS_HI_DWORD
#define THRS_HI_DWORD 1
#endif
    if constexpr (THRS_HI_DWORD != 0) {
      // The u8 plane in dwords: a wave's 64 x KPT bytes take KPT/4 + 1 dword
      // loads (from the dword-aligned address below its first byte), not KPT
      // byte loads -- with the KPT u16 loads a wave keeps 41 loads in flight
      // instead of 64, under the 63 a wave can have outstanding (the 64th
      // would wait for the first to return, ~2 us per tile).  Each lane then
      // takes its byte from the lane that loaded it (ds_bpermute).
      static_assert(KPT % 4 == 0, "whole dwords of the u8 plane per four items");
      constexpr int HQ = KPT / 4 + 1;
      const uintptr_t hb = reinterpret_cast<uintptr_t>(hiIn + chunkBase);
      const uint32_t a = (uint32_t)(hb & 3u);
      const uint32_t* hw = reinterpret_cast<const uint32_t*>(hb - a);
      // (clamped to the tile's last byte: never past the plane)
      const uintptr_t tileEnd = reinterpret_cast<uintptr_t>(hiIn + keyStart + (valid ? valid - 1 : 0));
      const int32_t lastW = (int32_t)(((tileEnd & ~(uintptr_t)3) - (hb - a)) >> 2);
      uint32_t hq[HQ];
#pragma unroll
      for (int q = 0; q < HQ; ++q) hq[q] = hw[max(0, min((int32_t)(64 * q + lane), lastW))];
      if (valid == T) {
#pragma unroll
        for (int j = 0; j < KPT; ++j) k[j] = (U)lo[chunkBase + j * 64 + lane];
      } else {
#pragma unroll
        for (int j = 0; j < KPT; ++j) k[j] = (j * 64 < lim) ? (U)lo[chunkBase + j * 64 + lane] : (U)0;
      }
      load_vals();
      // byte (a + 64j + lane) of the window: dword 16j + (a + lane) / 4 --
      // lane (that & 63) of load j/4, or of load j/4 + 1 past the end of a
      // 256-byte load (j % 4 == 3, a + lane >= 64)
      const uint32_t al = a + lane;                   // in [0, 66]
      const int src = (int)((al >> 2) << 2);          // 4 (al / 4), in [0, 64]
      const uint32_t e8 = (al & 3u) * 8u;
#pragma unroll
      for (int j = 0; j < KPT; ++j) {
        const int s = (src + 64 * (j & 3)) & 255;  // 4 x the source lane ((16 (j % 4) + al / 4) & 63)
        uint32_t x = (uint32_t)__builtin_amdgcn_ds_bpermute(s, (int)hq[j >> 2]);
        if ((j & 3) == 3) {
          const uint32_t y = (uint32_t)__builtin_amdgcn_ds_bpermute(s, (int)hq[(j >> 2) + 1]);
          x = al >= 64u ? y : x;
        }
        const uint32_t hi8 = (x >> e8) & 0xFFu;
        k[j] = (valid == T || j * 64 < lim) ? (U)((hi8 << 16) | (uint32_t)k[j]) : (U)0;
      }
      return;
    }
    auto ld = [&](uint64_t i) -> U { return (U)(((uint32_t)hiIn[i] << 16) | (uint32_t)lo[i]); };
    if (valid == T) {
#pragma unroll
      for (int j = 0; j < KPT; ++j) k[j] = ld(chunkBase + j * 64 + lane);
    } else {
#pragma unroll
      for (int j = 0; j < KPT; ++j) k[j] = (j * 64 < lim) ? ld(chunkBase + j * 64 + lane) : (U)0;
    }
    load_vals();
    return;
  }
  if (valid == T) {
#pragma unroll
    for (int j = 0; j < KPT; ++j) k[j] = keysIn[chunkBase + j * 64 + lane];
  } else {
#pragma unroll
    for (int j = 0; j < KPT; ++j) k[j] = (j * 64 < lim) ? keysIn[chunkBase + j * 64 + lane] : (U)0;
  }
  load_vals();
}

// keys in tile `tile` of an unsegmented pass over n keys
template <uint32_t T> __device__ __forceinline__ uint32_t tile_valid(uint32_t n, uint32_t tile) {
  return (uint32_t)min((uint64_t)T, (uint64_t)n - (uint64_t)tile * T);
}

struct NoMid {
  __device__ __forceinline__ void operator()() const {}
};

// GROUPED = false: the flat per-tile look-back (the per-bucket fallback,
// whose chains may be shorter than a group; thrs_fallback.hpp).
template <int KT, int VB, typename ST, bool ATOMIC_RANK, typename Mid, int CODEC = kCodecKeys, bool GROUPED = true,
          typename KM>
__device__ __forceinline__ void pass_tile(
    const typename KeyTraits<KT>::U* __restrict__ keysIn, typename KeyTraits<KT>::U* __restrict__ keysOut,
    const typename ValueWord<VB>::T* __restrict__ valsIn, typename ValueWord<VB>::T* __restrict__ valsOut,
    uint64_t keyStart, uint32_t valid, KM km, int shift, uint32_t myBase,
    uint32_t outEnd, ST* __restrict__ status, ST* __restrict__ statusNext, uint32_t* __restrict__ errFlag, uint32_t tile,
    uint32_t chainStart, const GroupTables<ST>& grp, unsigned char* smem, uint64_t* __restrict__ stamps,
    typename KeyTraits<KT>::U (&k)[PassGeom<sizeof(typename KeyTraits<KT>::U), VB>::KPT],
    typename ValueWord<VB>::T (&v)[VB ? PassGeom<sizeof(typename KeyTraits<KT>::U), VB>::KPT : 1], Mid mid,
    uint8_t* __restrict__ hiOut = nullptr) {
  using U = typename KeyTraits<KT>::U;
  using VW = typename ValueWord<VB>::T;
  using G = PassGeom<sizeof(U), VB>;
  static_assert(CODEC == kCodecKeys || (sizeof(U) == 4 && (VB == 0 || VB == 4)), "codecs: 4-byte keys, <= 4-byte values");
  constexpr int WAVES = G::WAVES, KPT = G::KPT, ROUNDS = G::ROUNDS, THREADS = G::THREADS;
  constexpr uint32_t T = G::TILE, STAGE = G::STAGE, CHUNK = 64 * KPT;
  constexpr int STAGE_SHIFT = __builtin_ctz(STAGE);
  // threads [PUB_LO, PUB_LO+256) publish the tile's status row (see phase B)
  constexpr uint32_t PUB_LO = WAVES >= 8 ? 256u : 0u;
  U* stage_k = reinterpret_cast<U*>(smem);
  VW* stage_v = reinterpret_cast<VW*>(smem + STAGE * sizeof(U));
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(smem + STAGE * (sizeof(U) + VB));  // [WAVES][256]
  uint32_t* s_gofs = s_cnt + WAVES * kBins;
  uint32_t* s_misc = s_gofs + kBins;
  // tid is re-derived per tile (pinned): in the persistent kernels the
  // addresses computed from it would otherwise be hoisted out of the tile
  // loop and spilled to scratch (this kernel is at its VGPR limit)
  uint32_t tid0 = threadIdx.x;
  pin(tid0);
  const uint32_t tid = tid0, lane = tid & 63, w = tid >> 6;
#ifdef THRS_STAMPS
  uint64_t* s_stamp = reinterpret_cast<uint64_t*>(s_misc + 16);  // flushed once per tile (a global
                                                                  // store mid-tile would perturb timing)
#endif
  // Diagnostic builds (-DTHRS_STAMPS) record s_memrealtime (100 MHz) per
  // phase for every tile into stamps[tile*kStampSlots + i]; normal builds compile none.
#ifdef THRS_STAMPS
#define THRS_STAMP(i)                                                                                  \
  do {                                                                                                 \
    if (stamps && threadIdx.x == 0) s_stamp[(i)] = __builtin_amdgcn_s_memrealtime();                     \
  } while (0)
#else
#define THRS_STAMP(i) \
  do {                \
  } while (0)
  (void)stamps;
#endif

  THRS_STAMP(1);
  const bool full = valid == T;
  const uint32_t d = tid & 255u;

  // partial tile: item j is real iff j*64 < lim (one register; pinned so the
  // per-item positions are never hoisted into 32 live registers)
  int32_t lim = (int32_t)valid - (int32_t)(w * CHUNK + lane);
  pin(reinterpret_cast<uint32_t&>(lim));
  // The split codec writes images: the keys become their images once, here,
  // and the count, rank and write-out read them as they are (float keys under
  // a key range or the squeeze: one map per key instead of four)
  constexpr bool kImg = CODEC == kCodecSplit;
  if constexpr (kImg) {
#pragma unroll
    for (int j = 0; j < KPT; ++j) k[j] = kimg<KT>(km, k[j]);
  }
  auto img_of = [&](U key) -> U {
    if constexpr (kImg) return key;
    else return kimg<KT>(km, key);
  };
  auto digit_of = [&](U key, int j) -> uint32_t {
    uint32_t dd = (uint32_t)(img_of(key) >> shift) & 0xFFu;
    if (!full) dd = (j * 64 < lim) ? dd : 0xFFu;  // padding sorts after every real key
    return dd;
  };

  // ---- B: per-wave histogram (order-free LDS atomics) -> tile counts.
  // A wave whose every item has one digit (sorted / constant input: one LDS
  // atomic per key would be a 64-way same-address conflict) adds 64*KPT to
  // the digit once instead; its slots are then base + 64j + lane.
  uint32_t* cnt = s_cnt + w * kBins;
  // hint: items 0 and KPT-1 carry one digit d0 in every lane (sorted input);
  // the count loop verifies the others, and a wrong hint recounts (rare).
  const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)digit_of(k[0], 0));
  const bool hint = full && __ballot(digit_of(k[0], 0) != d0 || digit_of(k[KPT - 1], KPT - 1) != d0) == 0;
  // (wave-uniform branches: random input runs only the plain loops)
  bool allU = false;
  if (hint) {
    uint32_t diff = 0;
#pragma unroll
    for (int j = 0; j < KPT; ++j) diff |= digit_of(k[j], j) ^ d0;
    allU = __ballot(diff != 0) == 0;
  }
  // Float keys: the count's digits, four per register, for the rank
  // (THRS_DIGIT_CACHE): a float key under the squeeze takes ~15 operations to
  // map, its cached digit two to unpack (kf32v32 -0.19 ms; integer keys map
  // in one to three operations, and the cache measured neutral to slower
  // there: docs/EXPERIMENTS.md row 98).
#ifndef THRS_DIGIT_CACHE
#define THRS_DIGIT_CACHE 1
#endif
  constexpr bool kDC = THRS_DIGIT_CACHE != 0 && !kImg && kSqueezable<KT>;
  uint32_t dg[kDC ? (KPT + 3) / 4 : 1];
#pragma unroll
  for (int q = 0; q < (kDC ? (KPT + 3) / 4 : 1); ++q) dg[q] = 0;
  auto cached_digit = [&](int j) -> uint32_t {
    if constexpr (kDC) return (dg[j >> 2] >> (8 * (j & 3))) & 0xFFu;
    else return digit_of(k[j], j);
  };
  if (allU) {
    if (lane == 0) __hip_atomic_fetch_add(&cnt[d0], 64u * KPT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      const uint32_t dd = digit_of(k[j], j);
      if constexpr (kDC) dg[j >> 2] |= dd << (8 * (j & 3));
      __hip_atomic_fetch_add(&cnt[dd], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  lds_barrier();
  THRS_STAMP(2);

  uint32_t tot = 0, realTot = 0;
  ST* myStatus = status + (uint64_t)tile * kBins + d;
  if (tid < 256) {
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) tot += s_cnt[ww * kBins + d];
    realTot = (d == 255u) ? tot - (T - valid) : tot;
  }
  // Publish the tile aggregate (and the group atomic) from waves 4-7: vmcnt
  // counts stores too on gfx9-family parts, so if the walkers (waves 0-3)
  // issued these write-through stores, their first wait on a look-back load
  // would also wait for the stores' acknowledgement -- several us under load.
  if (PUB_LO <= tid && tid < PUB_LO + 256) {
    const uint32_t dp = tid - PUB_LO;
    uint32_t t2 = 0;
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) t2 += s_cnt[ww * kBins + dp];
    const uint32_t real2 = (dp == 255u) ? t2 - (T - valid) : t2;
    ST* pub = status + (uint64_t)tile * kBins + dp;
    if (tile != chainStart) store_agent(pub, Status<ST>::agg(real2));
    else store_agent(pub, Status<ST>::pre(real2));
    if constexpr (kGroup > 0 && GROUPED)
      __hip_atomic_fetch_add(&grp.ga[(uint64_t)(tile / kGroup) * kBins + dp], real2 + kArrival, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
  GroupWalk<ST> gw(status, grp, tile, d);
  // Look-back window loader: rows j, j-1, ... of column d.  32-bit byte offsets
  // from the uniform base -> saddr loads, one VGPR each.
  ST win[kLookWindow];
  int64_t j = (int64_t)tile - 1;  // next predecessor to consume
  auto issue_window = [&]() __attribute__((always_inline)) {
    const uint32_t off0 = ((uint32_t)j * kBins + d) * (uint32_t)sizeof(ST);
#pragma unroll
    for (int q = 0; q < kLookWindow; ++q)
      win[q] = (j - q >= (int64_t)chainStart)
                   ? load_agent(reinterpret_cast<const ST*>(reinterpret_cast<const char*>(status) +
                                                            (off0 - (uint32_t)q * kBins * sizeof(ST))))
                   : (ST)0;
  };
  // local exclusive scan over the 256 digits (waves 0-3)
  uint32_t localStart = 0;
  {
    const uint32_t incl = wave_incl_scan(tot, lane);
    if (tid < 256 && lane == 63) s_misc[4 + w] = incl;
    lds_barrier();
    if (tid < 256) {
      const uint32_t w0 = s_misc[4], w1 = s_misc[5], w2 = s_misc[6];
      localStart = incl - tot + (w > 0 ? w0 : 0u) + (w > 1 ? w1 : 0u) + (w > 2 ? w2 : 0u);
      uint32_t run = localStart;
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) {
        const uint32_t c = s_cnt[ww * kBins + d];
        s_cnt[ww * kBins + d] = run;
        run += c;
      }
    }
  }
  lds_barrier();
  THRS_STAMP(3);

  // ---- C: stable rank = running per-wave offset + same-digit keys in lower
  // lanes of the item (wave_rank: one ds_add_rtn_u32 per key, or one per
  // wave when its digit is uniform; the ballot match without ATOMIC_RANK).
  // all-uniform wave: item j of lane l takes slot base + 64j + l, base = the
  // wave's running offset of d0 (a broadcast read), no atomics
  uint32_t sl[(KPT + 1) / 2];  // final slots, two 16-bit halves per register
#pragma unroll
  for (int j = 0; j < (KPT + 1) / 2; ++j) sl[j] = 0;
  const uint32_t ubase = (uint32_t)__builtin_amdgcn_readfirstlane((int)cnt[d0]);  // scalar
  // lane-ordered rank atomics kept RP in flight: item j+RP's atomic is issued
  // before item j's result is used (a wave's LDS operations execute in issue
  // order, so the ranks are those of the one-at-a-time loop); one at a time,
  // every item waited a full LDS round trip
  constexpr int RP = THRS_RANK_PIPE;
  auto rank_atomic = [&](int j) -> uint32_t {
    return __hip_atomic_fetch_add(&cnt[cached_digit(j)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  auto place = [&](int j, uint32_t slot) __attribute__((always_inline)) {
    if constexpr (ROUNDS == 1) {
      // one LDS round: place the key in sorted order now (frees its register
      // before the walk; the post-walk barrier orders it for phase E)
      stage_k[slot] = k[j];
      if constexpr (VB != 0) stage_v[slot] = v[j];
    } else {
      sl[j / 2] |= slot << (16 * (j & 1));
      pin(sl[j / 2]);  // materialise the slot now (else it is sunk to phase E, keeping masks alive)
    }
  };
  if (allU) {
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      place(j, ubase + 64u * j + lane);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    uint32_t rq[RP];
    if constexpr (ATOMIC_RANK) {
#pragma unroll
      for (int j = 0; j < RP && j < KPT; ++j) {
        pin(k[j]);
        rq[j] = rank_atomic(j);
      }
    }
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      uint32_t slot;
      if constexpr (ATOMIC_RANK) {
        slot = rq[j % RP];
        if (j + RP < KPT) {
          pin(k[j + RP]);  // keep item j+RP's digit/address math here (register pressure)
          rq[j % RP] = rank_atomic(j + RP);
        }
      } else {
        pin(k[j]);  // keep item j's digit/address math inside iteration j (register pressure)
        slot = wave_rank<false>(cnt, cached_digit(j), lane, false);
      }
      place(j, slot);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  auto slot_of = [&](int j) -> uint32_t { return (sl[j / 2] >> (16 * (j & 1))) & 0xFFFFu; };
  THRS_STAMP(4);


  // ---- D: decoupled look-back for digit d, kLookWindow rows per round trip;
  // a not-yet-published word stops the window and is re-polled.
  if constexpr (kGroup > 0 && GROUPED) {
    if (tid < 256) gw.finish(realTot, myBase, outEnd, localStart, s_gofs, s_misc, errFlag, stamps);
#ifdef THRS_STAMPS
    if (stamps && lane == 0 && w < 4) {  // slots 12..15: waves 0..3 arrive at the post-walk barrier
      uint32_t dep = s_gofs[d & 255];
      pin(dep);
      const uint64_t tnow = __builtin_amdgcn_s_memrealtime();
      s_stamp[12 + w] = tnow + (uint64_t)(dep == 0xFFFFFFFFu);
    }
#endif
  } else if (tid < 256) {
    uint32_t excl = 0;
#ifdef THRS_STAMPS
    uint32_t dbgRounds = 0;
#endif
    if (tile != chainStart) {
      uint32_t spins = 0;
      while (true) {
        issue_window();
#ifdef THRS_STAMPS
        ++dbgRounds;
#endif
        bool done = false, stall = false;
#pragma unroll
        for (int q = 0; q < kLookWindow; ++q) {
          if (!done && !stall) {
            const ST sw = win[q];
            if (sw == 0) {
              stall = true;
            } else {
              excl += Status<ST>::val(sw);
              if (Status<ST>::is_pre(sw)) done = true;
              else --j;
            }
          }
        }
        if (done) break;
        if (stall) {
          if (++spins > kSpinMax) {  // bounded spin: never hang the GPU
            atomicOr(errFlag, kErrSpin);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      store_agent(myStatus, Status<ST>::pre(excl + realTot));
#ifdef THRS_STAMPS
      if ((d & 63) == 0) {
        atomicMax(&s_misc[1], dbgRounds);
        atomicMax(&s_misc[2], spins);
        atomicMax(&s_misc[3], (uint32_t)(tile - 1 - j));
      }
#endif
    }
    s_gofs[d] = clamp_run(myBase, excl, realTot, outEnd, errFlag) - localStart;
  }
  lds_barrier();
  THRS_STAMP(5);

  mid();  // persistent kernel: take the next tile and start its loads (k/v are free)

  // ---- E: ROUNDS x (scatter this round's slots into the stage, write it out)
#pragma unroll 1
  for (int r = 0; r < ROUNDS; ++r) {
    if constexpr (ROUNDS > 1) {
      // keep slot-derived addresses inside the round (else they are hoisted
      // out of the round loop as 32 live registers and spilled)
#pragma unroll
      for (int j = 0; j < (KPT + 1) / 2; ++j) pin(sl[j]);
#pragma unroll
      for (int j = 0; j < KPT; ++j) {
        const uint32_t slot = slot_of(j);
        if ((slot >> STAGE_SHIFT) == (uint32_t)r) {
          stage_k[slot & (STAGE - 1)] = k[j];
          if constexpr (VB != 0) stage_v[slot & (STAGE - 1)] = v[j];
        }
      }
      lds_barrier();
    }
    // write one stage slot (i) to its global position (vv: its value, read by the caller)
    auto put = [&](U key, uint32_t i, uint32_t off, const VW& vv) __attribute__((always_inline)) {
      const uint32_t dst = off + (uint32_t)r * STAGE + i;
      if constexpr (CODEC == kCodecSplit) {
        const uint32_t img = (uint32_t)key;  // (an image already)
        reinterpret_cast<uint16_t*>(keysOut)[dst] = (uint16_t)img;
        hiOut[dst] = (uint8_t)(img >> 24);
      } else if constexpr (CODEC == kCodecPlanes) {
        reinterpret_cast<uint16_t*>(keysOut)[dst] = (uint16_t)key;
      } else {
        keysOut[dst] = key;
      }
      if constexpr (VB != 0) valsOut[dst] = vv;
    };
    if (VB == 0 && full) {
      // whole tile: no lane conditions, so each batch's stage reads,
      // then its offset reads, are issued back to back (a read under a lane
      // condition is waited for before the next one issues)
      constexpr int NS = (int)(STAGE / THREADS), WB = THRS_WO_BATCH;
#pragma unroll
      for (int j0 = 0; j0 < NS; j0 += WB) {
        U key[WB];
        uint32_t off[WB];
        VW val[VB ? WB : 1];
#pragma unroll
        for (int b = 0; b < WB; ++b)
          if (j0 + b < NS) {
            key[b] = stage_k[(j0 + b) * THREADS + tid];
            if constexpr (VB != 0) val[b] = stage_v[(j0 + b) * THREADS + tid];
          }
#pragma unroll
        for (int b = 0; b < WB; ++b)
          if (j0 + b < NS) off[b] = s_gofs[(uint32_t)(img_of(key[b]) >> shift) & 0xFFu];
#pragma unroll
        for (int b = 0; b < WB; ++b)
          if (j0 + b < NS) put(key[b], (j0 + b) * THREADS + tid, off[b], val[VB ? b : 0]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else
#pragma unroll
    for (int j = 0; j < (int)(STAGE / THREADS); ++j) {
      const uint32_t i = j * THREADS + tid;
      const uint32_t slot = (uint32_t)r * STAGE + i;
      if (full || slot < valid) {
        const U key = stage_k[i];
        const uint32_t dd = (uint32_t)(img_of(key) >> shift) & 0xFFu;
        VW vv{};
        if constexpr (VB != 0) vv = stage_v[i];
        put(key, i, s_gofs[dd], vv);
      }
      // bound the batch the scheduler hoists (LDS reads + 64-bit addresses):
      // in the persistent kernel the next tile's keys are live here
      if ((j % THRS_WO_BATCH) == THRS_WO_BATCH - 1) __builtin_amdgcn_sched_barrier(0);
    }
    if (r + 1 < ROUNDS) lds_barrier();
  }
  // Clear this tile's rows of the next pass's tables only now: a store issued
  // before the look-back barrier waits for room in the CU's in-order vector
  // memory queue (behind the other workgroup's loads) and holds the barrier.
  if (tid < 256) {
    if (statusNext) statusNext[(uint64_t)tile * kBins + d] = 0;
    if constexpr (kGroup > 0 && GROUPED) {
      const uint32_t gend = min((tile / kGroup + 1) * (uint32_t)kGroup, grp.nTiles);
      if (grp.gaNext && tile == gend - 1) {
        grp.gaNext[(uint64_t)(tile / kGroup) * kBins + d] = 0;
        grp.gpNext[(uint64_t)(tile / kGroup) * kBins + d] = 0;
      }
    }
  }
#ifdef THRS_STAMPS
#ifndef THRS_STAMPS_NOWAIT
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // slot 6 = stores drained (NOWAIT: issued)
#endif
  THRS_STAMP(6);
  if (stamps && tid == 0)  // slot 7: xcc | max rounds << 8 | max depth << 24 | max stalls << 40
    s_stamp[7] |= ((uint64_t)min(s_misc[1], 65535u) << 8) | ((uint64_t)min(s_misc[3], 65535u) << 24) |
                  ((uint64_t)s_misc[2] << 40);
  lds_barrier();
  if (stamps && tid < (uint32_t)kStampSlots) stamps[(uint64_t)tile * kStampSlots + tid] = s_stamp[tid];
#endif
#undef THRS_STAMP
}


// One workgroup per tile, tile ids in start order (dynamic): the chain is the
// whole tile range and status words go through the agent scope.
template <int KT, int VB, typename ST, bool ATOMIC_RANK>
__global__ __launch_bounds__((PassGeom<sizeof(typename KeyTraits<KT>::U), VB>::THREADS))
__attribute__((amdgpu_waves_per_eu(PassGeom<sizeof(typename KeyTraits<KT>::U), VB>::WPE))) void thrs_pass(
    const typename KeyTraits<KT>::U* __restrict__ keysIn, typename KeyTraits<KT>::U* __restrict__ keysOut,
    const typename ValueWord<VB>::T* __restrict__ valsIn, typename ValueWord<VB>::T* __restrict__ valsOut,
    uint32_t n, KeyMap<typename KeyTraits<KT>::U> km, int shift, const uint32_t* __restrict__ digitBase,
    ST* __restrict__ status, ST* __restrict__ statusNext, uint32_t* __restrict__ tileCounter,
    uint32_t* __restrict__ errFlag, GroupTables<ST> grp, uint64_t* __restrict__ stamps,
    const uint32_t* __restrict__ gate, uint32_t gateMask) {
  if (gate && !((gateMask >> *gate) & 1u)) return;  // not needed on this launch path (thrs_plan decides)
  using G = PassGeom<sizeof(typename KeyTraits<KT>::U), VB>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(smem + G::STAGE * (sizeof(typename KeyTraits<KT>::U) + VB));
  uint32_t* s_misc = s_cnt + (G::WAVES + 1) * kBins;
#ifdef THRS_STAMPS
  const uint64_t t_entry = __builtin_amdgcn_s_memrealtime();
#endif
  const uint32_t tid = threadIdx.x;
  if (tid == 0) {
    s_misc[0] = atomicAdd(tileCounter, 1u);
    s_misc[1] = s_misc[2] = s_misc[3] = 0;  // diagnostic maxima (THRS_STAMPS)
  }
  for (uint32_t i = tid; i < (uint32_t)(G::WAVES * kBins); i += G::THREADS) s_cnt[i] = 0;
  const uint32_t myBase = digitBase[tid & 255u];
  lds_barrier();
  const uint32_t tile = s_misc[0];
#ifdef THRS_STAMPS
  if (stamps && tid == 0) {
    uint64_t* s_stamp = reinterpret_cast<uint64_t*>(s_misc + 16);
    for (int i = 0; i < kStampSlots; ++i) s_stamp[i] = 0;
    s_stamp[0] = t_entry;
    s_stamp[7] = xcc_id();
  }
#endif
  typename KeyTraits<KT>::U k[G::KPT];
  typename ValueWord<VB>::T v[VB ? G::KPT : 1];
  load_tile<KT, VB>(keysIn, valsIn, (uint64_t)tile * G::TILE, tile_valid<G::TILE>(n, tile), k, v);
  pass_tile<KT, VB, ST, ATOMIC_RANK>(keysIn, keysOut, valsIn, valsOut, (uint64_t)tile * G::TILE,
                                     tile_valid<G::TILE>(n, tile), km, shift, myBase, n, status,
                                     statusNext, errFlag, tile, 0, grp, smem, stamps, k, v, NoMid{});
}

// ============================================================ XCD-block claims
// Tiles are claimed in BLOCKS of kXcdBlock consecutive tiles, one open block
// per XCD, so neighbouring tiles -- whose digit runs share the 128-B lines at
// their boundaries -- are written through the same L2, which merges the two
// partial halves before write-back.  (Consecutive tiles on different XCDs
// leave two partial line writes each, which HBM with ECC serves as
// read-modify-write: scripts/abut_probe.hip measured 2.7 vs 4.1 TB/s.)
// Lock-free claims: the k-th claim on XCD x gets offset k % B of that XCD's
// (k / B)-th block; the claimer with offset 0 opens the XCD's NEXT block (one
// global atomic on the block counter) and publishes it in the XCD's block
// table, so a claim costs one ticket atomic and one load of an entry that was
// published about B claims earlier.
// Deadlock-free without any placement assumption: blocks are opened in global
// order and each XCD claims its blocks in order, so the lowest unpublished
// tile is either held by a running workgroup or is the next tile of an opened
// block of some XCD, whose workgroups hold only lower (published) tiles and
// come back for it; an opened block always belongs to an XCD with running
// workgroups, which claim through it before they can see the DONE entry.
#ifndef THRS_XCD_BLOCK
#define THRS_XCD_BLOCK 8
#endif
constexpr uint32_t kXcdBlock = THRS_XCD_BLOCK;
constexpr uint32_t kXbDone = 0xFFFFFFFFu;
#ifndef THRS_XB_OPEN_AT
#define THRS_XB_OPEN_AT (THRS_XCD_BLOCK / 2)
#endif
constexpr uint32_t kXbOpenAt = THRS_XB_OPEN_AT;
static_assert(kXbOpenAt < kXcdBlock, "open the next block from inside the current one");

// claimState: [0..7] per-XCD tickets, [8] global block counter, [16..]
// per-XCD block tables of `stride` entries (0 = not yet published,
// kXbDone = no more blocks, else block + 1)
__device__ __forceinline__ void xb_open(uint32_t* gblock, uint32_t* entry, uint32_t nBlocks) {
  const uint32_t nb = atomicAdd(gblock, 1u);
  store_agent(entry, nb < nBlocks ? nb + 1 : kXbDone);
}

__device__ __forceinline__ uint32_t xb_claim(uint32_t* claimState, uint32_t stride, uint32_t nTiles,
                                             uint32_t* errFlag) {
  const uint32_t x = xcc_id() & 7u;
  const uint32_t nBlocks = (nTiles + kXcdBlock - 1) / kXcdBlock;
  uint32_t* gblock = claimState + 8;
  uint32_t* tab = claimState + 16 + x * stride;
  const uint32_t k = atomicAdd(&claimState[x], 1u);
  const uint32_t j = k / kXcdBlock, o = k % kXcdBlock;
  if (j + 1 >= stride) return kXbDone;  // cannot happen with stride = nBlocks + slack; never write past the table
  if (k == 0) xb_open(gblock, &tab[0], nBlocks);  // first claim on this XCD: its first block
  // open the XCD's next block once this one is partly claimed: early enough
  // that its claimers find it published, late enough that other XCDs' tiles
  // do not wait long on a block this XCD has not started
  if (o == kXbOpenAt) xb_open(gblock, &tab[j + 1], nBlocks);
  uint32_t e = load_agent(&tab[j]);
  for (uint32_t spin = 0; e == 0; ++spin) {
    if (spin >= kSpinMax) {  // bounded: never hang the GPU
      atomicOr(errFlag, kErrSpin);  // a claim spin that gave up: THRS_ERROR_LOOKBACK_TIMEOUT
      return kXbDone;
    }
    __builtin_amdgcn_s_sleep(1);
    e = load_agent(&tab[j]);
  }
  if (e == kXbDone) return kXbDone;
  const uint32_t tile = (e - 1) * kXcdBlock + o;
  return tile < nTiles ? tile : kXbDone;
}

// Persistent form with XCD-block claims (THRS_XB): one tile per iteration,
// exactly the work of thrs_pass.
template <int KT, int VB, typename ST, bool ATOMIC_RANK>
__global__ __launch_bounds__((PassGeom<sizeof(typename KeyTraits<KT>::U), VB>::THREADS))
__attribute__((amdgpu_waves_per_eu(PassGeom<sizeof(typename KeyTraits<KT>::U), VB>::WPE))) void thrs_pass_xb(
    const typename KeyTraits<KT>::U* __restrict__ keysIn, typename KeyTraits<KT>::U* __restrict__ keysOut,
    const typename ValueWord<VB>::T* __restrict__ valsIn, typename ValueWord<VB>::T* __restrict__ valsOut,
    uint32_t n, KeyMap<typename KeyTraits<KT>::U> km, int shift, const uint32_t* __restrict__ digitBase,
    ST* __restrict__ status, ST* __restrict__ statusNext, uint32_t* __restrict__ claimState,
    uint32_t* __restrict__ errFlag, GroupTables<ST> grp, uint64_t* __restrict__ stamps,
    const uint32_t* __restrict__ gate, uint32_t gateMask) {
  if (gate && !((gateMask >> *gate) & 1u)) return;  // not needed on this launch path (thrs_plan decides)
  using U = typename KeyTraits<KT>::U;
  using VW = typename ValueWord<VB>::T;
  using G = PassGeom<sizeof(U), VB>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(smem + G::STAGE * (sizeof(U) + VB));
  uint32_t* s_misc = s_cnt + (G::WAVES + 1) * kBins;
  const uint32_t tid = threadIdx.x;
  const uint32_t nTiles = (uint32_t)(((uint64_t)n + G::TILE - 1) / G::TILE);
  const uint32_t myBase = digitBase[tid & 255u];
  U k[G::KPT];
  VW v[VB ? G::KPT : 1];
  for (;;) {
    if (tid == 0) {
      s_misc[0] = xb_claim(claimState, (nTiles + kXcdBlock - 1) / kXcdBlock + 16, nTiles, errFlag);
#ifdef THRS_STAMPS
      if (stamps && s_misc[0] != kXbDone) {
        uint64_t* s_stamp = reinterpret_cast<uint64_t*>(s_misc + 16);
        for (int i = 0; i < kStampSlots; ++i) s_stamp[i] = 0;
        s_stamp[0] = __builtin_amdgcn_s_memrealtime();
        s_stamp[7] = xcc_id();
        s_misc[1] = s_misc[2] = s_misc[3] = 0;
      }
#endif
    }
    for (uint32_t i = tid; i < (uint32_t)(G::WAVES * kBins); i += G::THREADS) s_cnt[i] = 0;
    lds_barrier();
    const uint32_t tile = s_misc[0];
    if (tile == kXbDone) break;
    load_tile<KT, VB>(keysIn, valsIn, (uint64_t)tile * G::TILE, tile_valid<G::TILE>(n, tile), k, v);
    pass_tile<KT, VB, ST, ATOMIC_RANK>(keysIn, keysOut, valsIn, valsOut, (uint64_t)tile * G::TILE,
                                       tile_valid<G::TILE>(n, tile), km, shift, myBase, n, status,
                                       statusNext, errFlag, tile, 0, grp, smem, stamps, k, v, NoMid{});
    lds_barrier();  // stage, s_gofs and s_misc[0] are reused by the next tile
  }
}

// ============================================================ XCD segments
// Segmented pass (the 3-pass path's TOP-digit pass, thrs_hybrid.hpp): its
// input is sorted by the second digit, so it splits into 8 segments of
// second-digit ranges [32s, 32s+32) whose top-digit histograms -- column
// blocks of the bucket histogram -- give every segment its own digit bases.
// Segment s is tiled on its own (tile ids from segTiles[s], a multiple of
// kGroup, so groups never span segments) and its look-back chain starts at
// its first tile: segments never wait on each other.  The workgroups of XCD
// x claim segment x's tiles in order (one ticket counter per segment), so
// neighbouring tiles -- whose digit runs share 128-B lines -- are written
// through one L2 and the whole segment is one contiguous range per XCD
// (docs/EXPERIMENTS.md: abut probe 1.88 ms vs 2.08 for 8-tile blocks); a
// workgroup whose segment is exhausted steals from the next ones.
// Deadlock-free: a walk waits only on earlier tiles of its segment, which
// were claimed earlier (tickets are monotone) by running workgroups.
// segInfo: segPos[9] (key positions), segTiles[9] (first tile id); tickets[8] at word 64
// CODEC (kCodec*): keys, or the u32 bucket path's planes (hiPlane: the u8
// plane written by kCodecSplit / read by kCodecPlanes; keysIn / keysOut are
// then u16 planes).
constexpr int kSegs = 8;
// Aligned segments (segInfo[kSegAlignWord] = 1: the top-digit pass, whose
// segments start at data-dependent positions): tile t of a segment [pos, end)
// covers [max(pos, a + tT), min(end, a + (t+1)T)), a = pos rounded down to a
// multiple of T, so every interior tile starts at a multiple of T -- the
// planes codec's vector loads need a multiple of 4; the first tile (and the
// last) may be partial.  Otherwise tiles are counted from pos.
constexpr int kSegAlignWord = 32;
// segInfo[kSegVecWord]: tiles of the top-digit pass that took the planes
// codec's vector loads (zeroed by the plan; thrs_debug_vector_tiles)
constexpr int kSegVecWord = 96;
__host__ __device__ __forceinline__ uint64_t seg_tile_base(uint32_t pos, uint32_t T, bool align) {
  return align ? (uint64_t)pos / T * T : (uint64_t)pos;
}
__host__ __device__ __forceinline__ uint32_t seg_tiles(uint32_t pos, uint32_t end, uint32_t T, bool align) {
  return end > pos ? (uint32_t)(((uint64_t)end - seg_tile_base(pos, T, align) + T - 1) / T) : 0u;
}
template <int KT, int VB, typename ST, bool ATOMIC_RANK, int CODEC>
__device__ __forceinline__ void thrs_pass_seg_body(
    const typename KeyTraits<KT>::U* __restrict__ keysIn, typename KeyTraits<KT>::U* __restrict__ keysOut,
    const typename ValueWord<VB>::T* __restrict__ valsIn, typename ValueWord<VB>::T* __restrict__ valsOut,
    KeyMap<typename KeyTraits<KT>::U> km, int shift, uint32_t* __restrict__ segInfo,
    const uint32_t* __restrict__ segBase, ST* __restrict__ status, uint32_t* __restrict__ errFlag,
    GroupTables<ST> grp, uint8_t* __restrict__ hiPlane, uint64_t* __restrict__ stamps,
    const SqueezeWords* __restrict__ sq, const uint32_t* __restrict__ secondBase) {
  using U = typename KeyTraits<KT>::U;
  using VW = typename ValueWord<VB>::T;
  using G = PassGeom<sizeof(U), VB>;
  constexpr uint32_t T = G::TILE;
  // the planes codec (the top-digit pass over second-digit regions): whole,
  // aligned tiles inside one region take the vector loads (load_tile)
  // (keys only: with values the rank must walk the keys in input order)
  constexpr bool kVec = CODEC == kCodecPlanes && VB == 0 && G::KPT % 4 == 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(smem + G::STAGE * (sizeof(U) + VB));
  uint32_t* s_misc = s_cnt + (G::WAVES + 1) * kBins;
  __shared__ uint32_t segPos[kSegs + 1], segTiles[kSegs + 1], s_align;  // read once per workgroup
  __shared__ uint32_t s_b2[kVec ? kBins : 1];                            // second-digit region starts
  uint32_t* tickets = segInfo + 64;                                      // a cache line of their own
  const uint32_t tid = threadIdx.x;
  if (tid < 2 * (kSegs + 1)) (tid <= (uint32_t)kSegs ? segPos[tid] : segTiles[tid - kSegs - 1]) = segInfo[tid];
  if (tid == 0) s_align = segInfo[kSegAlignWord];
  if constexpr (kVec) {
    if (secondBase)
      for (uint32_t i = tid; i < kBins; i += G::THREADS) s_b2[i] = secondBase[i];
  }
  __syncthreads();
  const bool salign = s_align != 0;
  const uint32_t home = xcc_id() & (kSegs - 1);
  with_map<KT>(km, sq, [&](auto kmx) __attribute__((always_inline)) {
  uint32_t done = 0;  // thread 0: segments found exhausted
  uint32_t nVec = 0;  // thread 0: vector-load tiles (kVec)
  U k[G::KPT];
  VW v[VB ? G::KPT : 1];
  for (;;) {
    if (tid == 0) {
      uint32_t seg = kSegs, t = 0;
      for (int q = 0; q < kSegs; ++q) {
        const uint32_t s = (home + q) & (kSegs - 1);
        if (done & (1u << s)) continue;
        const uint32_t nT = seg_tiles(segPos[s], segPos[s + 1], T, salign);
        const uint32_t x = nT ? atomicAdd(&tickets[s], 1u) : nT;
        if (x < nT) {
          seg = s;
          t = x;
          break;
        }
        done |= 1u << s;
      }
      s_misc[8] = seg;
      s_misc[9] = t;
#ifdef THRS_STAMPS
      if (stamps && seg < (uint32_t)kSegs) {  // slot 7: xcc | segment << 4 (| walk maxima, pass_tile)
        uint64_t* s_stamp = reinterpret_cast<uint64_t*>(s_misc + 16);
        for (int i = 0; i < kStampSlots; ++i) s_stamp[i] = 0;
        s_stamp[0] = __builtin_amdgcn_s_memrealtime();
        s_stamp[7] = xcc_id() | (seg << 4);
        s_misc[1] = s_misc[2] = s_misc[3] = 0;
      }
#endif
    }
    for (uint32_t i = tid; i < (uint32_t)(G::WAVES * kBins); i += G::THREADS) s_cnt[i] = 0;
    lds_barrier();
    const uint32_t seg = s_misc[8], t = s_misc[9];
    if (seg >= (uint32_t)kSegs) {
      if (kVec && tid == 0 && nVec) atomicAdd(&segInfo[kSegVecWord], nVec);  // one add per workgroup
      break;
    }
    const uint32_t segStart = segPos[seg], segEnd = segPos[seg + 1];
    const uint64_t t0 = seg_tile_base(segStart, T, salign) + (uint64_t)t * T;
    const uint64_t keyStart = max((uint64_t)segStart, t0);
    const uint32_t valid = (uint32_t)(min((uint64_t)segEnd, t0 + T) - keyStart);
    bool vec = false;
    if constexpr (kVec) {
      // no second-digit region boundary inside the tile (its keys all go to
      // the buckets of one second digit): the segment's 31 inner boundaries,
      // one per lane, checked by every wave
      if (secondBase && valid == T && (keyStart & 3u) == 0) {
        const uint32_t lane = tid & 63u;
        const uint32_t b = lane < kBins / kSegs - 1 ? s_b2[(kBins / kSegs) * seg + 1 + lane] : 0u;
        vec = __ballot(lane < kBins / kSegs - 1 && b > keyStart && (uint64_t)b < keyStart + T) == 0;
      }
      nVec += vec ? 1u : 0u;
    }
    const uint32_t chain = segTiles[seg];
    GroupTables<ST> g = grp;
    g.nTiles = chain + seg_tiles(segStart, segEnd, T, salign);  // end of this segment's tile ids
    g.gmin = chain / kGroup;
    g.gaNext = nullptr;
    g.gpNext = nullptr;
    const uint32_t myBase = segBase[seg * kBins + (tid & 255u)];
    load_tile<KT, VB, CODEC>(keysIn, valsIn, keyStart, valid, k, v, hiPlane, vec);
    pass_tile<KT, VB, ST, ATOMIC_RANK, NoMid, CODEC>(keysIn, keysOut, valsIn, valsOut, keyStart, valid, kmx,
                                                     shift, myBase, segPos[kSegs], status, nullptr, errFlag, chain + t, chain, g, smem,
                                                     stamps, k, v, NoMid{}, hiPlane);
    lds_barrier();  // stage, s_gofs and s_misc are reused by the next tile
  }
  });
}

template <int KT, int VB, typename ST, bool ATOMIC_RANK, int CODEC = kCodecKeys>
__global__ __launch_bounds__((PassGeom<sizeof(typename KeyTraits<KT>::U), VB>::THREADS))
__attribute__((amdgpu_waves_per_eu(PassGeom<sizeof(typename KeyTraits<KT>::U), VB>::WPE))) void thrs_pass_seg(
    const typename KeyTraits<KT>::U* __restrict__ keysIn, typename KeyTraits<KT>::U* __restrict__ keysOut,
    const typename ValueWord<VB>::T* __restrict__ valsIn, typename ValueWord<VB>::T* __restrict__ valsOut,
    KeyMap<typename KeyTraits<KT>::U> km, int shift, uint32_t* __restrict__ segInfo,
    const uint32_t* __restrict__ segBase, ST* __restrict__ status, uint32_t* __restrict__ errFlag,
    GroupTables<ST> grp, const uint32_t* __restrict__ gate, uint32_t gateMask, uint8_t* __restrict__ hiPlane,
    uint64_t* __restrict__ stamps, const SqueezeWords* __restrict__ sq, const uint32_t* __restrict__ secondBase) {
  if (gate && !((gateMask >> *gate) & 1u)) return;
  thrs_pass_seg_body<KT, VB, ST, ATOMIC_RANK, CODEC>(keysIn, keysOut, valsIn, valsOut, km, shift, segInfo, segBase,
                                                      status, errFlag, grp, hiPlane, stamps, sq, secondBase);
}

// The bucket path's two launches of one top-digit pass in ONE (u32 / f32 keys
// without values, or with 4-byte values, planes on; the values move
// the same way in both bodies): the plan's mode picks the body -- mode 0 the
// key-plane codec CODEC_A (kCodecSplit: keys in, planes out; kCodecPlanes:
// planes in, a plane out, image space KTA), modes 1 / 3 whole keys
// (kCodecKeys, KTB), mode 2 neither.  A gated launch that does nothing still
// costs ~4.7 us of device time (rocprof timeline, docs/EXPERIMENTS.md row
// 124), so each top-digit pass is one launch whatever the plan decides.
template <int KTA, int KTB, int VB, typename ST, bool ATOMIC_RANK, int CODEC_A>
__global__ __launch_bounds__((PassGeom<4, VB>::THREADS))
__attribute__((amdgpu_waves_per_eu(PassGeom<4, VB>::WPE))) void thrs_pass_seg2(
    const uint32_t* __restrict__ kinA, uint32_t* __restrict__ koutA, KeyMap<uint32_t> kmA, int shiftA,
    const uint32_t* __restrict__ secondBaseA, const uint32_t* __restrict__ kinB, uint32_t* __restrict__ koutB,
    KeyMap<uint32_t> kmB, int shiftB, uint32_t* __restrict__ segInfo, const uint32_t* __restrict__ segBase,
    ST* __restrict__ status, uint32_t* __restrict__ errFlag, GroupTables<ST> grp, const uint32_t* __restrict__ mode,
    uint8_t* __restrict__ hiPlane, uint64_t* __restrict__ stamps, const SqueezeWords* __restrict__ sq,
    const typename ValueWord<VB>::T* __restrict__ valsIn, typename ValueWord<VB>::T* __restrict__ valsOut) {
  static_assert(sizeof(typename KeyTraits<KTA>::U) == 4 && sizeof(typename KeyTraits<KTB>::U) == 4 &&
                    (VB == 0 || VB == 4),
                "4-byte keys, no values or 4-byte values");
  const uint32_t m = *mode;
  if (m == 0)
    thrs_pass_seg_body<KTA, VB, ST, ATOMIC_RANK, CODEC_A>(kinA, koutA, valsIn, valsOut, kmA, shiftA, segInfo, segBase,
                                                          status, errFlag, grp, hiPlane, stamps, sq, secondBaseA);
  else if (m == 1 || m == 3)
    thrs_pass_seg_body<KTB, VB, ST, ATOMIC_RANK, kCodecKeys>(kinB, koutB, valsIn, valsOut, kmB, shiftB, segInfo,
                                                             segBase, status, errFlag, grp, nullptr, stamps, sq,
                                                             nullptr);
}

// Zeroing of up to three 16-byte-aligned ranges in one launch (the scratch
// header and look-back tables at the start of every sort).
struct ZeroRanges {
  char* ptr[3] = {};
  uint64_t words[3] = {};  // 16-byte words
};
__global__ __launch_bounds__(256) void thrs_zero_ranges(ZeroRanges z) {
  const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x, stride = (uint64_t)gridDim.x * 256;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    uint4* p = reinterpret_cast<uint4*>(z.ptr[r]);
    for (uint64_t i = g; i < z.words[r]; i += stride) p[i] = make_uint4(0, 0, 0, 0);
  }
}

// Last launch of every sort: ORs the sort's device error word into the
// device's sticky word (host-mapped, thrs_capi.h "Device-side failures").
__global__ void thrs_err_publish(const uint32_t* __restrict__ err, uint32_t* __restrict__ sticky) {
  const uint32_t e = *err;
  if (e) __hip_atomic_fetch_or(sticky, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ================================================================ self-probe
// Does ds_add_rtn_u32 hand out values in lane order when several lanes of one
// fully active wave hit the same LDS word?  Compared against the ballot-match
// rank over random, heavily conflicting and all-equal digit patterns.
// *bad counts disagreeing lanes (0 => ATOMIC_RANK is safe on this device).
__global__ __launch_bounds__(256) void thrs_probe_lds_order(uint32_t* bad, int iters) {
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
    const int mode = it & 3;
    if (mode == 1) d &= 0x3u;
    if (mode == 2) d = 0x5Au;
    if (mode == 3) d &= 0x1Fu;
    uint32_t mlo, mhi;
    match_digit(d, mlo, mhi);
    const uint32_t want = (uint32_t)it + __builtin_amdgcn_mbcnt_hi(mhi, __builtin_amdgcn_mbcnt_lo(mlo, 0u));
    const uint32_t got = __hip_atomic_fetch_add(&cnt[w][d], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    b += got != want;
  }
  if (b) atomicAdd(bad, b);
}

}  // namespace
}  // namespace thrs_dev
