// thrs_host.hpp -- host side of libthrs.so shared by its translation units:
// temporary-buffer layout, the launch plan and the launch sequence (run_sort)
// for one key type.  The sequence is instantiated per key type in
// thrs_run.hip (compiled once per key type, in parallel); thrs_capi.hip holds
// the C-ABI and the process-wide state (profiling events, rank probe, error
// words).
//
// The pass loop follows RadixSort::sort (tinyhipradixsort.hpp:854-944): one
// pass per bitLocation = startBits + 8i < endBits, ping-pong between the
// caller's buffers and the keyOut/valueOut regions of the temporary buffer,
// and a copy-back when the pass count is odd so the result always lands in the
// caller's buffers.  Differences, all deliberate:
//   * one histogram launch for all passes + one tiny scan, then ONE launch per
//     pass (the reference launches blockCount + prefixSumExclusiveInplace +
//     reorder per pass, :872-922);
//   * the odd-pass copy is stream-ordered (hipMemcpyAsync on `stream`); the
//     reference's oroMemcpyDtoD (:938-941) is not;
//   * a pass whose bit location is at or past the key width reads only zero
//     bits, is the identity permutation, and is skipped;
//   * errors are returned, never __debugbreak (:14-15).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "thrs/thrs_capi.h"
#include "thrs_kernels.hpp"
#include "thrs_hybrid.hpp"
#include "thrs_fallback.hpp"

namespace thrs_host {
using namespace thrs_dev;


constexpr uint64_t kAlign = 256;
// the bucket path's lower bounds (default path; docs/EXPERIMENTS.md rows 87,
// 112, 115, 129)
constexpr uint64_t kBucketMinKeys4 = 40000000ull;    // f32 keys without values (rows 129, 132)
constexpr uint64_t kBucketMinKeysU32 = 60000000ull;  // u32 keys without values (4096-key chunks: rows 112, 132)
constexpr uint64_t kTiny16MaxKeys = 3ull << 26;      // u32 keys-only, 4-byte pairs: 4096-key chunks up to here
constexpr uint64_t kTiny16MaxKeysF32 = 1ull << 27;   // f32 keys-only: 4096-key chunks up to here (row 131)
constexpr uint64_t kBucketMinPairs4 = 32000000ull;   // f32 keys with 4-byte values (key planes, 4096-key chunks: rows 129, 132)
constexpr uint64_t kBucketMinPairsU32 = 35000000ull;  // u32 keys + 4-byte values (4096-key chunks, key planes: rows 115, 129)
// thrs_local_kv's types (8-byte keys, 8/16-byte values), with its 8704- and
// 4352-key chunks (row 130)
constexpr uint64_t kBucketMinK8 = 20000000ull;       // 8-byte keys alone or with 4-byte values
constexpr uint64_t kBucketMinK8V8 = 12000000ull;     // u64 keys + 8-byte values (f64: 15M)
constexpr uint64_t kBucketMinF64V8 = 15000000ull;
constexpr uint64_t kBucketMinK8V16 = 8000000ull;     // 8-byte keys + 16-byte values
constexpr uint64_t kBucketMinK4V8 = 32000000ull;     // 4-byte keys + 8-byte values
constexpr uint64_t kBucketMinK4V16 = 25000000ull;    // 4-byte keys + 16-byte values
constexpr uint64_t kHistOff = 0;                       // u32 [8][256]
constexpr uint64_t kBaseOff = 8 * 256 * 4;             // u32 [8][256]
constexpr uint64_t kCounterOff = 2 * 8 * 256 * 4;      // u32 [8]
constexpr uint64_t kErrOff = kCounterOff + 8 * 4;      // u32
constexpr uint64_t kHeaderBytes = 16640;               // 65 * 256

inline uint64_t round_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }
constexpr uint64_t round_up_c(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

inline bool valid_key(int k) { return k >= THRS_KEY_U32 && k <= THRS_KEY_F64; }
inline bool valid_value(int v) { return v >= THRS_VALUE_U32 && v <= THRS_VALUE_U128; }
inline int key_bytes_of(int k) { return (k == THRS_KEY_U32 || k == THRS_KEY_F32) ? 4 : 8; }
inline int value_bytes_of(int v) { return v == THRS_VALUE_U32 ? 4 : v == THRS_VALUE_U64 ? 8 : 16; }

// keys per tile of the pass kernel, per (key bytes, value bytes) -- PassCfg in
// thrs_kernels.hpp
inline uint64_t tile_keys(int kb, int vb) {
  switch (kb * 100 + vb) {
    case 400: return PassGeom<4, 0>::TILE;
    case 404: return PassGeom<4, 4>::TILE;
    case 408: return PassGeom<4, 8>::TILE;
    case 416: return PassGeom<4, 16>::TILE;
    case 800: return PassGeom<8, 0>::TILE;
    case 804: return PassGeom<8, 4>::TILE;
    case 808: return PassGeom<8, 8>::TILE;
    default: return PassGeom<8, 16>::TILE;
  }
}


// keys per tile of the bucket path's segmented passes
inline uint64_t seg_tile_keys(int kb, int vb) {
  return tile_keys(kb, vb);
}

struct Plan {
  int kb, vb;         // key / value bytes (vb = 0 for sortKeys)
  uint64_t tileKeys;  // keys per tile of the pass kernel
  uint64_t nTiles;
  bool wideStatus;    // 64-bit look-back words (n >= 2^31)
  uint64_t statusBytes;   // per-tile rows [nTiles + extra][256]
  uint64_t statusUsedBytes;  // the rows the LSD / top-digit passes use (nTiles + kSegTilePad)
  uint64_t gaBytes;       // group aggregates [nGroups][256] u32 (kGroup > 0)
  uint64_t gpBytes;       // group prefixes   [nGroups][256] status words
  uint64_t setBytes;      // one look-back table set = status + ga + gp
  uint64_t claimBytes;    // per pass: XCD-block claim state (tickets, block counter, 8 block tables)
  uint64_t hybridOff;     // 3-pass path (thrs_hybrid.hpp): bucket histogram, chunk table, meta
  uint64_t bigMax;        // most big chunks the per-bucket fallback can meet (thrs_fallback.hpp)
  uint64_t bigHistOff;    // their low digits' counts [bigMax][key bytes - 2][256]
  uint64_t hiPlaneOff;    // u32 keys without values: the bucket path's u8 plane (n bytes)
  uint64_t scratchBytes;  // header + 2 sets (ping-pong between passes) + 8 claim areas + hybrid area +
                          // fallback area [+ u8 plane]
};

// hybrid area: u32 joint[65536] | segHistA[8][256] | rowHist[256] | the same
// three for a squeezed second histogram | meta[64] (all zeroed up front) | chunkOff[65537] | chunkB0[65537] | segment tables
// of the two top-digit passes
constexpr uint64_t kJointBytes = kBuckets * 4;
constexpr uint64_t kSegHistAOff = kJointBytes;                    // per position segment: second-digit counts
constexpr uint64_t kRowHistOff = kSegHistAOff + kSegs * 256 * 4;  // top-digit counts (thrs_hist_joint)
// the second histogram of a squeezed sort (float keys: thrs_plan_rows, KeyMap<U, true>): joint | segHistA | rowHist
constexpr uint64_t kJoint2Off = kRowHistOff + 256 * 4;
constexpr uint64_t kSegHistA2Off = kJoint2Off + kJointBytes;
constexpr uint64_t kRowHist2Off = kSegHistA2Off + kSegs * 256 * 4;
constexpr uint64_t kMetaOff = kRowHist2Off + 256 * 4;             // zero: thrs_plan_rows raises its flags atomically
constexpr uint64_t kJointZero = kMetaOff + 256;
// the sampled squeeze (thrs_squeeze_sample: written whole every float sort, not zeroed)
constexpr uint64_t kSampleOff = kJointZero;
constexpr uint64_t kChunkOffOff = kJointZero + 256;
constexpr uint64_t kChunkB0Off = kChunkOffOff + round_up_c((kBuckets + 1) * 4, 256);
constexpr uint64_t kSegInfoOff = kChunkB0Off + round_up_c((kBuckets + 1) * 4, 256);  // segPos[9] | segTiles[9] ... tickets[8] at +256 B (thrs_pass_seg)
constexpr uint64_t kSegBaseOff = kSegInfoOff + 512;   // u32 [8][256] per-segment top-digit bases
constexpr uint64_t kSegInfoAOff = kSegBaseOff + kSegs * 256 * 4;  // the same two for the second-digit pass
constexpr uint64_t kSegBaseAOff = kSegInfoAOff + 512;
// big chunks of the per-bucket fallback: chunk ids, size prefix, tile prefix
constexpr uint64_t kBigBOff = kSegBaseAOff + kSegs * 256 * 4;
constexpr uint64_t kBigPosOff = kBigBOff + round_up_c((kBuckets + 1) * 4, 256);
constexpr uint64_t kBigTileOff = kBigPosOff + round_up_c((kBuckets + 1) * 4, 256);
constexpr uint64_t kZeroLogOff = kBigTileOff + round_up_c((kBuckets + 1) * 4, 256);  // f32: +-0 keys (thrs_hist_joint)
constexpr uint64_t kHybridBytes = kZeroLogOff + round_up_c(kZeroLogCap * 4, 256);
// the smallest local-sort capacity (LocSmall): a big chunk holds more keys
constexpr uint64_t kMinLocalCap = LocKVS::CAP;  // (8-byte keys or 8/16-byte values: the smallest thrs_local_kv chunk)
// tile ids of the segmented pass: each of the 8 segments adds at most two
// partial tiles (its first and last: seg_tiles) and rounds its id range up
// to a multiple of kGroup
constexpr uint64_t kSegTilePad = kSegs * (kGroup + 1);

inline Plan make_plan(int keyType, int valueBytesOrZero, uint32_t n) {
  Plan p{};
  p.kb = key_bytes_of(keyType);
  p.vb = valueBytesOrZero;
  p.tileKeys = tile_keys(p.kb, p.vb);
  p.nTiles = std::max<uint64_t>(1, ((uint64_t)n + p.tileKeys - 1) / p.tileKeys);
  p.wideStatus = (uint64_t)n >= (1ull << 31);
  // the per-bucket fallback (thrs_fallback.hpp): big chunks hold more keys
  // than the smallest local capacity each (4-byte keys-only: Loc16Tiny's),
  // and there are at most 65536 buckets
  static_assert(LocTiny::CAP == Loc16Tiny::CAP, "one smallest capacity for 4-byte keys");
  const uint64_t minCap = (p.kb == 4 && p.vb <= 4) ? (uint64_t)Loc16Tiny::CAP : kMinLocalCap;
  p.bigMax = std::min<uint64_t>(kBuckets, (uint64_t)n / (minCap + 1) + 1);
  // status rows: a tile id per tile, + the segmented passes' extra ids (each
  // segment rounds up to a look-back group) or the fallback's (a partial tile
  // per big chunk; the fallback passes use the same two table sets)
  // (the segmented passes may use smaller tiles: seg_tile_keys)
  const uint64_t segTiles = std::max<uint64_t>(p.nTiles, ((uint64_t)n + seg_tile_keys(p.kb, p.vb) - 1) /
                                                             seg_tile_keys(p.kb, p.vb));
  const uint64_t rows = segTiles + std::max<uint64_t>(kSegTilePad, p.bigMax);
  p.statusBytes = round_up(rows * kBins * (p.wideStatus ? 8 : 4), kAlign);
  p.statusUsedBytes = round_up((segTiles + kSegTilePad) * kBins * (p.wideStatus ? 8 : 4), kAlign);
  const uint64_t nGroups = kGroup > 0 ? (rows + kGroup - 1) / kGroup : 0;
  p.gaBytes = round_up(nGroups * kBins * 4, kAlign);
  p.gpBytes = round_up(nGroups * kBins * (p.wideStatus ? 8 : 4), kAlign);
  p.setBytes = p.statusBytes + p.gaBytes + p.gpBytes;
  const uint64_t nXb = (p.nTiles + kXcdBlock - 1) / kXcdBlock + 16;  // table stride (see xb_claim)
  p.claimBytes = round_up((16 + 8 * nXb) * 4, kAlign);
  p.hybridOff = kHeaderBytes + 2 * p.setBytes + 8 * p.claimBytes;
  p.bigHistOff = p.hybridOff + kHybridBytes;
  p.scratchBytes = p.bigHistOff + round_up(p.bigMax * (p.kb - 2) * kBins * 4, kAlign);
  // the u8 plane of the planes codecs (thrs_kernels.hpp kCodecSplit): the u16
  // planes fill keyOut, which is all a sortKeys caller must allocate
  // (getTemporaryBufferBytesForSortKeys = pSumBuffer + keyOutBuffer).  For
  // u32 / f32 keys-only at every n up to 2^31 + 2^25 (the bucket path's
  // range): the default takes it from kBucketMinKeysU32 / kBucketMinKeys4, and
  // a bucket path forced below that carries the planes too, so the codecs the
  // headline runs are tested element-wise at sizes the oracle finishes.
  // u32 / f32 keys with 4-byte values likewise, up to 2^30 + 2^26 (the u16 planes
  // fill keyOut, the values take valueOut as ever).
  p.hiPlaneOff = p.scratchBytes;
  if ((keyType == THRS_KEY_U32 || keyType == THRS_KEY_F32) &&
      ((valueBytesOrZero == 0 && (uint64_t)n <= (1ull << 31) + (1ull << 25)) ||
       (valueBytesOrZero == 4 && (uint64_t)n <= (1ull << 30) + (1ull << 26))))
    p.scratchBytes += round_up(n, kAlign);
  return p;
}

// ---- process-wide state, defined in thrs_capi.hip
int cu_count();
// HIP-event timing of the launches (thrs_profile_*): kind 0 = histogram +
// plan, 1 = device-wide digit pass, 2 = local sort, 3 = fallback-only launches
hipEvent_t prof_begin(hipStream_t s);
void prof_end(hipEvent_t a, hipStream_t s, int kind, int kernel, uint64_t bytes);
// records [a, b) around the launches issued in its lifetime, with the
// kernel's id (THRS_PK_*) and algorithmic bytes (0 = data-dependent)
struct ProfScope {
  hipStream_t s;
  int kind, kernel;
  uint64_t bytes;
  hipEvent_t a;
  ProfScope(hipStream_t s_, int k, int kern, uint64_t b) : s(s_), kind(k), kernel(kern), bytes(b), a(prof_begin(s_)) {}
  ~ProfScope() {
    if (a) prof_end(a, s, kind, kernel, bytes);
  }
};
extern uint64_t* g_stamps;   // THRS_STAMPS diagnostic builds only (thrs_debug_set_stamps)
// fault injection (THRS_FAULT_INJECT builds only, thrs_debug_inject; else 0):
// bit 0 = the plan's first big-chunk entry is made stale
extern int g_inject;
extern uint64_t* g_lstamps;  // same, local sort: [chunk][8] (thrs_debug_set_local_stamps)
// 1 = lane-ordered LDS atomics on this device (fast rank), 0 = ballot match
int probe_rank_mode(hipStream_t stream);
// device view of the current device's sticky error word, or nullptr (not
// set up: the sort then runs without publishing to it)
uint32_t* sticky_dev(hipStream_t stream);

template <typename F>
hipError_t allow_lds(F kernel, size_t bytes) {
  if (bytes <= 65536) return hipSuccess;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)bytes);
}

// One launch sequence.  Sort mode (counts == nullptr): the result lands in
// keys/vals.  Partition mode (counts != nullptr, nPass == 1,
// thrs_partition_pass): the pass writes keyOutBuf/valOutBuf, which are the
// caller's, and the digit's 256 bucket counts go to `counts`.
//   LSD path:    histogram of every digit + scan, nPass ping-pong passes,
//                copy-back after an odd pass count.
//   bucket path: 4-byte keys (u32 keys + 4-byte values over the whole key),
//                nPass >= 3 (thrs_hybrid.hpp): bucket histogram + plan,
//                [low-digit passes + copy, gated on the fallback flag], the
//                two top-digit passes (skipped when one bucket holds every
//                key), local sort.
// Every hipFuncSetAttribute happens before the first enqueue, so a failure
// there leaves the caller's buffers untouched.
// The path one sort takes (host decision, no device work): run_sort and
// thrs_path_info (thrs_capi.hip) share it.
struct PathSel {
  bool bucket, fullWindow, smallLocal, local16, wide16, tiny16, tinyPairs, small16, count16, local32, segTop, segA, planes, ranged, useXb;
  int nLow;
  int kvGeom;  // thrs_local_kv's geometry: 0 LocKV, 1 LocKVM, 2 LocKVS
  uint32_t cap;
};
template <int KT, int VB>
PathSel select_path(uint32_t n, int startBits, int nPass, const thrs_options& opt, const Plan& plan, bool partition) {
  using U = typename KeyTraits<KT>::U;
  const bool counts = partition;  // (a partition pass is one plain pass)
  // Bucket path (thrs_hybrid.hpp, thrs_fallback.hpp): a bucket histogram,
  // device passes for the window's TOP two digits only, then one in-LDS sort
  // of every 16-bit bucket.  Key / value types and their local sorts:
  //   4-byte keys, no values    any window with >= 3 digits: thrs_local16
  //                             (16-bit items; full window) or thrs_local
  //                             (32-bit items; windows, or when asked)
  //   4-byte keys, 4-B values   full window: thrs_local_pairs (items carry
  //                             positions; values -- and f32 keys -- permuted)
  //   4-byte keys, 8/16-B vals  full window: thrs_local_kv
  //   8-byte keys, any values   full window: thrs_local_kv
  constexpr int KB = (int)sizeof(U);
  constexpr bool kKeys4 = KB == 4 && VB == 0;
  constexpr bool kKV = KB == 8 || VB >= 8;
  const bool fullWindow = startBits == 0 && nPass * 8 >= (int)(8 * sizeof(U));
  // Size window of the default (uniform keys: n / 65536 keys per bucket;
  // docs/EXPERIMENTS.md row 29): the local sort costs about the same per chunk
  // whatever its size, so below a measured bound per key / value type (the
  // kBucketMin* constants) the two passes it replaces are cheaper;
  // above 2^30 + 2^26 the largest of 65536 uniform buckets (mean + ~4.5 sigma)
  // outgrows the chunk capacity and big chunks would take the per-bucket
  // fallback.  THRS_PATH_BUCKET forces the path for any n (tests).
  // Local geometries: 9216-key chunks for n <= 2^29, 18432 above (thrs_local_kv:
  // 4352 / 8704 / 17408, the last up to 2^30 + 2^24, the largest uniform
  // bucket ~3 sigma below the capacity); 4-byte keys-only up to 2^31 + 2^25
  // in 34816-key chunks (Loc16Wide).
  const uint64_t nn = n;
  // a key range (the multi-GPU finish: its keys fill the image space, so the
  // buckets are uniform whatever the global distribution) takes the bucket
  // path from 2^27 (C2's 2^30 keys over 8 GPUs; docs/EXPERIMENTS.md row 84)
  const bool rangedReq = opt.keyRange == 1 && fullWindow && !counts;
  // lower bounds by measurement (docs/EXPERIMENTS.md rows 87, 112, 115, 129,
  // 130; the kBucketMin* constants) (the 2^27 bound of a ranged finish is
  // measured for 4-byte keys without values, the C2 finish; other key /
  // value types keep their own bounds)
  const uint64_t minN = (rangedReq && kKeys4) ? (1ull << 27)
                        : kKeys4  ? (KT == 0 ? kBucketMinKeysU32 : kBucketMinKeys4)
                        : (KB == 4 && VB == 4) ? (KT == 0 ? kBucketMinPairsU32 : kBucketMinPairs4)
                        : KB == 4 ? (VB == 8 ? kBucketMinK4V8 : kBucketMinK4V16)
                        : VB == 16 ? kBucketMinK8V16
                        : VB == 8 ? (KT == 3 ? kBucketMinF64V8 : kBucketMinK8V8)
                                  : kBucketMinK8;
  const bool sizeOk = nn >= minN && nn <= (1ull << 30) + (kKV ? (1ull << 24) : (1ull << 26));
  const bool wideOk = kKeys4 && fullWindow && nn > (1ull << 30) + (1ull << 26) && nn <= (1ull << 31) + (1ull << 25);
  // the local geometry follows the keys per USED bucket: a range whose span
  // is just above a power of two fills only about half of the image space
  // ((img - lo) << sh keeps its top bit clear for most keys), so its
  // buckets hold up to twice n / 65536 keys (the multi-GPU finish at 2
  // GPUs: rank 1's range is [~2^31, 2^32 - 1])
  double fill = 1.0;
  if (rangedReq && opt.rangeHi > opt.rangeLo) {
    const U span = (U)opt.rangeHi - (U)opt.rangeLo;
    const int sh = sizeof(U) == 4 ? __builtin_clz((uint32_t)span) : __builtin_clzll((uint64_t)span);
    fill = std::ldexp((double)span, sh - (int)(8 * sizeof(U)));  // in [0.5, 1)
  }
  const double nEff = (double)nn / std::max(fill, 0.5);
  const bool smallLocal = opt.localGeometry == THRS_LOCAL_SMALL ? true
                          : opt.localGeometry != THRS_LOCAL_AUTO  // BIG, BIG32 and the 16-bit kernels
                              ? false
                              : nEff <= (double)(1ull << 29);
  const bool bucket = !counts && nPass >= 3 &&
                      (opt.path == THRS_PATH_BUCKET || (opt.path == THRS_PATH_AUTO && (sizeOk || wideOk))) &&
                      (kKeys4 || fullWindow);
  const int nLow = nPass - 2;
  // 4-byte keys over the whole key: the local sort on 16-bit items
  // (thrs_local16) over single-bucket chunks, unless 32-bit items are asked
  const bool local16 = kKeys4 && bucket && fullWindow && opt.localGeometry != THRS_LOCAL_BIG32;
  // ... in 34816-key chunks (explicitly, or by default above 2^30 + 2^26);
  // 9216-key chunks for n <= 2^29 (or asked: SMALL)
  const bool wide16 = local16 && (opt.localGeometry == THRS_LOCAL_WIDE16 ||
                                  (opt.localGeometry == THRS_LOCAL_AUTO && nEff > (double)((1ull << 30) + (1ull << 26))));
  // ... in 4096-key chunks for u32 up to 3 x 2^26 keys, f32 up to 2^27 (or
  // asked: TINY16; docs/EXPERIMENTS.md rows 112, 131)
  const bool tiny16 = local16 && !wide16 &&
                      (opt.localGeometry == THRS_LOCAL_TINY16 ||
                       (opt.localGeometry == THRS_LOCAL_AUTO &&
                        nEff <= (double)(KT == 0 ? kTiny16MaxKeys : kTiny16MaxKeysF32)));
  const bool small16 = local16 && !wide16 && !tiny16 && smallLocal;
  // u32 keys + 4-byte values likewise (thrs_local_pairs in LocTiny chunks)
  const bool tinyPairs = KB == 4 && VB == 4 && bucket && fullWindow &&
                         (opt.localGeometry == THRS_LOCAL_TINY16 ||
                          (opt.localGeometry == THRS_LOCAL_AUTO && nEff <= (double)kTiny16MaxKeys));
  // ... u32 only: sorted by counting (thrs_local_count16) when asked (it
  // measured slower, docs/EXPERIMENTS.md row 56)
  const bool count16 = local16 && KT == 0 && !wide16 && !small16 && opt.localGeometry == THRS_LOCAL_COUNT16;
  const bool local32 = kKeys4 && bucket && !local16;
  // thrs_local_kv (8-byte keys, 8/16-byte values): 17408-key chunks from 2^29
  // keys, 8704 up to there, 4352 up to 3 x 2^26 (mean bucket + ~5 sigma below
  // the capacity; docs/EXPERIMENTS.md row 130); asked: BIG / SMALL / TINY16
  const int kvGeom = !kKV                                           ? 0
                     : opt.localGeometry == THRS_LOCAL_TINY16       ? 2
                     : opt.localGeometry == THRS_LOCAL_SMALL        ? 1
                     : opt.localGeometry != THRS_LOCAL_AUTO         ? 0
                     : nEff <= (double)kTiny16MaxKeys               ? 2
                     : nEff <= (double)(1ull << 29)                 ? 1
                                                                    : 0;
  const bool segTop = opt.segmented != THRS_SEG_NONE;
  const bool segA = opt.segmented == THRS_SEG_AUTO;
  // u32 / f32 local16 with both top-digit passes segmented: the passes carry
  // the keys' IMAGES as planes (thrs_kernels.hpp kCodecSplit / kCodecPlanes):
  // keyOut (4n bytes) = lo u16[n] | lo2 u16[n], the u8 plane hi[n] at the end
  // of the scratch.  f32: -0 and +0 share one image, so the local sort takes
  // the zeros' signs from the zero log (thrs_hist_joint), and a plan that saw
  // a -0 among more zeros than the log holds runs the whole-key passes
  // instead (mode 3).  u32 / f32 keys + 4-byte values likewise
  // (thrs_local_pairs over the lo2 plane; the values move as they are).
  const bool planes = (KT == 0 || KT == 2) && (local16 || (VB == 4 && bucket && fullWindow)) && segA &&
                      opt.planes != THRS_PLANES_OFF && plan.scratchBytes - plan.hiPlaneOff >= (uint64_t)n;
  // the local sort's chunk capacity (a bigger bucket is a big chunk)
  const uint32_t cap = kKV ? (kvGeom == 2 ? LocKVS::CAP : kvGeom == 1 ? LocKVM::CAP : LocKV::CAP)
                       : local16 ? (wide16    ? Loc16Wide::CAP
                                    : tiny16  ? Loc16Tiny::CAP
                                    : small16 ? Loc16Small::CAP
                                              : Loc16::CAP)
                       : tinyPairs ? LocTiny::CAP
                                   : (smallLocal ? LocSmall::CAP : LocBig::CAP);
  // The key range (thrs_options.keyRange, thrs_kernels.hpp KeyMap): for
  // full-window sorts, except the 32-bit local sort (it sorts the keys
  // themselves and pads with keys)
  const bool ranged = opt.keyRange == 1 && fullWindow && !counts && !local32;
  // XCD-block claims (thrs_pass_xb) pay off where runs are short and the
  // grid is large: 4-byte keys without values, n >= 2^29 (docs/EXPERIMENTS.md
  // row 19: +4-6% there, neutral at 2^28, -2..-6% for pairs / f32 at 2^28).
  const bool useXb = opt.tileClaims == THRS_CLAIMS_XCD_BLOCKS ? true
                     : opt.tileClaims == THRS_CLAIMS_TICKET ? false
                                                            : (sizeof(U) == 4 && VB == 0 && n >= (1u << 29));
  PathSel P{};
  P.bucket = bucket;
  P.fullWindow = fullWindow;
  P.smallLocal = smallLocal;
  P.local16 = local16;
  P.wide16 = wide16;
  P.tiny16 = tiny16;
  P.tinyPairs = tinyPairs;
  P.small16 = small16;
  P.count16 = count16;
  P.local32 = local32;
  P.segTop = segTop;
  P.segA = segA;
  P.planes = planes;
  P.ranged = ranged;
  P.useXb = useXb;
  P.nLow = nLow;
  P.kvGeom = kvGeom;
  P.cap = cap;
  return P;
}

#ifdef THRS_RUN_KT
template <int KT, int VB, typename ST>
int run_sort(void* keys, void* vals, uint32_t n, void* tmp, void* keyOutBuf, void* valOutBuf, int startBits, int nPass,
             bool desc, const Plan& plan, const thrs_options& opt, hipStream_t stream, uint32_t* counts = nullptr) {
  using U = typename KeyTraits<KT>::U;
  using VW = typename ValueWord<VB>::T;
  using G = PassGeom<sizeof(U), VB>;

  char* scratch = static_cast<char*>(tmp);
  uint32_t* hist = reinterpret_cast<uint32_t*>(scratch + kHistOff);
  uint32_t* base = reinterpret_cast<uint32_t*>(scratch + kBaseOff);
  uint32_t* counters = reinterpret_cast<uint32_t*>(scratch + kCounterOff);
  uint32_t* err = reinterpret_cast<uint32_t*>(scratch + kErrOff);
  // table sets: [status | ga | gp] x 2; pass p uses set p&1 and clears its
  // rows of set (p+1)&1 for the next pass
  ST* status[2];
  GroupTables<ST> grp[2];
  for (int i = 0; i < 2; ++i) {
    char* set = scratch + kHeaderBytes + i * plan.setBytes;
    status[i] = reinterpret_cast<ST*>(set);
    grp[i].ga = reinterpret_cast<uint32_t*>(set + plan.statusBytes);
    grp[i].gp = reinterpret_cast<ST*>(set + plan.statusBytes + plan.gaBytes);
    grp[i].nTiles = (uint32_t)plan.nTiles;
  }
  char* hyb = scratch + plan.hybridOff;
  uint32_t* joint = reinterpret_cast<uint32_t*>(hyb);
  uint32_t* chunkOff = reinterpret_cast<uint32_t*>(hyb + kChunkOffOff);
  uint32_t* chunkB0 = reinterpret_cast<uint32_t*>(hyb + kChunkB0Off);
  uint32_t* meta = reinterpret_cast<uint32_t*>(hyb + kMetaOff);
  U* keyOut = static_cast<U*>(keyOutBuf);
  VW* valOut = static_cast<VW*>(valOutBuf);

  const U orderMask = desc ? (U)~(U)0 : (U)0;
  constexpr int KB = (int)sizeof(U);
  constexpr bool kKeys4 = KB == 4 && VB == 0;
  constexpr bool kPairs4 = KB == 4 && VB == 4;
  constexpr bool kKV = KB == 8 || VB >= 8;
  const PathSel P = select_path<KT, VB>(n, startBits, nPass, opt, plan, counts != nullptr);
  const bool bucket = P.bucket, smallLocal = P.smallLocal, local16 = P.local16, wide16 = P.wide16;
  const bool small16 = P.small16, count16 = P.count16, local32 = P.local32, segTop = P.segTop, segA = P.segA;
  const bool planes = P.planes, ranged = P.ranged, useXb = P.useXb;
  const int nLow = P.nLow;
  const uint32_t cap = P.cap;
  // the device-chosen squeeze (float keys over the whole key, single-bucket
  // chunks: thrs_plan_rows; KeyMap<U, true> in thrs_kernels.hpp)
  // (both top passes segmented: the squeeze-aware pass kernel)
  const bool squeeze = kSqueezable<KT> && bucket && P.fullWindow && !local32 && P.segA &&
                       opt.squeeze == THRS_SQUEEZE_AUTO;
  const SqueezeWords* sqw =
      squeeze ? reinterpret_cast<const SqueezeWords*>(scratch + plan.hybridOff + kMetaOff + kMetaSqueeze * 4) : nullptr;
  SqueezeWords* sample = squeeze ? reinterpret_cast<SqueezeWords*>(scratch + plan.hybridOff + kSampleOff) : nullptr;
  // f32 on the bucket path: the zero log (+-0 keys' positions and signs;
  // the planes restore the signs from it) and the -0 flag (pairs rebuild
  // their keys from the images unless it is set)
  uint32_t* zeroLog = (KT == 2 && bucket && !local32) ? reinterpret_cast<uint32_t*>(scratch + plan.hybridOff + kZeroLogOff)
                                                     : nullptr;
  KeyMap<U> km{orderMask, (U)0, 0u};
  if (ranged) {
    const U span = (U)opt.rangeHi - (U)opt.rangeLo;  // > 0 (sort_impl returns at once for 0)
    km.lo = (U)opt.rangeLo;
    km.sh = sizeof(U) == 4 ? (uint32_t)__builtin_clz((uint32_t)span) : (uint32_t)__builtin_clzll((uint64_t)span);
  }
  const KeyMap<uint32_t> km32{(uint32_t)km.mask, (uint32_t)km.lo, km.sh};
  uint16_t* loP = static_cast<uint16_t*>(keyOutBuf);
  uint16_t* lo2P = loP + n;
  uint8_t* hiP = reinterpret_cast<uint8_t*>(scratch + plan.hiPlaneOff);
  const bool atomicRank = opt.rank == THRS_RANK_ATOMIC ? true
                          : opt.rank == THRS_RANK_BALLOT ? false
                                                         : probe_rank_mode(stream) != 0;
  uint32_t* sticky = sticky_dev(stream);
  // Partition mode by a digit at bit 8 or above (thrs_partition_pass, the
  // multi-GPU exchange): the bucket histogram in segRows mode gives the digit's
  // counts per position segment, and one segmented pass (thrs_pass_seg, keys
  // codec, as the bucket path's second-digit pass) moves the keys.
  const bool segPart = counts != nullptr && startBits >= 8 && opt.segmented != THRS_SEG_NONE;

  // ---- kernels and their LDS opt-ins, before anything is enqueued
  const size_t lds = G::LDS_BYTES;
  auto kernelXb = atomicRank ? thrs_pass_xb<KT, VB, ST, true> : thrs_pass_xb<KT, VB, ST, false>;
  auto kernelBig = atomicRank ? thrs_pass_big<KT, VB, ST, true> : thrs_pass_big<KT, VB, ST, false>;
  auto kernel = useXb ? kernelXb : (atomicRank ? thrs_pass<KT, VB, ST, true> : thrs_pass<KT, VB, ST, false>);
  auto sk = atomicRank ? thrs_pass_seg<KT, VB, ST, true> : thrs_pass_seg<KT, VB, ST, false>;
  // plane codecs, each top-digit pass one launch with its whole-key body
  // (thrs_pass_seg2; u32 / f32 keys without values or with 4-byte values
  // only: `planes` is false elsewhere, and the other instantiations are
  // never launched).  The planes codec reads images (identity map): the u32
  // kernel serves both key types.
  constexpr bool kPlanesK = (KT == 0 || KT == 2) && VB == 0;
  constexpr bool kPlanesP = (KT == 0 || KT == 2) && VB == 4;
  constexpr int kKT4 = kPlanesK || kPlanesP ? KT : 0;
  constexpr int kVB4 = kPlanesP ? 4 : 0;
  auto sk2Split = atomicRank ? thrs_pass_seg2<kKT4, kKT4, kVB4, ST, true, kCodecSplit>
                             : thrs_pass_seg2<kKT4, kKT4, kVB4, ST, false, kCodecSplit>;
  auto sk2Planes = atomicRank ? thrs_pass_seg2<0, kKT4, kVB4, ST, true, kCodecPlanes>
                              : thrs_pass_seg2<0, kKT4, kVB4, ST, false, kCodecPlanes>;
  const uint32_t segTileKeys = (uint32_t)seg_tile_keys(KB, VB);
  const int histPasses = nPass;
  const size_t histLds = (size_t)histPasses * kBins * hist_copies<(int)sizeof(U)>() * 4;
  if (allow_lds(thrs_hist<KT>, histLds) != hipSuccess || allow_lds(kernel, lds) != hipSuccess ||
      allow_lds(kernelXb, lds) != hipSuccess || allow_lds(kernelBig, lds) != hipSuccess)
    return THRS_ERROR_HIP;
  if (bucket || segPart) {
    if (allow_lds(thrs_hist_joint<KT>, kJointLds) != hipSuccess || allow_lds(sk, lds) != hipSuccess ||
        (squeeze && allow_lds(thrs_hist_joint<KT, true>, kJointLds) != hipSuccess))
      return THRS_ERROR_HIP;
    if (planes && (allow_lds(sk2Split, lds) != hipSuccess || allow_lds(sk2Planes, lds) != hipSuccess))
      return THRS_ERROR_HIP;
    if constexpr (kKV) {
      if (allow_lds(atomicRank ? thrs_local_kv<KT, VB, true, LocKV> : thrs_local_kv<KT, VB, false, LocKV>,
                    LocKV::LDS) != hipSuccess ||
          allow_lds(atomicRank ? thrs_local_kv<KT, VB, true, LocKVM> : thrs_local_kv<KT, VB, false, LocKVM>,
                    LocKVM::LDS) != hipSuccess ||
          allow_lds(atomicRank ? thrs_local_kv<KT, VB, true, LocKVS> : thrs_local_kv<KT, VB, false, LocKVS>,
                    LocKVS::LDS) != hipSuccess)
        return THRS_ERROR_HIP;
    } else if constexpr (kPairs4) {
      if (allow_lds(atomicRank ? thrs_local_pairs<KT, true, LocBig> : thrs_local_pairs<KT, false, LocBig>,
                    LocBig::lds<U>()) != hipSuccess ||
          allow_lds(atomicRank ? thrs_local_pairs<KT, true, LocSmall> : thrs_local_pairs<KT, false, LocSmall>,
                    LocSmall::lds<U>()) != hipSuccess)
        return THRS_ERROR_HIP;
    } else if constexpr (kKeys4) {
      if (allow_lds(atomicRank ? thrs_local16<KT, true, Loc16> : thrs_local16<KT, false, Loc16>, Loc16::LDS) !=
              hipSuccess ||
          allow_lds(atomicRank ? thrs_local16<KT, true, Loc16Wide> : thrs_local16<KT, false, Loc16Wide>,
                    Loc16Wide::LDS) != hipSuccess ||
          allow_lds(atomicRank ? thrs_local<KT, true, LocBig> : thrs_local<KT, false, LocBig>, LocBig::lds<U>()) !=
              hipSuccess ||
          allow_lds(atomicRank ? thrs_local<KT, true, LocSmall> : thrs_local<KT, false, LocSmall>,
                    LocSmall::lds<U>()) != hipSuccess)
        return THRS_ERROR_HIP;
      if constexpr (KT == 0) {
        if (allow_lds(thrs_local_count16<true>, LocCount::LDS) != hipSuccess ||
            allow_lds(thrs_local_count16<false>, LocCount::LDS) != hipSuccess)
          return THRS_ERROR_HIP;
      }
    }
  }
  // persistent grids (occupancy x CUs): the XCD-block kernel, and the
  // per-bucket fallback's passes (thrs_pass_big): a launch of nTiles
  // workgroups that all exit at once would cost ~0.1 ms at 2^18 tiles
  auto persistent_grid = [&](auto kern) -> uint32_t {
    int perCU = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, kern, G::THREADS, lds) != hipSuccess || perCU < 1)
      perCU = 1;
    return (uint32_t)std::min<uint64_t>(plan.nTiles, (uint64_t)perCU * cu_count());
  };
  const uint32_t gridXb = useXb ? persistent_grid(kernelXb) : (uint32_t)plan.nTiles;
  const uint32_t gridBig = bucket ? persistent_grid(kernelBig) : 1u;
  const uint32_t grid = useXb ? gridXb : (uint32_t)plan.nTiles;
  int segPerCU = 0;
  if ((bucket || segPart) &&
      (hipOccupancyMaxActiveBlocksPerMultiprocessor(&segPerCU, sk, G::THREADS, lds) != hipSuccess || segPerCU < 1))
    segPerCU = 1;

  // header (histograms, tile counters, error word) + first status table; the
  // bucket path with an odd number of (skippable) low passes starts on set 1
  // too, and zeroes its bucket histogram
  // Bucket path: ONE memset from the header through the bucket histogram --
  // both table sets (the top-digit passes use set nLow&1 and the other one,
  // and no launch before them dirties the other unless it also cleans it:
  // fallback passes clear their successor's rows), all 8 claim areas, joint.
  // (one zeroing launch over up to three ranges: a set's status rows past
  // statusUsedBytes serve only the per-bucket fallback, which zeroes them)
  // Bucket path: the look-back tables are zeroed by thrs_hist_joint (`tables`)
  ZeroRanges tables{};
  {
    const uint64_t set0 = kHeaderBytes, set1 = kHeaderBytes + plan.setBytes;
    ZeroRanges z{};
    if (bucket || segPart) {
      z.ptr[0] = scratch;  // header
      z.words[0] = kHeaderBytes / 16;
      z.ptr[1] = scratch + set1 + plan.setBytes;  // claim areas, bucket histogram, meta
      z.words[1] = (plan.hybridOff + kJointZero - (set1 + plan.setBytes)) / 16;
      tables.ptr[0] = scratch + set0;  // set 0's used rows
      tables.words[0] = plan.statusUsedBytes / 16;
      tables.ptr[1] = scratch + set0 + plan.statusBytes;  // set 0's group tables .. set 1's used rows
      tables.words[1] = (set1 + plan.statusUsedBytes - (set0 + plan.statusBytes)) / 16;
      tables.ptr[2] = scratch + set1 + plan.statusBytes;  // set 1's group tables
      tables.words[2] = (plan.setBytes - plan.statusBytes) / 16;
    } else {
      z.ptr[0] = scratch;
      z.words[0] = (set0 + plan.statusUsedBytes) / 16;
      z.ptr[1] = scratch + set0 + plan.statusBytes;  // set 0's group tables
      z.words[1] = (plan.gaBytes + plan.gpBytes) / 16;
      if (useXb) {  // the XCD-block claim areas of every pass
        z.ptr[2] = scratch + kHeaderBytes + 2 * plan.setBytes;
        z.words[2] = (uint64_t)nPass * plan.claimBytes / 16;
      }
    }
    ProfScope prof(stream, 0, THRS_PK_ZERO, 16 * (z.words[0] + z.words[1] + z.words[2]));
    hipLaunchKernelGGL(thrs_zero_ranges, dim3(std::min<uint32_t>(2048, 8 * cu_count())), dim3(256), 0, stream, z);
  }
  char* claim = scratch + kHeaderBytes + 2 * plan.setBytes;  // 8 per-pass claim areas

  const uint64_t keyBytes = (uint64_t)n * sizeof(U), moveBytes = 2 * (uint64_t)n * (sizeof(U) + VB);
  {  // histograms of every pass in one read of the keys
    const int vec = (reinterpret_cast<uintptr_t>(keys) % 16) == 0;
    const uint64_t want = ((uint64_t)n + kHistThreads * 64 - 1) / (kHistThreads * 64);
    const int hgrid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)cu_count() * THRS_HIST_GRID_MULT));
    if (bucket) {
      if (squeeze) {  // the sample's guess at the squeeze, for the first histogram
        ProfScope prof(stream, 0, THRS_PK_SQUEEZE_SAMPLE, (uint64_t)kSqSample * sizeof(U));
        hipLaunchKernelGGL(thrs_squeeze_sample<KT>, dim3(kSqBlocks), dim3(kSqSampleThreads), 0, stream,
                           static_cast<const U*>(keys), n, km, cap, sample, meta);
      }
      // the histogram workgroups' partial counts go to keyOut (free until
      // the first pass) and thrs_hist_reduce sums them, where they fit
      uint32_t* partial = (uint64_t)hgrid * kJointWords * 4 <= (uint64_t)n * sizeof(U)
                              ? reinterpret_cast<uint32_t*>(keyOutBuf)
                              : nullptr;
      {
        ProfScope prof(stream, 0, THRS_PK_HIST_JOINT, keyBytes);
        hipLaunchKernelGGL(thrs_hist_joint<KT>, dim3(hgrid), dim3(kHistThreads), kJointLds, stream,
                         static_cast<const U*>(keys), n, km, startBits + 8 * nLow, vec, joint,
                         reinterpret_cast<uint32_t*>(hyb + kSegHistAOff), reinterpret_cast<uint32_t*>(hyb + kRowHistOff),
                         tables, meta, sample, zeroLog, partial, 0);
      }
      if (partial) {
        ProfScope prof(stream, 0, THRS_PK_HIST_REDUCE, (uint64_t)hgrid * kJointWords * 4);
        hipLaunchKernelGGL(thrs_hist_reduce, dim3(kJointWords / 128), dim3(kHistReduceThreads), 0, stream, partial,
                           (uint32_t)hgrid, joint);
      }
      // single-bucket chunks: one workgroup per top digit; float keys with
      // the whole key decide the squeeze (sqMode 1) and, if it went on,
      // histogram and plan once more under it (gated: a few us otherwise)
      auto plan_rows = [&](int sqMode, uint64_t jOff, uint64_t sOff, uint64_t rOff) {
        ProfScope prof(stream, 0, THRS_PK_PLAN, 3 * kJointBytes);
        hipLaunchKernelGGL(thrs_plan_rows, dim3(kBins), dim3(kPlanRowThreads), 0, stream,
                           reinterpret_cast<const uint32_t*>(hyb + jOff), reinterpret_cast<const uint32_t*>(hyb + rOff),
                           reinterpret_cast<const uint32_t*>(hyb + sOff), n, cap, base + nLow * kBins,
                           chunkOff, chunkB0, meta, reinterpret_cast<uint32_t*>(hyb + kSegInfoOff),
                           reinterpret_cast<uint32_t*>(hyb + kSegBaseOff), segTileKeys, (uint32_t)hgrid,
                           reinterpret_cast<uint32_t*>(hyb + kSegInfoAOff), reinterpret_cast<uint32_t*>(hyb + kSegBaseAOff),
                           reinterpret_cast<uint32_t*>(hyb + kBigBOff), sqMode, 8 * KB,
                           reinterpret_cast<uint32_t*>(hyb + kBigPosOff), reinterpret_cast<uint32_t*>(hyb + kBigTileOff),
                           reinterpret_cast<uint4*>(scratch + plan.bigHistOff), nLow,
                           sqMode == 1 ? static_cast<const SqueezeWords*>(sample) : nullptr,
                           planes ? (VB ? 2 : 1) : 0,  // (2: with values, no aligned tiles)
                           err, g_inject);
      };
      if (!local32 && squeeze) {
        plan_rows(1, 0, kSegHistAOff, kRowHistOff);
        // (the second histogram runs only on a wrong guess: it flushes with
        // global atomics, so no gated reduce launch follows it every sort)
        {
          ProfScope prof(stream, 0, THRS_PK_HIST_JOINT, keyBytes);
          hipLaunchKernelGGL((thrs_hist_joint<KT, true>), dim3(hgrid), dim3(kHistThreads), kJointLds, stream,
                             static_cast<const U*>(keys), n, km, startBits + 8 * nLow, vec,
                             reinterpret_cast<uint32_t*>(hyb + kJoint2Off), reinterpret_cast<uint32_t*>(hyb + kSegHistA2Off),
                             reinterpret_cast<uint32_t*>(hyb + kRowHist2Off), ZeroRanges{}, meta, sqw, nullptr, nullptr, 0);
        }
        plan_rows(2, kJoint2Off, kSegHistA2Off, kRowHist2Off);
      } else if (!local32) {
        plan_rows(0, 0, kSegHistAOff, kRowHistOff);
      } else {
        ProfScope prof(stream, 0, THRS_PK_PLAN, 3 * kJointBytes);
        // chunks: whole buckets; neighbouring buckets below kLocCap/2 keys share one
        hipLaunchKernelGGL(thrs_plan, dim3(1), dim3(kPlanThreads), 0, stream, joint, n, base + nLow * kBins, chunkOff,
                           chunkB0, meta, cap, smallLocal ? kLocSmallLogT : kLocLogT,
                           reinterpret_cast<uint32_t*>(hyb + kSegInfoOff), reinterpret_cast<uint32_t*>(hyb + kSegBaseOff),
                           segTileKeys, reinterpret_cast<const uint32_t*>(hyb + kSegHistAOff), (uint32_t)hgrid,
                           reinterpret_cast<uint32_t*>(hyb + kSegInfoAOff), reinterpret_cast<uint32_t*>(hyb + kSegBaseAOff),
                           reinterpret_cast<uint32_t*>(hyb + kBigBOff));
      }
    } else if (segPart) {
      {
        ProfScope prof(stream, 0, THRS_PK_HIST_JOINT, keyBytes);
        hipLaunchKernelGGL(thrs_hist_joint<KT>, dim3(hgrid), dim3(kHistThreads), kJointLds, stream,
                           static_cast<const U*>(keys), n, km, startBits - 8, vec, nullptr,
                           reinterpret_cast<uint32_t*>(hyb + kSegHistAOff), reinterpret_cast<uint32_t*>(hyb + kRowHistOff),
                           tables, meta, nullptr, nullptr, nullptr, 1);
      }
      ProfScope prof(stream, 0, THRS_PK_PLAN, 3 * kBins * 4);
      hipLaunchKernelGGL(thrs_partition_plan, dim3(1), dim3(kBins), 0, stream,
                         reinterpret_cast<const uint32_t*>(hyb + kRowHistOff),
                         reinterpret_cast<const uint32_t*>(hyb + kSegHistAOff), n, (uint32_t)hgrid, segTileKeys, counts,
                         reinterpret_cast<uint32_t*>(hyb + kSegInfoAOff), reinterpret_cast<uint32_t*>(hyb + kSegBaseAOff));
    } else {
      {
        ProfScope prof(stream, 0, THRS_PK_HIST, keyBytes);
        hipLaunchKernelGGL(thrs_hist<KT>, dim3(hgrid), dim3(kHistThreads), histLds, stream,
                           static_cast<const U*>(keys), n, km, startBits, nPass, vec, hist);
      }
      ProfScope prof(stream, 0, THRS_PK_SCAN, 2 * (uint64_t)nPass * kBins * 4);
      hipLaunchKernelGGL(thrs_scan, dim3(1), dim3(kThreads), 0, stream, hist, base, nPass);
    }
    if (counts && !segPart &&
        hipMemcpyAsync(counts, hist, kBins * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream) != hipSuccess)
      return THRS_ERROR_HIP;
  }


  // pass p: digit at startBits + 8p, tables of set p&1; gate != nullptr runs
  // it only if bit *gate of gateMask is set (meta words written by thrs_plan)
  auto launch_pass = [&](int p, U* kin, U* kout, VW* vin, VW* vout, const uint32_t* gate, uint32_t gateMask) {
    const bool more = p + 1 < nPass;
    ST* next = more ? status[(p + 1) & 1] : nullptr;
    GroupTables<ST> g = grp[p & 1];
    g.gaNext = more ? grp[(p + 1) & 1].ga : nullptr;
    g.gpNext = more ? grp[(p + 1) & 1].gp : nullptr;
    ProfScope prof(stream, 1, useXb ? THRS_PK_PASS_XB : THRS_PK_PASS, moveBytes);
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(G::THREADS), lds, stream, kin, kout, vin, vout, n, km, startBits + 8 * p,
                       base + p * kBins, status[p & 1], next,
                       useXb ? reinterpret_cast<uint32_t*>(claim + p * plan.claimBytes) : counters + p, err, g,
                       g_stamps ? g_stamps + (uint64_t)p * plan.nTiles * kStampSlots : nullptr, gate, gateMask);
  };
  auto publish_error = [&]() -> int {
    if (sticky) hipLaunchKernelGGL(thrs_err_publish, dim3(1), dim3(1), 0, stream, err, sticky);
    return hipGetLastError() == hipSuccess ? THRS_SUCCESS : THRS_ERROR_HIP;
  };

  if (segPart) {  // the one pass: keys (and values) to the caller's output buffers
    ProfScope prof(stream, 1, THRS_PK_PASS_SEG, moveBytes);
    hipLaunchKernelGGL(sk, dim3((uint32_t)segPerCU * cu_count()), dim3(G::THREADS), lds, stream,
                       static_cast<const U*>(keys), keyOut, static_cast<const VW*>(vals), valOut, km, startBits,
                       reinterpret_cast<uint32_t*>(hyb + kSegInfoAOff), reinterpret_cast<const uint32_t*>(hyb + kSegBaseAOff),
                       status[0], err, grp[0], nullptr, 0u, nullptr,
                       g_stamps ? g_stamps : nullptr, nullptr, nullptr);
    if (hipGetLastError() != hipSuccess) return THRS_ERROR_HIP;
    return publish_error();
  }
  if (!bucket) {
    U* kin = static_cast<U*>(keys);
    U* kout = keyOut;
    VW* vin = static_cast<VW*>(vals);
    VW* vout = valOut;
    for (int p = 0; p < nPass; ++p) {
      launch_pass(p, kin, kout, vin, vout, nullptr, 0u);
      std::swap(kin, kout);
      std::swap(vin, vout);
    }
    if (hipGetLastError() != hipSuccess) return THRS_ERROR_HIP;
    if ((nPass & 1) && !counts) {  // result must end in the caller's buffers (hpp:936-943), stream-ordered here
      if (hipMemcpyAsync(keys, keyOut, (size_t)n * sizeof(U), hipMemcpyDeviceToDevice, stream) != hipSuccess)
        return THRS_ERROR_HIP;
      if (VB && hipMemcpyAsync(vals, valOut, (size_t)n * VB, hipMemcpyDeviceToDevice, stream) != hipSuccess)
        return THRS_ERROR_HIP;
    }
    return publish_error();
  }

  // ---- bucket path: the two top digits, the local sort, the per-bucket fallback
  {
    U* K = static_cast<U*>(keys);
    VW* V = static_cast<VW*>(vals);
    uint32_t* mode = meta + kMetaMode;
    // The two top digits: XCD-segmented passes (thrs_kernels.hpp
    // thrs_pass_seg) -- the second digit over position segments (the bucket
    // histogram's workgroup ranges), the top digit over second-digit ranges.
    // Gates on meta[kMetaMode]: mode 0 (every bucket fits its local sort) and
    // mode 1 (some big chunks: the per-bucket fallback needs the full keys,
    // so the key-plane codecs run in mode 0 only); mode 2 (one bucket holds
    // every key: both top digits constant) neither -- both are identities,
    // and skipping both keeps the keys in K.
    auto launch_seg = [&](int p, U* kin, U* kout, VW* vin, VW* vout, uint64_t infoOff, uint64_t baseOff,
                          const uint32_t* gate, uint32_t gateMask) {
      ProfScope prof(stream, 1, THRS_PK_PASS_SEG, moveBytes);
      hipLaunchKernelGGL(sk, dim3((uint32_t)segPerCU * cu_count()), dim3(G::THREADS), lds, stream, kin, kout, vin,
                         vout, km, startBits + 8 * p, reinterpret_cast<uint32_t*>(hyb + infoOff),
                         reinterpret_cast<const uint32_t*>(hyb + baseOff), status[p & 1], err, grp[p & 1], gate,
                         gateMask, hiP,
                         g_stamps ? g_stamps + (uint64_t)(p - nLow) * (plan.nTiles + kSegTilePad) * kStampSlots
                                  : nullptr,
                         sqw, nullptr);
    };
    // planes: the codec and the whole-key body of one pass in one launch
    // (thrs_pass_seg2, mode-dispatched; kCodecPlanes: image-space input,
    // identity map, digit at bits 16-23 of k')
    auto launch_seg2 = [&](int p, bool top) {
      ProfScope prof(stream, 1, THRS_PK_PASS_SEG, moveBytes);
      uint32_t* kA = top ? reinterpret_cast<uint32_t*>(loP) : reinterpret_cast<uint32_t*>(K);
      uint32_t* oA = reinterpret_cast<uint32_t*>(top ? lo2P : loP);
      uint32_t* kB = reinterpret_cast<uint32_t*>(top ? keyOut : K);
      uint32_t* oB = reinterpret_cast<uint32_t*>(top ? K : keyOut);
      hipLaunchKernelGGL(top ? sk2Planes : sk2Split, dim3((uint32_t)segPerCU * cu_count()), dim3(G::THREADS), lds,
                         stream, kA, oA, top ? KeyMap<uint32_t>{} : km32, top ? 16 : startBits + 8 * p,
                         top ? base + nLow * kBins : nullptr, kB, oB, km32, startBits + 8 * p,
                         reinterpret_cast<uint32_t*>(hyb + (top ? kSegInfoOff : kSegInfoAOff)),
                         reinterpret_cast<const uint32_t*>(hyb + (top ? kSegBaseOff : kSegBaseAOff)), status[p & 1], err,
                         grp[p & 1], static_cast<const uint32_t*>(mode), hiP,
                         g_stamps ? g_stamps + (uint64_t)(p - nLow) * (plan.nTiles + kSegTilePad) * kStampSlots
                                  : nullptr,
                         sqw, reinterpret_cast<const typename ValueWord<kVB4>::T*>(top ? valOut : V),
                         reinterpret_cast<typename ValueWord<kVB4>::T*>(top ? V : valOut));
    };
    const uint64_t sw = plan.wideStatus ? 8 : 4;
    const int setB = (nLow + 1) & 1;
    if (segA) {
      // Both table sets are clean (zeroed up front); the segmented passes'
      // extra tile ids (rows past nTiles) are touched by nothing else.
      if (planes) {
        launch_seg2(nLow, false);
      } else {
        launch_seg(nLow, K, keyOut, V, valOut, kSegInfoAOff, kSegBaseAOff, mode, kGateMode0 | kGateMode1 | kGateMode3);
      }
    } else {
      launch_pass(nLow, K, keyOut, V, valOut, mode, kGateMode0 | kGateMode1 | kGateMode3);
      // the segmented pass's tile ids reach past nTiles (per-segment
      // rounding): clear those rows (pass nLow cleared rows [0, nTiles))
      const uint64_t nGroups0 = (plan.nTiles + kGroup - 1) / kGroup;
      constexpr uint64_t kPadGroups = (kSegTilePad + kGroup - 1) / kGroup + 1;
      if (hipMemsetAsync(reinterpret_cast<char*>(status[setB]) + plan.nTiles * kBins * sw, 0,
                         kSegTilePad * kBins * sw, stream) != hipSuccess ||
          hipMemsetAsync(grp[setB].ga + nGroups0 * kBins, 0, kPadGroups * kBins * 4, stream) != hipSuccess ||
          hipMemsetAsync(reinterpret_cast<char*>(grp[setB].gp) + nGroups0 * kBins * sw, 0, kPadGroups * kBins * sw,
                         stream) != hipSuccess)
        return THRS_ERROR_HIP;
    }
    if (planes) {  // mode 0: planes -> lo2; mode 1 (big chunks) / 3 (f32 -0): keys
      launch_seg2(nLow + 1, true);
    } else if (segTop)
      launch_seg(nLow + 1, keyOut, K, valOut, V, kSegInfoOff, kSegBaseOff, mode, kGateMode0 | kGateMode1 | kGateMode3);
    else
      launch_pass(nLow + 1, keyOut, K, valOut, V, mode, kGateMode0 | kGateMode1 | kGateMode3);
    {
      ProfScope prof(stream, 2,
                     kKV ? THRS_PK_LOCAL_KV
                     : kPairs4 ? THRS_PK_LOCAL_PAIRS
                     : count16 ? THRS_PK_LOCAL_COUNT16
                     : local16 ? THRS_PK_LOCAL16 : THRS_PK_LOCAL,
                     moveBytes);
      // never more workgroups than chunks can exist: <= 256 (one per top digit)
      // + 2 per non-empty bucket, and <= the number of buckets (single-bucket
      // chunks -- every local sort but the 32-bit one: thrs_plan_rows makes
      // every bucket a chunk, empty or not)
      const uint64_t maxChunks = !local32 ? kBuckets : std::min<uint64_t>(kBuckets, 256 + 2 * (uint64_t)n);
      const dim3 lgrid((uint32_t)maxChunks);
      if constexpr (kKV) {
        auto launch_kv = [&](auto geom) {
          using LK = decltype(geom);
          auto lk = atomicRank ? thrs_local_kv<KT, VB, true, LK> : thrs_local_kv<KT, VB, false, LK>;
          hipLaunchKernelGGL(lk, lgrid, dim3(LK::THREADS), LK::LDS, stream, K, V, km, chunkOff, chunkB0, meta, sqw,
                             g_lstamps);
        };
        if (P.kvGeom == 2) launch_kv(LocKVS{});
        else if (P.kvGeom == 1) launch_kv(LocKVM{});
        else launch_kv(LocKV{});
      } else if constexpr (kPairs4) {
        auto launch_pairs = [&](auto geom) {
          using LG = decltype(geom);
          auto lk = atomicRank ? thrs_local_pairs<KT, true, LG> : thrs_local_pairs<KT, false, LG>;
          hipLaunchKernelGGL(lk, lgrid, dim3(LG::THREADS), LG::template lds<U>(), stream,
                             reinterpret_cast<uint32_t*>(K), reinterpret_cast<uint32_t*>(V), km32, chunkOff, chunkB0,
                             meta, sqw, zeroLog ? meta + kMetaNegZero : nullptr,
                             planes ? static_cast<const uint16_t*>(lo2P) : nullptr, zeroLog);
        };
        if (P.tinyPairs) launch_pairs(LocTiny{});
        else if (smallLocal) launch_pairs(LocSmall{});
        else launch_pairs(LocBig{});
      } else if constexpr (kKeys4) {
        auto launch16 = [&](auto geom) {
          using LG = decltype(geom);
          auto lk = atomicRank ? thrs_local16<KT, true, LG> : thrs_local16<KT, false, LG>;
          hipLaunchKernelGGL(lk, lgrid, dim3(LG::THREADS), LG::LDS, stream, reinterpret_cast<uint32_t*>(K), km32,
                             chunkOff, chunkB0, meta, planes ? static_cast<const uint16_t*>(lo2P) : nullptr, sqw,
                             zeroLog);
        };
        auto launch32 = [&](auto geom) {
          using LG = decltype(geom);
          auto lk = atomicRank ? thrs_local<KT, true, LG> : thrs_local<KT, false, LG>;
          hipLaunchKernelGGL(lk, lgrid, dim3(LG::THREADS), LG::template lds<U>(), stream, K, km, startBits, nLow,
                             chunkOff, chunkB0, meta, g_lstamps);
        };
        if (count16) {
          if constexpr (KT == 0) {
            // persistent: one 128-KiB workgroup per CU walks the chunks
            const uint32_t cgrid = (uint32_t)std::min<uint64_t>(maxChunks, (uint64_t)cu_count());
            // planes off (or mode 1, big chunks): the items are the keys
            // themselves (in place)
            auto lk = planes ? thrs_local_count16<true> : thrs_local_count16<false>;
            hipLaunchKernelGGL(lk, dim3(cgrid), dim3(LocCount::THREADS), LocCount::LDS, stream,
                               reinterpret_cast<uint32_t*>(K), n, km32, chunkOff, chunkB0, meta,
                               static_cast<const uint16_t*>(lo2P), joint);
          }
        } else if (wide16) {
          launch16(Loc16Wide{});
        } else if (P.tiny16) {
          launch16(Loc16Tiny{});
        } else if (small16) {
          launch16(Loc16Small{});
        } else if (local16) {
          launch16(Loc16{});
        } else if (smallLocal) {
          launch32(LocSmall{});
        } else {
          launch32(LocBig{});
        }
      }
    }
    // ---- the per-bucket fallback (thrs_fallback.hpp): big chunks only,
    // gated on meta[kMetaFallback]
    {  // (profiled per launch: the bench line shows which of them ran)
      uint32_t* bigB = reinterpret_cast<uint32_t*>(hyb + kBigBOff);
      uint32_t* bigPos = reinterpret_cast<uint32_t*>(hyb + kBigPosOff);
      uint32_t* bigTile = reinterpret_cast<uint32_t*>(hyb + kBigTileOff);
      uint32_t* bigHist = reinterpret_cast<uint32_t*>(scratch + plan.bigHistOff);
      // (the low passes reuse both look-back table sets: zeroed by
      // thrs_big_hist; the big chunks' prefixes and counts' zeroing are
      // thrs_plan_rows's -- thrs_plan's multi-bucket chunks take thrs_big_plan)
      if (local32) {
        ProfScope prof(stream, 3, THRS_PK_BIG_PLAN, 0);
        hipLaunchKernelGGL(thrs_big_plan, dim3(std::min<uint32_t>(256, cu_count())), dim3(kBigPlanThreads), 0, stream,
                           chunkOff, meta, bigB, bigPos, bigTile, (uint32_t)G::TILE, reinterpret_cast<uint4*>(bigHist),
                           nLow, reinterpret_cast<uint4*>(scratch + kHeaderBytes), (uint64_t)(2 * plan.setBytes / 16));
      }
      {
        ProfScope prof(stream, 3, THRS_PK_BIG_HIST, 0);
        hipLaunchKernelGGL(thrs_big_hist<KT>, dim3(cu_count()), dim3(kHistThreads),
                           (size_t)nLow * kBins * kBigCopies * 4, stream, static_cast<const U*>(keys), km, startBits,
                           nLow, chunkOff, meta, bigB, bigPos, bigHist, sqw,
                           local32 ? nullptr : reinterpret_cast<uint4*>(scratch + kHeaderBytes),
                           (uint64_t)(2 * plan.setBytes / 16));
      }
      for (int p = 0; p < nLow; ++p) {
        ProfScope prof(stream, 3, THRS_PK_PASS_BIG, 0);
        hipLaunchKernelGGL(kernelBig, dim3(gridBig), dim3(G::THREADS), lds, stream, K, keyOut, V, valOut, km,
                           startBits + 8 * p, p, nLow, chunkOff, meta, bigB, bigPos, bigTile, bigHist, status[0],
                           status[1], err, sqw);
      }
      ProfScope prof(stream, 3, THRS_PK_BIG_COPY, 0);
      // (also publishes the sort's error word: no thrs_err_publish launch)
      hipLaunchKernelGGL((thrs_big_copy<U, VW>), dim3(2048), dim3(256), 0, stream, K, keyOut, VB ? V : nullptr, valOut,
                         chunkOff, meta, bigB, bigPos, err, sticky);
    }
  }
  return hipGetLastError() == hipSuccess ? THRS_SUCCESS : THRS_ERROR_HIP;
}

template <int KT, int VB>
int run_st(void* keys, void* vals, uint32_t n, void* tmp, void* ko, void* vo, int startBits, int nPass, bool desc,
           const Plan& plan, const thrs_options& opt, hipStream_t stream, uint32_t* counts) {
  if (plan.wideStatus)
    return run_sort<KT, VB, uint64_t>(keys, vals, n, tmp, ko, vo, startBits, nPass, desc, plan, opt, stream, counts);
  return run_sort<KT, VB, uint32_t>(keys, vals, n, tmp, ko, vo, startBits, nPass, desc, plan, opt, stream, counts);
}

template <int KT>
int run_vb(int vb, void* keys, void* vals, uint32_t n, void* tmp, void* ko, void* vo, int startBits, int nPass,
           bool desc, const Plan& plan, const thrs_options& opt, hipStream_t stream, uint32_t* counts = nullptr) {
  switch (vb) {
    case 0: return run_st<KT, 0>(keys, vals, n, tmp, ko, vo, startBits, nPass, desc, plan, opt, stream, counts);
    case 4: return run_st<KT, 4>(keys, vals, n, tmp, ko, vo, startBits, nPass, desc, plan, opt, stream, counts);
    case 8: return run_st<KT, 8>(keys, vals, n, tmp, ko, vo, startBits, nPass, desc, plan, opt, stream, counts);
    case 16: return run_st<KT, 16>(keys, vals, n, tmp, ko, vo, startBits, nPass, desc, plan, opt, stream, counts);
  }
  return THRS_ERROR_INVALID_VALUE;
}

#else
template <int KT>
int run_vb(int vb, void* keys, void* vals, uint32_t n, void* tmp, void* ko, void* vo, int startBits, int nPass,
           bool desc, const Plan& plan, const thrs_options& opt, hipStream_t stream, uint32_t* counts = nullptr);
#endif

}  // namespace thrs_host
