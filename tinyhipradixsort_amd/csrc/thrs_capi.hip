// thrs_capi.hip -- host side of libthrs.so: the C-ABI declared in
// include/thrs/thrs_capi.h, launching the gfx950 kernels of thrs_kernels.hpp.
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
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "thrs/thrs_capi.h"
#include "thrs_kernels.hpp"
#include "thrs_hybrid.hpp"


using namespace thrs_dev;

namespace {

constexpr uint64_t kAlign = 256;
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

#ifndef THRS_WIDE16_AUTO
#define THRS_WIDE16_AUTO 1  // AUTO takes the bucket path (wide 16-bit local sort) for u32 keys-only up to 2^31 + 2^25
#endif
#ifndef THRS_COUNT16_DEFAULT
// u32 keys-only local sort over 16-bit items: 1 = counting (thrs_local_count16)
// unless RANK16 is asked; 0 = two LSD rounds (thrs_local16) unless COUNT16 is
// asked.  Counting measured slower (docs/EXPERIMENTS.md row 56: 2.63 vs 1.78 ms)
#define THRS_COUNT16_DEFAULT 0
#endif

struct Plan {
  int kb, vb;         // key / value bytes (vb = 0 for sortKeys)
  uint64_t tileKeys;  // keys per tile of the pass kernel
  uint64_t nTiles;
  bool wideStatus;    // 64-bit look-back words (n >= 2^31)
  uint64_t statusBytes;   // per-tile rows [nTiles][256]
  uint64_t gaBytes;       // group aggregates [nGroups][256] u32 (kGroup > 0)
  uint64_t gpBytes;       // group prefixes   [nGroups][256] status words
  uint64_t setBytes;      // one look-back table set = status + ga + gp
  uint64_t claimBytes;    // per pass: XCD-block claim state (tickets, block counter, 8 block tables)
  uint64_t hybridOff;     // 3-pass path (thrs_hybrid.hpp): bucket histogram, chunk table, meta
  uint64_t hiPlaneOff;    // u32 keys without values: the bucket path's u8 plane (n bytes)
  uint64_t scratchBytes;  // header + 2 sets (ping-pong between passes) + 8 claim areas + hybrid area [+ u8 plane]
};

// hybrid area: u32 joint[65536] | segHistA[8][256] | rowHist[256] | meta[64]
// (all zeroed up front) | chunkOff[65537] | chunkB0[65537] | segment tables
// of the two top-digit passes
constexpr uint64_t kJointBytes = kBuckets * 4;
constexpr uint64_t kSegHistAOff = kJointBytes;                    // per position segment: second-digit counts
constexpr uint64_t kRowHistOff = kSegHistAOff + kSegs * 256 * 4;  // top-digit counts (thrs_hist_joint)
constexpr uint64_t kMetaOff = kRowHistOff + 256 * 4;              // zero: thrs_plan_rows raises its flags atomically
constexpr uint64_t kJointZero = kMetaOff + 256;
constexpr uint64_t kChunkOffOff = kJointZero;
constexpr uint64_t kChunkB0Off = kChunkOffOff + round_up_c((kBuckets + 1) * 4, 256);
constexpr uint64_t kSegInfoOff = kChunkB0Off + round_up_c((kBuckets + 1) * 4, 256);  // segPos[9] | segTiles[9] ... tickets[8] at +256 B (thrs_pass_seg)
constexpr uint64_t kSegBaseOff = kSegInfoOff + 512;   // u32 [8][256] per-segment top-digit bases
constexpr uint64_t kSegInfoAOff = kSegBaseOff + kSegs * 256 * 4;  // the same two for the second-digit pass
constexpr uint64_t kSegBaseAOff = kSegInfoAOff + 512;
constexpr uint64_t kHybridBytes = kSegBaseAOff + kSegs * 256 * 4;
// tile ids of the segmented pass: each of the 8 segments adds at most one
// partial tile and rounds its id range up to a multiple of kGroup
constexpr uint64_t kSegTilePad = kSegs * kGroup;

Plan make_plan(int keyType, int valueBytesOrZero, uint32_t n) {
  Plan p{};
  p.kb = key_bytes_of(keyType);
  p.vb = valueBytesOrZero;
  p.tileKeys = tile_keys(p.kb, p.vb);
  p.nTiles = std::max<uint64_t>(1, ((uint64_t)n + p.tileKeys - 1) / p.tileKeys);
  p.wideStatus = (uint64_t)n >= (1ull << 31);
  const uint64_t rows = p.nTiles + kSegTilePad;  // + the segmented pass's extra tile ids
  p.statusBytes = round_up(rows * kBins * (p.wideStatus ? 8 : 4), kAlign);
  const uint64_t nGroups = kGroup > 0 ? (rows + kGroup - 1) / kGroup : 0;
  p.gaBytes = round_up(nGroups * kBins * 4, kAlign);
  p.gpBytes = round_up(nGroups * kBins * (p.wideStatus ? 8 : 4), kAlign);
  p.setBytes = p.statusBytes + p.gaBytes + p.gpBytes;
  const uint64_t nXb = (p.nTiles + kXcdBlock - 1) / kXcdBlock + 16;  // table stride (see xb_claim)
  p.claimBytes = round_up((16 + 8 * nXb) * 4, kAlign);
  p.hybridOff = kHeaderBytes + 2 * p.setBytes + 8 * p.claimBytes;
  p.scratchBytes = p.hybridOff + kHybridBytes;
  // the u8 plane of the planes codecs (thrs_kernels.hpp kCodecSplit): the u16
  // planes fill keyOut, which is all a sortKeys caller must allocate
  // (getTemporaryBufferBytesForSortKeys = pSumBuffer + keyOutBuffer)
  p.hiPlaneOff = p.scratchBytes;
  if (keyType == THRS_KEY_U32 && valueBytesOrZero == 0) p.scratchBytes += round_up(n, kAlign);
  return p;
}

int cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    cached[dev] = c;
  }
  return cached[dev];
}

// ---- optional event timing (thrs_profile_*) ----------------------------------
struct ProfRec {
  hipEvent_t a, b;
  int kind;  // 0 = histogram + scan, 1 = pass
};
std::mutex g_prof_mu;
bool g_prof_on = false;
std::vector<ProfRec> g_prof;
std::vector<hipEvent_t> g_prof_pool;

hipEvent_t prof_event() {
  hipEvent_t e = nullptr;
  if (!g_prof_pool.empty()) {
    e = g_prof_pool.back();
    g_prof_pool.pop_back();
  } else if (hipEventCreate(&e) != hipSuccess) {
    e = nullptr;
  }
  return e;
}
struct ProfScope {  // records [a, b) around the launches issued in its lifetime
  hipStream_t s;
  int kind;
  hipEvent_t a = nullptr;
  ProfScope(hipStream_t s_, int k) : s(s_), kind(k) {
    if (!g_prof_on) return;
    std::lock_guard<std::mutex> g(g_prof_mu);
    a = prof_event();
    if (a) (void)hipEventRecord(a, s);
  }
  ~ProfScope() {
    if (!a) return;
    std::lock_guard<std::mutex> g(g_prof_mu);
    hipEvent_t b = prof_event();
    if (!b) return;
    (void)hipEventRecord(b, s);
    g_prof.push_back({a, b, kind});
  }
};

uint64_t* g_stamps = nullptr;   // THRS_STAMPS diagnostic builds only (thrs_debug_set_stamps)
uint64_t* g_lstamps = nullptr;  // same, local sort: [chunk][8] (thrs_debug_set_local_stamps)

// Per-device result of thrs_probe_lds_order: 1 = lane-ordered LDS atomics
// (fast rank), 0 = ballot-match rank.
int g_rank_mode[64];
std::once_flag g_rank_once[64];

int probe_rank_mode(hipStream_t stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  std::call_once(g_rank_once[dev], [&] {
    g_rank_mode[dev] = 0;
    // never probe (synchronising) inside a stream capture: stay on the ballot path
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
    uint32_t* d = nullptr;
    if (hipMalloc(&d, 4) != hipSuccess) return;
    uint32_t h = 1;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess) {
      if (hipMemsetAsync(d, 0, 4, s) == hipSuccess) {
        hipLaunchKernelGGL(thrs_probe_lds_order, dim3(256), dim3(256), 0, s, d, 64);
        if (hipGetLastError() == hipSuccess && hipMemcpyAsync(&h, d, 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
            hipStreamSynchronize(s) == hipSuccess && h == 0)
          g_rank_mode[dev] = 1;
      }
      (void)hipStreamDestroy(s);
    }
    (void)hipFree(d);
  });
  return g_rank_mode[dev];
}

// Per-device sticky error word in host memory (mapped): thrs_err_publish
// ORs a sort's device error word into it at the end of every sort; the next
// thrs_sort_* call reads and clears it (thrs_capi.h, "Device-side failures").
uint32_t* g_sticky[64];          // host view
uint32_t* g_sticky_dev[64];      // device view
std::once_flag g_sticky_once[64];

uint32_t* sticky_dev() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::call_once(g_sticky_once[dev], [&] {
    void* h = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      (void)hipHostFree(h);
      return;
    }
    std::memset(h, 0, 64);
    g_sticky[dev] = static_cast<uint32_t*>(h);
    g_sticky_dev[dev] = static_cast<uint32_t*>(d);
  });
  return g_sticky_dev[dev];
}
// read-and-clear of the current device's sticky word (0 = no failure)
uint32_t take_sticky() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || !g_sticky[dev]) return 0;
  return __atomic_exchange_n(g_sticky[dev], 0u, __ATOMIC_ACQ_REL);
}

__global__ void thrs_err_publish(const uint32_t* __restrict__ err, uint32_t* __restrict__ sticky) {
  const uint32_t e = *err;
  if (e) __hip_atomic_fetch_or(sticky, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

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
  // 4-byte keys without values; u32 keys with 4-byte values over the whole
  // key; 8-byte keys without values or with 8-byte values over the whole key
  constexpr bool kBucket32 = sizeof(U) == 4 && (VB == 0 || (VB == 4 && KT == 0));
  constexpr bool kBucket64 = sizeof(U) == 8 && (VB == 0 || VB == 8);
  constexpr bool kBucketType = kBucket32 || kBucket64;
  const bool fullWindow = startBits == 0 && nPass * 8 >= (int)(8 * sizeof(U));
  // Size window of the default (uniform keys: n / 65536 keys per bucket;
  // docs/EXPERIMENTS.md row 29): the local sort costs about the same per chunk
  // whatever its size, so below 2^28 the two passes it replaces are cheaper;
  // above 2^30 + 2^26 the largest of 65536 uniform buckets (mean + ~4.5 sigma)
  // outgrows the chunk capacity and the fallback would pay for the bucket
  // histogram in vain.  THRS_PATH_BUCKET forces the path for any n (tests).
  // Local geometries (thrs_hybrid.hpp LocG): LocSmall (9216-key chunks,
  // uniform buckets of 4-8K keys) for n <= 2^29, LocBig (18432) above.
  const uint64_t nn = n;
  // (8-byte keys: one 17408-slot chunk per bucket, so up to 2^30 + 2^24: the
  // largest uniform bucket stays ~3 sigma below the capacity)
  const bool sizeOk = nn >= (1ull << 28) && nn <= (1ull << 30) + (sizeof(U) == 8 ? (1ull << 24) : (1ull << 26));
  // u32 keys without values over the whole key: up to 2^31 + 2^25 with the
  // wide 16-bit local sort (Loc16Wide: 34816-key chunks)
  const bool wideOk = THRS_WIDE16_AUTO && KT == 0 && VB == 0 && fullWindow && nn > (1ull << 30) + (1ull << 26) &&
                      nn <= (1ull << 31) + (1ull << 25);
  const bool smallLocal = opt.localGeometry == THRS_LOCAL_SMALL ? true
                          : opt.localGeometry != THRS_LOCAL_AUTO  // BIG, BIG32 and the 16-bit kernels
                              ? false
                              : nn <= (1ull << 29);
  const bool bucket = kBucketType && !counts && nPass >= 3 &&
                      (opt.path == THRS_PATH_BUCKET || (opt.path == THRS_PATH_AUTO && (sizeOk || wideOk))) &&
                      ((kBucket32 && VB == 0) || fullWindow);
  const int nLow = nPass - 2;
  // u32 keys over the whole key, large chunks: the local sort on 16-bit items
  // (thrs_hybrid.hpp thrs_local16) over single-bucket chunks
  const bool local16 = bucket && KT == 0 && VB == 0 && fullWindow && !smallLocal &&
                       opt.localGeometry != THRS_LOCAL_BIG32;
  // ... sorted by counting (thrs_local_count16) or by two LSD rounds (thrs_local16)
  // ... in 34816-key chunks (explicitly, or by default above 2^30 + 2^26)
  const bool wide16 = local16 && (opt.localGeometry == THRS_LOCAL_WIDE16 ||
                                  (opt.localGeometry == THRS_LOCAL_AUTO && nn > (1ull << 30) + (1ull << 26)));
  const bool count16 = local16 && !wide16 &&
                       (opt.localGeometry == THRS_LOCAL_COUNT16 ||
                        (opt.localGeometry != THRS_LOCAL_RANK16 && THRS_COUNT16_DEFAULT));
  const bool segTop = opt.segmented != THRS_SEG_NONE;
  const bool segA = opt.segmented == THRS_SEG_AUTO;
  // local16 with both top-digit passes segmented: the passes carry the keys
  // as planes (thrs_kernels.hpp kCodecSplit / kCodecPlanes): keyOut (4n bytes)
  // = lo u16[n] | lo2 u16[n], the u8 plane hi[n] at the end of the scratch
  const bool planes = local16 && segA && opt.planes != THRS_PLANES_OFF &&
                      plan.scratchBytes - plan.hiPlaneOff >= (uint64_t)n;
  uint16_t* loP = static_cast<uint16_t*>(keyOutBuf);
  uint16_t* lo2P = loP + n;
  uint8_t* hiP = reinterpret_cast<uint8_t*>(scratch + plan.hiPlaneOff);
  const bool atomicRank = opt.rank == THRS_RANK_ATOMIC ? true
                          : opt.rank == THRS_RANK_BALLOT ? false
                                                         : probe_rank_mode(stream) != 0;
  // XCD-block claims (thrs_pass_xb) pay off where runs are short and the
  // grid is large: 4-byte keys without values, n >= 2^29 (docs/EXPERIMENTS.md
  // row 19: +4-6% there, neutral at 2^28, -2..-6% for pairs / f32 at 2^28).
  const bool useXb = opt.tileClaims == THRS_CLAIMS_XCD_BLOCKS ? true
                     : opt.tileClaims == THRS_CLAIMS_TICKET ? false
                                                            : (sizeof(U) == 4 && VB == 0 && n >= (1u << 29));
  uint32_t* sticky = sticky_dev();
  if (!sticky) return THRS_ERROR_HIP;

  // ---- kernels and their LDS opt-ins, before anything is enqueued
  const size_t lds = G::LDS_BYTES;
  auto kernelXb = atomicRank ? thrs_pass_xb<KT, VB, ST, true> : thrs_pass_xb<KT, VB, ST, false>;
  auto kernelPersist = atomicRank ? thrs_pass_persist<KT, VB, ST, true> : thrs_pass_persist<KT, VB, ST, false>;
  auto kernel = useXb ? kernelXb : (atomicRank ? thrs_pass<KT, VB, ST, true> : thrs_pass<KT, VB, ST, false>);
  auto sk = atomicRank ? thrs_pass_seg<KT, VB, ST, true> : thrs_pass_seg<KT, VB, ST, false>;
  // plane codecs (u32 keys-only instantiations only; `planes` is false elsewhere)
  auto skSplit = atomicRank ? thrs_pass_seg<KT, VB, ST, true, (KT == 0 && VB == 0) ? kCodecSplit : kCodecKeys>
                            : thrs_pass_seg<KT, VB, ST, false, (KT == 0 && VB == 0) ? kCodecSplit : kCodecKeys>;
  auto skPlanes = atomicRank ? thrs_pass_seg<KT, VB, ST, true, (KT == 0 && VB == 0) ? kCodecPlanes : kCodecKeys>
                             : thrs_pass_seg<KT, VB, ST, false, (KT == 0 && VB == 0) ? kCodecPlanes : kCodecKeys>;
  const int histPasses = bucket ? nLow : nPass;
  const size_t histLds = (size_t)histPasses * kBins * hist_copies<(int)sizeof(U)>() * 4;
  if (allow_lds(thrs_hist<KT>, histLds) != hipSuccess || allow_lds(kernel, lds) != hipSuccess ||
      allow_lds(kernelXb, lds) != hipSuccess || allow_lds(kernelPersist, lds) != hipSuccess)
    return THRS_ERROR_HIP;
  if (bucket) {
    if (allow_lds(thrs_hist_joint<KT>, kJointLds) != hipSuccess || allow_lds(sk, lds) != hipSuccess)
      return THRS_ERROR_HIP;
    if (planes && (allow_lds(skSplit, lds) != hipSuccess || allow_lds(skPlanes, lds) != hipSuccess))
      return THRS_ERROR_HIP;
    if constexpr (kBucket64) {
      if (allow_lds(atomicRank ? thrs_local64<KT, VB, true> : thrs_local64<KT, VB, false>, Loc64::LDS) != hipSuccess)
        return THRS_ERROR_HIP;
    } else if constexpr (kBucketType) {
      if (local16) {
        if constexpr (KT == 0 && VB == 0) {
          if (allow_lds(atomicRank ? thrs_local16<true, Loc16> : thrs_local16<false, Loc16>, Loc16::LDS) !=
                  hipSuccess ||
              allow_lds(atomicRank ? thrs_local16<true, Loc16Wide> : thrs_local16<false, Loc16Wide>,
                        Loc16Wide::LDS) != hipSuccess ||
              allow_lds(thrs_local_count16<true>, LocCount::LDS) != hipSuccess ||
              allow_lds(thrs_local_count16<false>, LocCount::LDS) != hipSuccess)
            return THRS_ERROR_HIP;
        }
      } else if constexpr (VB == 4) {
        if (allow_lds(atomicRank ? thrs_local_pairs<true, LocBig> : thrs_local_pairs<false, LocBig>,
                      LocBig::lds<U>()) != hipSuccess ||
            allow_lds(atomicRank ? thrs_local_pairs<true, LocSmall> : thrs_local_pairs<false, LocSmall>,
                      LocSmall::lds<U>()) != hipSuccess)
          return THRS_ERROR_HIP;
      } else {
        if (allow_lds(atomicRank ? thrs_local<KT, true, LocBig> : thrs_local<KT, false, LocBig>, LocBig::lds<U>()) !=
                hipSuccess ||
            allow_lds(atomicRank ? thrs_local<KT, true, LocSmall> : thrs_local<KT, false, LocSmall>,
                      LocSmall::lds<U>()) != hipSuccess)
          return THRS_ERROR_HIP;
      }
    }
  }
  // persistent grids (occupancy x CUs): the XCD-block kernel, and the bucket
  // path's fallback-only passes (thrs_pass_persist): a launch of nTiles
  // workgroups that all exit at once still costs ~0.1 ms at 2^18 tiles
  auto persistent_grid = [&](auto kern) -> uint32_t {
    int perCU = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, kern, G::THREADS, lds) != hipSuccess || perCU < 1)
      perCU = 1;
    return (uint32_t)std::min<uint64_t>(plan.nTiles, (uint64_t)perCU * cu_count());
  };
  const uint32_t gridXb = useXb ? persistent_grid(kernelXb) : (uint32_t)plan.nTiles;
  const uint32_t gridPersist = bucket ? persistent_grid(kernelPersist) : (uint32_t)plan.nTiles;
  const uint32_t grid = useXb ? gridXb : (uint32_t)plan.nTiles;
  int segPerCU = 0;
  if (bucket &&
      (hipOccupancyMaxActiveBlocksPerMultiprocessor(&segPerCU, sk, G::THREADS, lds) != hipSuccess || segPerCU < 1))
    segPerCU = 1;

  // header (histograms, tile counters, error word) + first status table; the
  // bucket path with an odd number of (skippable) low passes starts on set 1
  // too, and zeroes its bucket histogram
  // Bucket path: ONE memset from the header through the bucket histogram --
  // both table sets (the top-digit passes use set nLow&1 and the other one,
  // and no launch before them dirties the other unless it also cleans it:
  // fallback passes clear their successor's rows), all 8 claim areas, joint.
  if (bucket) {
    if (hipMemsetAsync(scratch, 0, plan.hybridOff + kJointZero, stream) != hipSuccess) return THRS_ERROR_HIP;
  } else if (hipMemsetAsync(scratch, 0, kHeaderBytes + plan.setBytes, stream) != hipSuccess) {
    return THRS_ERROR_HIP;
  }
  char* claim = scratch + kHeaderBytes + 2 * plan.setBytes;  // 8 per-pass claim areas

  {  // histograms of every pass in one read of the keys
    ProfScope prof(stream, 0);
    const int vec = (reinterpret_cast<uintptr_t>(keys) % 16) == 0;
    const uint64_t want = ((uint64_t)n + kHistThreads * 64 - 1) / (kHistThreads * 64);
    const int hgrid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)cu_count() * THRS_HIST_GRID_MULT));
    if (bucket) {
      hipLaunchKernelGGL(thrs_hist_joint<KT>, dim3(hgrid), dim3(kHistThreads), kJointLds, stream,
                         static_cast<const U*>(keys), n, orderMask, startBits + 8 * nLow, vec, joint,
                         reinterpret_cast<uint32_t*>(hyb + kSegHistAOff), reinterpret_cast<uint32_t*>(hyb + kRowHistOff));
      const uint32_t cap = kBucket64 ? Loc64::CAP : smallLocal ? LocSmall::CAP : wide16 ? Loc16Wide::CAP : LocBig::CAP;
#ifndef THRS_PLAN_ROWS
#define THRS_PLAN_ROWS 1
#endif
      if (THRS_PLAN_ROWS && (VB || local16 || kBucket64)) {
        // single-bucket chunks: one workgroup per top digit
        hipLaunchKernelGGL(thrs_plan_rows, dim3(kBins), dim3(kPlanRowThreads), 0, stream, joint,
                           reinterpret_cast<const uint32_t*>(hyb + kRowHistOff),
                           reinterpret_cast<const uint32_t*>(hyb + kSegHistAOff), n, cap, base + nLow * kBins,
                           chunkOff, chunkB0, meta, reinterpret_cast<uint32_t*>(hyb + kSegInfoOff),
                           reinterpret_cast<uint32_t*>(hyb + kSegBaseOff), (uint32_t)G::TILE, (uint32_t)hgrid,
                           reinterpret_cast<uint32_t*>(hyb + kSegInfoAOff), reinterpret_cast<uint32_t*>(hyb + kSegBaseAOff));
      } else {
        // chunks: whole buckets; neighbouring buckets below kLocCap/2 keys share one
        hipLaunchKernelGGL(thrs_plan, dim3(1), dim3(kPlanThreads), 0, stream, joint, n, base + nLow * kBins, chunkOff,
                           chunkB0, meta, cap, (VB || local16 || kBucket64) ? -1 : smallLocal ? kLocSmallLogT : kLocLogT,
                           reinterpret_cast<uint32_t*>(hyb + kSegInfoOff), reinterpret_cast<uint32_t*>(hyb + kSegBaseOff),
                           (uint32_t)G::TILE, reinterpret_cast<const uint32_t*>(hyb + kSegHistAOff), (uint32_t)hgrid,
                           reinterpret_cast<uint32_t*>(hyb + kSegInfoAOff), reinterpret_cast<uint32_t*>(hyb + kSegBaseAOff));
      }
      // the low digits' histograms + bases: needed only on the fallback path
      hipLaunchKernelGGL(thrs_hist<KT>, dim3(hgrid), dim3(kHistThreads), histLds, stream, static_cast<const U*>(keys),
                         n, orderMask, startBits, nLow, vec, hist, meta + kMetaFallback);
      hipLaunchKernelGGL(thrs_scan, dim3(1), dim3(kThreads), 0, stream, hist, base, nLow, meta + kMetaFallback);
    } else {
      hipLaunchKernelGGL(thrs_hist<KT>, dim3(hgrid), dim3(kHistThreads), histLds, stream, static_cast<const U*>(keys),
                         n, orderMask, startBits, nPass, vec, hist, nullptr);
      hipLaunchKernelGGL(thrs_scan, dim3(1), dim3(kThreads), 0, stream, hist, base, nPass, nullptr);
    }
    if (counts && hipMemcpyAsync(counts, hist, kBins * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream) != hipSuccess)
      return THRS_ERROR_HIP;
  }

  if (useXb && !bucket && hipMemsetAsync(claim, 0, (size_t)nPass * plan.claimBytes, stream) != hipSuccess)
    return THRS_ERROR_HIP;

  // pass p: digit at startBits + 8p, tables of set p&1; gate != nullptr runs
  // it only if bit *gate of gateMask is set (meta words written by thrs_plan)
  auto launch_pass = [&](int p, U* kin, U* kout, VW* vin, VW* vout, const uint32_t* gate, uint32_t gateMask) {
    const bool more = p + 1 < nPass;
    ST* next = more ? status[(p + 1) & 1] : nullptr;
    GroupTables<ST> g = grp[p & 1];
    g.gaNext = more ? grp[(p + 1) & 1].ga : nullptr;
    g.gpNext = more ? grp[(p + 1) & 1].gp : nullptr;
    ProfScope prof(stream, gate && (gateMask == kGateFallback || gateMask == kGateMode1) ? 3 : 1);  // fallback-only passes are timed apart
    // fallback-only launches (most exit at once): persistent ticket kernel,
    // unless the XCD-block kernel runs anyway
    const bool fallbackOnly = gate && (gateMask == kGateFallback || gateMask == kGateMode1);
    const bool persist = bucket && fallbackOnly && !useXb;
    hipLaunchKernelGGL(persist ? kernelPersist : kernel, dim3(persist ? gridPersist : grid), dim3(G::THREADS), lds,
                       stream, kin, kout, vin, vout, n, orderMask, startBits + 8 * p, base + p * kBins, status[p & 1],
                       next, useXb ? reinterpret_cast<uint32_t*>(claim + p * plan.claimBytes) : counters + p, err, g,
                       g_stamps ? g_stamps + (uint64_t)p * plan.nTiles * kStampSlots : nullptr, gate, gateMask);
  };
  auto publish_error = [&]() -> int {
    hipLaunchKernelGGL(thrs_err_publish, dim3(1), dim3(1), 0, stream, err, sticky);
    return hipGetLastError() == hipSuccess ? THRS_SUCCESS : THRS_ERROR_HIP;
  };

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

  // ---- bucket path: fallback-only low passes, the two top digits, local sort
  if constexpr (kBucketType) {
    U* K = static_cast<U*>(keys);
    VW* V = static_cast<VW*>(vals);
    uint32_t* fallback = meta + kMetaFallback;
    uint32_t* mode = meta + kMetaMode;
    {
      U* kin = K;
      U* kout = keyOut;
      VW* vin = V;
      VW* vout = valOut;
      for (int p = 0; p < nLow; ++p) {
        launch_pass(p, kin, kout, vin, vout, fallback, kGateFallback);
        std::swap(kin, kout);
        std::swap(vin, vout);
      }
      if (nLow & 1) {  // fallback result is in keyOut: the top-digit passes read K
        hipLaunchKernelGGL(thrs_copy_gated, dim3(2048), dim3(256), 0, stream,
                           reinterpret_cast<const uint32_t*>(keyOut), reinterpret_cast<uint32_t*>(K),
                           (uint64_t)n * sizeof(U) / 4, fallback, 1u);
        if (VB)
          hipLaunchKernelGGL(thrs_copy_gated, dim3(2048), dim3(256), 0, stream,
                             reinterpret_cast<const uint32_t*>(valOut), reinterpret_cast<uint32_t*>(V),
                             (uint64_t)n * VB / 4, fallback, 1u);
      }
    }
    // The two top digits: XCD-segmented passes (thrs_kernels.hpp
    // thrs_pass_seg) -- the second digit over position segments (the bucket
    // histogram's workgroup ranges), the top digit over second-digit ranges.
    // Gates on meta[kMetaMode]: mode 0 (local path) the segmented second-digit
    // pass, mode 1 (fallback) the plain one (the position segments' counts are
    // those of the INPUT order, not the low passes' output), mode 2 (one
    // bucket holds every key: both top digits constant) neither, and no
    // top-digit pass either (both are identities, and skipping both keeps the
    // result in K).
    auto launch_seg = [&](int p, U* kin, U* kout, VW* vin, VW* vout, uint64_t infoOff, uint64_t baseOff,
                          const uint32_t* gate, uint32_t gateMask, int codec = kCodecKeys) {
      ProfScope prof(stream, gateMask == kGateMode1 ? 3 : 1);  // fallback-only launches are timed apart
      auto kern = codec == kCodecSplit ? skSplit : codec == kCodecPlanes ? skPlanes : sk;
      // kCodecPlanes: image-space input (orderMask 0), digit at bits 16-23 of k'
      hipLaunchKernelGGL(kern, dim3((uint32_t)segPerCU * cu_count()), dim3(G::THREADS), lds, stream, kin, kout, vin,
                         vout, codec == kCodecPlanes ? (U)0 : orderMask, codec == kCodecPlanes ? 16 : startBits + 8 * p,
                         reinterpret_cast<uint32_t*>(hyb + infoOff), reinterpret_cast<const uint32_t*>(hyb + baseOff),
                         status[p & 1], err, grp[p & 1], gate, gateMask, hiP);
    };
    const uint64_t sw = plan.wideStatus ? 8 : 4;
    const int setB = (nLow + 1) & 1;
    if (segA) {
      // Both table sets are clean: zeroed up front, and on the fallback each
      // low pass clears its successor's rows; the segmented passes' extra
      // tile ids (rows past nTiles) are touched by nothing else.
      if (planes)
        launch_seg(nLow, K, reinterpret_cast<U*>(loP), V, valOut, kSegInfoAOff, kSegBaseAOff, mode, kGateMode0,
                   kCodecSplit);
      else
        launch_seg(nLow, K, keyOut, V, valOut, kSegInfoAOff, kSegBaseAOff, mode, kGateMode0);
      launch_pass(nLow, K, keyOut, V, valOut, mode, kGateMode1);
    } else {
      launch_pass(nLow, K, keyOut, V, valOut, mode, kGateMode0 | kGateMode1);
      // the segmented pass's tile ids reach past nTiles (per-segment
      // rounding): clear those rows (pass nLow cleared rows [0, nTiles))
      const uint64_t nGroups0 = (plan.nTiles + kGroup - 1) / kGroup;
      if (hipMemsetAsync(reinterpret_cast<char*>(status[setB]) + plan.nTiles * kBins * sw, 0,
                         kSegTilePad * kBins * sw, stream) != hipSuccess ||
          hipMemsetAsync(grp[setB].ga + nGroups0 * kBins, 0, (kSegs + 1) * kBins * 4, stream) != hipSuccess ||
          hipMemsetAsync(reinterpret_cast<char*>(grp[setB].gp) + nGroups0 * kBins * sw, 0, (kSegs + 1) * kBins * sw,
                         stream) != hipSuccess)
        return THRS_ERROR_HIP;
    }
    if (planes) {  // mode 0: planes -> lo2; mode 1 (fallback): keys
      launch_seg(nLow + 1, reinterpret_cast<U*>(loP), reinterpret_cast<U*>(lo2P), valOut, V, kSegInfoOff, kSegBaseOff,
                 mode, kGateMode0, kCodecPlanes);
      launch_seg(nLow + 1, keyOut, K, valOut, V, kSegInfoOff, kSegBaseOff, mode, kGateMode1);
    } else if (segTop)
      launch_seg(nLow + 1, keyOut, K, valOut, V, kSegInfoOff, kSegBaseOff, mode, kGateMode0 | kGateMode1);
    else
      launch_pass(nLow + 1, keyOut, K, valOut, V, mode, kGateMode0 | kGateMode1);
    {
      ProfScope prof(stream, 2);
      // never more workgroups than chunks can exist: <= 256 (one per top digit)
      // + 2 per non-empty bucket, and <= the number of buckets
      // (single-bucket chunks -- pairs, local16, 8-byte keys: thrs_plan makes
      // every bucket a chunk, empty or not)
      const bool singleChunks = VB || local16 || kBucket64;
      const uint64_t maxChunks = singleChunks ? kBuckets : std::min<uint64_t>(kBuckets, 256 + 2 * (uint64_t)n);
      auto launch_local = [&](auto geom) {
        using LG = decltype(geom);
        const size_t llds = LG::template lds<U>();
        if constexpr (kBucket64) {
          (void)llds;
        } else if constexpr (VB == 4) {
          auto lk = atomicRank ? thrs_local_pairs<true, LG> : thrs_local_pairs<false, LG>;
          hipLaunchKernelGGL(lk, dim3((uint32_t)maxChunks), dim3(LG::THREADS), llds, stream,
                             reinterpret_cast<uint32_t*>(K), reinterpret_cast<uint32_t*>(V), (uint32_t)orderMask,
                             chunkOff, chunkB0, meta);
        } else {
          auto lk = atomicRank ? thrs_local<KT, true, LG> : thrs_local<KT, false, LG>;
          hipLaunchKernelGGL(lk, dim3((uint32_t)maxChunks), dim3(LG::THREADS), llds, stream, K, orderMask, startBits,
                             nLow, chunkOff, chunkB0, meta, g_lstamps);
        }
      };
      if constexpr (kBucket64) {
        auto lk = atomicRank ? thrs_local64<KT, VB, true> : thrs_local64<KT, VB, false>;
        hipLaunchKernelGGL(lk, dim3((uint32_t)maxChunks), dim3(Loc64::THREADS), Loc64::LDS, stream,
                           reinterpret_cast<uint64_t*>(K), reinterpret_cast<uint64_t*>(V), (uint64_t)orderMask,
                           chunkOff, chunkB0, meta);
      } else if (local16) {
        if constexpr (KT == 0 && VB == 0) {
          if (count16) {
            // persistent: one 128-KiB workgroup per CU walks the chunks
            const uint32_t cgrid = (uint32_t)std::min<uint64_t>(maxChunks, (uint64_t)cu_count());
            // planes off / mode 2: the items are the keys themselves (in place)
            auto lk = planes ? thrs_local_count16<true> : thrs_local_count16<false>;
            hipLaunchKernelGGL(lk, dim3(cgrid), dim3(LocCount::THREADS), LocCount::LDS, stream,
                               reinterpret_cast<uint32_t*>(K), n, (uint32_t)orderMask, chunkOff, chunkB0, meta,
                               static_cast<const uint16_t*>(lo2P), joint);
          } else if (wide16) {
            auto lk = atomicRank ? thrs_local16<true, Loc16Wide> : thrs_local16<false, Loc16Wide>;
            hipLaunchKernelGGL(lk, dim3((uint32_t)maxChunks), dim3(Loc16Wide::THREADS), Loc16Wide::LDS, stream,
                               reinterpret_cast<uint32_t*>(K), (uint32_t)orderMask, chunkOff, chunkB0, meta,
                               planes ? static_cast<const uint16_t*>(lo2P) : nullptr);
          } else {
            auto lk = atomicRank ? thrs_local16<true, Loc16> : thrs_local16<false, Loc16>;
            hipLaunchKernelGGL(lk, dim3((uint32_t)maxChunks), dim3(Loc16::THREADS), Loc16::LDS, stream,
                               reinterpret_cast<uint32_t*>(K), (uint32_t)orderMask, chunkOff, chunkB0, meta,
                               planes ? static_cast<const uint16_t*>(lo2P) : nullptr);
          }
        }
      } else if (smallLocal) {
        launch_local(LocSmall{});
      } else {
        launch_local(LocBig{});
      }
    }
    if (hipGetLastError() != hipSuccess) return THRS_ERROR_HIP;
  }
  return publish_error();
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

bool valid_options(const thrs_options& o) {
  return o.path >= THRS_PATH_AUTO && o.path <= THRS_PATH_BUCKET && o.localGeometry >= THRS_LOCAL_AUTO &&
         o.localGeometry <= THRS_LOCAL_WIDE16 && o.segmented >= THRS_SEG_AUTO && o.segmented <= THRS_SEG_NONE &&
         o.tileClaims >= THRS_CLAIMS_AUTO && o.tileClaims <= THRS_CLAIMS_TICKET && o.rank >= THRS_RANK_AUTO &&
         o.rank <= THRS_RANK_BALLOT && o.planes >= THRS_PLANES_AUTO && o.planes <= THRS_PLANES_OFF;
}

// Scratch is sized for the larger of the keys-only and pairs tile plans so
// one buffer serves both sortKeys and sortPairs, like the reference's.
int temp_def(int keyType, int valueType, uint32_t n, thrs_temp_def* out) {
  if (!out || !valid_key(keyType)) return THRS_ERROR_INVALID_VALUE;
  const int vbytes = valid_value(valueType) ? value_bytes_of(valueType) : 16;
  const Plan pk = make_plan(keyType, 0, n);
  const Plan pp = make_plan(keyType, vbytes, n);
  out->pSumBuffer = round_up(std::max(pk.scratchBytes, pp.scratchBytes), 16);
  out->keyOutBuffer = round_up((uint64_t)key_bytes_of(keyType) * n, 16);
  out->valueOutBuffer = round_up((uint64_t)vbytes * n, 16);
  return THRS_SUCCESS;
}

int sort_impl(const thrs_config* cfg, const thrs_options* options, void* keys, void* vals, bool pairs, uint32_t n,
              void* tmp, int startBits, int endBits, hipStream_t stream) {
  // a failure of an earlier sort on this device is reported first (and cleared)
  if (take_sticky()) return THRS_ERROR_LOOKBACK_TIMEOUT;
  const thrs_options opt = options ? *options : thrs_options{};
  if (!valid_options(opt)) return THRS_ERROR_INVALID_VALUE;
  if (!cfg || !valid_key(cfg->keyType) || (pairs && !valid_value(cfg->valueType))) return THRS_ERROR_INVALID_VALUE;
  if (cfg->sortOrder != THRS_ORDER_ASCENDING && cfg->sortOrder != THRS_ORDER_DESCENDING) return THRS_ERROR_INVALID_VALUE;
  if (((endBits - startBits) % 8) != 0) return THRS_ERROR_BIT_RANGE;  // tinyhipradixsort.hpp:856
  if (startBits < 0) return THRS_ERROR_INVALID_VALUE;
  if (n == 0 || startBits >= endBits) return THRS_SUCCESS;
  const int kb = key_bytes_of(cfg->keyType);
  const int width = kb * 8;
  int nPass = 0;  // passes that read at least one key bit; the rest are identities
  for (int i = 0; startBits + 8 * i < endBits; ++i)
    if (startBits + 8 * i < width) ++nPass;
  if (nPass == 0) return THRS_SUCCESS;
  if (!keys || !tmp || (pairs && !vals)) return THRS_ERROR_INVALID_VALUE;
  const int vb = pairs ? value_bytes_of(cfg->valueType) : 0;
  const Plan plan = make_plan(cfg->keyType, vb, n);
  const bool desc = cfg->sortOrder == THRS_ORDER_DESCENDING;
  // [pSumBuffer = scratch][keyOut][valueOut], exactly as getTemporaryBufferBytes
  // reports it (TemporaryBufferDef accessors, tinyhipradixsort.hpp:820-831).
  thrs_temp_def def;
  const int rc = temp_def(cfg->keyType, cfg->valueType, n, &def);
  if (rc) return rc;
  void* ko = static_cast<char*>(tmp) + def.pSumBuffer;
  void* vo = static_cast<char*>(tmp) + def.pSumBuffer + def.keyOutBuffer;
  switch (cfg->keyType) {
    case THRS_KEY_U32: return run_vb<0>(vb, keys, vals, n, tmp, ko, vo, startBits, nPass, desc, plan, opt, stream);
    case THRS_KEY_U64: return run_vb<1>(vb, keys, vals, n, tmp, ko, vo, startBits, nPass, desc, plan, opt, stream);
    case THRS_KEY_F32: return run_vb<2>(vb, keys, vals, n, tmp, ko, vo, startBits, nPass, desc, plan, opt, stream);
    case THRS_KEY_F64: return run_vb<3>(vb, keys, vals, n, tmp, ko, vo, startBits, nPass, desc, plan, opt, stream);
  }
  return THRS_ERROR_INVALID_VALUE;
}

int partition_impl(const thrs_config* cfg, const void* keysIn, const void* valsIn, uint32_t n, void* tmp,
                   void* keysOut, void* valsOut, int bitLocation, uint32_t* counts, hipStream_t stream) {
  if (take_sticky()) return THRS_ERROR_LOOKBACK_TIMEOUT;
  if (!cfg || !valid_key(cfg->keyType)) return THRS_ERROR_INVALID_VALUE;
  if (cfg->sortOrder != THRS_ORDER_ASCENDING && cfg->sortOrder != THRS_ORDER_DESCENDING) return THRS_ERROR_INVALID_VALUE;
  const bool pairs = valsIn != nullptr;
  if (pairs && (!valid_value(cfg->valueType) || !valsOut)) return THRS_ERROR_INVALID_VALUE;
  const int kb = key_bytes_of(cfg->keyType);
  if (bitLocation < 0 || bitLocation >= kb * 8 || !counts || !tmp) return THRS_ERROR_INVALID_VALUE;
  if (n == 0) return hipMemsetAsync(counts, 0, kBins * sizeof(uint32_t), stream) == hipSuccess ? THRS_SUCCESS
                                                                                                : THRS_ERROR_HIP;
  if (!keysIn || !keysOut || keysIn == keysOut || (pairs && valsIn == valsOut)) return THRS_ERROR_INVALID_VALUE;
  const int vb = pairs ? value_bytes_of(cfg->valueType) : 0;
  const Plan plan = make_plan(cfg->keyType, vb, n);
  const bool desc = cfg->sortOrder == THRS_ORDER_DESCENDING;
  const thrs_options opt{};
  void* ki = const_cast<void*>(keysIn);
  void* vi = const_cast<void*>(valsIn);
  switch (cfg->keyType) {
    case THRS_KEY_U32: return run_vb<0>(vb, ki, vi, n, tmp, keysOut, valsOut, bitLocation, 1, desc, plan, opt, stream, counts);
    case THRS_KEY_U64: return run_vb<1>(vb, ki, vi, n, tmp, keysOut, valsOut, bitLocation, 1, desc, plan, opt, stream, counts);
    case THRS_KEY_F32: return run_vb<2>(vb, ki, vi, n, tmp, keysOut, valsOut, bitLocation, 1, desc, plan, opt, stream, counts);
    case THRS_KEY_F64: return run_vb<3>(vb, ki, vi, n, tmp, keysOut, valsOut, bitLocation, 1, desc, plan, opt, stream, counts);
  }
  return THRS_ERROR_INVALID_VALUE;
}

}  // namespace

#define THRS_API __attribute__((visibility("default")))

extern "C" {

THRS_API int thrs_abi_version(void) { return THRS_ABI_VERSION; }

THRS_API const char* thrs_status_string(int s) {
  switch (s) {
    case THRS_SUCCESS: return "THRS_SUCCESS";
    case THRS_ERROR_INVALID_VALUE: return "THRS_ERROR_INVALID_VALUE";
    case THRS_ERROR_BIT_RANGE: return "THRS_ERROR_BIT_RANGE: (endBits - startBits) % 8 != 0";
    case THRS_ERROR_HIP: return "THRS_ERROR_HIP";
    case THRS_ERROR_OUT_OF_MEMORY: return "THRS_ERROR_OUT_OF_MEMORY";
    case THRS_ERROR_LOOKBACK_TIMEOUT: return "THRS_ERROR_LOOKBACK_TIMEOUT";
  }
  return "THRS_UNKNOWN_STATUS";
}

THRS_API uint64_t thrs_key_bytes(int keyType) { return valid_key(keyType) ? (uint64_t)key_bytes_of(keyType) : 0; }
THRS_API uint64_t thrs_value_bytes(int valueType) { return valid_value(valueType) ? (uint64_t)value_bytes_of(valueType) : 0; }

THRS_API int thrs_get_temporary_buffer_bytes(const thrs_config* cfg, uint32_t n, thrs_temp_def* out) {
  if (!cfg || !valid_value(cfg->valueType)) return THRS_ERROR_INVALID_VALUE;
  return temp_def(cfg->keyType, cfg->valueType, n, out);
}

THRS_API int thrs_sort_keys(const thrs_config* config, void* keys, uint32_t n, void* tmp, int startBits, int endBits,
                            hipStream_t stream) {
  return sort_impl(config, nullptr, keys, nullptr, false, n, tmp, startBits, endBits, stream);
}

THRS_API int thrs_sort_pairs(const thrs_config* config, void* keys, void* values, uint32_t n, void* tmp, int startBits,
                             int endBits, hipStream_t stream) {
  return sort_impl(config, nullptr, keys, values, true, n, tmp, startBits, endBits, stream);
}

THRS_API int thrs_sort_keys_ex(const thrs_config* config, const thrs_options* options, void* keys, uint32_t n,
                               void* tmp, int startBits, int endBits, hipStream_t stream) {
  return sort_impl(config, options, keys, nullptr, false, n, tmp, startBits, endBits, stream);
}

THRS_API int thrs_sort_pairs_ex(const thrs_config* config, const thrs_options* options, void* keys, void* values,
                                uint32_t n, void* tmp, int startBits, int endBits, hipStream_t stream) {
  return sort_impl(config, options, keys, values, true, n, tmp, startBits, endBits, stream);
}

THRS_API int thrs_partition_pass(const thrs_config* config, const void* keysIn, const void* valuesIn, uint32_t n,
                                 void* tmp, void* keysOut, void* valuesOut, int bitLocation, uint32_t* counts,
                                 hipStream_t stream) {
  return partition_impl(config, keysIn, valuesIn, n, tmp, keysOut, valuesOut, bitLocation, counts, stream);
}

THRS_API int thrs_digit_histogram(const thrs_config* config, const void* keys, uint32_t n, uint64_t prefixMask,
                                  uint64_t prefixValue, int bitLocation, uint32_t* counts, hipStream_t stream) {
  if (!config || !valid_key(config->keyType) || !counts) return THRS_ERROR_INVALID_VALUE;
  if (config->sortOrder != THRS_ORDER_ASCENDING && config->sortOrder != THRS_ORDER_DESCENDING)
    return THRS_ERROR_INVALID_VALUE;
  const int kb = key_bytes_of(config->keyType);
  if (bitLocation < 0 || bitLocation + 8 > kb * 8) return THRS_ERROR_INVALID_VALUE;
  if (n && !keys) return THRS_ERROR_INVALID_VALUE;
  if (hipMemsetAsync(counts, 0, kBins * sizeof(uint32_t), stream) != hipSuccess) return THRS_ERROR_HIP;
  if (n == 0) return THRS_SUCCESS;
  const bool desc = config->sortOrder == THRS_ORDER_DESCENDING;
  const uint64_t want = ((uint64_t)n + kHistThreads * 8 - 1) / (kHistThreads * 8);
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)cu_count()));
  if (kb == 4)
    hipLaunchKernelGGL(thrs_digit_hist_u32, dim3(grid), dim3(kHistThreads), 0, stream,
                       static_cast<const uint32_t*>(keys), n, config->keyType, desc ? 0xFFFFFFFFu : 0u,
                       (uint32_t)prefixMask, (uint32_t)prefixValue, bitLocation, counts);
  else
    hipLaunchKernelGGL(thrs_digit_hist_u64, dim3(grid), dim3(kHistThreads), 0, stream,
                       static_cast<const uint64_t*>(keys), n, config->keyType, desc ? ~0ull : 0ull, prefixMask,
                       prefixValue, bitLocation, counts);
  return hipGetLastError() == hipSuccess ? THRS_SUCCESS : THRS_ERROR_HIP;
}

THRS_API int thrs_check_device_error(void* tmp, hipStream_t stream) {
  if (!tmp) return THRS_ERROR_INVALID_VALUE;
  uint32_t err = 0;
  if (hipMemcpyAsync(&err, static_cast<char*>(tmp) + kErrOff, sizeof(err), hipMemcpyDeviceToHost, stream) !=
          hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess)
    return THRS_ERROR_HIP;
  if (err) {
    (void)take_sticky();  // reported here: the next sort does not repeat it
    return THRS_ERROR_LOOKBACK_TIMEOUT;
  }
  return THRS_SUCCESS;
}

THRS_API int thrs_take_device_error(void) { return take_sticky() ? THRS_ERROR_LOOKBACK_TIMEOUT : THRS_SUCCESS; }

THRS_API int thrs_profile_enable(int enable) {
  std::lock_guard<std::mutex> g(g_prof_mu);
  for (auto& r : g_prof) {
    g_prof_pool.push_back(r.a);
    g_prof_pool.push_back(r.b);
  }
  g_prof.clear();
  g_prof_on = enable != 0;
  return THRS_SUCCESS;
}

// kind: 0 = histogram + scan/plan, 1 = device-wide digit pass, 2 = local sort
THRS_API int thrs_profile_read_kind(int kind, double* ms, int* launches) {
  std::lock_guard<std::mutex> g(g_prof_mu);
  double t = 0;
  int c = 0;
  for (auto& r : g_prof) {
    if (r.kind != kind) continue;
    if (hipEventSynchronize(r.b) != hipSuccess) return THRS_ERROR_HIP;
    float x = 0;
    if (hipEventElapsedTime(&x, r.a, r.b) != hipSuccess) return THRS_ERROR_HIP;
    t += x;
    ++c;
  }
  if (ms) *ms = t;
  if (launches) *launches = c;
  return THRS_SUCCESS;
}

THRS_API int thrs_profile_read(double* histMs, int* histLaunches, double* passMs, int* passLaunches) {
  const int rc = thrs_profile_read_kind(0, histMs, histLaunches);
  return rc ? rc : thrs_profile_read_kind(1, passMs, passLaunches);
}

// Diagnostic hook, not part of the drop-in boundary: in -DTHRS_STAMPS builds
// the pass kernel writes per-tile phase timestamps to buf[(pass*nTiles+tile)*16+i].
THRS_API int thrs_debug_set_stamps(void* buf) {
  g_stamps = static_cast<uint64_t*>(buf);
  return THRS_SUCCESS;
}

// Diagnostic hook: in -DTHRS_STAMPS builds the local sort kernel writes
// per-chunk phase timestamps to buf[chunk*8+i] (thrs_hybrid.hpp loc_stamp).
THRS_API int thrs_debug_set_local_stamps(void* buf) {
  g_lstamps = static_cast<uint64_t*>(buf);
  return THRS_SUCCESS;
}

// Diagnostic: keys per tile of the pass kernel for (key type, value bytes).
THRS_API uint64_t thrs_debug_tile_keys(int keyType, int valueBytes) {
  return valid_key(keyType) ? tile_keys(key_bytes_of(keyType), valueBytes) : 0;
}

// Diagnostic: resident workgroups per CU of the local (in-LDS) bucket sort
// kernel for 4-byte keys, as the runtime computes it from its LDS and VGPRs.
THRS_API int thrs_debug_local_occupancy(void) {
  const size_t lds = local_lds_bytes<uint32_t>();
  if (allow_lds(thrs_local<0, true, LocBig>, lds) != hipSuccess) return -1;
  int perCU = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, thrs_local<0, true, LocBig>, kLocThreads, lds) != hipSuccess)
    return -1;
  return perCU;
}

// Which rank path the current device uses (1 = LDS-atomic, 0 = ballot match);
// runs the one-time probe if needed.
THRS_API int thrs_rank_mode(void) { return probe_rank_mode(nullptr); }

THRS_API int thrs_malloc(void** ptr, int64_t bytes) {
  if (!ptr) return THRS_ERROR_INVALID_VALUE;
  *ptr = nullptr;
  if (hipMalloc(ptr, (size_t)std::max<int64_t>(bytes, 1)) != hipSuccess) {
    *ptr = nullptr;
    return THRS_ERROR_OUT_OF_MEMORY;
  }
  return THRS_SUCCESS;
}
THRS_API int thrs_free(void* ptr) { return hipFree(ptr) == hipSuccess ? THRS_SUCCESS : THRS_ERROR_HIP; }

THRS_API int thrs_memcpy_htod_async(void* dst, const void* src, uint64_t bytes, hipStream_t stream) {
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream) == hipSuccess ? THRS_SUCCESS : THRS_ERROR_HIP;
}
THRS_API int thrs_memcpy_dtoh(void* dst, const void* src, uint64_t bytes) {
  return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) == hipSuccess ? THRS_SUCCESS : THRS_ERROR_HIP;
}
THRS_API int thrs_memcpy_dtod_async(void* dst, const void* src, uint64_t bytes, hipStream_t stream) {
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, stream) == hipSuccess ? THRS_SUCCESS
                                                                                          : THRS_ERROR_HIP;
}
THRS_API int thrs_stream_create(hipStream_t* s) {
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking) == hipSuccess ? THRS_SUCCESS : THRS_ERROR_HIP;
}
THRS_API int thrs_stream_destroy(hipStream_t s) { return hipStreamDestroy(s) == hipSuccess ? THRS_SUCCESS : THRS_ERROR_HIP; }
THRS_API int thrs_stream_synchronize(hipStream_t s) {
  return hipStreamSynchronize(s) == hipSuccess ? THRS_SUCCESS : THRS_ERROR_HIP;
}

}  // extern "C"
