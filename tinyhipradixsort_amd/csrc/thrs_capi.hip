// thrs_capi.hip -- the C-ABI of libthrs.so declared in include/thrs/thrs_capi.h,
// and the process-wide state of the library (profiling events, the per-device
// rank probe and error words).  The launch sequences are in thrs_host.hpp,
// instantiated per key type in thrs_run.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>

#include "thrs_host.hpp"

namespace thrs_host {

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

// ---- optional event timing (thrs_profile_*) ----------------------------------
namespace {
struct ProfRec {
  hipEvent_t a, b;
  int kind;
  int kernel;      // THRS_PK_*
  uint64_t bytes;  // algorithmic bytes of the launch (0 = data-dependent)
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
}  // namespace

hipEvent_t prof_begin(hipStream_t s) {
  if (!g_prof_on) return nullptr;
  std::lock_guard<std::mutex> g(g_prof_mu);
  hipEvent_t a = prof_event();
  if (a) (void)hipEventRecord(a, s);
  return a;
}
void prof_end(hipEvent_t a, hipStream_t s, int kind, int kernel, uint64_t bytes) {
  std::lock_guard<std::mutex> g(g_prof_mu);
  hipEvent_t b = prof_event();
  if (!b) return;
  (void)hipEventRecord(b, s);
  g_prof.push_back({a, b, kind, kernel, bytes});
}

uint64_t* g_stamps = nullptr;
int g_inject = 0;
uint64_t* g_lstamps = nullptr;

// Per-device result of thrs_probe_lds_order: 1 = lane-ordered LDS atomics
// (fast rank), 0 = ballot-match rank, -1 = not probed yet.  Never probed
// (synchronising) inside a stream capture: such a call takes the ballot path
// and the probe runs at the next call outside a capture.
int g_rank_mode[64];
bool g_rank_known[64];
std::mutex g_rank_mu;

int probe_rank_mode(hipStream_t stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  std::lock_guard<std::mutex> g(g_rank_mu);
  if (g_rank_known[dev]) return g_rank_mode[dev];
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return 0;
  int mode = 0;
  uint32_t* d = nullptr;
  if (hipMalloc(&d, 4) != hipSuccess) return 0;
  uint32_t h = 1;
  hipStream_t s = nullptr;
  bool ran = false;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess) {
    if (hipMemsetAsync(d, 0, 4, s) == hipSuccess) {
      hipLaunchKernelGGL(thrs_probe_lds_order, dim3(256), dim3(256), 0, s, d, 64);
      if (hipGetLastError() == hipSuccess && hipMemcpyAsync(&h, d, 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
          hipStreamSynchronize(s) == hipSuccess) {
        ran = true;
        mode = h == 0 ? 1 : 0;
      }
    }
    (void)hipStreamDestroy(s);
  }
  (void)hipFree(d);
  if (ran) {  // a probe that could not run is retried at the next call
    g_rank_mode[dev] = mode;
    g_rank_known[dev] = true;
  }
  return mode;
}

// Per-device sticky error word in host memory (mapped): thrs_err_publish
// ORs a sort's device error word into it at the end of every sort;
// thrs_take_device_error reads and clears it (thrs_capi.h, "Device-side
// failures").  Set up on first use, retried after a failure and never inside
// a stream capture; a sort runs without it (no publish) rather than fail.
uint32_t* g_sticky[64];      // host view
uint32_t* g_sticky_dev[64];  // device view
std::mutex g_sticky_mu;

uint32_t* sticky_dev(hipStream_t stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> g(g_sticky_mu);
  if (g_sticky_dev[dev]) return g_sticky_dev[dev];
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  void* h = nullptr;
  if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
    (void)hipHostFree(h);
    return nullptr;
  }
  std::memset(h, 0, 64);
  g_sticky[dev] = static_cast<uint32_t*>(h);
  g_sticky_dev[dev] = static_cast<uint32_t*>(d);
  return g_sticky_dev[dev];
}
// read-and-clear of the current device's sticky word (0 = no failure)
uint32_t take_sticky() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  uint32_t* h = nullptr;
  {
    std::lock_guard<std::mutex> g(g_sticky_mu);
    h = g_sticky[dev];
  }
  return h ? __atomic_exchange_n(h, 0u, __ATOMIC_ACQ_REL) : 0u;
}

namespace {
// the error word's bits (thrs_kernels.hpp kErrSpin / kErrRunClamped) -> status
int status_of_error_word(uint32_t e) {
  if (e & thrs_dev::kErrSpin) return THRS_ERROR_LOOKBACK_TIMEOUT;
  return e ? THRS_ERROR_DEVICE_CHECK : THRS_SUCCESS;
}

bool valid_options(const thrs_options& o) {
  return o.path >= THRS_PATH_AUTO && o.path <= THRS_PATH_BUCKET && o.localGeometry >= THRS_LOCAL_AUTO &&
         o.localGeometry <= THRS_LOCAL_TINY16 && o.segmented >= THRS_SEG_AUTO && o.segmented <= THRS_SEG_NONE &&
         o.tileClaims >= THRS_CLAIMS_AUTO && o.tileClaims <= THRS_CLAIMS_TICKET && o.rank >= THRS_RANK_AUTO &&
         o.rank <= THRS_RANK_BALLOT && o.planes >= THRS_PLANES_AUTO && o.planes <= THRS_PLANES_OFF &&
         (o.squeeze == THRS_SQUEEZE_AUTO || o.squeeze == THRS_SQUEEZE_OFF) &&
         (o.keyRange == 0 || (o.keyRange == 1 && o.rangeLo <= o.rangeHi));
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
  const thrs_options opt = options ? *options : thrs_options{};
  if (!valid_options(opt)) return THRS_ERROR_INVALID_VALUE;
  if (!cfg || !valid_key(cfg->keyType) || (pairs && !valid_value(cfg->valueType))) return THRS_ERROR_INVALID_VALUE;
  if (cfg->sortOrder != THRS_ORDER_ASCENDING && cfg->sortOrder != THRS_ORDER_DESCENDING) return THRS_ERROR_INVALID_VALUE;
  if (((endBits - startBits) % 8) != 0) return THRS_ERROR_BIT_RANGE;  // tinyhipradixsort.hpp:856
  if (startBits < 0) return THRS_ERROR_INVALID_VALUE;
  // a sort with nothing to do launches nothing; its temporary buffer (sized
  // for n > 0, so it holds the header) reports no device failure afterwards
  auto noop = [&]() -> int {
    if (n == 0 || !tmp) return THRS_SUCCESS;
    return hipMemsetAsync(static_cast<char*>(tmp) + kErrOff, 0, 4, stream) == hipSuccess ? THRS_SUCCESS
                                                                                         : THRS_ERROR_HIP;
  };
  if (n == 0 || startBits >= endBits) return noop();
  const int kb = key_bytes_of(cfg->keyType);
  const int width = kb * 8;
  int nPass = 0;  // passes that read at least one key bit; the rest are identities
  for (int i = 0; startBits + 8 * i < endBits; ++i)
    if (startBits + 8 * i < width) ++nPass;
  if (nPass == 0) return noop();
  if (!keys || !tmp || (pairs && !vals)) return THRS_ERROR_INVALID_VALUE;
  const int vb = pairs ? value_bytes_of(cfg->valueType) : 0;
  if (opt.keyRange == 1) {
    if (kb == 4 && opt.rangeHi > 0xFFFFFFFFull) return THRS_ERROR_INVALID_VALUE;
    // every key has one image: the stable sort is the identity (full window)
    if (opt.rangeLo == opt.rangeHi && startBits == 0 && endBits >= width) return noop();
  }
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
}  // namespace thrs_host

using namespace thrs_host;

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
    case THRS_ERROR_DEVICE_CHECK: return "THRS_ERROR_DEVICE_CHECK: a device-side range check clamped a run";
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

THRS_API int thrs_digit_histogram_batch(const thrs_config* config, const void* keys, const thrs_hist_target* targets,
                                        int nTargets, int bitLocation, uint32_t* counts, hipStream_t stream) {
  if (!config || !valid_key(config->keyType) || nTargets < 0 || (nTargets && (!targets || !counts)))
    return THRS_ERROR_INVALID_VALUE;
  if (config->sortOrder != THRS_ORDER_ASCENDING && config->sortOrder != THRS_ORDER_DESCENDING)
    return THRS_ERROR_INVALID_VALUE;
  const int kb = key_bytes_of(config->keyType);
  if (bitLocation < 0 || bitLocation + 8 > kb * 8) return THRS_ERROR_INVALID_VALUE;
  uint64_t most = 0;
  for (int i = 0; i < nTargets; ++i) {
    if (targets[i].count && !keys) return THRS_ERROR_INVALID_VALUE;
    most = std::max<uint64_t>(most, targets[i].count);
  }
  if (nTargets == 0) return THRS_SUCCESS;
  if (hipMemsetAsync(counts, 0, (size_t)nTargets * kBins * sizeof(uint32_t), stream) != hipSuccess)
    return THRS_ERROR_HIP;
  if (most == 0) return THRS_SUCCESS;
  const bool desc = config->sortOrder == THRS_ORDER_DESCENDING;
  const uint64_t want = (most + kHistThreads * 8 - 1) / (kHistThreads * 8);
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)cu_count()));
  for (int t0 = 0; t0 < nTargets; t0 += kMaxHistTargets) {  // one launch per kMaxHistTargets ranges
    const int cnt = std::min(kMaxHistTargets, nTargets - t0);
    HistTargets tg{};
    for (int i = 0; i < cnt; ++i) {
      tg.off[i] = targets[t0 + i].offset;
      tg.n[i] = targets[t0 + i].count;
      tg.mask[i] = targets[t0 + i].prefixMask;
      tg.value[i] = targets[t0 + i].prefixValue;
    }
    uint32_t* out = counts + (uint64_t)t0 * kBins;
    if (kb == 4)
      hipLaunchKernelGGL(thrs_digit_hist<uint32_t>, dim3(grid, cnt), dim3(kHistThreads), 0, stream,
                         static_cast<const uint32_t*>(keys), tg, config->keyType, desc ? 0xFFFFFFFFu : 0u, bitLocation,
                         out);
    else
      hipLaunchKernelGGL(thrs_digit_hist<uint64_t>, dim3(grid, cnt), dim3(kHistThreads), 0, stream,
                         static_cast<const uint64_t*>(keys), tg, config->keyType, desc ? ~0ull : 0ull, bitLocation,
                         out);
  }
  return hipGetLastError() == hipSuccess ? THRS_SUCCESS : THRS_ERROR_HIP;
}

THRS_API int thrs_digit_histogram(const thrs_config* config, const void* keys, uint32_t n, uint64_t prefixMask,
                                  uint64_t prefixValue, int bitLocation, uint32_t* counts, hipStream_t stream) {
  if (!counts) return THRS_ERROR_INVALID_VALUE;
  const thrs_hist_target t{0, n, 0, prefixMask, prefixValue};
  return thrs_digit_histogram_batch(config, keys, &t, 1, bitLocation, counts, stream);
}

THRS_API int thrs_debug_bucket_mode(const void* tmp, int keyType, int valueBytes, uint32_t n, hipStream_t stream,
                                    int* mode, int* bigChunks) {
  if (!tmp || !mode || !bigChunks || !valid_key(keyType) ||
      !(valueBytes == 0 || valueBytes == 4 || valueBytes == 8 || valueBytes == 16))
    return THRS_ERROR_INVALID_VALUE;
  const Plan plan = make_plan(keyType, valueBytes, n);
  uint32_t meta[8] = {};
  if (hipMemcpyAsync(meta, static_cast<const char*>(tmp) + plan.hybridOff + kMetaOff, sizeof(meta),
                     hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess)
    return THRS_ERROR_HIP;
  *mode = (int)meta[kMetaMode];
  *bigChunks = (int)meta[kMetaBigCount];
  return THRS_SUCCESS;
}

THRS_API int thrs_debug_big_keys(const void* tmp, int keyType, int valueBytes, uint32_t n, hipStream_t stream,
                                 uint64_t* keys) {
  if (!tmp || !keys || !valid_key(keyType) ||
      !(valueBytes == 0 || valueBytes == 4 || valueBytes == 8 || valueBytes == 16))
    return THRS_ERROR_INVALID_VALUE;
  const Plan plan = make_plan(keyType, valueBytes, n);
  const char* hyb = static_cast<const char*>(tmp) + plan.hybridOff;
  uint32_t meta[8] = {};
  if (hipMemcpyAsync(meta, hyb + kMetaOff, sizeof(meta), hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess)
    return THRS_ERROR_HIP;
  *keys = 0;
  const uint32_t m = meta[kMetaBigCount];
  // (mode 1: big chunks beside local ones; mode 2: one bucket holds every key
  // and is the one big chunk -- the fallback sorts all n keys)
  if ((meta[kMetaMode] != 1 && meta[kMetaMode] != 2) || m == 0 || m > kBuckets) return THRS_SUCCESS;
  uint32_t total = 0;
  if (hipMemcpyAsync(&total, hyb + kBigPosOff + (uint64_t)m * 4, 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess)
    return THRS_ERROR_HIP;
  *keys = total;
  return THRS_SUCCESS;
}

THRS_API int thrs_debug_vector_tiles(const void* tmp, int keyType, uint32_t n, hipStream_t stream, uint32_t* tiles) {
  if (!tmp || !tiles || !valid_key(keyType)) return THRS_ERROR_INVALID_VALUE;
  const Plan plan = make_plan(keyType, 0, n);
  uint32_t v = 0;
  if (hipMemcpyAsync(&v, static_cast<const char*>(tmp) + plan.hybridOff + kSegInfoOff + kSegVecWord * 4, 4,
                     hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess)
    return THRS_ERROR_HIP;
  *tiles = v;
  return THRS_SUCCESS;
}

THRS_API int thrs_check_device_error(void* tmp, hipStream_t stream) {
  if (!tmp) return THRS_ERROR_INVALID_VALUE;
  uint32_t err = 0;
  if (hipMemcpyAsync(&err, static_cast<char*>(tmp) + kErrOff, sizeof(err), hipMemcpyDeviceToHost, stream) !=
          hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess)
    return THRS_ERROR_HIP;
  return status_of_error_word(err);
}

THRS_API int thrs_accumulate_device_error(const void* tmp, uint32_t* acc, hipStream_t stream) {
  if (!tmp || !acc) return THRS_ERROR_INVALID_VALUE;
  hipLaunchKernelGGL(thrs_dev::thrs_err_publish, dim3(1), dim3(1), 0, stream,
                     reinterpret_cast<const uint32_t*>(static_cast<const char*>(tmp) + kErrOff), acc);
  return hipGetLastError() == hipSuccess ? THRS_SUCCESS : THRS_ERROR_HIP;
}

THRS_API int thrs_take_device_error(void) { return status_of_error_word(take_sticky()); }

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

THRS_API int thrs_profile_read_launches(int kind, double* ms, int cap, int* count) {
  std::lock_guard<std::mutex> g(g_prof_mu);
  int c = 0;
  for (auto& r : g_prof) {
    if (r.kind != kind) continue;
    if (ms && c < cap) {
      if (hipEventSynchronize(r.b) != hipSuccess) return THRS_ERROR_HIP;
      float x = 0;
      if (hipEventElapsedTime(&x, r.a, r.b) != hipSuccess) return THRS_ERROR_HIP;
      ms[c] = x;
    }
    ++c;
  }
  if (count) *count = c;
  return THRS_SUCCESS;
}

THRS_API int thrs_profile_read_launch_kernels(int kind, int32_t* kernel, uint64_t* bytes, int cap, int* count) {
  std::lock_guard<std::mutex> g(g_prof_mu);
  int c = 0;
  for (auto& r : g_prof) {
    if (r.kind != kind) continue;
    if (c < cap) {
      if (kernel) kernel[c] = r.kernel;
      if (bytes) bytes[c] = r.bytes;
    }
    ++c;
  }
  if (count) *count = c;
  return THRS_SUCCESS;
}

THRS_API const char* thrs_profile_kernel_name(int kernel) {
  static const char* names[] = {"thrs_zero_ranges", "thrs_hist", "thrs_scan", "thrs_hist_joint", "thrs_plan",
                                "thrs_pass", "thrs_pass_xb", "thrs_pass_seg", "thrs_local16", "thrs_local",
                                "thrs_local_pairs", "thrs_local_kv", "thrs_local_count16", "thrs_big_plan",
                                "thrs_big_hist", "thrs_pass_big", "thrs_big_copy", "copy-back",
                                "thrs_squeeze_sample", "thrs_hist_reduce"};
  return kernel >= 0 && kernel < (int)(sizeof(names) / sizeof(names[0])) ? names[kernel] : "";
}

THRS_API int thrs_get_path_info(const thrs_config* cfg, const thrs_options* options, int pairs, uint32_t n,
                            int startBits, int endBits, thrs_path_info* out) {
  const thrs_options opt = options ? *options : thrs_options{};
  if (!out || !cfg || !valid_key(cfg->keyType) || (pairs && !valid_value(cfg->valueType)) || !valid_options(opt))
    return THRS_ERROR_INVALID_VALUE;
  if (((endBits - startBits) % 8) != 0) return THRS_ERROR_BIT_RANGE;
  const int kb = key_bytes_of(cfg->keyType), vb = pairs ? value_bytes_of(cfg->valueType) : 0;
  int nPass = 0;
  for (int i = 0; startBits + 8 * i < endBits; ++i)
    if (startBits + 8 * i < kb * 8) ++nPass;
  *out = thrs_path_info{};
  if (n == 0 || nPass == 0) return THRS_SUCCESS;
  const Plan plan = make_plan(cfg->keyType, vb, n);
  PathSel P{};
  auto sel = [&](auto kt) {
    constexpr int KT = decltype(kt)::value;
    switch (vb) {
      case 0: P = select_path<KT, 0>(n, startBits, nPass, opt, plan, false); break;
      case 4: P = select_path<KT, 4>(n, startBits, nPass, opt, plan, false); break;
      case 8: P = select_path<KT, 8>(n, startBits, nPass, opt, plan, false); break;
      default: P = select_path<KT, 16>(n, startBits, nPass, opt, plan, false); break;
    }
  };
  switch (cfg->keyType) {
    case THRS_KEY_U32: sel(std::integral_constant<int, 0>{}); break;
    case THRS_KEY_U64: sel(std::integral_constant<int, 1>{}); break;
    case THRS_KEY_F32: sel(std::integral_constant<int, 2>{}); break;
    default: sel(std::integral_constant<int, 3>{}); break;
  }
  const uint64_t N = n, K = kb, V = vb;
  out->path = P.bucket ? 1 : 0;
  if (!P.bucket) {
    out->devicePasses = nPass;
    out->minBytes = N * K + (uint64_t)nPass * 2 * N * (K + V) + ((nPass & 1) ? 2 * N * (K + V) : 0);
    return THRS_SUCCESS;
  }
  out->devicePasses = 2;
  out->planes = P.planes ? 1 : 0;
  out->localCap = P.cap;
  out->local = P.count16 ? THRS_LOCALK_COUNT16
               : P.local16 ? THRS_LOCALK_16
               : P.local32 ? THRS_LOCALK_32
               : (kb == 4 && vb == 4) ? THRS_LOCALK_PAIRS : THRS_LOCALK_KV;
  // bucket histogram read; pass A (second digit) reads keys, writes KA per
  // key; pass B reads KA, writes KB; the local sort reads KB, writes keys
  const uint64_t KA = P.planes ? 3 : K, KBy = P.planes ? 2 : K;
  uint64_t bytes = N * K + N * (K + V) + N * (KA + V) + N * (KA + V) + N * (KBy + V) + N * (KBy + V) + N * (K + V);
  const bool floatKeys = cfg->keyType == THRS_KEY_F32 || cfg->keyType == THRS_KEY_F64;
  if (floatKeys && vb) bytes += N * K;  // the local sort re-reads float keys to permute them
  out->minBytes = bytes;
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

#ifdef THRS_FAULT_INJECT
// Fault-injection builds only (libthrs_spin0.so; not in libthrs.so): bit 0 =
// every bucket-path plan with big chunks gets a stale first entry, which its
// check must catch (THRS_ERROR_DEVICE_CHECK, no out-of-bounds access).
THRS_API int thrs_debug_inject(int what) {
  g_inject = what;
  return THRS_SUCCESS;
}
#endif

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
