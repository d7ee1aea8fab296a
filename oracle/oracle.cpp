// oracle.cpp -- CPU restatement of the tinyhipradixsort hot path.
//
// TEST INFRASTRUCTURE ONLY.  Nothing in the product path (libthrs.so, the
// header-only API, the Python mirror's sort calls) may link, load or call this
// file.  It is imported only by tests/, by __graft_entry__.smoke() and by the
// cpu_baseline leg of bench.py, always as the checker, never as the thing
// measured for `value`.
//
// What it restates (all citations are into /root/reference):
//   * splitmix64                       unittest.cpp:24-35
//   * randomizeValues generators       unittest.cpp:96-116
//   * getKeyBits (host, no order mask) fpKey.hpp:15-38
//   * getKeyBits ^ ORDER_MASK (device) tinyhipradixsort.hpp:64-115 (== kernel.cu:18-69)
//   * digit = (keyBits >> bitLocation) & 0xFF
//                                      tinyhipradixsort.hpp:131, 306, 321
//   * the pass loop: one stable 8-bit counting pass per
//     bitLocation = startBits + 8i < endBits, result in the caller's buffers
//                                      tinyhipradixsort.hpp:854-944
//   * the reference tests' own oracles: std::sort (unittest.cpp:154-161),
//     std::stable_sort by a window digit (unittest.cpp:283-291, 343-348) and
//     stableSortPairs (unittest.cpp:358-377).
//
// Each reference pass (blockCount + prefixSumExclusiveInplace + reorder) is a
// stable counting sort on one 8-bit digit; the restatement below performs
// exactly that, pass by pass, so intermediate ping-pong states match too.
//
// Shift semantics: a digit shift at or beyond the key width reads zero bits.
// The reference only exercises this for 64-bit keys (StartBits.u64 with
// startBit > 56, unittest.cpp:266) where C++ shifts are defined; for 32-bit
// keys a shift >= 32 is UB in the reference (kernel.cu:85) and out of
// contract, and both this oracle and libthrs define it as zero bits.

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>
#include <parallel/algorithm>

extern "C" {

enum { ORC_U32 = 0, ORC_U64 = 1, ORC_F32 = 2, ORC_F64 = 3 };  // == thrs::KeyType order (tinyhipradixsort.hpp:638-644)

// ---- splitmix64 (unittest.cpp:24-35) -------------------------------------
uint64_t orc_splitmix64_next(uint64_t* state) {
  uint64_t z = (*state += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

void orc_splitmix64_fill(uint64_t* state, uint64_t* out, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) out[i] = orc_splitmix64_next(state);
}

// randomizeValues<T> (unittest.cpp:96-116) for each key type, consuming n
// draws from *state.  out must hold n elements of the key's width.
void orc_randomize_keys(int keyType, uint64_t* state, void* out, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t r = orc_splitmix64_next(state);
    switch (keyType) {
      case ORC_U32: ((uint32_t*)out)[i] = (uint32_t)r; break;
      case ORC_F32: ((uint32_t*)out)[i] = (uint32_t)(r & 0xFF7FFFFFull); break;
      case ORC_U64: ((uint64_t*)out)[i] = r; break;
      case ORC_F64: ((uint64_t*)out)[i] = r & 0xFFEFFFFFFFFFFFFFull; break;
    }
  }
}

// ---- key transform --------------------------------------------------------
// fpKey.hpp:23-30 / kernel.cu:54-61.  `x == 0.0f` is restated on the bits
// ((b & 0x7FFFFFFF) == 0) so that denormals are never flushed to zero.
static inline uint32_t key_bits_f32(uint32_t b) {
  if ((b & 0x7FFFFFFFu) == 0) b = 0;
  uint32_t flip = (uint32_t)((int32_t)b >> 31) | 0x80000000u;
  return b ^ flip;
}
static inline uint64_t key_bits_f64(uint64_t b) {
  if ((b & 0x7FFFFFFFFFFFFFFFull) == 0) b = 0;
  uint64_t flip = (uint64_t)((int64_t)b >> 63) | 0x8000000000000000ull;
  return b ^ flip;
}

// getKeyBits(x) ^ ORDER_MASK for every element, widened to u64.
void orc_key_bits(int keyType, const void* in, uint64_t* out, uint64_t n, int descending) {
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t b = 0;
    switch (keyType) {
      case ORC_U32: b = ((const uint32_t*)in)[i]; if (descending) b ^= 0xFFFFFFFFull; break;
      case ORC_F32: b = key_bits_f32(((const uint32_t*)in)[i]); if (descending) b ^= 0xFFFFFFFFull; break;
      case ORC_U64: b = ((const uint64_t*)in)[i]; if (descending) b = ~b; break;
      case ORC_F64: b = key_bits_f64(((const uint64_t*)in)[i]); if (descending) b = ~b; break;
    }
    out[i] = b;
  }
}

static inline int key_bytes(int keyType) { return (keyType == ORC_U32 || keyType == ORC_F32) ? 4 : 8; }

static inline uint32_t digit_of(uint64_t bits, int keyWidth, int bitLocation) {
  if (bitLocation >= keyWidth) return 0;
  return (uint32_t)((bits >> bitLocation) & 0xFFu);
}

// ---- the pass loop (tinyhipradixsort.hpp:854-944) -------------------------
// keys/values are sorted in place.  valueBytes = 0 for sortKeys, else 4/8/16.
// Returns the number of passes run, or -1 if (endBits-startBits)%8 != 0
// (the reference's THRS_ASSERT at tinyhipradixsort.hpp:856).
int orc_lsd_sort(int keyType, int valueBytes, void* keys, void* values, uint64_t n,
                 int startBits, int endBits, int descending) {
  if (((endBits - startBits) % 8) != 0) return -1;
  const int kb = key_bytes(keyType);
  const int width = kb * 8;
  std::vector<uint64_t> bits(n), bitsTmp(n);
  orc_key_bits(keyType, keys, bits.data(), n, descending);
  std::vector<uint8_t> kIn((uint8_t*)keys, (uint8_t*)keys + n * kb), kOut(n * kb);
  std::vector<uint8_t> vIn, vOut;
  if (valueBytes) {
    vIn.assign((uint8_t*)values, (uint8_t*)values + n * valueBytes);
    vOut.resize(n * valueBytes);
  }
  int passes = 0;
  for (int i = 0; (startBits + i * 8) < endBits; ++i) {
    const int bitLocation = startBits + i * 8;
    uint64_t count[257] = {0};
    for (uint64_t j = 0; j < n; ++j) count[digit_of(bits[j], width, bitLocation) + 1]++;
    for (int d = 0; d < 256; ++d) count[d + 1] += count[d];  // exclusive offsets in count[0..255]
    for (uint64_t j = 0; j < n; ++j) {
      uint64_t dst = count[digit_of(bits[j], width, bitLocation)]++;
      std::memcpy(&kOut[dst * kb], &kIn[j * kb], kb);
      bitsTmp[dst] = bits[j];
      if (valueBytes) std::memcpy(&vOut[dst * valueBytes], &vIn[j * valueBytes], valueBytes);
    }
    kIn.swap(kOut);
    bits.swap(bitsTmp);
    if (valueBytes) vIn.swap(vOut);
    ++passes;
  }
  // The reference leaves the result in the caller's buffers (ping-pong plus
  // the odd-pass copy-back at :936-943).
  std::memcpy(keys, kIn.data(), n * kb);
  if (valueBytes) std::memcpy(values, vIn.data(), n * valueBytes);
  return passes;
}

// ---- the reference tests' own oracles -------------------------------------
// std::sort with operator< / operator> (unittest.cpp:154-161, 218).
void orc_std_sort_keys(int keyType, void* keys, uint64_t n, int descending) {
  switch (keyType) {
    case ORC_U32: { auto* p = (uint32_t*)keys;
      if (descending) std::sort(p, p + n, [](uint32_t a, uint32_t b) { return a > b; }); else std::sort(p, p + n); } break;
    case ORC_U64: { auto* p = (uint64_t*)keys;
      if (descending) std::sort(p, p + n, [](uint64_t a, uint64_t b) { return a > b; }); else std::sort(p, p + n); } break;
    case ORC_F32: { auto* p = (float*)keys;
      if (descending) std::sort(p, p + n, [](float a, float b) { return a > b; }); else std::sort(p, p + n); } break;
    case ORC_F64: { auto* p = (double*)keys;
      if (descending) std::sort(p, p + n, [](double a, double b) { return a > b; }); else std::sort(p, p + n); } break;
  }
}

// Stand-in for concurrency::parallel_sort / parallel_radixsort
// (unittest.cpp:526, 563, 711): libstdc++ parallel mode over OpenMP.
void orc_parallel_sort_u32(uint32_t* keys, uint64_t n) { __gnu_parallel::sort(keys, keys + n); }
void orc_parallel_sort_u64(uint64_t* keys, uint64_t n) { __gnu_parallel::sort(keys, keys + n); }
void orc_parallel_sort_keys(int keyType, void* keys, uint64_t n) {
  switch (keyType) {
    case ORC_U32: __gnu_parallel::sort((uint32_t*)keys, (uint32_t*)keys + n); break;
    case ORC_U64: __gnu_parallel::sort((uint64_t*)keys, (uint64_t*)keys + n); break;
    case ORC_F32: __gnu_parallel::sort((float*)keys, (float*)keys + n); break;
    case ORC_F64: __gnu_parallel::sort((double*)keys, (double*)keys + n); break;
  }
}

}  // extern "C"

// stableSortPairs<K,V> (unittest.cpp:358-377): std::stable_sort of (key,value)
// pairs by key with operator<.  valueBytes 4/8/16.
template <class K, int VB, bool PAR = false>
static void stable_pairs_t(void* keys, void* values, uint64_t n) {
  struct V { uint8_t b[VB]; };
  std::vector<std::pair<K, V>> pairs(n);
  for (uint64_t i = 0; i < n; ++i) {
    pairs[i].first = ((K*)keys)[i];
    std::memcpy(pairs[i].second.b, (uint8_t*)values + i * VB, VB);
  }
  auto less = [](const std::pair<K, V>& a, const std::pair<K, V>& b) { return a.first < b.first; };
  if constexpr (PAR) __gnu_parallel::stable_sort(pairs.begin(), pairs.end(), less);
  else std::stable_sort(pairs.begin(), pairs.end(), less);
  for (uint64_t i = 0; i < n; ++i) {
    ((K*)keys)[i] = pairs[i].first;
    std::memcpy((uint8_t*)values + i * VB, pairs[i].second.b, VB);
  }
}
template <class K, bool PAR = false>
static void stable_pairs_k(void* keys, void* values, uint64_t n, int valueBytes) {
  if (valueBytes == 4) stable_pairs_t<K, 4, PAR>(keys, values, n);
  else if (valueBytes == 8) stable_pairs_t<K, 8, PAR>(keys, values, n);
  else stable_pairs_t<K, 16, PAR>(keys, values, n);
}
extern "C" {
void orc_std_stable_sort_pairs(int keyType, int valueBytes, void* keys, void* values, uint64_t n) {
  switch (keyType) {
    case ORC_U32: stable_pairs_k<uint32_t>(keys, values, n, valueBytes); break;
    case ORC_U64: stable_pairs_k<uint64_t>(keys, values, n, valueBytes); break;
    case ORC_F32: stable_pairs_k<float>(keys, values, n, valueBytes); break;
    case ORC_F64: stable_pairs_k<double>(keys, values, n, valueBytes); break;
  }
}

// the same with __gnu_parallel::stable_sort (all OpenMP threads): the all-core
// CPU baseline for sortPairs workloads (bench.py cpu_baseline)
void orc_parallel_stable_sort_pairs(int keyType, int valueBytes, void* keys, void* values, uint64_t n) {
  switch (keyType) {
    case ORC_U32: stable_pairs_k<uint32_t, true>(keys, values, n, valueBytes); break;
    case ORC_U64: stable_pairs_k<uint64_t, true>(keys, values, n, valueBytes); break;
    case ORC_F32: stable_pairs_k<float, true>(keys, values, n, valueBytes); break;
    case ORC_F64: stable_pairs_k<double, true>(keys, values, n, valueBytes); break;
  }
}

// std::stable_sort by the window digit (k >> s) & 0xFF, u64 keys
// (unittest.cpp:283-291, keys asc/desc; :343-348 pairs asc with u32 values).
void orc_std_stable_sort_window_u64(uint64_t* keys, uint32_t* values, uint64_t n, int startBit, int descending) {
  std::vector<std::pair<uint64_t, uint32_t>> pairs(n);
  for (uint64_t i = 0; i < n; ++i) pairs[i] = {keys[i], values ? values[i] : 0u};
  std::stable_sort(pairs.begin(), pairs.end(), [startBit, descending](const std::pair<uint64_t, uint32_t>& a,
                                                                      const std::pair<uint64_t, uint32_t>& b) {
    uint32_t bitA = (uint32_t)((a.first >> startBit) & 0xFF);
    uint32_t bitB = (uint32_t)((b.first >> startBit) & 0xFF);
    return descending ? bitA > bitB : bitA < bitB;
  });
  for (uint64_t i = 0; i < n; ++i) {
    keys[i] = pairs[i].first;
    if (values) values[i] = pairs[i].second;
  }
}

}  // extern "C"
