// unittest_thrs.cpp -- the reference's GPU test matrix (/root/reference/
// unittest.cpp) re-run against the drop-in header <thrs/tinyhipradixsort.hpp>.
//
// Same cases, same splitmix64 streams (state 0, recreated per test), same
// sizes (TEST_ITERATION = 128, n in [1, 99999]) and the same CPU oracles
// (std::sort, std::stable_sort, stableSortPairs).  Orochi calls become the
// C-ABI helpers (oroMemcpyHtoDAsync -> thrs_memcpy_htod_async, ...).  The
// runner is a small one of our own (no utest.h); `--filter=<substr>`,
// `--list`, exit code = number of failed cases.  Compiled with plain g++: the
// header needs no HIP headers.
#include <thrs/fpKey.hpp>
#include <thrs/tinyhipradixsort.hpp>

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <limits>
#include <parallel/algorithm>
#include <string>
#include <vector>

static thrs_options g_opts{};  // set from the command line (main)

#define TEST_ITERATION 128
#define TEST_MAX_ARRAY_SIZE 100000

struct splitmix64 {  // unittest.cpp:24-35
  uint64_t x = 0;
  uint64_t next() {
    uint64_t z = (x += 0x9e3779b97f4a7c15);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9;
    z = (z ^ (z >> 27)) * 0x94d049bb133111eb;
    return z ^ (z >> 31);
  }
};

static hipStream_t stream;
static std::vector<std::string> extraArgs;  // ignored by the AOT build, kept for signature parity
static int g_failures_in_case = 0;

#define ASSERT_TRUE(e)                                                   \
  do {                                                                   \
    if (!(e)) {                                                          \
      if (g_failures_in_case++ < 5)                                      \
        std::printf("    assertion failed: %s (%s:%d)\n", #e, __FILE__, __LINE__); \
      return;                                                            \
    }                                                                    \
  } while (0)

struct Case {
  const char* name;
  std::function<void()> fn;
  bool large;
};
static std::vector<Case>& cases() {
  static std::vector<Case> c;
  return c;
}
struct Reg {
  Reg(const char* n, std::function<void()> f, bool large = false) { cases().push_back({n, f, large}); }
};
#define UTEST(S, N) \
  static void S##_##N(); \
  static Reg reg_##S##_##N(#S "." #N, S##_##N); \
  static void S##_##N()
#define UTEST_LARGE(S, N) \
  static void S##_##N(); \
  static Reg reg_##S##_##N(#S "." #N, S##_##N, true); \
  static void S##_##N()

template <class T>
static void randomizeValues(splitmix64* rng, std::vector<T>* data) {  // unittest.cpp:96-116
  for (size_t i = 0; i < data->size(); i++) {
    if (std::is_same<T, float>::value) {
      uint32_t b = rng->next() & 0xFF7FFFFF;
      std::memcpy(&(*data)[i], &b, 4);
    } else if (std::is_same<T, double>::value) {
      uint64_t b = rng->next() & 0xFFEFFFFFFFFFFFFFllu;
      std::memcpy(&(*data)[i], &b, 8);
    } else {
      (*data)[i] = static_cast<T>(rng->next());
    }
  }
}

static void h2d(void* d, const void* h, size_t bytes) { thrs::check(thrs_memcpy_htod_async(d, h, bytes, stream)); }
static void d2h(void* h, const void* d, size_t bytes) { thrs::check(thrs_memcpy_dtoh(h, d, bytes)); }
static void sync() { thrs::check(thrs_stream_synchronize(stream)); }

// ---------------------------------------------------------------- FPKeys
UTEST(FPKeys, float) {  // unittest.cpp:81-94 (10^7 pairs instead of 10^8)
  ASSERT_TRUE((-0.0f < 0.0f) == (getKeyBits(-0.0f) < getKeyBits(0.0f)));
  ASSERT_TRUE((FLT_MAX < std::numeric_limits<float>::infinity()) ==
              (getKeyBits(FLT_MAX) < getKeyBits(std::numeric_limits<float>::infinity())));
  splitmix64 rng;
  for (int i = 0; i < 10000000; i++) {
    float a = (rng.next() % 2 == 0 ? -1.0 : 1.0) * rng.next() * 0.1;
    float b = (rng.next() % 2 == 0 ? -1.0 : 1.0) * rng.next() * 0.1;
    ASSERT_TRUE((a < b) == (getKeyBits(a) < getKeyBits(b)));
  }
}

// ---------------------------------------------------------------- SortKeys
template <class KeyType>
static void testSortKeys(thrs::SortOrder sortOrder = thrs::SortOrder::Ascending) {  // unittest.cpp:127-168
  thrs::RadixSort::Config config;
  config.configureWithKey<KeyType>();
  config.sortOrder = sortOrder;
  thrs::RadixSort radixsort(extraArgs, config);
  radixsort.setOptions(g_opts);

  splitmix64 rng;
  for (int i = 0; i < TEST_ITERATION; i++) {
    int numberOfInputs = 1 + rng.next() % (TEST_MAX_ARRAY_SIZE - 1);
    std::vector<KeyType> inputKeys(numberOfInputs);
    randomizeValues(&rng, &inputKeys);

    thrs::Buffer inputKeyBuffer(sizeof(KeyType) * numberOfInputs);
    h2d(inputKeyBuffer.data(), inputKeys.data(), sizeof(KeyType) * inputKeys.size());
    thrs::Buffer tmpBuffer(radixsort.getTemporaryBufferBytes(numberOfInputs).getTemporaryBufferBytesForSortKeys());
    radixsort.sortKeys(inputKeyBuffer.data(), numberOfInputs, tmpBuffer.data(), 0, sizeof(KeyType) * 8, stream);
    sync();
    std::vector<KeyType> outputKeys(inputKeys.size());
    d2h(outputKeys.data(), inputKeyBuffer.data(), sizeof(KeyType) * numberOfInputs);

    if (sortOrder == thrs::SortOrder::Ascending) std::sort(inputKeys.begin(), inputKeys.end());
    else std::sort(inputKeys.begin(), inputKeys.end(), [](KeyType a, KeyType b) { return a > b; });
    for (size_t j = 0; j < inputKeys.size(); j++) ASSERT_TRUE(inputKeys[j] == outputKeys[j]);
  }
}

UTEST(SortKeys, u32) { testSortKeys<uint32_t>(); }
UTEST(SortKeysDescending, u32) { testSortKeys<uint32_t>(thrs::SortOrder::Descending); }
UTEST(SortKeys, f32) { testSortKeys<float>(); }
UTEST(SortKeys, u64) { testSortKeys<uint64_t>(); }
UTEST(SortKeys, f64) { testSortKeys<double>(); }
UTEST(SortKeysDescending, f64) { testSortKeys<double>(thrs::SortOrder::Descending); }
// coverage the reference lacks
UTEST(SortKeysDescending, f32) { testSortKeys<float>(thrs::SortOrder::Descending); }
UTEST(SortKeysDescending, u64) { testSortKeys<uint64_t>(thrs::SortOrder::Descending); }

UTEST(SortKeys, extremeCase) {  // unittest.cpp:191-225
  using KeyType = uint32_t;
  thrs::RadixSort::Config config;
  config.configureWithKey<KeyType>();
  thrs::RadixSort radixsort(extraArgs, config);
  radixsort.setOptions(g_opts);
  splitmix64 rng;
  for (int i = 0; i < TEST_ITERATION; i++) {
    int numberOfInputs = 1 + rng.next() % (TEST_MAX_ARRAY_SIZE - 1);
    std::vector<KeyType> inputKeys(numberOfInputs);
    inputKeys[rng.next() % inputKeys.size()] = 1;
    inputKeys[rng.next() % inputKeys.size()] = 42;
    thrs::Buffer inputKeyBuffer(sizeof(KeyType) * numberOfInputs);
    h2d(inputKeyBuffer.data(), inputKeys.data(), sizeof(KeyType) * inputKeys.size());
    thrs::Buffer tmpBuffer(radixsort.getTemporaryBufferBytes(numberOfInputs).getTemporaryBufferBytesForSortKeys());
    radixsort.sortKeys(inputKeyBuffer.data(), numberOfInputs, tmpBuffer.data(), 0, sizeof(KeyType) * 8, stream);
    sync();
    std::vector<KeyType> outputKeys(inputKeys.size());
    d2h(outputKeys.data(), inputKeyBuffer.data(), sizeof(KeyType) * numberOfInputs);
    std::sort(inputKeys.begin(), inputKeys.end());
    for (size_t j = 0; j < inputKeys.size(); j++) ASSERT_TRUE(inputKeys[j] == outputKeys[j]);
  }
}

// ---------------------------------------------------------------- StartBits
UTEST(StartBits, u64) {  // unittest.cpp:248-355
  using KeyType = uint64_t;
  using ValueType = uint32_t;
  for (auto sortOrder : {thrs::SortOrder::Ascending, thrs::SortOrder::Descending}) {
    thrs::RadixSort::Config config;
    config.configureWithKey<KeyType>();
    config.sortOrder = sortOrder;
    thrs::RadixSort radixsort(extraArgs, config);
    radixsort.setOptions(g_opts);
    splitmix64 rng;
    for (int i = 0; i < TEST_ITERATION; i++) {
      int numberOfInputs = 1 + rng.next() % (TEST_MAX_ARRAY_SIZE - 1);
      int startBit = rng.next() % 64;
      std::vector<KeyType> inputKeys(numberOfInputs);
      randomizeValues(&rng, &inputKeys);
      thrs::Buffer inputKeyBuffer(sizeof(KeyType) * numberOfInputs);
      h2d(inputKeyBuffer.data(), inputKeys.data(), sizeof(KeyType) * inputKeys.size());
      thrs::Buffer tmpBuffer(radixsort.getTemporaryBufferBytes(numberOfInputs).getTemporaryBufferBytesForSortKeys());
      radixsort.sortKeys(inputKeyBuffer.data(), numberOfInputs, tmpBuffer.data(), startBit, startBit + 8, stream);
      sync();
      std::vector<KeyType> outputKeys(inputKeys.size());
      d2h(outputKeys.data(), inputKeyBuffer.data(), sizeof(KeyType) * numberOfInputs);
      std::stable_sort(inputKeys.begin(), inputKeys.end(), [startBit, sortOrder](KeyType a, KeyType b) {
        uint32_t bitA = (a >> startBit) & 0xFF;
        uint32_t bitB = (b >> startBit) & 0xFF;
        if (sortOrder == thrs::SortOrder::Descending) return bitA > bitB;
        return bitA < bitB;
      });
      for (size_t j = 0; j < inputKeys.size(); j++) ASSERT_TRUE(inputKeys[j] == outputKeys[j]);
    }
  }
  thrs::RadixSort::Config config;
  config.configureWithKeyPair<KeyType, ValueType>();
  thrs::RadixSort radixsort(extraArgs, config);
  radixsort.setOptions(g_opts);
  splitmix64 rng;
  for (int i = 0; i < TEST_ITERATION; i++) {
    int numberOfInputs = 1 + rng.next() % (TEST_MAX_ARRAY_SIZE - 1);
    int startBit = rng.next() % 64;
    std::vector<KeyType> inputKeys(numberOfInputs);
    std::vector<ValueType> inputValues(numberOfInputs);
    randomizeValues(&rng, &inputKeys);
    for (size_t j = 0; j < inputValues.size(); j++) inputValues[j] = ValueType(j);
    thrs::Buffer inputKeyBuffer(sizeof(KeyType) * numberOfInputs);
    h2d(inputKeyBuffer.data(), inputKeys.data(), sizeof(KeyType) * inputKeys.size());
    thrs::Buffer inputValueBuffer(sizeof(ValueType) * numberOfInputs);
    h2d(inputValueBuffer.data(), inputValues.data(), sizeof(ValueType) * inputValues.size());
    thrs::Buffer tmpBuffer(radixsort.getTemporaryBufferBytes(numberOfInputs).getTemporaryBufferBytesForSortPairs());
    radixsort.sortPairs(inputKeyBuffer.data(), inputValueBuffer.data(), numberOfInputs, tmpBuffer.data(), startBit,
                        startBit + 8, stream);
    sync();
    std::vector<KeyType> outputKeys(inputKeys.size());
    d2h(outputKeys.data(), inputKeyBuffer.data(), sizeof(KeyType) * numberOfInputs);
    std::vector<ValueType> outputValues(inputValues.size());
    d2h(outputValues.data(), inputValueBuffer.data(), sizeof(ValueType) * numberOfInputs);
    std::vector<std::pair<KeyType, ValueType>> pairs(inputKeys.size());
    for (size_t j = 0; j < inputKeys.size(); j++) pairs[j] = {inputKeys[j], inputValues[j]};
    std::stable_sort(pairs.begin(), pairs.end(), [startBit](std::pair<KeyType, ValueType> a, std::pair<KeyType, ValueType> b) {
      uint32_t bitA = (a.first >> startBit) & 0xFF;
      uint32_t bitB = (b.first >> startBit) & 0xFF;
      return bitA < bitB;
    });
    for (size_t j = 0; j < outputKeys.size(); j++) {
      ASSERT_TRUE(outputKeys[j] == pairs[j].first);
      ASSERT_TRUE(outputValues[j] == pairs[j].second);
    }
  }
}

// ---------------------------------------------------------------- SortPairs
template <class KeyType, class ValueType>
static void stableSortPairs(std::vector<KeyType>* keys, std::vector<ValueType>* values) {  // unittest.cpp:358-377
  size_t n = keys->size();
  std::vector<std::pair<KeyType, ValueType>> pairs(n);
  for (size_t i = 0; i < n; i++) pairs[i] = {(*keys)[i], (*values)[i]};
  std::stable_sort(pairs.begin(), pairs.end(),
                   [](std::pair<KeyType, ValueType> a, std::pair<KeyType, ValueType> b) { return a.first < b.first; });
  for (size_t i = 0; i < n; i++) {
    (*keys)[i] = pairs[i].first;
    (*values)[i] = pairs[i].second;
  }
}

template <class KeyType, class ValueType>
static void testSortPairs() {  // unittest.cpp:379-424
  thrs::RadixSort::Config config;
  config.configureWithKeyPair<KeyType, ValueType>();
  thrs::RadixSort radixsort(extraArgs, config);
  radixsort.setOptions(g_opts);
  splitmix64 rng;
  for (int i = 0; i < TEST_ITERATION; i++) {
    int numberOfInputs = 1 + rng.next() % (TEST_MAX_ARRAY_SIZE - 1);
    std::vector<KeyType> inputKeys(numberOfInputs);
    std::vector<ValueType> inputValues(numberOfInputs);
    randomizeValues(&rng, &inputKeys);
    for (size_t j = 0; j < inputValues.size(); j++) inputValues[j] = ValueType(j);
    thrs::Buffer inputKeyBuffer(sizeof(KeyType) * numberOfInputs);
    h2d(inputKeyBuffer.data(), inputKeys.data(), sizeof(KeyType) * inputKeys.size());
    thrs::Buffer inputValueBuffer(sizeof(ValueType) * numberOfInputs);
    h2d(inputValueBuffer.data(), inputValues.data(), sizeof(ValueType) * inputValues.size());
    thrs::Buffer tmpBuffer(radixsort.getTemporaryBufferBytes(numberOfInputs).getTemporaryBufferBytesForSortPairs());
    radixsort.sortPairs(inputKeyBuffer.data(), inputValueBuffer.data(), numberOfInputs, tmpBuffer.data(), 0,
                        sizeof(KeyType) * 8, stream);
    sync();
    std::vector<KeyType> outputKeys(inputKeys.size());
    d2h(outputKeys.data(), inputKeyBuffer.data(), sizeof(KeyType) * numberOfInputs);
    std::vector<ValueType> outputValues(inputValues.size());
    d2h(outputValues.data(), inputValueBuffer.data(), sizeof(ValueType) * numberOfInputs);
    stableSortPairs<KeyType, ValueType>(&inputKeys, &inputValues);
    for (size_t j = 0; j < outputKeys.size(); j++) {
      ASSERT_TRUE(outputKeys[j] == inputKeys[j]);
      ASSERT_TRUE(outputValues[j] == inputValues[j]);
    }
  }
}

UTEST(SortPairs, K32V32) { testSortPairs<uint32_t, uint32_t>(); }
UTEST(SortPairs, KF32V32) { testSortPairs<float, uint32_t>(); }
UTEST(SortPairs, K64V32) { testSortPairs<uint64_t, uint32_t>(); }
UTEST(SortPairs, KF64V32) { testSortPairs<double, uint32_t>(); }
UTEST(SortPairs, K32V64) { testSortPairs<uint32_t, uint64_t>(); }
UTEST(SortPairs, K64V64) { testSortPairs<uint64_t, uint64_t>(); }
struct u128 {  // unittest.cpp:471-481
  uint64_t a;
  uint64_t b;
  u128() : a(0), b(0) {}
  u128(uint64_t x) : a(x), b(x) {}
  bool operator==(const u128& rhs) const { return a == rhs.a && b == rhs.b; }
};
UTEST(SortPairs, K64V128) { testSortPairs<uint64_t, u128>(); }
UTEST(SortPairs, K32V128) { testSortPairs<uint32_t, u128>(); }

// ---------------------------------------------------------------- beyond the reference
UTEST(Edge, emptyAndNoop) {
  thrs::RadixSort::Config config;
  thrs::RadixSort radixsort(extraArgs, config);
  radixsort.setOptions(g_opts);
  thrs::Buffer tmp(radixsort.getTemporaryBufferBytes(0).getTemporaryBufferBytesForSortKeys());
  thrs::Buffer keys(4);
  radixsort.sortKeys(keys.data(), 0, tmp.data(), 0, 32, stream);       // n = 0
  uint32_t one = 7;
  h2d(keys.data(), &one, 4);
  radixsort.sortKeys(keys.data(), 1, tmp.data(), 8, 8, stream);        // start == end
  radixsort.sortKeys(keys.data(), 1, tmp.data(), 0, 32, stream);
  sync();
  uint32_t back = 0;
  d2h(&back, keys.data(), 4);
  ASSERT_TRUE(back == 7);
  bool threw = false;
  try {
    radixsort.sortKeys(keys.data(), 1, tmp.data(), 0, 31, stream);     // hpp:856 assert
  } catch (const thrs::Error& e) {
    threw = e.status == THRS_ERROR_BIT_RANGE;
  }
  ASSERT_TRUE(threw);
}

UTEST(Edge, f32SpecialValues) {  // NaN / Inf / +-0 / denormals, pinned by the bit transform
  thrs::RadixSort::Config config;
  config.configureWithKeyPair<float, uint32_t>();
  thrs::RadixSort radixsort(extraArgs, config);
  radixsort.setOptions(g_opts);
  splitmix64 rng;
  const uint32_t specials[] = {0x00000000u, 0x80000000u, 0x00000001u, 0x80000001u, 0x007FFFFFu, 0x807FFFFFu,
                               0x7F800000u, 0xFF800000u, 0x7FC00000u, 0xFFC00000u, 0x7F800001u, 0xFFFFFFFFu,
                               0x3F800000u, 0xBF800000u};
  for (int it = 0; it < 16; ++it) {
    const int n = 1 + rng.next() % 30000;
    std::vector<uint32_t> keys(n), vals(n);
    for (int j = 0; j < n; ++j) {
      const uint64_t r = rng.next();
      keys[j] = (r & 3) ? specials[(r >> 8) % 14] : (uint32_t)(r >> 32);
      vals[j] = j;
    }
    thrs::Buffer kb(4 * n), vb(4 * n);
    h2d(kb.data(), keys.data(), 4 * n);
    h2d(vb.data(), vals.data(), 4 * n);
    thrs::Buffer tmp(radixsort.getTemporaryBufferBytes(n).getTemporaryBufferBytesForSortPairs());
    radixsort.sortPairs(kb.data(), vb.data(), n, tmp.data(), 0, 32, stream);
    sync();
    std::vector<uint32_t> ok(n), ov(n);
    d2h(ok.data(), kb.data(), 4 * n);
    d2h(ov.data(), vb.data(), 4 * n);
    std::vector<uint32_t> order(n);
    for (int j = 0; j < n; ++j) order[j] = j;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
      float fa, fb;
      std::memcpy(&fa, &keys[a], 4);
      std::memcpy(&fb, &keys[b], 4);
      return getKeyBits(fa) < getKeyBits(fb);
    });
    for (int j = 0; j < n; ++j) {
      ASSERT_TRUE(ov[j] == order[j]);
      ASSERT_TRUE(ok[j] == keys[order[j]]);
    }
  }
}

UTEST(Edge, pairsDescendingU32) {
  thrs::RadixSort::Config config;
  config.configureWithKeyPair<uint32_t, uint32_t>();
  config.sortOrder = thrs::SortOrder::Descending;
  thrs::RadixSort radixsort(extraArgs, config);
  radixsort.setOptions(g_opts);
  splitmix64 rng;
  for (int it = 0; it < 16; ++it) {
    const int n = 1 + rng.next() % 99999;
    std::vector<uint32_t> keys(n), vals(n);
    for (int j = 0; j < n; ++j) {
      keys[j] = (uint32_t)rng.next() & 0xFFF;  // many ties -> stability visible
      vals[j] = j;
    }
    thrs::Buffer kb(4 * n), vb(4 * n);
    h2d(kb.data(), keys.data(), 4 * n);
    h2d(vb.data(), vals.data(), 4 * n);
    thrs::Buffer tmp(radixsort.getTemporaryBufferBytes(n).getTemporaryBufferBytesForSortPairs());
    radixsort.sortPairs(kb.data(), vb.data(), n, tmp.data(), 0, 32, stream);
    sync();
    std::vector<uint32_t> ok(n), ov(n);
    d2h(ok.data(), kb.data(), 4 * n);
    d2h(ov.data(), vb.data(), 4 * n);
    std::vector<std::pair<uint32_t, uint32_t>> p(n);
    for (int j = 0; j < n; ++j) p[j] = {keys[j], vals[j]};
    std::stable_sort(p.begin(), p.end(), [](auto a, auto b) { return a.first > b.first; });
    for (int j = 0; j < n; ++j) {
      ASSERT_TRUE(ok[j] == p[j].first);
      ASSERT_TRUE(ov[j] == p[j].second);
    }
  }
}

UTEST(Edge, misalignedKeys) {  // keyIs16byteAligned=false and a 4-byte-offset base
  thrs::RadixSort::Config config;
  config.configureWithKey<uint32_t>();
  config.keyIs16byteAligned = false;
  thrs::RadixSort radixsort(extraArgs, config);
  radixsort.setOptions(g_opts);
  splitmix64 rng;
  const int n = 77777;
  std::vector<uint32_t> keys(n);
  randomizeValues(&rng, &keys);
  thrs::Buffer kb(4 * (n + 1));
  char* base = kb.data() + 4;
  h2d(base, keys.data(), 4 * n);
  thrs::Buffer tmp(radixsort.getTemporaryBufferBytes(n).getTemporaryBufferBytesForSortKeys());
  radixsort.sortKeys(base, n, tmp.data(), 0, 32, stream);
  sync();
  std::vector<uint32_t> out(n);
  d2h(out.data(), base, 4 * n);
  std::sort(keys.begin(), keys.end());
  for (int j = 0; j < n; ++j) ASSERT_TRUE(out[j] == keys[j]);
}

UTEST(Edge, windowsU32) {  // multi-pass windows, odd and even pass counts, u32
  thrs::RadixSort::Config config;
  config.configureWithKeyPair<uint32_t, uint32_t>();
  thrs::RadixSort radixsort(extraArgs, config);
  radixsort.setOptions(g_opts);
  splitmix64 rng;
  const int windows[][2] = {{0, 8}, {0, 16}, {4, 28}, {8, 32}, {16, 32}, {24, 32}, {3, 27}, {0, 24}};
  for (auto& w : windows) {
    const int n = 1 + rng.next() % 99999;
    std::vector<uint32_t> keys(n), vals(n);
    randomizeValues(&rng, &keys);
    for (int j = 0; j < n; ++j) vals[j] = j;
    thrs::Buffer kb(4 * n), vb(4 * n);
    h2d(kb.data(), keys.data(), 4 * n);
    h2d(vb.data(), vals.data(), 4 * n);
    thrs::Buffer tmp(radixsort.getTemporaryBufferBytes(n).getTemporaryBufferBytesForSortPairs());
    radixsort.sortPairs(kb.data(), vb.data(), n, tmp.data(), w[0], w[1], stream);
    sync();
    std::vector<uint32_t> ok(n), ov(n);
    d2h(ok.data(), kb.data(), 4 * n);
    d2h(ov.data(), vb.data(), 4 * n);
    const int s = w[0], len = w[1] - w[0];
    std::vector<std::pair<uint32_t, uint32_t>> p(n);
    for (int j = 0; j < n; ++j) p[j] = {keys[j], vals[j]};
    std::stable_sort(p.begin(), p.end(), [s, len](auto a, auto b) {
      const uint64_t m = (1ull << len) - 1;
      return ((a.first >> s) & m) < ((b.first >> s) & m);
    });
    for (int j = 0; j < n; ++j) {
      ASSERT_TRUE(ok[j] == p[j].first);
      ASSERT_TRUE(ov[j] == p[j].second);
    }
  }
}

UTEST_LARGE(SortKeys, u32Large) {  // unittest.cpp:688-717 (parallel_sort -> __gnu_parallel::sort)
  using KeyType = uint32_t;
  thrs::RadixSort::Config config;
  config.configureWithKey<KeyType>();
  thrs::RadixSort radixsort(extraArgs, config);
  radixsort.setOptions(g_opts);
  splitmix64 rng;
  uint32_t numberOfInputs = 1024llu * 1024 * 1024 * 2 + 100;
  thrs::Buffer tmpBuffer(radixsort.getTemporaryBufferBytes(numberOfInputs).getTemporaryBufferBytesForSortKeys());
  std::vector<KeyType> inputKeys(numberOfInputs);
  randomizeValues(&rng, &inputKeys);
  thrs::Buffer inputKeyBuffer(sizeof(KeyType) * (uint64_t)numberOfInputs);
  h2d(inputKeyBuffer.data(), inputKeys.data(), sizeof(KeyType) * inputKeys.size());
  radixsort.sortKeys(inputKeyBuffer.data(), numberOfInputs, tmpBuffer.data(), 0, sizeof(KeyType) * 8, stream);
  sync();
  thrs::check(thrs_check_device_error(tmpBuffer.data(), stream));
  std::vector<KeyType> outputKeys(inputKeys.size());
  d2h(outputKeys.data(), inputKeyBuffer.data(), sizeof(KeyType) * (uint64_t)numberOfInputs);
  __gnu_parallel::sort(inputKeys.begin(), inputKeys.end());
  for (size_t i = 0; i < inputKeys.size(); i++) ASSERT_TRUE(inputKeys[i] == outputKeys[i]);
}

int main(int argc, char** argv) {
  std::string filter;
  bool list = false, large = false;
  // path / claim / rank choices for the whole matrix (thrs_options): the
  // tests run it with each non-default choice forced
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a.rfind("--filter=", 0) == 0) filter = a.substr(9);
    else if (a == "--list") list = true;
    else if (a == "--large") large = true;
    else if (a == "--path=lsd") g_opts.path = THRS_PATH_LSD;
    else if (a == "--path=bucket") g_opts.path = THRS_PATH_BUCKET;
    else if (a == "--claims=xcd") g_opts.tileClaims = THRS_CLAIMS_XCD_BLOCKS;
    else if (a == "--claims=ticket") g_opts.tileClaims = THRS_CLAIMS_TICKET;
    else if (a == "--rank=atomic") g_opts.rank = THRS_RANK_ATOMIC;
    else if (a == "--rank=ballot") g_opts.rank = THRS_RANK_BALLOT;
    else {
      std::printf("unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  if (list) {
    for (auto& c : cases()) std::printf("%s%s\n", c.name, c.large ? " (--large)" : "");
    return 0;
  }
  thrs::check(thrs_stream_create(&stream));
  int failed = 0, ran = 0;
  for (auto& c : cases()) {
    if (!filter.empty() && std::string(c.name).find(filter) == std::string::npos) continue;
    if (c.large && !large && filter != c.name) continue;
    g_failures_in_case = 0;
    auto t0 = std::chrono::steady_clock::now();
    try {
      c.fn();
    } catch (const std::exception& e) {
      std::printf("    exception: %s\n", e.what());
      g_failures_in_case++;
    }
    double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    ++ran;
    if (g_failures_in_case) ++failed;
    std::printf("[%s] %s (%.1f ms)\n", g_failures_in_case ? "FAILED" : "    OK", c.name, ms);
  }
  thrs_stream_destroy(stream);
  std::printf("%d/%d cases passed\n", ran - failed, ran);
  return failed;
}
