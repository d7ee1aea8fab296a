// thrs_vendor.hip -- libthrs_vendor.so: hipCUB/rocPRIM DeviceRadixSort on the
// same inputs, as the vendor comparator for benchmarks (the MI355X analogue of
// the reference's CUB baseline, cudaEnv.cu:95-116).  Benchmark-only; never
// used by the sort path.  Keys are sorted as their own type (f32 / f64 keys
// as floats: rocPRIM's float order is the reference's getKeyBits order), values
// are 4-, 8- or 16-byte payloads.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#define THRS_API __attribute__((visibility("default")))

namespace {

struct V16 {
  uint64_t lo, hi;
};

// keys/values ping-pong between a and b; *selector tells where the result is.
template <typename K, typename V>
hipError_t run(void* tmp, size_t& t, void* ka, void* kb, void* va, void* vb, uint32_t n, int* selector,
               hipStream_t stream) {
  hipcub::DoubleBuffer<K> k(static_cast<K*>(ka), static_cast<K*>(kb));
  hipError_t e;
  if constexpr (std::is_void<V>::value) {
    e = hipcub::DeviceRadixSort::SortKeys(tmp, t, k, n, 0, 8 * (int)sizeof(K), stream);
  } else {
    hipcub::DoubleBuffer<V> v(static_cast<V*>(va), static_cast<V*>(vb));
    e = hipcub::DeviceRadixSort::SortPairs(tmp, t, k, v, n, 0, 8 * (int)sizeof(K), stream);
  }
  if (selector) *selector = k.selector;
  return e;
}

template <typename K>
hipError_t by_value(int valueBytes, void* tmp, size_t& t, void* ka, void* kb, void* va, void* vb, uint32_t n,
                    int* selector, hipStream_t stream, bool* ok) {
  *ok = true;
  switch (valueBytes) {
    case 0: return run<K, void>(tmp, t, ka, kb, va, vb, n, selector, stream);
    case 4: return run<K, uint32_t>(tmp, t, ka, kb, va, vb, n, selector, stream);
    case 8: return run<K, uint64_t>(tmp, t, ka, kb, va, vb, n, selector, stream);
    case 16: return run<K, V16>(tmp, t, ka, kb, va, vb, n, selector, stream);
  }
  *ok = false;
  return hipErrorInvalidValue;
}

// keyType: 0 u32, 1 u64, 2 f32, 3 f64 (thrs_capi.h THRS_KEY_*)
hipError_t dispatch(int keyType, int valueBytes, void* tmp, size_t& t, void* ka, void* kb, void* va, void* vb,
                    uint32_t n, int* selector, hipStream_t stream, bool* ok) {
  switch (keyType) {
    case 0: return by_value<uint32_t>(valueBytes, tmp, t, ka, kb, va, vb, n, selector, stream, ok);
    case 1: return by_value<uint64_t>(valueBytes, tmp, t, ka, kb, va, vb, n, selector, stream, ok);
    case 2: return by_value<float>(valueBytes, tmp, t, ka, kb, va, vb, n, selector, stream, ok);
    case 3: return by_value<double>(valueBytes, tmp, t, ka, kb, va, vb, n, selector, stream, ok);
  }
  *ok = false;
  return hipErrorInvalidValue;
}

}  // namespace

extern "C" {

THRS_API int thrsv_temp_bytes(int keyType, int valueBytes, uint32_t n, uint64_t* bytes) {
  size_t t = 0;
  bool ok = false;
  const hipError_t e = dispatch(keyType, valueBytes, nullptr, t, nullptr, nullptr, nullptr, nullptr, n, nullptr,
                                nullptr, &ok);
  if (!ok) return -1;
  *bytes = t;
  return e == hipSuccess ? 0 : -3;
}

THRS_API int thrsv_sort(int keyType, int valueBytes, void* ka, void* kb, void* va, void* vb, uint32_t n, void* tmp,
                        uint64_t tmpBytes, int* selector, hipStream_t stream) {
  size_t t = tmpBytes;
  bool ok = false;
  const hipError_t e = dispatch(keyType, valueBytes, tmp, t, ka, kb, va, vb, n, selector, stream, &ok);
  if (!ok) return -1;
  return e == hipSuccess ? 0 : -3;
}

}  // extern "C"
