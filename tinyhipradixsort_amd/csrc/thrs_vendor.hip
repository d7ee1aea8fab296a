// thrs_vendor.hip -- libthrs_vendor.so: hipCUB/rocPRIM DeviceRadixSort on the
// same inputs, as the vendor comparator for benchmarks (the MI355X analogue of
// the reference's CUB baseline, cudaEnv.cu:95-116).  Benchmark-only; never
// used by the sort path.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#define THRS_API __attribute__((visibility("default")))

extern "C" {

// keys/values ping-pong between a and b; *selector tells where the result is.
THRS_API int thrsv_temp_bytes(int keyBytes, int valueBytes, uint32_t n, uint64_t* bytes) {
  size_t t = 0;
  hipcub::DoubleBuffer<uint32_t> k32(nullptr, nullptr);
  hipcub::DoubleBuffer<uint64_t> k64(nullptr, nullptr);
  hipcub::DoubleBuffer<uint32_t> v32(nullptr, nullptr);
  hipcub::DoubleBuffer<uint64_t> v64(nullptr, nullptr);
  hipError_t e;
  if (keyBytes == 4 && valueBytes == 0) e = hipcub::DeviceRadixSort::SortKeys(nullptr, t, k32, n);
  else if (keyBytes == 8 && valueBytes == 0) e = hipcub::DeviceRadixSort::SortKeys(nullptr, t, k64, n);
  else if (keyBytes == 4 && valueBytes == 4) e = hipcub::DeviceRadixSort::SortPairs(nullptr, t, k32, v32, n);
  else if (keyBytes == 8 && valueBytes == 8) e = hipcub::DeviceRadixSort::SortPairs(nullptr, t, k64, v64, n);
  else return -1;
  *bytes = t;
  return e == hipSuccess ? 0 : -3;
}

THRS_API int thrsv_sort(int keyBytes, int valueBytes, void* ka, void* kb, void* va, void* vb, uint32_t n, void* tmp,
                        uint64_t tmpBytes, int* selector, hipStream_t stream) {
  size_t t = tmpBytes;
  hipError_t e;
  if (keyBytes == 4 && valueBytes == 0) {
    hipcub::DoubleBuffer<uint32_t> k((uint32_t*)ka, (uint32_t*)kb);
    e = hipcub::DeviceRadixSort::SortKeys(tmp, t, k, n, 0, 32, stream);
    *selector = k.selector;
  } else if (keyBytes == 8 && valueBytes == 0) {
    hipcub::DoubleBuffer<uint64_t> k((uint64_t*)ka, (uint64_t*)kb);
    e = hipcub::DeviceRadixSort::SortKeys(tmp, t, k, n, 0, 64, stream);
    *selector = k.selector;
  } else if (keyBytes == 4 && valueBytes == 4) {
    hipcub::DoubleBuffer<uint32_t> k((uint32_t*)ka, (uint32_t*)kb);
    hipcub::DoubleBuffer<uint32_t> v((uint32_t*)va, (uint32_t*)vb);
    e = hipcub::DeviceRadixSort::SortPairs(tmp, t, k, v, n, 0, 32, stream);
    *selector = k.selector;
  } else if (keyBytes == 8 && valueBytes == 8) {
    hipcub::DoubleBuffer<uint64_t> k((uint64_t*)ka, (uint64_t*)kb);
    hipcub::DoubleBuffer<uint64_t> v((uint64_t*)va, (uint64_t*)vb);
    e = hipcub::DeviceRadixSort::SortPairs(tmp, t, k, v, n, 0, 64, stream);
    *selector = k.selector;
  } else {
    return -1;
  }
  return e == hipSuccess ? 0 : -3;
}

}  // extern "C"
