// tinyhipradixsort.hpp -- header-only drop-in for the reference's host API
// (/root/reference/tinyhipradixsort.hpp:44-948), MI355X-native underneath.
//
// Same namespace, class, enum, struct and method names and signatures as the
// reference:
//   thrs::KeyType / ValueType / SortOrder, bytesOf, div_round_up64,
//   next_multiple64                                 (reference :638-692)
//   thrs::Buffer                                    (reference :501-528)
//   thrs::RadixSort::Config, configureWithKey<K>, configureWithKeyPair<K,V>
//                                                   (reference :697-749)
//   thrs::RadixSort(extraArgs, config)              (reference :751-804)
//   TemporaryBufferDef / getTemporaryBufferBytes    (reference :806-843)
//   sortKeys / sortPairs                            (reference :845-852)
//
// Extensions (no reference counterpart): setOptions / options (explicit path
// and tuning choices, thrs_options; defaults = the library's choice), and
// THRS_CHECKED: defined before including this header, every sortKeys /
// sortPairs synchronises its stream and throws (aborts) on a device-side
// failure of that sort (thrs_check_device_error) -- without it the caller
// checks a sort with checkDeviceError(temporaryBuffer, stream) (thrs_capi.h,
// "Device-side failures"); a sort never fails because of an earlier one.
//
// What changed underneath: no Orochi and no hipRTC.  Every call goes through
// the C-ABI of libthrs.so (<thrs/thrs_capi.h>), whose kernels are compiled
// ahead of time for gfx950.  `extraArgs` (hipRTC flags in the reference) are
// accepted and ignored.  Errors the reference turned into __debugbreak()
// (THRS_ASSERT, :14-15) throw thrs::Error here (or abort() when
// THRS_NO_EXCEPTIONS is defined).  This header needs no HIP headers: link with
// -lthrs (and the HIP runtime it pulls in).
#pragma once

#include <stdint.h>

#include <algorithm>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#ifndef THRS_NO_EXCEPTIONS
#include <stdexcept>
#else
#include <cstdio>
#include <cstdlib>
#endif

#include "thrs_capi.h"

// On the HIP backend the reference's oroStream is the HIP stream handle.
#ifndef THRS_HAVE_OROCHI
typedef hipStream_t oroStream;
#endif

namespace thrs {

#ifndef THRS_NO_EXCEPTIONS
struct Error : std::runtime_error {
  int status;
  explicit Error(int s) : std::runtime_error(thrs_status_string(s)), status(s) {}
};
inline void check(int status) {
  if (status != THRS_SUCCESS) throw Error(status);
}
#else
inline void check(int status) {
  if (status != THRS_SUCCESS) {
    std::fprintf(stderr, "thrs: %s\n", thrs_status_string(status));
    std::abort();
  }
}
#endif

// -------------------------------------------------------------- enums
enum class KeyType { U32 = THRS_KEY_U32, U64 = THRS_KEY_U64, F32 = THRS_KEY_F32, F64 = THRS_KEY_F64 };
enum class ValueType { U32 = THRS_VALUE_U32, U64 = THRS_VALUE_U64, U128 = THRS_VALUE_U128 };
enum class SortOrder { Ascending = THRS_ORDER_ASCENDING, Descending = THRS_ORDER_DESCENDING };

inline uint64_t bytesOf(KeyType t) {
  const uint64_t b = thrs_key_bytes(static_cast<int>(t));
  if (!b) check(THRS_ERROR_INVALID_VALUE);
  return b;
}
inline uint64_t bytesOf(ValueType t) {
  const uint64_t b = thrs_value_bytes(static_cast<int>(t));
  if (!b) check(THRS_ERROR_INVALID_VALUE);
  return b;
}
inline uint64_t div_round_up64(uint64_t val, uint64_t divisor) { return (val + divisor - 1) / divisor; }
inline uint64_t next_multiple64(uint64_t val, uint64_t divisor) { return div_round_up64(val, divisor) * divisor; }

// -------------------------------------------------------------- Buffer
class Buffer {
 public:
  Buffer(const Buffer&) = delete;
  void operator=(const Buffer&) = delete;

  Buffer(int64_t bytes) : m_bytes(std::max<int64_t>(bytes, 1)) { check(thrs_malloc(&m_ptr, m_bytes)); }
  ~Buffer() { thrs_free(m_ptr); }
  int64_t bytes() const { return m_bytes; }
  char* data() { return static_cast<char*>(m_ptr); }

 private:
  int64_t m_bytes;
  void* m_ptr = nullptr;
};

// -------------------------------------------------------------- RadixSort
class RadixSort {
 public:
  struct Config {
    // strongly recommended (a hint here: alignment is re-checked per call)
    bool keyIs16byteAligned = true;

    KeyType keyType = KeyType::U32;
    ValueType valueType = ValueType::U32;

    SortOrder sortOrder = SortOrder::Ascending;

    template <class KEY>
    void configureWithKey() {
      static_assert(sizeof(KEY) == 4 || sizeof(KEY) == 8, "");
      if (std::is_same<KEY, float>::value) keyType = KeyType::F32;
      else if (std::is_same<KEY, double>::value) keyType = KeyType::F64;
      else if (sizeof(KEY) == 4) keyType = KeyType::U32;
      else keyType = KeyType::U64;
    }
    template <class KEY, class VALUE>
    void configureWithKeyPair() {
      configureWithKey<KEY>();
      static_assert(sizeof(VALUE) == 4 || sizeof(VALUE) == 8 || sizeof(VALUE) == 16, "");
      valueType = sizeof(VALUE) == 4 ? ValueType::U32 : sizeof(VALUE) == 8 ? ValueType::U64 : ValueType::U128;
    }
  };

  // (the reference's `const Config& config = Config()` default argument is
  // spelled as a delegating overload: GCC rejects the default argument for a
  // nested class with default member initialisers, PR c++/96645)
  RadixSort(std::vector<std::string> extraArgs) : RadixSort(std::move(extraArgs), Config{}) {}
  RadixSort(std::vector<std::string> extraArgs, const Config& config) : m_config(config) {
    (void)extraArgs;  // hipRTC options in the reference; kernels are AOT-compiled here
    check(thrs_abi_version() == THRS_ABI_VERSION ? THRS_SUCCESS : THRS_ERROR_INVALID_VALUE);
  }

  struct TemporaryBufferDef {
    uint64_t pSumBuffer;
    uint64_t keyOutBuffer;
    uint64_t valueOutBuffer;

    uint64_t getTemporaryBufferBytesForSortKeys() const { return pSumBuffer + keyOutBuffer; }
    uint64_t getTemporaryBufferBytesForSortPairs() const { return pSumBuffer + keyOutBuffer + valueOutBuffer; }
    void* getPSumBuffer(void* p) const { return p; }
    void* getOutputKeyBuffer(void* p) const { return (void*)((uint8_t*)p + pSumBuffer); }
    void* getOutputValueBuffer(void* p) const { return (void*)((uint8_t*)p + pSumBuffer + keyOutBuffer); }
  };

  TemporaryBufferDef getTemporaryBufferBytes(uint32_t numberOfMaxInputs) const {
    const thrs_config c = cconfig();
    thrs_temp_def d{};
    check(thrs_get_temporary_buffer_bytes(&c, numberOfMaxInputs, &d));
    return TemporaryBufferDef{d.pSumBuffer, d.keyOutBuffer, d.valueOutBuffer};
  }

  void sortKeys(void* inputKeyBuffer, uint32_t numberOfInputs, void* temporaryBuffer, int startBits, int endBits,
                oroStream stream) {
    const thrs_config c = cconfig();
    check(thrs_sort_keys_ex(&c, &m_options, inputKeyBuffer, numberOfInputs, temporaryBuffer, startBits, endBits,
                            reinterpret_cast<hipStream_t>(stream)));
    checked(temporaryBuffer, stream);
  }
  void sortPairs(void* inputKeyBuffer, void* inputValueBuffer, uint32_t numberOfInputs, void* temporaryBuffer,
                 int startBits, int endBits, oroStream stream) {
    const thrs_config c = cconfig();
    check(thrs_sort_pairs_ex(&c, &m_options, inputKeyBuffer, inputValueBuffer, numberOfInputs, temporaryBuffer,
                             startBits, endBits, reinterpret_cast<hipStream_t>(stream)));
    checked(temporaryBuffer, stream);
  }

  const Config& config() const { return m_config; }

  // extension: explicit path / tuning choices (thrs_capi.h thrs_options)
  void setOptions(const thrs_options& options) { m_options = options; }
  const thrs_options& options() const { return m_options; }

 private:
  thrs_config cconfig() const {
    return thrs_config{m_config.keyIs16byteAligned ? 1 : 0, static_cast<int32_t>(m_config.keyType),
                       static_cast<int32_t>(m_config.valueType), static_cast<int32_t>(m_config.sortOrder)};
  }
  static void checked(void* temporaryBuffer, oroStream stream) {
#ifdef THRS_CHECKED
    check(thrs_check_device_error(temporaryBuffer, reinterpret_cast<hipStream_t>(stream)));
#else
    (void)temporaryBuffer;
    (void)stream;
#endif
  }
  Config m_config;
  thrs_options m_options{};
};

}  // namespace thrs
