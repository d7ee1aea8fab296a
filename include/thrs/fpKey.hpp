// fpKey.hpp -- host-side order-preserving key transform, drop-in for the
// reference's fpKey.hpp (/root/reference/fpKey.hpp:15-38).
//
// Same overload set: getKeyBits(uint32_t / uint64_t / float / double).  Two
// deliberate fixes over the reference file:
//   * the reference defines NON-inline __float_as_int / __float_as_uint /
//     __double_as_longlong (:3-14), which breaks the ODR when included from
//     two translation units and collides with the HIP device builtins; here
//     the bit casts are memcpy-based and private;
//   * `x == 0.0f` (:25) is evaluated on the bits ((b & 0x7FFFFFFF) == 0), so a
//     build with flush-to-zero cannot fold denormals into zero.
// The resulting order is -NaN < -Inf < ... < -denorm < -0 == +0 < +denorm <
// ... < +Inf < +NaN, identical to libthrs's device transform (descending order
// additionally XORs all ones, which the device applies and this host helper,
// like the reference's, does not).
#pragma once

#include <stdint.h>
#include <string.h>

namespace thrs_fpkey_detail {
inline uint32_t bits_of(float x) { uint32_t b; memcpy(&b, &x, 4); return b; }
inline uint64_t bits_of(double x) { uint64_t b; memcpy(&b, &x, 8); return b; }
}  // namespace thrs_fpkey_detail

inline uint32_t getKeyBits(uint32_t x) { return x; }
inline uint64_t getKeyBits(uint64_t x) { return x; }
inline uint32_t getKeyBits(float x) {
  uint32_t b = thrs_fpkey_detail::bits_of(x);
  if ((b & 0x7FFFFFFFu) == 0) b = 0;  // -0 -> +0
  const uint32_t flip = (uint32_t)((int32_t)b >> 31) | 0x80000000u;
  return b ^ flip;
}
inline uint64_t getKeyBits(double x) {
  uint64_t b = thrs_fpkey_detail::bits_of(x);
  if ((b & 0x7FFFFFFFFFFFFFFFull) == 0) b = 0;
  const uint64_t flip = (uint64_t)((int64_t)b >> 63) | 0x8000000000000000ull;
  return b ^ flip;
}
