// fpkey_shim.cpp -- C-ABI over the REFERENCE's own host code, compiled from
// the reference sources where they lie (oracle/ref/Makefile; outputs only in
// oracle/_ref/, never committed).  TEST INFRASTRUCTURE ONLY: it pins the
// oracle (oracle/oracle.cpp) -- tests compare the two; nothing in the product
// path loads it.
//   getKeyBits(u32/u64/float/double)   /root/reference/fpKey.hpp:15-38, as-is
//   struct splitmix64                  /root/reference/unittest.cpp:24-35,
//                                      extracted verbatim by extract_splitmix64.py
#include <cstdint>

#include "fpKey.hpp"
#include "splitmix64_ref.inc"

extern "C" {

void ref_key_bits_u32(const uint32_t* in, uint32_t* out, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) out[i] = getKeyBits(in[i]);
}
void ref_key_bits_u64(const uint64_t* in, uint64_t* out, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) out[i] = getKeyBits(in[i]);
}
void ref_key_bits_f32(const float* in, uint32_t* out, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) out[i] = getKeyBits(in[i]);
}
void ref_key_bits_f64(const double* in, uint64_t* out, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) out[i] = getKeyBits(in[i]);
}

// n draws of the reference's splitmix64 from state *x (advanced)
void ref_splitmix64_fill(uint64_t* x, uint64_t* out, uint64_t n) {
  splitmix64 rng;
  rng.x = *x;
  for (uint64_t i = 0; i < n; ++i) out[i] = rng.next();
  *x = rng.x;
}

}  // extern "C"
