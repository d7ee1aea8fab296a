// Host-side check of the kernel-argument structs (thrs_kernels.hpp): a struct
// the launch sequence (thrs_host.hpp run_sort) declares and then fills field
// by field must not carry indeterminate bytes into a kernel -- the class of
// bug behind docs/EXPERIMENTS.md row 106 (uninitialised GroupTables next-pass
// pointers, an illegal address on the GPU).
//
// Each struct is default-initialised (`T x;`, no braces: only the default
// member initialisers run) over memory pre-filled with 0xAA and, separately,
// 0x55; the two objects must be byte-identical.  That holds only if every
// field has an initialiser AND the struct has no implicit padding (padding
// keeps the fill byte), so a field added later without one fails here.
// Compiled host-only by tests/test_capi_cpu.py; prints one line per struct.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <new>
#include <type_traits>

#include "thrs_kernels.hpp"

using namespace thrs_dev;

template <typename T>
static int check(const char* name) {
  static_assert(std::is_trivially_copyable<T>::value, "kernel arguments are copied bytewise");
  alignas(T) unsigned char a[sizeof(T)], b[sizeof(T)];
  std::memset(a, 0xAA, sizeof(T));
  std::memset(b, 0x55, sizeof(T));
  T* x = new (a) T;
  T* y = new (b) T;
  (void)x;
  (void)y;
  const bool noPad = std::has_unique_object_representations<T>::value;
  const bool same = std::memcmp(a, b, sizeof(T)) == 0;
  std::printf("%-28s %3zu B  no padding: %s  determinate: %s\n", name, sizeof(T), noPad ? "yes" : "NO",
              same ? "yes" : "NO");
  return noPad && same ? 0 : 1;
}

int main() {
  int bad = 0;
  bad += check<KeyMap<uint32_t>>("KeyMap<u32>");
  bad += check<KeyMap<uint64_t>>("KeyMap<u64>");
  bad += check<KeyMap<uint32_t, true>>("KeyMap<u32, squeeze>");
  bad += check<KeyMap<uint64_t, true>>("KeyMap<u64, squeeze>");
  bad += check<SqueezeWords>("SqueezeWords");
  bad += check<HistTargets>("HistTargets");
  bad += check<GroupTables<uint32_t>>("GroupTables<u32>");
  bad += check<GroupTables<uint64_t>>("GroupTables<u64>");
  bad += check<ZeroRanges>("ZeroRanges");
  std::printf(bad ? "FAILED: %d struct(s)\n" : "all kernel-argument structs determinate\n", bad);
  return bad ? 1 : 0;
}
