// ref_runner.cpp -- liboracle_refk.so: runs the REFERENCE's own kernels
// (kernel.cu, compiled by rtc_build with hipRTC into oracle/_ref/*.co) with the
// reference's launch sequence.  TEST INFRASTRUCTURE AND BASELINE ONLY: the GPU
// parity tests compare libthrs against it bit for bit, and bench.py can time it
// as the reference's own MI355X speed.  Nothing in the product path loads it.
//
// The reference's host code (tinyhipradixsort.hpp) needs Orochi, which is not
// vendored, so the pass loop is restated here, launch for launch:
//   TemporaryBufferDef           tinyhipradixsort.hpp:833-843
//   RadixSort::sort pass loop    tinyhipradixsort.hpp:854-944
//     blockCount                 grid nb, block 256                  :870-879
//     prefixSumExclusiveInplace  grid ceil(256*nb / 16384), block 512 :881-894
//     reorderKey / reorderKeyPair grid nb, block 256                 :897-928
//     ping-pong, odd-pass copy-back                                  :932-943
// Kernel arguments are passed in the ShaderArgument order of those launches.
// The one difference: the copy-back is stream-ordered (the reference's
// oroMemcpyDtoD is synchronous); the result after a synchronisation is the same.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <fstream>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

namespace {

constexpr uint32_t kBlockSize = 2048;     // RADIX_SORT_BLOCK_SIZE (kernel.cu:6)
constexpr uint32_t kScanBlock = 16384;    // RADIX_SORT_PREFIX_SCAN_BLOCK (kernel.cu:7)

struct Module {
  hipModule_t mod = nullptr;
  hipFunction_t count = nullptr, scan = nullptr, reorderKey = nullptr, reorderKeyPair = nullptr;
};

std::mutex g_mu;
std::map<std::tuple<int, int, int, int, int>, Module> g_mods;  // (device, key, value, desc, aligned)

std::string self_dir() {
  Dl_info info;
  if (dladdr(reinterpret_cast<void*>(&self_dir), &info) && info.dli_fname) {
    std::string p = info.dli_fname;
    const size_t s = p.rfind('/');
    if (s != std::string::npos) return p.substr(0, s);
  }
  return ".";
}

int get_module(int kt, int vt, int desc, int al, Module** out) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -3;
  std::lock_guard<std::mutex> g(g_mu);
  auto key = std::make_tuple(dev, kt, vt, desc, al);
  auto it = g_mods.find(key);
  if (it != g_mods.end()) {
    *out = &it->second;
    return 0;
  }
  char name[64];
  std::snprintf(name, sizeof(name), "/refk_k%d_v%d_d%d_a%d.co", kt, vt, desc, al);
  std::ifstream f(self_dir() + name, std::ios::binary);
  std::vector<char> code((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (code.empty()) return -4;
  Module m;
  if (hipModuleLoadData(&m.mod, code.data()) != hipSuccess) return -3;
  if (hipModuleGetFunction(&m.count, m.mod, "blockCount") != hipSuccess ||
      hipModuleGetFunction(&m.scan, m.mod, "prefixSumExclusiveInplace") != hipSuccess ||
      hipModuleGetFunction(&m.reorderKey, m.mod, "reorderKey") != hipSuccess ||
      hipModuleGetFunction(&m.reorderKeyPair, m.mod, "reorderKeyPair") != hipSuccess)
    return -3;
  *out = &(g_mods[key] = m);
  return 0;
}

uint64_t key_bytes(int kt) { return (kt == 0 || kt == 2) ? 4 : 8; }
uint64_t value_bytes(int vt) { return vt == 0 ? 4 : vt == 1 ? 8 : 16; }
uint64_t next_multiple(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

}  // namespace

extern "C" {

// TemporaryBufferDef (tinyhipradixsort.hpp:833-843): out = {pSum, keyOut, valueOut}
__attribute__((visibility("default"))) int refk_temp_bytes(int keyType, int valueType, uint32_t n, uint64_t* out) {
  const uint64_t nb = (n + (uint64_t)kBlockSize - 1) / kBlockSize;
  out[0] = next_multiple(4ull * 256 * nb, 16);
  out[1] = next_multiple(key_bytes(keyType) * n, 16);
  out[2] = next_multiple(value_bytes(valueType) * n, 16);
  return 0;
}

// RadixSort::sortKeys / sortPairs with the reference's kernels.
// keyType/valueType as thrs::KeyType / ValueType; values == NULL: sortKeys.
// Returns 0, -1 bad argument, -3 HIP error, -4 code object missing.
__attribute__((visibility("default"))) int refk_sort(int keyType, int valueType, int descending, int aligned16,
                                                      void* keys, void* values, uint32_t n, void* tmp, int startBits,
                                                      int endBits, hipStream_t stream) {
  if (keyType < 0 || keyType > 3 || valueType < 0 || valueType > 2) return -1;
  if (((endBits - startBits) % 8) != 0) return -1;  // THRS_ASSERT (tinyhipradixsort.hpp:856)
  if (n == 0) return 0;                             // the reference would launch an empty grid
  Module* m = nullptr;
  const int rc = get_module(keyType, valueType, descending ? 1 : 0, aligned16 ? 1 : 0, &m);
  if (rc) return rc;
  uint64_t def[3];
  refk_temp_bytes(keyType, valueType, n, def);
  void* pSum = tmp;
  void* keyOut = static_cast<char*>(tmp) + def[0];
  void* valueOut = static_cast<char*>(tmp) + def[0] + def[1];
  const bool pair = values != nullptr;
  uint32_t numberOfBlocks = (uint32_t)((n + (uint64_t)kBlockSize - 1) / kBlockSize);
  int iteration = 0;
  void* inK = keys;
  void* inV = values;
  for (int i = 0; startBits + i * 8 < endBits; ++i) {
    uint32_t bitLocation = (uint32_t)(startBits + i * 8);
    {
      void* args[] = {&inK, &n, &pSum, &bitLocation};
      if (hipModuleLaunchKernel(m->count, numberOfBlocks, 1, 1, 256, 1, 1, 0, stream, args, nullptr) != hipSuccess)
        return -3;
    }
    {
      uint32_t counters = numberOfBlocks * 256;
      void* args[] = {&pSum, &counters};
      const uint32_t grid = (uint32_t)((counters + (uint64_t)kScanBlock - 1) / kScanBlock);
      if (hipModuleLaunchKernel(m->scan, grid, 1, 1, 512, 1, 1, 0, stream, args, nullptr) != hipSuccess) return -3;
    }
    if (pair) {
      void* args[] = {&inK, &keyOut, &inV, &valueOut, &n, &pSum, &bitLocation};
      if (hipModuleLaunchKernel(m->reorderKeyPair, numberOfBlocks, 1, 1, 256, 1, 1, 0, stream, args, nullptr) !=
          hipSuccess)
        return -3;
    } else {
      void* args[] = {&inK, &keyOut, &n, &pSum, &bitLocation};
      if (hipModuleLaunchKernel(m->reorderKey, numberOfBlocks, 1, 1, 256, 1, 1, 0, stream, args, nullptr) !=
          hipSuccess)
        return -3;
    }
    ++iteration;
    std::swap(inK, keyOut);
    std::swap(inV, valueOut);
  }
  if (iteration % 2 == 1) {
    if (hipMemcpyAsync(keyOut, inK, key_bytes(keyType) * n, hipMemcpyDeviceToDevice, stream) != hipSuccess) return -3;
    if (pair && hipMemcpyAsync(valueOut, inV, value_bytes(valueType) * n, hipMemcpyDeviceToDevice, stream) != hipSuccess)
      return -3;
  }
  return 0;
}

}  // extern "C"
