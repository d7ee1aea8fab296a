// rtc_build.cpp -- compile the REFERENCE's device code (kernel.cu, read where
// it lies under /root/reference) with hipRTC for gfx950, once per
// configuration, with exactly the -D options RadixSort's constructor passes
// (tinyhipradixsort.hpp:751-791) and Shader's hipRTC sequence (:564-607).
// The reference JIT-compiles the same source at run time through Orochi
// (absent here); this writes the code objects ahead of time into
// oracle/_ref/ (never committed).  TEST INFRASTRUCTURE ONLY.
//
// usage: rtc_build <kernel.cu> <out dir>
#include <hip/hiprtc.h>

#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: %s <kernel.cu> <out dir>\n", argv[0]);
    return 2;
  }
  std::ifstream f(argv[1]);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string src = ss.str();
  if (src.empty()) {
    std::fprintf(stderr, "cannot read %s\n", argv[1]);
    return 1;
  }
  // KeyType / ValueType order of tinyhipradixsort.hpp:638-650 (== thrs_capi.h)
  const char* keyTypes[] = {"uint32_t", "uint64_t", "float", "double"};
  const char* valueTypes[] = {"uint32_t", "uint64_t", "uint4"};
  int built = 0;
  for (int k = 0; k < 4; ++k)
    for (int v = 0; v < 3; ++v)
      for (int desc = 0; desc < 2; ++desc)
        for (int al = 0; al < 2; ++al) {
          std::vector<std::string> opts = {"--gpu-architecture=gfx950",
                                           std::string("-DRADIX_SORT_KEY_TYPE=") + keyTypes[k],
                                           std::string("-DRADIX_SORT_VALUE_TYPE=") + valueTypes[v]};
          if (al) opts.push_back("-DKEY_IS_16BYTE_ALIGNED=1");
          if (desc) opts.push_back("-DDESCENDING_ORDER=1");
          std::vector<const char*> o;
          for (auto& s : opts) o.push_back(s.c_str());
          hiprtcProgram prog = nullptr;
          if (hiprtcCreateProgram(&prog, src.c_str(), "kernel.cu", 0, nullptr, nullptr) != HIPRTC_SUCCESS) return 1;
          const hiprtcResult rc = hiprtcCompileProgram(prog, (int)o.size(), o.data());
          size_t logSize = 0;
          hiprtcGetProgramLogSize(prog, &logSize);
          if (logSize > 1) {
            std::vector<char> log(logSize);
            hiprtcGetProgramLog(prog, log.data());
            std::fprintf(stderr, "%s", log.data());
          }
          if (rc != HIPRTC_SUCCESS) {
            std::fprintf(stderr, "hipRTC failed for key %s value %s desc %d aligned %d\n", keyTypes[k], valueTypes[v],
                         desc, al);
            return 1;
          }
          size_t size = 0;
          hiprtcGetCodeSize(prog, &size);
          std::vector<char> code(size);
          hiprtcGetCode(prog, code.data());
          hiprtcDestroyProgram(&prog);
          char name[512];
          std::snprintf(name, sizeof(name), "%s/refk_k%d_v%d_d%d_a%d.co", argv[2], k, v, desc, al);
          std::ofstream out(name, std::ios::binary);
          out.write(code.data(), (std::streamsize)code.size());
          ++built;
        }
  std::printf("rtc_build: %d code objects from %s\n", built, argv[1]);
  return 0;
}
