// vis_probe.hip -- how long until a status word written by one workgroup is
// seen by another, per store/load cache-policy flavour, same XCD vs other XCD.
// Experiment support for the look-back design, not product code.
//
// Each workgroup (one wave does the work) registers in arrival order
// (global atomic), publishes flag[slot] = slot+1 with store flavour S, and then
// spins on the flag of a partner that arrived earlier (same XCD: the previous
// arrival on its own XCD; other XCD: the previous arrival on XCD+1 mod 8)
// with load flavour L.  It records the s_memrealtime ticks (100 MHz) between
// its own arrival and seeing the partner's flag, minus the partner's
// publication time -> visibility latency.  Bounded spins.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 7u;
}

template <int S>
__device__ __forceinline__ void st(uint32_t* p, uint32_t v) {
  if constexpr (S == 0) asm volatile("global_store_dword %0, %1, off" ::"v"(p), "v"(v) : "memory");
  if constexpr (S == 1) asm volatile("global_store_dword %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
  if constexpr (S == 2) asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  if constexpr (S == 3) asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  if constexpr (S == 4) asm volatile("global_store_dword %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
}
template <int L>
__device__ __forceinline__ uint32_t ld(const uint32_t* p) {
  uint32_t v;
  if constexpr (L == 0) asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  if constexpr (L == 1) asm volatile("global_load_dword %0, %1, off sc0\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  if constexpr (L == 2) asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  if constexpr (L == 3) asm volatile("global_load_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  if constexpr (L == 4)
    asm volatile("buffer_inv sc0\n\tglobal_load_dword %0, %1, off sc0\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  if constexpr (L == 5)
    asm volatile("buffer_inv sc1\n\tglobal_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}

struct Rec {
  uint32_t xcc, partner_xcc, seen, spins;
  uint64_t t_pub, t_seen;
};

// slots: [0..7] per-XCD arrival counters, [8] global arrival counter
template <int S, int L>
__global__ void probe(uint32_t* counters, uint32_t* perXcdSlot /*[8][cap]*/, uint32_t* flags, uint64_t* tpub,
                      Rec* rec, uint32_t cap, int cross) {
  if (threadIdx.x != 0) return;
  const uint32_t x = xcc_id();
  const uint32_t g = atomicAdd(&counters[8], 1u);
  const uint32_t k = atomicAdd(&counters[x], 1u);
  if (k < cap) __hip_atomic_store(&perXcdSlot[x * cap + k], g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  // busy work so the partner's store is in flight while we start looking
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  __hip_atomic_store(&tpub[g], t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  st<S>(&flags[g], g + 1);
  // partner: previous arrival on the same XCD (or on XCD x+1)
  const uint32_t px = cross ? (x + 1) & 7u : x;
  uint32_t pk = cross ? 0xFFFFFFFFu : (k ? k - 1 : 0xFFFFFFFFu);
  if (cross) {
    const uint32_t c = __hip_atomic_load(&counters[px], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    pk = (c && c - 1 < cap) ? c - 1 : 0xFFFFFFFFu;
  }
  Rec r{x, px, 0, 0, 0, 0};
  if (pk != 0xFFFFFFFFu && pk < cap) {
    uint32_t pg = 0;
    for (int i = 0; i < 100000 && !pg; ++i)
      pg = __hip_atomic_load(&perXcdSlot[px * cap + pk], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (pg) {
      pg -= 1;
      uint32_t spins = 0, v = 0;
      while (spins < 200000) {
        v = ld<L>(&flags[pg]);
        if (v == pg + 1) break;
        ++spins;
      }
      r.seen = v == pg + 1;
      r.spins = spins;
      r.t_seen = __builtin_amdgcn_s_memrealtime();
      r.t_pub = __hip_atomic_load(&tpub[pg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  rec[g] = r;
}

// background HBM load: a streaming copy on a second stream
__global__ void stream_copy(const uint4* a, uint4* b, size_t n, int reps) {
  for (int r = 0; r < reps; ++r)
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
      b[i] = a[i];
}

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

template <int S, int L>
void run(const char* name, int cross, bool load, uint32_t* counters, uint32_t* slots, uint32_t* flags, uint64_t* tpub,
         Rec* rec, uint32_t nwg, uint32_t cap, hipStream_t s, hipStream_t bg, const uint4* a, uint4* b, size_t nn) {
  CK(hipMemsetAsync(counters, 0, 64, s));
  CK(hipMemsetAsync(slots, 0, 8ull * cap * 4, s));
  CK(hipMemsetAsync(flags, 0, nwg * 4ull, s));
  CK(hipStreamSynchronize(s));
  if (load) hipLaunchKernelGGL(stream_copy, dim3(1024), dim3(256), 0, bg, a, b, nn, 4);
  hipLaunchKernelGGL((probe<S, L>), dim3(nwg), dim3(64), 0, s, counters, slots, flags, tpub, rec, cap, cross);
  CK(hipStreamSynchronize(s));
  CK(hipStreamSynchronize(bg));
  std::vector<Rec> h(nwg);
  CK(hipMemcpy(h.data(), rec, nwg * sizeof(Rec), hipMemcpyDeviceToHost));
  std::vector<double> lat;
  int unseen = 0, sameX = 0;
  for (auto& r : h) {
    if (!r.t_pub) continue;
    if (!r.seen) { ++unseen; continue; }
    sameX += r.xcc == r.partner_xcc;
    lat.push_back(r.t_seen > r.t_pub ? (r.t_seen - r.t_pub) * 10.0 : 0.0);  // ns
  }
  std::sort(lat.begin(), lat.end());
  auto q = [&](double f) { return lat.empty() ? -1.0 : lat[(size_t)(f * (lat.size() - 1))]; };
  printf("{\"case\": \"%s\", \"cross\": %d, \"load\": %d, \"pairs\": %zu, \"unseen\": %d, \"p50_ns\": %.0f, "
         "\"p90_ns\": %.0f, \"p99_ns\": %.0f}\n",
         name, cross, (int)load, lat.size(), unseen, q(0.5), q(0.9), q(0.99));
  fflush(stdout);
}

int main() {
  const uint32_t nwg = 4096, cap = 4096;
  uint32_t *counters, *slots, *flags;
  uint64_t* tpub;
  Rec* rec;
  CK(hipMalloc(&counters, 64));
  CK(hipMalloc(&slots, 8ull * cap * 4));
  CK(hipMalloc(&flags, nwg * 4ull));
  CK(hipMalloc(&tpub, nwg * 8ull));
  CK(hipMalloc(&rec, nwg * sizeof(Rec)));
  const size_t nn = (1ull << 30) / 16;
  uint4 *a, *b;
  CK(hipMalloc(&a, nn * 16));
  CK(hipMalloc(&b, nn * 16));
  CK(hipMemset(a, 1, nn * 16));
  hipStream_t s, bg;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&bg, hipStreamNonBlocking));
  for (int load = 0; load < 2; ++load)
    for (int cross = 0; cross < 2; ++cross) {
#define R(S, L, nm) run<S, L>(nm, cross, load, counters, slots, flags, tpub, rec, nwg, cap, s, bg, a, b, nn)
      R(0, 2, "st_plain/ld_sc1");
      R(1, 2, "st_sc0/ld_sc1");
      R(2, 2, "st_sc1/ld_sc1");
      R(0, 1, "st_plain/ld_sc0");
      R(1, 1, "st_sc0/ld_sc0");
      R(2, 1, "st_sc1/ld_sc0");
      R(1, 4, "st_sc0/inv0+ld_sc0");
      R(0, 4, "st_plain/inv0+ld_sc0");
      R(2, 0, "st_sc1/ld_plain");
      R(3, 3, "st_sc0sc1/ld_sc0sc1");
      R(4, 2, "st_nt/ld_sc1");
      R(1, 5, "st_sc0/inv1+ld_plain");
#undef R
    }
  return 0;
}
