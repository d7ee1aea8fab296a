// Infinity Cache reuse probe: does a produce -> consume hand-off of G MB
// groups (kernel 1 writes tmp[g], kernel 2 reads tmp[g] and writes it back in
// place / to dst[g]) cost less HBM time than the same two kernels over the
// whole 4 GiB?  (MI355X_MICROARCH.md "Infinity Cache": 256 MiB die-level.)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int UN>
__global__ void k_copy(v4u* __restrict__ d, const v4u* __restrict__ s, uint64_t n) {
  const uint64_t per = (uint64_t)UN * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * per; base < n; base += (uint64_t)gridDim.x * per) {
    v4u q[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) q[u] = s[base + (uint64_t)u * blockDim.x + threadIdx.x];
#pragma unroll
    for (int u = 0; u < UN; ++u) d[base + (uint64_t)u * blockDim.x + threadIdx.x] = q[u] ^ 1u;
  }
}

int main() {
  const uint64_t bytes = 4ull << 30, n = bytes / 16;
  v4u *s, *t, *d;
  CK(hipMalloc(&s, bytes)); CK(hipMalloc(&t, bytes)); CK(hipMalloc(&d, bytes));
  CK(hipMemset(s, 1, bytes)); CK(hipMemset(t, 0, bytes)); CK(hipMemset(d, 0, bytes));
  hipStream_t st[2];
  CK(hipStreamCreateWithFlags(&st[0], hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&st[1], hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(4096);
  for (auto& evx : ev) CK(hipEventCreateWithFlags(&evx, hipEventDisableTiming));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto grid = [](uint64_t m) { return (unsigned)std::max<uint64_t>(1, m / 1024); };
  auto run = [&](const char* name, auto launch) {
    std::vector<float> ms;
    for (int r = 0; r < 7; ++r) {
      CK(hipDeviceSynchronize());
      (void)hipEventRecord(a, st[0]); launch();
      (void)hipEventRecord(ev[4095], st[1]); (void)hipStreamWaitEvent(st[0], ev[4095], 0);
      (void)hipEventRecord(b, st[0]); (void)hipEventSynchronize(b);
      float x; (void)hipEventElapsedTime(&x, a, b); ms.push_back(x);
    }
    std::sort(ms.begin(), ms.end());
    printf("%-40s %8.3f ms  (16 GiB moved: %5.2f TB/s equiv)\n", name, ms[3], 4.0 * bytes / (ms[3] * 1e-3) / 1e12);
    return 0;
  };
  run("whole: copy s->t, then t->t in place", [&] {
    k_copy<4><<<grid(n), 256, 0, st[0]>>>(t, s, n);
    k_copy<4><<<grid(n), 256, 0, st[0]>>>(t, t, n);
  });
  run("whole: copy s->t, then t->d", [&] {
    k_copy<4><<<grid(n), 256, 0, st[0]>>>(t, s, n);
    k_copy<4><<<grid(n), 256, 0, st[0]>>>(d, t, n);
  });
  for (uint64_t gmb : {8ull, 16ull, 32ull, 64ull, 128ull, 256ull}) {
    const uint64_t gn = (gmb << 20) / 16, groups = n / gn;
    char nm[96];
    snprintf(nm, 96, "groups %3llu MB, 1 stream, in place", (unsigned long long)gmb);
    run(nm, [&] {
      for (uint64_t g = 0; g < groups; ++g) {
        k_copy<4><<<grid(gn), 256, 0, st[0]>>>(t + g * gn, s + g * gn, gn);
        k_copy<4><<<grid(gn), 256, 0, st[0]>>>(t + g * gn, t + g * gn, gn);
      }
    });
    snprintf(nm, 96, "groups %3llu MB, 1 stream, t->d", (unsigned long long)gmb);
    run(nm, [&] {
      for (uint64_t g = 0; g < groups; ++g) {
        k_copy<4><<<grid(gn), 256, 0, st[0]>>>(t + g * gn, s + g * gn, gn);
        k_copy<4><<<grid(gn), 256, 0, st[0]>>>(d + g * gn, t + g * gn, gn);
      }
    });
    snprintf(nm, 96, "groups %3llu MB, 2 streams, in place", (unsigned long long)gmb);
    run(nm, [&] {
      for (uint64_t g = 0; g < groups; ++g) {
        k_copy<4><<<grid(gn), 256, 0, st[0]>>>(t + g * gn, s + g * gn, gn);
        (void)hipEventRecord(ev[g], st[0]);
        (void)hipStreamWaitEvent(st[1], ev[g], 0);
        k_copy<4><<<grid(gn), 256, 0, st[1]>>>(t + g * gn, t + g * gn, gn);
      }
    });
  }
  // launch cost alone: the same group counts on 1 MB
  for (uint64_t groups : {64ull, 256ull}) {
    char nm[96];
    snprintf(nm, 96, "launch floor: %llu x2 tiny kernels", (unsigned long long)groups);
    const uint64_t gn = (1ull << 20) / 16;
    run(nm, [&] {
      for (uint64_t g = 0; g < groups; ++g) {
        k_copy<4><<<grid(gn), 256, 0, st[0]>>>(t, s, gn);
        k_copy<4><<<grid(gn), 256, 0, st[0]>>>(t, t, gn);
      }
    });
  }
  CK(hipDeviceSynchronize());
  return 0;
}
