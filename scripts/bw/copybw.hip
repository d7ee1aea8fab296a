// HBM copy-rate probe: what access pattern reaches the guide's ~6.3 TB/s
// (MI355X_MICROARCH.md "HBM") on this box.  4 GiB -> 4 GiB, hipEvent timing.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_gs1(v4u* __restrict__ d, const v4u* __restrict__ s, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) d[i] = s[i];
}
// block-contiguous tiles of UN*blockDim v4u, UN loads in flight per lane; NT: nontemporal stores/loads
template <int UN, int NTS, int NTL>
__global__ void k_tile(v4u* __restrict__ d, const v4u* __restrict__ s, uint64_t n) {
  const uint64_t per = (uint64_t)UN * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * per; base < n; base += (uint64_t)gridDim.x * per) {
    v4u q[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const uint64_t i = base + (uint64_t)u * blockDim.x + threadIdx.x;
      if (NTL) q[u] = __builtin_nontemporal_load(s + i); else q[u] = s[i];
    }
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const uint64_t i = base + (uint64_t)u * blockDim.x + threadIdx.x;
      if (NTS) __builtin_nontemporal_store(q[u], d + i); else d[i] = q[u];
    }
  }
}
template <int UN>
__global__ void k_read(const v4u* __restrict__ s, uint64_t n, uint32_t* out) {
  const uint64_t per = (uint64_t)UN * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t base = (uint64_t)blockIdx.x * per; base < n; base += (uint64_t)gridDim.x * per) {
    v4u q[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) q[u] = s[base + (uint64_t)u * blockDim.x + threadIdx.x];
#pragma unroll
    for (int u = 0; u < UN; ++u) acc ^= q[u].x ^ q[u].y ^ q[u].z ^ q[u].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
template <int UN, int NTS>
__global__ void k_write(v4u* __restrict__ d, uint64_t n) {
  const uint64_t per = (uint64_t)UN * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * per; base < n; base += (uint64_t)gridDim.x * per) {
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const uint64_t i = base + (uint64_t)u * blockDim.x + threadIdx.x;
      const v4u v = v4u{(uint32_t)i, 1u, 2u, 3u};
      if (NTS) __builtin_nontemporal_store(v, d + i); else d[i] = v;
    }
  }
}

int main() {
  const uint64_t bytes = 4ull << 30, n = bytes / 16;
  v4u *s, *d; uint32_t* o;
  CK(hipMalloc(&s, bytes)); CK(hipMalloc(&d, bytes)); CK(hipMalloc(&o, 4));
  CK(hipMemset(s, 1, bytes)); CK(hipMemset(d, 0, bytes));
  int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto run = [&](const char* name, double moved, auto launch) {
    std::vector<float> ms;
    for (int r = 0; r < 7; ++r) {
      (void)hipEventRecord(a); launch(); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
      float t; (void)hipEventElapsedTime(&t, a, b); ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    printf("%-34s %8.3f ms  %6.2f TB/s\n", name, ms[3], moved / (ms[3] * 1e-3) / 1e12);
  };
  const double rw = 2.0 * bytes, r1 = bytes;
  run("gs1 4096x256", rw, [&] { k_gs1<<<4096, 256>>>(d, s, n); });
  for (int wpc : {1, 2, 4, 8}) {
    char nm[64];
    const int g = wpc * cus;
    snprintf(nm, 64, "tile4 1024t %d/CU", wpc);   run(nm, rw, [&] { k_tile<4, 0, 0><<<g, 1024>>>(d, s, n); });
    snprintf(nm, 64, "tile4 256t %d/CU", 4 * wpc); run(nm, rw, [&] { k_tile<4, 0, 0><<<4 * g, 256>>>(d, s, n); });
    snprintf(nm, 64, "tile8 256t %d/CU", 4 * wpc); run(nm, rw, [&] { k_tile<8, 0, 0><<<4 * g, 256>>>(d, s, n); });
    snprintf(nm, 64, "tile4 256t nts %d/CU", 4 * wpc); run(nm, rw, [&] { k_tile<4, 1, 0><<<4 * g, 256>>>(d, s, n); });
    snprintf(nm, 64, "tile4 256t ntl+nts %d/CU", 4 * wpc); run(nm, rw, [&] { k_tile<4, 1, 1><<<4 * g, 256>>>(d, s, n); });
  }
  run("tile4 256t big grid n/1024", rw, [&] { k_tile<4, 0, 0><<<(unsigned)(n / 1024), 256>>>(d, s, n); });
  run("tile4 256t nts big grid", rw, [&] { k_tile<4, 1, 0><<<(unsigned)(n / 1024), 256>>>(d, s, n); });
  run("read4 256t 16/CU", r1, [&] { k_read<4><<<16 * cus, 256>>>(s, n, o); });
  run("read8 256t 16/CU", r1, [&] { k_read<8><<<16 * cus, 256>>>(s, n, o); });
  run("write4 256t 16/CU", r1, [&] { k_write<4, 0><<<16 * cus, 256>>>(d, n); });
  run("write4 nts 256t 16/CU", r1, [&] { k_write<4, 1><<<16 * cus, 256>>>(d, n); });
  CK(hipDeviceSynchronize());
  return 0;
}
