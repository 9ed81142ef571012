// Copy-ceiling probe #2 (diagnostic): loads in flight per lane, workgroup size,
// grid size, store/load cache policy.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, int T>
__global__ __launch_bounds__(T) void copy_k(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  const size_t stride = size_t(gridDim.x) * T;
  size_t i = size_t(blockIdx.x) * T + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = a[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) b[i + u * stride] = v[u];
  }
  for (; i < n; i += stride) b[i] = a[i];
}
template <int U, int T>
__global__ __launch_bounds__(T) void copy_ntl(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
  const size_t stride = size_t(gridDim.x) * T;
  size_t i = size_t(blockIdx.x) * T + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(a + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) b[i + u * stride] = v[u];
  }
}
// contiguous chunk per workgroup (each WG copies CH bytes, lanes interleaved)
template <int U, int T>
__global__ __launch_bounds__(T) void copy_chunk(const uint4* __restrict__ a, uint4* __restrict__ b, size_t per) {
  const size_t base = size_t(blockIdx.x) * per;
  for (size_t j = threadIdx.x; j < per; j += U * T) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) if (j + u * T < per) v[u] = a[base + j + u * T];
#pragma unroll
    for (int u = 0; u < U; ++u) if (j + u * T < per) b[base + j + u * T] = v[u];
  }
}

int main() {
  const size_t bytes = size_t(4) << 30, n = bytes / 16;
  uint4 *a, *b;
  hipMalloc(&a, bytes);
  hipMalloc(&b, bytes);
  hipMemset(a, 1, bytes);
  hipMemset(b, 0, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, auto launch) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("%-34s %8.3f ms  %8.1f GB/s\n", name, ms, 2.0 * bytes / ms / 1e6);
  };
  char nm[80];
#define RUNK(U, T, G)                                                          \
  snprintf(nm, 80, "copy U=%d T=%d grid=%d", U, T, G);                        \
  run(nm, [&] { copy_k<U, T><<<G, T>>>(a, b, n); });
  RUNK(1, 256, 1024) RUNK(2, 256, 1024) RUNK(4, 256, 1024) RUNK(8, 256, 1024)
  RUNK(4, 256, 512) RUNK(8, 256, 512) RUNK(8, 256, 256) RUNK(16, 256, 256)
  RUNK(4, 512, 512) RUNK(8, 512, 256) RUNK(4, 1024, 256) RUNK(8, 1024, 256)
  RUNK(2, 256, 2048) RUNK(4, 256, 2048)
#define RUNN(U, T, G)                                                          \
  snprintf(nm, 80, "copy_ntload U=%d T=%d grid=%d", U, T, G);                 \
  run(nm, [&] { copy_ntl<U, T><<<G, T>>>((const u32x4*)a, (u32x4*)b, n); });
  RUNN(4, 256, 1024) RUNN(8, 256, 512)
#define RUNC(U, T, KB)                                                         \
  snprintf(nm, 80, "copy_chunk U=%d T=%d %dKiB/WG", U, T, KB);                \
  run(nm, [&] { copy_chunk<U, T><<<bytes / (KB * 1024), T>>>(a, b, KB * 64); });
  RUNC(4, 256, 64) RUNC(8, 256, 64) RUNC(4, 256, 256) RUNC(8, 512, 256) RUNC(4, 256, 1024)
  run("hipMemcpyDtoD", [&] { hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0); });
  return 0;
}
