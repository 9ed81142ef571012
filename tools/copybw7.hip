// Copy-ceiling probe #7 (diagnostic, not product): can a decode pass keep the
// one-shot copy's rate (4 KiB per workgroup, dispatch order = address order)
// when every workgroup also needs per-tile metadata that costs dependent trips?
//   reg : data loaded into VGPRs; its address depends on the metadata
//         (TRIPS dependent loads before the data load)
//   dma : data DMA'd into LDS by global_load_lds_dwordx4 at an address known
//         from blockIdx alone, metadata trips in parallel; stores from LDS with
//         the metadata-dependent shift
// U = 4 KiB tiles per workgroup.
// Build: hipcc --offload-arch=gfx950 -O3 tools/copybw7.hip -o tools/copybw7
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

template <int TRIPS>
__device__ __forceinline__ uint32_t meta_chain(const uint32_t* __restrict__ m1,
                                               const uint32_t* __restrict__ m2, uint32_t t) {
  uint32_t s = 0;
  if (TRIPS >= 1) s = m1[t];                                  // tile -> first run
  if (TRIPS >= 2) s = m2[s + t * 4 + (threadIdx.x & 3)];      // the run (lane-varying)
  if (TRIPS >= 3) s = m2[s + t * 4 + 1];                       // one more hop
  return s;  // always 0 at run time (zeroed tables)
}

template <int TRIPS, int U>
__global__ __launch_bounds__(256) void tile_reg(const uint4* __restrict__ a, uint4* __restrict__ b,
                                                const uint32_t* __restrict__ m1,
                                                const uint32_t* __restrict__ m2) {
  const uint32_t t = blockIdx.x;
  const uint32_t s = meta_chain<TRIPS>(m1, m2, t);
  const size_t base = size_t(t) * (U * 256) + threadIdx.x;
  uint4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = a[base + u * 256 + s];
#pragma unroll
  for (int u = 0; u < U; ++u) b[base + u * 256] = v[u];
}

template <int TRIPS, int U>
__global__ __launch_bounds__(256) void tile_dma(const uint4* __restrict__ a, uint4* __restrict__ b,
                                                const uint32_t* __restrict__ m1,
                                                const uint32_t* __restrict__ m2) {
  __shared__ uint4 st[U * 256 + 16];
  const uint32_t t = blockIdx.x;
  const size_t base = size_t(t) * (U * 256);
  const uint32_t w = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < U; ++u)
    __builtin_amdgcn_global_load_lds(a + base + u * 256 + threadIdx.x,
                                     LDS_PTR(st + u * 256 + w * 64), 16, 0, 0);
  const uint32_t s = meta_chain<TRIPS>(m1, m2, t);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int u = 0; u < U; ++u) b[base + u * 256 + threadIdx.x] = st[u * 256 + threadIdx.x + s];
}

int main() {
  const size_t bytes = size_t(4) << 30;
  uint4 *a, *b;
  uint32_t *m1, *m2;
  const size_t ntile = bytes / 4096;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess ||
      hipMalloc(&m1, ntile * 4) != hipSuccess || hipMalloc(&m2, ntile * 16 + 64) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(a, 1, bytes);
  (void)hipMemset(b, 0, bytes);
  (void)hipMemset(m1, 0, ntile * 4);
  (void)hipMemset(m2, 0, ntile * 16 + 64);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int reps = 10;
  auto run = [&](const char* name, auto launch) {
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    printf("%-40s %8.3f ms  %8.1f GB/s\n", name, ms, 2.0 * bytes / ms / 1e6);
    fflush(stdout);
  };
  const size_t n = bytes / 16;
#define RUN(K, T, U)                                                              \
  run(#K " trips=" #T " U=" #U, [&] {                                             \
    K<T, U><<<uint32_t(n / (256 * U)), 256>>>(a, b, m1, m2);                      \
  })
  for (int rep = 0; rep < 2; ++rep) {
    RUN(tile_reg, 0, 1);
    RUN(tile_reg, 1, 1);
    RUN(tile_reg, 2, 1);
    RUN(tile_reg, 3, 1);
    RUN(tile_reg, 2, 2);
    RUN(tile_reg, 2, 4);
    RUN(tile_dma, 0, 1);
    RUN(tile_dma, 1, 1);
    RUN(tile_dma, 2, 1);
    RUN(tile_dma, 3, 1);
    RUN(tile_dma, 0, 2);
    RUN(tile_dma, 2, 2);
    RUN(tile_dma, 2, 4);
  }
  (void)hipFree(a);
  (void)hipFree(b);
  (void)hipFree(m1);
  (void)hipFree(m2);
  return 0;
}
