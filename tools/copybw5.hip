// Copy-ceiling probe #5 (diagnostic, not product): why does a one-shot copy
// with one 16-byte chunk per lane (4 KiB per workgroup) beat every looping or
// wider shape?  Two candidate causes are separated here:
//   (a) bytes in flight: U chunks per lane at an occupancy capped through a
//       dynamic LDS allocation (fewer workgroups per CU);
//   (b) the chip's concurrent footprint: the same U=1 kernel with its
//       workgroup -> tile mapping permuted so consecutive workgroups land S
//       streams apart (same bytes in flight, wide footprint).
// Build: hipcc --offload-arch=gfx950 -O3 tools/copybw5.hip -o tools/copybw5
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

template <int U>
__global__ __launch_bounds__(256) void copy_chunk(const uint4* __restrict__ a,
                                                  uint4* __restrict__ b, uint32_t streams,
                                                  uint32_t ntiles) {
  extern __shared__ uint32_t occ[];
  uint32_t t = blockIdx.x;
  if (streams > 1) t = (t % streams) * (ntiles / streams) + t / streams;
  const uint64_t base = uint64_t(t) * (U * 256) + threadIdx.x;
  uint4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = a[base + u * 256];
  if (v[0].x == 0xdeadbeefu) occ[threadIdx.x] = 1;  // keeps the LDS allocation
#pragma unroll
  for (int u = 0; u < U; ++u) b[base + u * 256] = v[u];
}

int main() {
  const size_t bytes = size_t(4) << 30;
  uint4 *a, *b;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(a, 1, bytes);
  (void)hipMemset(b, 0, bytes);
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
    printf("%-56s %8.3f ms  %8.1f GB/s\n", name, ms, 2.0 * bytes / ms / 1e6);
    fflush(stdout);
  };
  const size_t n = bytes / 16;
  char nm[128];
  for (int rep = 0; rep < 2; ++rep) {
    // (a) occupancy caps: LDS bytes per WG -> WGs per CU (160 KiB / lds)
    for (uint32_t lds : {0u, 20480u, 40960u, 81920u}) {
      const uint32_t t1 = uint32_t(n / 256), t2 = uint32_t(n / 512), t4 = uint32_t(n / 1024);
      snprintf(nm, sizeof nm, "U1 lds=%u", lds);
      run(nm, [&] { copy_chunk<1><<<t1, 256, lds>>>(a, b, 1, t1); });
      snprintf(nm, sizeof nm, "U2 lds=%u", lds);
      run(nm, [&] { copy_chunk<2><<<t2, 256, lds>>>(a, b, 1, t2); });
      snprintf(nm, sizeof nm, "U4 lds=%u", lds);
      run(nm, [&] { copy_chunk<4><<<t4, 256, lds>>>(a, b, 1, t4); });
    }
    // (b) footprint: U=1, consecutive WGs S streams apart
    for (uint32_t s : {2u, 16u, 256u, 1024u, 4096u}) {
      const uint32_t t1 = uint32_t(n / 256);
      snprintf(nm, sizeof nm, "U1 streams=%u", s);
      run(nm, [&] { copy_chunk<1><<<t1, 256, 0>>>(a, b, s, t1); });
    }
  }
  (void)hipFree(a);
  (void)hipFree(b);
  return 0;
}
