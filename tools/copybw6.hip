// Copy-ceiling probe #6 (diagnostic, not product): do looping copies lose to
// the one-shot form because each iteration's wait for its loads also waits for
// the previous iteration's stores (gfx9 has one vmcnt for both)?  Software-
// pipelined loops issue iteration i+1's loads before iteration i's stores, so
// the compiler's vmcnt(N) skips the stores.
// Build: hipcc --offload-arch=gfx950 -O3 tools/copybw6.hip -o tools/copybw6
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

// grid-stride, U chunks per lane per iteration; PIPE: next loads before stores
template <int U, bool PIPE>
__global__ __launch_bounds__(256) void copy_gs(const uint4* __restrict__ a, uint4* __restrict__ b,
                                               size_t n) {
  const size_t stride = size_t(gridDim.x) * 256 * U;
  size_t i = size_t(blockIdx.x) * 256 * U + threadIdx.x;
  if (!PIPE) {
    for (; i < n; i += stride) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = a[i + u * 256];
#pragma unroll
      for (int u = 0; u < U; ++u) b[i + u * 256] = v[u];
    }
    return;
  }
  if (i >= n) return;
  uint4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = a[i + u * 256];
  for (;;) {
    const size_t j = i + stride;
    const bool more = j < n;
    uint4 w[U];
    if (more) {
#pragma unroll
      for (int u = 0; u < U; ++u) w[u] = a[j + u * 256];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) b[i + u * 256] = v[u];
    if (!more) break;
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = w[u];
    i = j;
  }
}

// the gather's block shape (64 KiB per WG, wave = contiguous quarter, kU tiles
// per iteration), plain or pipelined
template <int kU, bool PIPE>
__global__ __launch_bounds__(256) void copy_block(const uint4* __restrict__ a,
                                                  uint4* __restrict__ b) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t base = size_t(blockIdx.x) * 4096 + size_t(wave) * 1024 + lane;
  if (!PIPE) {
    for (int t = 0; t < 16; t += kU) {
      uint4 v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) v[u] = a[base + (t + u) * 64];
#pragma unroll
      for (int u = 0; u < kU; ++u) b[base + (t + u) * 64] = v[u];
    }
    return;
  }
  uint4 v[kU];
#pragma unroll
  for (int u = 0; u < kU; ++u) v[u] = a[base + u * 64];
#pragma unroll
  for (int t = 0; t < 16; t += kU) {
    uint4 w[kU];
    if (t + kU < 16) {
#pragma unroll
      for (int u = 0; u < kU; ++u) w[u] = a[base + (t + kU + u) * 64];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) b[base + (t + u) * 64] = v[u];
#pragma unroll
    for (int u = 0; u < kU; ++u) v[u] = w[u];
  }
}

template <int U>
__global__ __launch_bounds__(256) void copy_chunk(const uint4* __restrict__ a,
                                                  uint4* __restrict__ b) {
  const size_t base = size_t(blockIdx.x) * (U * 256) + threadIdx.x;
  uint4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = a[base + u * 256];
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
    run("chunk U1 (control)", [&] { copy_chunk<1><<<n / 256, 256>>>(a, b); });
    for (int g : {512, 1024, 2048}) {
      snprintf(nm, sizeof nm, "gs U1 plain grid=%d", g);
      run(nm, [&] { copy_gs<1, false><<<g, 256>>>(a, b, n); });
      snprintf(nm, sizeof nm, "gs U1 pipe  grid=%d", g);
      run(nm, [&] { copy_gs<1, true><<<g, 256>>>(a, b, n); });
      snprintf(nm, sizeof nm, "gs U2 plain grid=%d", g);
      run(nm, [&] { copy_gs<2, false><<<g, 256>>>(a, b, n); });
      snprintf(nm, sizeof nm, "gs U2 pipe  grid=%d", g);
      run(nm, [&] { copy_gs<2, true><<<g, 256>>>(a, b, n); });
    }
    const uint32_t nb = uint32_t(bytes / 65536);
    run("block kU4 plain", [&] { copy_block<4, false><<<nb, 256>>>(a, b); });
    run("block kU4 pipe", [&] { copy_block<4, true><<<nb, 256>>>(a, b); });
    run("block kU2 plain", [&] { copy_block<2, false><<<nb, 256>>>(a, b); });
    run("block kU2 pipe", [&] { copy_block<2, true><<<nb, 256>>>(a, b); });
    run("block kU1 pipe", [&] { copy_block<1, true><<<nb, 256>>>(a, b); });
  }
  (void)hipFree(a);
  (void)hipFree(b);
  return 0;
}
