// Copy-ceiling probe #4 (diagnostic, not product): the two questions the
// round-2 gather redesign depends on.
//   1. A byte-shifted copy (source misaligned by s bytes) with ONE unaligned
//      global_load_dwordx4 per lane (gfx950 unaligned access mode) vs the
//      product's two aligned 16-byte loads + byte funnel.
//   2. How a 64 KiB-per-workgroup copy depends on the workgroup width
//      (4 / 8 / 16 waves: a block finishes sooner, fewer blocks are open at
//      once, the chip's concurrent footprint narrows).
// Build: hipcc --offload-arch=gfx950 -O3 tools/copybw4.hip -o tools/copybw4
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ uint4 ld_unaligned(const uint8_t* p) {
  uint4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}

__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) {
  return (a & m) | (b & ~m);
}
__device__ __forceinline__ uint4 funnel32(const uint4& x, const uint4& y, uint32_t s) {
  const uint32_t m8 = 0u - ((s >> 3) & 1u), m4 = 0u - ((s >> 2) & 1u), r = s & 3u;
  const uint32_t a0 = bsel(m8, x.z, x.x), a1 = bsel(m8, x.w, x.y), a2 = bsel(m8, y.x, x.z),
                 a3 = bsel(m8, y.y, x.w), a4 = bsel(m8, y.z, y.x), a5 = bsel(m8, y.w, y.y);
  const uint32_t b0 = bsel(m4, a1, a0), b1 = bsel(m4, a2, a1), b2 = bsel(m4, a3, a2),
                 b3 = bsel(m4, a4, a3), b4 = bsel(m4, a5, a4);
  return make_uint4(__builtin_amdgcn_alignbyte(b1, b0, r), __builtin_amdgcn_alignbyte(b2, b1, r),
                    __builtin_amdgcn_alignbyte(b3, b2, r), __builtin_amdgcn_alignbyte(b4, b3, r));
}
__device__ __forceinline__ uint4 ld_funnel(const uint8_t* base, uint64_t x) {
  const uint4* p = reinterpret_cast<const uint4*>(base + (x & ~uint64_t(15)));
  return funnel32(p[0], p[1], uint32_t(x & 15));
}

// One workgroup of W waves per 64 KiB destination block, wave w copies its
// contiguous share, kU 1 KiB tiles per iteration (loads before stores).
// MODE 0: aligned loads, 1: unaligned dwordx4, 2: two aligned loads + funnel.
template <int W, int kU, int MODE>
__global__ __launch_bounds__(W * 64) void copy_block(const uint8_t* __restrict__ a,
                                                     uint4* __restrict__ b, uint32_t shift) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int T = 64, per = T / W;
  const uint64_t base = uint64_t(blockIdx.x) * 4096;  // uint4 units
  for (int t = wave * per; t < wave * per + per; t += kU) {
    uint4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint64_t c = base + uint64_t(t + u) * 64 + lane;
      if (MODE == 0) v[u] = reinterpret_cast<const uint4*>(a)[c];
      else if (MODE == 1) v[u] = ld_unaligned(a + c * 16 + shift);
      else v[u] = ld_funnel(a, c * 16 + shift);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) b[base + uint64_t(t + u) * 64 + lane] = v[u];
  }
}

// One-shot: one 16-byte chunk per lane, U chunks per lane, 256 threads.
template <int U, int MODE>
__global__ __launch_bounds__(256) void copy_chunk(const uint8_t* __restrict__ a,
                                                  uint4* __restrict__ b, uint32_t shift) {
  const uint64_t base = uint64_t(blockIdx.x) * (U * 256) + threadIdx.x;
  uint4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t c = base + u * 256;
    if (MODE == 0) v[u] = reinterpret_cast<const uint4*>(a)[c];
    else if (MODE == 1) v[u] = ld_unaligned(a + c * 16 + shift);
    else v[u] = ld_funnel(a, c * 16 + shift);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) b[base + u * 256] = v[u];
}

int main(int argc, char** argv) {
  const size_t bytes = size_t(4) << 30;
  uint8_t* a;
  uint4* b;
  if (hipMalloc(&a, bytes + 4096) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(a, 1, bytes + 4096);
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
    printf("%-52s %8.3f ms  %8.1f GB/s\n", name, ms, 2.0 * bytes / ms / 1e6);
    fflush(stdout);
  };
  const size_t n = bytes / 16;
  const uint32_t nb = uint32_t(bytes / 65536);
  for (int rep = 0; rep < 2; ++rep) {
    run("block W4 kU4 aligned", [&] { copy_block<4, 4, 0><<<nb, 256>>>(a, b, 0); });
    run("block W4 kU4 unaligned s=5", [&] { copy_block<4, 4, 1><<<nb, 256>>>(a, b, 5); });
    run("block W4 kU4 unaligned s=0", [&] { copy_block<4, 4, 1><<<nb, 256>>>(a, b, 0); });
    run("block W4 kU4 funnel s=5", [&] { copy_block<4, 4, 2><<<nb, 256>>>(a, b, 5); });
    run("block W4 kU8 unaligned s=5", [&] { copy_block<4, 8, 1><<<nb, 256>>>(a, b, 5); });
    run("block W8 kU4 aligned", [&] { copy_block<8, 4, 0><<<nb, 512>>>(a, b, 0); });
    run("block W8 kU4 unaligned s=5", [&] { copy_block<8, 4, 1><<<nb, 512>>>(a, b, 5); });
    run("block W8 kU4 funnel s=5", [&] { copy_block<8, 4, 2><<<nb, 512>>>(a, b, 5); });
    run("block W16 kU4 aligned", [&] { copy_block<16, 4, 0><<<nb, 1024>>>(a, b, 0); });
    run("block W16 kU4 unaligned s=5", [&] { copy_block<16, 4, 1><<<nb, 1024>>>(a, b, 5); });
    run("block W16 kU4 funnel s=5", [&] { copy_block<16, 4, 2><<<nb, 1024>>>(a, b, 5); });
    run("block W16 kU2 unaligned s=5", [&] { copy_block<16, 2, 1><<<nb, 1024>>>(a, b, 5); });
    run("chunk U1 aligned", [&] { copy_chunk<1, 0><<<n / 256, 256>>>(a, b, 0); });
    run("chunk U1 unaligned s=5", [&] { copy_chunk<1, 1><<<n / 256, 256>>>(a, b, 5); });
    run("chunk U1 funnel s=5", [&] { copy_chunk<1, 2><<<n / 256, 256>>>(a, b, 5); });
    run("chunk U4 unaligned s=5", [&] { copy_chunk<4, 1><<<n / 1024, 256>>>(a, b, 5); });
    run("chunk U4 funnel s=5", [&] { copy_chunk<4, 2><<<n / 1024, 256>>>(a, b, 5); });
  }
  (void)hipFree(a);
  (void)hipFree(b);
  return 0;
}
