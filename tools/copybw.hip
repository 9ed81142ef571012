// Read+write ceiling microbenchmark for MI355X (diagnostic, not product code).
// Variants: grid-stride uint4 copy; unrolled x4; nontemporal; per-64KiB-block
// workgroups (the decode's shape); write-only; read-only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void copy_gs(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) b[i] = a[i];
}
__global__ void copy_u4(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  const size_t stride = gridDim.x * 256ull;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i + 3 * stride < n; i += 4 * stride) {
    uint4 x0 = a[i], x1 = a[i + stride], x2 = a[i + 2 * stride], x3 = a[i + 3 * stride];
    b[i] = x0; b[i + stride] = x1; b[i + 2 * stride] = x2; b[i + 3 * stride] = x3;
  }
}
__global__ void copy_nt(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
}
// one workgroup per 64 KiB block (4096 uint4), 256 threads x 16
__global__ void copy_blk(const uint4* __restrict__ a, uint4* __restrict__ b) {
  const size_t base = size_t(blockIdx.x) * 4096;
  uint4 v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = a[base + threadIdx.x + 256 * k];
#pragma unroll
  for (int k = 0; k < 16; ++k) b[base + threadIdx.x + 256 * k] = v[k];
}
__global__ void copy_blk4(const uint4* __restrict__ a, uint4* __restrict__ b) {
  const size_t base = size_t(blockIdx.x) * 4096;
  for (int k0 = 0; k0 < 16; k0 += 4) {
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = a[base + threadIdx.x + 256 * (k0 + k)];
#pragma unroll
    for (int k = 0; k < 4; ++k) b[base + threadIdx.x + 256 * (k0 + k)] = v[k];
  }
}
__device__ __forceinline__ uint32_t fsh(uint32_t hi, uint32_t lo, uint32_t s) {
  return __builtin_amdgcn_alignbyte(hi, lo, s);
}
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }
__device__ __forceinline__ uint4 funnel32(const uint4& x, const uint4& y, uint32_t s) {
  const uint32_t m8 = 0u - ((s >> 3) & 1u), m4 = 0u - ((s >> 2) & 1u), r = s & 3u;
  const uint32_t a0 = bsel(m8, x.z, x.x), a1 = bsel(m8, x.w, x.y), a2 = bsel(m8, y.x, x.z),
                 a3 = bsel(m8, y.y, x.w), a4 = bsel(m8, y.z, y.x), a5 = bsel(m8, y.w, y.y);
  const uint32_t b0 = bsel(m4, a1, a0), b1 = bsel(m4, a2, a1), b2 = bsel(m4, a3, a2),
                 b3 = bsel(m4, a4, a3), b4 = bsel(m4, a5, a4);
  return make_uint4(fsh(b1, b0, r), fsh(b2, b1, r), fsh(b3, b2, r), fsh(b4, b3, r));
}
// misaligned source: 2 aligned loads per 16 B + funnel (the decode's window16)
__global__ void copy_shift(const uint8_t* __restrict__ a, uint4* __restrict__ b, size_t n, uint32_t sh) {
  const size_t stride = gridDim.x * 256ull;
  for (size_t i0 = blockIdx.x * 256ull + threadIdx.x; i0 < n; i0 += 4 * stride) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      size_t i = i0 + u * stride;
      if (i + 1 >= n) i = i0;
      const uint4* p = reinterpret_cast<const uint4*>(a) + i;
      v[u] = funnel32(p[0], p[1], sh);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) if (i0 + u * stride + 1 < n) b[i0 + u * stride] = v[u];
  }
}
// misaligned source, per-64KiB workgroup, one aligned load + neighbour via shuffle
__global__ void copy_shift_blk(const uint4* __restrict__ a, uint4* __restrict__ b, uint32_t sh) {
  const size_t base = size_t(blockIdx.x) * 4096;
  uint4 v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = a[base + threadIdx.x + 256 * k];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    uint4 nx;
    nx.x = __shfl_down(v[k].x, 1, 64); nx.y = __shfl_down(v[k].y, 1, 64);
    nx.z = __shfl_down(v[k].z, 1, 64); nx.w = __shfl_down(v[k].w, 1, 64);
    b[base + threadIdx.x + 256 * k] = funnel32(v[k], nx, sh);
  }
}
__global__ void fill(uint4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    b[i] = make_uint4(i, 1, 2, 3);
}
__global__ void readsum(const uint4* __restrict__ a, size_t n, uint32_t* out) {
  uint32_t s = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    uint4 x = a[i];
    s ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  if (s == 0x12345678u) out[0] = s;
}

int main() {
  const size_t bytes = size_t(4) << 30, n = bytes / 16;
  uint4 *a, *b;
  uint32_t* o;
  hipMalloc(&a, bytes);
  hipMalloc(&b, bytes);
  hipMalloc(&o, 4);
  hipMemset(a, 1, bytes);
  hipMemset(b, 0, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, double moved, auto launch) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("%-28s %8.3f ms  %8.1f GB/s\n", name, ms, moved / ms / 1e6);
  };
  for (int g : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, 64, "copy_gs grid=%d", g);
    run(nm, 2.0 * bytes, [&] { copy_gs<<<g, 256>>>(a, b, n); });
  }
  for (int g : {2048, 8192}) {
    char nm[64];
    snprintf(nm, 64, "copy_u4 grid=%d", g);
    run(nm, 2.0 * bytes, [&] { copy_u4<<<g, 256>>>(a, b, n); });
    snprintf(nm, 64, "copy_nt grid=%d", g);
    run(nm, 2.0 * bytes, [&] { copy_nt<<<g, 256>>>((const u32x4*)a, (u32x4*)b, n); });
  }
  run("copy_blk (64KiB/WG)", 2.0 * bytes, [&] { copy_blk<<<n / 4096, 256>>>(a, b); });
  run("copy_blk4 (64KiB/WG)", 2.0 * bytes, [&] { copy_blk4<<<n / 4096, 256>>>(a, b); });
  for (int g : {1024, 2048, 8192}) {
    char nm[64];
    snprintf(nm, 64, "copy_shift5 grid=%d", g);
    run(nm, 2.0 * bytes, [&] { copy_shift<<<g, 256>>>((const uint8_t*)a, b, n, 5); });
  }
  run("copy_shift_blk (shfl)", 2.0 * bytes, [&] { copy_shift_blk<<<n / 4096, 256>>>(a, b, 5); });
  run("fill grid=8192", 1.0 * bytes, [&] { fill<<<8192, 256>>>(b, n); });
  run("readsum grid=8192", 1.0 * bytes, [&] { readsum<<<8192, 256>>>(a, n, o); });
  return 0;
}
