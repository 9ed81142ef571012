// okv_kernels.hpp -- device-side building blocks for the SST block decode
// (gfx950 / CDNA4, wave64).  Byte and index work only: no MFMA.
//
// Record format restated from the reference writer/reader:
//   [u16 LE klen][u32 LE vlen][key][value]      segment_writer.go:121-125
// decode loop `for consumed < OriginalSize`     segment_reader.go:338-352
// each read must be satisfied in full or Go panics (mustReadBytes :506-512);
// zero-length reads read nothing and yield nil (readBytes :490-493).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "okv_sst.h"

namespace okv {

constexpr int kThreads = 256;      // 4 waves per workgroup
constexpr int kTile = 256;         // blocks per pass-1 workgroup (one lane each)
constexpr int kRowBatch = 256;     // rows per LDS row-table batch (general path)
constexpr int kFastRows = 1024;    // max rows of a staged block on its fast path
constexpr int kRCap = 64;          // record positions pass 1 keeps per block
constexpr int kStage = 65536;      // LDS staging capacity for one block (bytes)
constexpr int kStagePad = 64;      // guard bytes around the staged image

struct BlockCount {   // pass-1 result per block
  uint64_t rows;      // records decoded
  uint64_t kbytes;    // sum of key lengths
  uint64_t vbytes;    // sum of value lengths
  uint64_t pend;      // final walk position (>= OriginalSize; <= buffer length)
  int32_t status;     // OKV_BLK_*
  int32_t pad;
};

struct Prefix {       // exclusive prefixes (rows, padded key bytes, padded value bytes)
  uint64_t rows, kb, vb, bad;
};

struct Totals {
  uint64_t rows, kb, vb, bad;
};

struct Desc {         // == okv_block_desc
  uint64_t offset, block_size, original_size, compressed_size;
};

struct SpanHint {  // okv_decode_plan's longest walk (host side)
  const uint8_t* seg = nullptr;
  const Desc* descs = nullptr;
  uint64_t seg_bytes = 0;
  uint32_t nblk = 0;
  uint64_t span = 0;
};

__host__ __device__ inline uint64_t round16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

// Go's int() conversions at the block boundary (segment_reader.go:303-340),
// shared by every walk:
// * make([]byte, stat.BlockSize) (:309) panics ("makeslice: len out of range")
//   for a length above the runtime's maxAlloc = 1 << heapAddrBits = 2^48 on
//   64-bit linux (runtime/malloc.go, runtime/slice.go), which also covers the
//   lengths that are negative as int;
// * `totalReadBytes < int(stat.OriginalSize)` (:340) has a negative bound
//   from 2^63 on: the loop runs no iteration (nil rows, no error).
constexpr uint64_t kGoMaxAlloc = uint64_t(1) << 48;
__host__ __device__ inline uint64_t go_walk_bound(uint64_t original_size) {
  return int64_t(original_size) < 0 ? 0 : original_size;
}
// The raw-block outcome of :303-316 in Go's order: Seek(int64(Offset))
// (negative -> error), make (panic), Read (io.EOF at / past the end, short).
// OKV_BLK_OK when the block's BlockSize bytes are in the segment.
__host__ __device__ inline int32_t go_read_status(const Desc& d, uint64_t seg_bytes) {
  if (int64_t(d.offset) < 0) return OKV_BLK_EOF;                // Seek error
  if (d.block_size > kGoMaxAlloc) return OKV_BLK_PANIC;           // makeslice
  if (d.offset >= seg_bytes) return OKV_BLK_EOF;                  // io.EOF
  if (seg_bytes - d.offset < d.block_size) return OKV_BLK_SHORT;  // short read
  return OKV_BLK_OK;
}

// Bytes [pos, pos+4) from two consecutive aligned dwords.
// An LDS pointer for __builtin_amdgcn_global_load_lds (LDS DMA destination).
#define OKV_LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// Read the 6-byte record header at absolute segment position pos (the caller
// has checked pos + 6 <= buffer end <= seg_bytes).  Only dwords containing a
// needed byte are loaded, so no load leaves the segment's last dword.
__device__ __forceinline__ void header_global(const uint8_t* __restrict__ seg, uint64_t pos,
                                              uint32_t& klen, uint32_t& vlen) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(seg + (pos & ~uint64_t(3)));
  const uint32_t sh = uint32_t(pos & 3);
  const uint32_t w0 = w[0];
  const uint32_t w1 = w[1];
  const uint32_t w2 = (sh == 3) ? w[2] : 0u;
  const uint32_t a = funnel(w1, w0, sh);  // bytes pos..pos+3
  const uint32_t b = funnel(w2, w1, sh);  // bytes pos+4..pos+7
  klen = a & 0xffffu;
  vlen = (a >> 16) | (b << 16);
}

// Same, from an LDS byte image (word-addressed, byte index bi).
__device__ __forceinline__ void header_lds(const uint32_t* sw, uint32_t bi, uint32_t& klen,
                                           uint32_t& vlen) {
  const uint32_t* w = sw + (bi >> 2);
  const uint32_t sh = bi & 3;
  const uint32_t a = funnel(w[1], w[0], sh);
  const uint32_t b = funnel(w[2], w[1], sh);
  klen = a & 0xffffu;
  vlen = (a >> 16) | (b << 16);
}

// 16 bytes starting at LDS byte index bi (any alignment): 5 dword reads + funnels.
__device__ __forceinline__ uint4 load16_lds(const uint32_t* sw, uint32_t bi) {
  const uint32_t* w = sw + (bi >> 2);
  const uint32_t sh = bi & 3;
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
  return make_uint4(funnel(w1, w0, sh), funnel(w2, w1, sh), funnel(w3, w2, sh),
                    funnel(w4, w3, sh));
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Branch-free bit select: m ? a : b per bit (one v_bfi_b32).  Plain ternary
// chains on runtime indices compile to exec-mask branches on gfx950.
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) {
  return (a & m) | (b & ~m);
}

// Bytes [s, s+16) of the 32-byte window (x, y), s in 0..15.
__device__ __forceinline__ uint4 funnel32(const uint4& x, const uint4& y, uint32_t s) {
  const uint32_t m8 = 0u - ((s >> 3) & 1u), m4 = 0u - ((s >> 2) & 1u), r = s & 3u;
  const uint32_t a0 = bsel(m8, x.z, x.x), a1 = bsel(m8, x.w, x.y), a2 = bsel(m8, y.x, x.z),
                 a3 = bsel(m8, y.y, x.w), a4 = bsel(m8, y.z, y.x), a5 = bsel(m8, y.w, y.y);
  const uint32_t b0 = bsel(m4, a1, a0), b1 = bsel(m4, a2, a1), b2 = bsel(m4, a3, a2),
                 b3 = bsel(m4, a4, a3), b4 = bsel(m4, a5, a4);
  return make_uint4(funnel(b1, b0, r), funnel(b2, b1, r), funnel(b3, b2, r), funnel(b4, b3, r));
}

// 16 bytes starting at LDS byte index bi (relative to s4): two aligned
// 16-byte reads + the branch-free funnel.
__device__ __forceinline__ uint4 load16_lds_b128(const uint4* s4, uint32_t bi) {
  const uint4 x = s4[bi >> 4];
  const uint4 y = s4[(bi >> 4) + 1];
  return funnel32(x, y, bi & 15u);
}

// Mask of bytes [a, b) (0 <= a <= b <= 16) that fall in dword k of a chunk.
__device__ __forceinline__ uint32_t byte_mask(int32_t a, int32_t b, int k) {
  const int32_t lo = min(max(a - 4 * k, 0), 4), hi = min(max(b - 4 * k, 0), 4);
  const uint32_t mh = hi >= 4 ? 0xffffffffu : ((1u << (8 * hi)) - 1u);
  const uint32_t ml = lo >= 4 ? 0xffffffffu : ((1u << (8 * lo)) - 1u);
  return mh & ~ml;
}

// out with bytes [a, b) replaced by those of v.
__device__ __forceinline__ uint4 merge_bytes(uint4 out, const uint4& v, int32_t a, int32_t b) {
  uint32_t m;
  m = byte_mask(a, b, 0); out.x = (out.x & ~m) | (v.x & m);
  m = byte_mask(a, b, 1); out.y = (out.y & ~m) | (v.y & m);
  m = byte_mask(a, b, 2); out.z = (out.z & ~m) | (v.z & m);
  m = byte_mask(a, b, 3); out.w = (out.w & ~m) | (v.w & m);
  return out;
}

// 16 bytes starting at absolute segment position pos (may be < 0 or run past
// the end for masked head/tail chunks): dwords wholly outside [0, seg_bytes)
// are not loaded.
__device__ __forceinline__ uint4 load16_global(const uint8_t* __restrict__ seg, uint64_t seg_bytes,
                                               int64_t pos) {
  const int64_t a = pos & ~int64_t(3);
  const uint32_t sh = uint32_t(pos & 3);
  uint32_t w[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int64_t at = a + 4 * i;
    w[i] = (at >= 0 && uint64_t(at) < seg_bytes)
               ? *reinterpret_cast<const uint32_t*>(seg + at)
               : 0u;
  }
  return make_uint4(funnel(w[1], w[0], sh), funnel(w[2], w[1], sh), funnel(w[3], w[2], sh),
                    funnel(w[4], w[3], sh));
}

// 16-byte streaming load (nontemporal: the block is read once).
__device__ __forceinline__ uint4 load_nt16(const uint4* p) {
  const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(t.x, t.y, t.z, t.w);
}

// 16-byte streaming store (nontemporal).
__device__ __forceinline__ void store_nt16(uint4* p, const uint4& v) {
  u32x4 t;
  t.x = v.x;
  t.y = v.y;
  t.z = v.z;
  t.w = v.w;
  __builtin_nontemporal_store(t, reinterpret_cast<u32x4*>(p));
}

// Dword of v starting at byte o (0..15) without runtime-indexed arrays.
__device__ __forceinline__ uint32_t dword_at(const uint4& v, uint32_t o) {
  return funnel32(v, make_uint4(0, 0, 0, 0), o).x;
}

// Store bytes [lo, hi) of the 16-byte vector v to the 16-byte aligned dst,
// using the widest naturally aligned stores (no read-modify-write: bytes
// outside [lo, hi) belong to a neighbouring row and are not touched).
__device__ __forceinline__ void store_partial(uint8_t* dst, const uint4& v, uint32_t lo,
                                              uint32_t hi) {
  uint32_t o = lo;
  while (o < hi) {
    if ((o & 7) == 0 && o + 8 <= hi) {
      const uint64_t q = uint64_t(dword_at(v, o)) | (uint64_t(dword_at(v, o + 4)) << 32);
      *reinterpret_cast<uint64_t*>(dst + o) = q;
      o += 8;
    } else if ((o & 3) == 0 && o + 4 <= hi) {
      *reinterpret_cast<uint32_t*>(dst + o) = dword_at(v, o);
      o += 4;
    } else if ((o & 1) == 0 && o + 2 <= hi) {
      *reinterpret_cast<uint16_t*>(dst + o) = uint16_t(dword_at(v, o));
      o += 2;
    } else {
      dst[o] = uint8_t(dword_at(v, o));
      o += 1;
    }
  }
}

// 16 bytes of seg starting at absolute position x from two aligned 16-byte
// loads and the byte funnel.  16-byte lines wholly outside [0, seg_bytes)
// are not loaded and read as zero (only masked bytes ever come from them).
__device__ __forceinline__ uint4 window16(const uint8_t* __restrict__ seg, uint64_t seg_bytes,
                                         int64_t x) {
  const int64_t a = x & ~int64_t(15);
  const uint32_t s = uint32_t(x & 15);
  const bool v0 = a >= 0 && uint64_t(a) < seg_bytes;
  const bool v1 = s != 0 && a + 16 >= 0 && uint64_t(a + 16) < seg_bytes;
  const uint4 lo = *reinterpret_cast<const uint4*>(seg + (v0 ? a : 0));
  const uint4 hi = *reinterpret_cast<const uint4*>(seg + (v1 ? a + 16 : 0));
  const uint32_t m0 = 0u - uint32_t(v0), m1 = 0u - uint32_t(v1);
  return funnel32(make_uint4(lo.x & m0, lo.y & m0, lo.z & m0, lo.w & m0),
                  make_uint4(hi.x & m1, hi.y & m1, hi.z & m1, hi.w & m1), s);
}

// Wave64 inclusive scan of a 32-bit value.
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t x, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// Wave64 inclusive scan by DPP (no LDS round trips): Hillis-Steele inside
// each 16-lane row, then row 0 -> 1, 2 -> 3 (row_bcast:15) and the first
// half's total into the second (row_bcast:31).  All 64 lanes must be active.
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t x) {
  x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, true);   // row_shr:1
  x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, true);   // row_shr:2
  x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, true);   // row_shr:4
  x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, true);   // row_shr:8
  x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

// Wave64 inclusive scan of a 64-bit value (DPP-free shuffle form).
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// XXH64 (cespare/xxhash v2.2.0 == canonical XXH64, seed 0) building blocks.
__device__ constexpr uint64_t XP1 = 11400714785074694791ULL, XP2 = 14029467366897019727ULL,
                              XP3 = 1609587929392839161ULL, XP4 = 9650029242287828579ULL,
                              XP5 = 2870177450012600261ULL;
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) {
  return (x << r) | (x >> (64 - r));
}
__device__ __forceinline__ uint64_t xround(uint64_t acc, uint64_t in) {
  acc += in * XP2;
  acc = rotl64(acc, 31);
  return acc * XP1;
}
__device__ __forceinline__ uint64_t ld64u(const uint8_t* p) {  // unaligned LE load
  uint64_t v = 0;
#pragma unroll
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

}  // namespace okv
