// okv_zstd.hip -- zstd block decompression on the GPU (gfx950), for segments
// whose meta compression byte is 1.
//
// The reference reads a zstd block as
//   zstd.NewReader(bytes.NewReader(rawBlockBytes[:stat.CompressedSize])); io.Copy
// (/root/reference/sst/segment_reader.go:320-330) with klauspost/compress
// v1.17.9: every frame in the slice is decoded (RFC 8878), skippable frames are
// skipped, content checksums and frame content sizes are verified, and any
// failure is an error returned from ReadBlockWithStat.  This file restates that
// decoding; the record walk then runs unchanged on the decompressed bytes.
//
// One wave (64 lanes) per segment block, persistent over the batch.  Entropy
// decoding (FSE sequences, Huffman weights, headers) is sequential and runs
// wave-uniform (every lane computes the same values: no broadcasts); Huffman
// literal streams run one per lane (4 streams -> lanes 0..3); literal and match
// copies run lane-parallel.  Output goes to a per-block scratch region in HBM;
// a match whose source overlaps bytes written since the last commit point first
// waits for this wave's stores (s_waitcnt vmcnt(0) + workgroup fence).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <cstdio>
#include <cstdlib>

#include "okv_ctx.hpp"
#include "okv_kernels.hpp"
#include "okv_sst.h"

namespace okv {
namespace zst {

constexpr int kHufMaxBits = 11;          // Max_Number_of_Bits for literals (RFC 8878 4.2.1)
constexpr uint32_t kBlockMax = 1u << 17;  // Block_Maximum_Size (128 KiB)
constexpr int kLLMaxAL = 9, kMLMaxAL = 9, kOFMaxAL = 8;
constexpr uint32_t kSeqChunk = 256;      // sequences decoded before a parallel execution pass
constexpr uint32_t kChunkOut = 4096;     // output bytes per chunk covered by the byte map
constexpr uint32_t kChunkClose = 3072;   // a chunk takes no more sequences past this output

enum : int32_t { kOK = 0, kErr = 1, kCap = 2, kSlow = 3, kDefer = 4 };
#ifdef OKV_ZSTD_TRACE
// diagnostic build (make ablate ZTRACE=1): every corrupt-input exit records
// its source line (okv_debug_zstd_err, tools/zdebug.py).  The records change
// the inlined code's shape, and with them the failures of DESIGN.md 13.2.
__device__ int g_zerr[4];  // last line, count
__device__ __forceinline__ int32_t zerr_at(int line) {
  if ((threadIdx.x & 63) == 0) {
    g_zerr[0] = line;
    atomicAdd(&g_zerr[1], 1);
  }
  return kErr;
}
#define ZERR zerr_at(__LINE__)
__device__ __forceinline__ int32_t zfail_at(int line, int32_t v) {
  if ((threadIdx.x & 63) == 0) {
    if (g_zerr[2] == 0) g_zerr[2] = line;  // the innermost failure (first recorded)
    g_zerr[3] = line;
  }
  return v;
}
#define ZFAIL(v) zfail_at(__LINE__, (v))
#else
#define ZERR kErr
#define ZFAIL(v) (v)
#endif
// kSlow: the prologue stage hands the block to the general kernel; kDefer: its
// sequences are decoded by the lane-per-block stage and executed by the
// parallel executor (okv_zstd_seq_kernel, okv_zstd_exec_kernel).

// Literals_Length and Match_Length baselines / extra bits (RFC 8878 3.1.1.3.2.1.1).
__constant__ uint32_t LL_BASE[36] = {0,  1,  2,   3,   4,   5,    6,    7,    8,    9,     10,    11,
                                     12, 13, 14,  15,  16,  18,   20,   22,   24,   28,    32,    40,
                                     48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t LL_BITS[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t ML_BASE[53] = {3,  4,  5,  6,  7,  8,  9,  10,  11,  12,  13,   14,   15,   16,
                                     17, 18, 19, 20, 21, 22, 23, 24,  25,  26,  27,   28,   29,   30,
                                     31, 32, 33, 34, 35, 37, 39, 41,  43,  47,  51,   59,   67,   83,
                                     99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t ML_BITS[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                                    2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
// Predefined distributions (RFC 8878 3.1.1.3.2.2).
__constant__ int16_t LL_DEF[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1,  1,  2,  2,
                                   2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t ML_DEF[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1,  1,  1,  1,  1,  1,  1,  1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,  1,  1,  1,  1,  1,  1,  1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t OF_DEF[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1,  1,  1,  1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

// FSE decoding table entry: symbol | nbBits << 8 | baseline << 16.
__device__ __forceinline__ uint32_t fse_sym(uint32_t e) { return e & 0xff; }
__device__ __forceinline__ uint32_t fse_nb(uint32_t e) { return (e >> 8) & 0xff; }
__device__ __forceinline__ uint32_t fse_base(uint32_t e) { return (e >> 16) & 0x1ff; }
__device__ __forceinline__ uint32_t fse_xb(uint32_t e) { return e >> 25; }

struct __align__(16) SmemCore {
  // FSE states: symbol | nbBits << 8 | nextState baseline << 16 (9 bits) | extra bits << 25
  uint32_t ll[1 << kLLMaxAL];
  uint32_t ml[1 << kMLMaxAL];
  uint32_t of[1 << kOFMaxAL];
  uint32_t hw[1 << 6];         // FSE table of the Huffman weights (AL <= 6)
  uint16_t huf[1 << kHufMaxBits];
  uint16_t next[64];           // FSE build scratch (symbolNext)
  int16_t norm[64];            // normalized counts
  uint8_t wgt[256];            // Huffman weights
  uint16_t hstart[256];        // first decoding-table entry of each symbol
  uint32_t rank[kHufMaxBits + 2];
};
struct __align__(16) Smem : SmemCore {
  // one chunk of decoded sequences (phase A) for parallel execution (phase B):
  // phase A writes {ll, ml, off, -}; the scan rewrites {opre, ll, off, lpre}
  // (output / literal prefix of the chunk); rec[cnt] = {osum, 0, 0, lsum}
  uint4 rec[kSeqChunk + 1];
  uint8_t map[kChunkOut];      // chunk output byte -> its sequence (low 8 bits)
};

// ---- byte access -------------------------------------------------------------
// Bytes [i, i+4) of p with every byte outside [0, n) read as 0; only aligned
// dwords holding a byte of [0, n) are loaded.
__device__ __forceinline__ uint32_t ld32z(const uint8_t* p, int64_t i, int64_t n) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p) + uintptr_t(i);
  const uintptr_t base = reinterpret_cast<uintptr_t>(p);
  const uintptr_t end = base + uintptr_t(n);
  const uintptr_t w0 = a & ~uintptr_t(3), w1 = w0 + 4;
  const uint32_t sh = uint32_t(a & 3);
  uint32_t x = 0, y = 0;
  if (int64_t(w0 + 4) > int64_t(base) && w0 < end) x = *reinterpret_cast<const uint32_t*>(w0);
  if (sh && int64_t(w1 + 4) > int64_t(base) && w1 < end) y = *reinterpret_cast<const uint32_t*>(w1);
  uint32_t v = sh ? __builtin_amdgcn_alignbyte(y, x, sh) : x;
  // zero the bytes outside [0, n)
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (i + k < 0 || i + k >= n) v &= ~(0xffu << (8 * k));
  return v;
}
__device__ __forceinline__ uint64_t ld64z(const uint8_t* p, int64_t i, int64_t n) {
  return uint64_t(ld32z(p, i, n)) | (uint64_t(ld32z(p, i + 4, n)) << 32);
}
__device__ __forceinline__ uint32_t rd8(const uint8_t* p) { return *p; }

// Wave-uniform values into scalar registers: the sequential decode then runs
// on the SALU instead of 4-cycle wave64 VALU instructions.
__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
  return uint64_t(rfl(uint32_t(x))) | (uint64_t(rfl(uint32_t(x >> 32))) << 32);
}
// Values the compiler cannot prove wave-uniform (anything derived from a flat
// load) are re-declared uniform, so the serial decode stays in SGPRs / SALU.
__device__ __forceinline__ int64_t rfls64(int64_t x) { return int64_t(rfl64(uint64_t(x))); }
template <class T>
__device__ __forceinline__ T* rflp(T* p) {
  return reinterpret_cast<T*>(rfl64(reinterpret_cast<uint64_t>(p)));
}

// ---- backward bit reader (FSE / Huffman streams) --------------------------------
// Stream bytes [0, n) of p; bit i of the stream = bit (i & 7) of byte i >> 3.
// Reading consumes from the top: read(n) returns bits [pos - n, pos) and
// lowers pos; bits below 0 read as 0 (the "overflow" tail of RFC 8878 4.2.1.2).
struct BitR {
  const uint8_t* p;
  int64_t n;     // stream bytes
  int64_t pos;   // remaining bits
  int64_t lo;    // container holds bits [lo, lo + 64)
  uint64_t c;
};

__device__ __forceinline__ bool bitr_init(BitR& b, const uint8_t* p, int64_t n) {
  b.p = p;
  b.n = n;
  b.lo = INT64_MAX / 4;  // forces the first fill
  b.c = 0;
  b.pos = 0;
  if (n <= 0) return false;
  const uint32_t last = p[n - 1];
  if (last == 0) return false;  // the final byte holds the end marker
  b.pos = (n - 1) * 8 + (31 - __builtin_clz(last));
  return true;
}
// Container = the 8 bytes ending at the byte boundary at or above bit `top`.
__device__ __forceinline__ void bitr_fill(BitR& b, int64_t top) {
  const int64_t top_byte = (top + 7) >> 3;  // floor division for negatives is fine here
  const int64_t lo_byte = top_byte - 8;
  b.lo = lo_byte * 8;
  b.c = ld64z(b.p, lo_byte, b.n);
}
// Bits [pos - nb, pos) (nb <= 32), consumed.
__device__ __forceinline__ uint32_t bitr_read(BitR& b, uint32_t nb) {
  if (nb == 0) return 0;
  b.pos -= nb;
  if (b.pos < b.lo || b.pos + nb > b.lo + 64) bitr_fill(b, b.pos + nb);
  return uint32_t((b.c >> (b.pos - b.lo)) & ((uint64_t(1) << nb) - 1));
}
// Wave-uniform variant (sequence streams): container and positions in SGPRs.
__device__ __forceinline__ uint32_t bitr_read_u(BitR& b, uint32_t nb) {
  if (nb == 0) return 0;
  b.pos -= nb;
  if (b.pos < b.lo || b.pos + nb > b.lo + 64) {
    const int64_t top_byte = (b.pos + nb + 7) >> 3;
    const int64_t lo_byte = top_byte - 8;
    b.lo = lo_byte * 8;
    b.c = rfl64(ld64z(b.p, lo_byte, b.n));
  }
  return uint32_t((b.c >> (b.pos - b.lo)) & ((uint64_t(1) << nb) - 1));
}
// Bits [pos - nb, pos), not consumed.
__device__ __forceinline__ uint32_t bitr_peek(BitR& b, uint32_t nb) {
  const int64_t p0 = b.pos - nb;
  if (p0 < b.lo || b.pos > b.lo + 64) bitr_fill(b, b.pos);
  return uint32_t((b.c >> (p0 - b.lo)) & ((uint64_t(1) << nb) - 1));
}
__device__ __forceinline__ void bitr_skip(BitR& b, uint32_t nb) { b.pos -= nb; }

// Wave register window over a short stream (table descriptions): 256 bytes
// from the stream's aligned base, one dword per lane, bytes outside [0, n)
// zero.  Reads are wave-uniform: v_readlane of the two dwords around a bit
// position, so a serial header decode waits on no memory after the one load.
struct RegWin {
  uint32_t w;     // this lane's dword
  int32_t boff;   // window bit of the stream's bit 0
};
// Every lane's dword is computed with the whole wave active and no branch:
// the window is read back by v_readlane from arbitrary lanes, and a lane that
// was inactive when its VGPR was written holds no defined value (DESIGN.md
// 15.3).  Lanes past the stream load the stream's first dword (always
// readable) and select 0.
__device__ __forceinline__ RegWin regwin_load(const uint8_t* p, int64_t n) {
  const uintptr_t pa = reinterpret_cast<uintptr_t>(p), base = pa & ~uintptr_t(3);
  const uintptr_t a = base + 4 * (threadIdx.x & 63);
  const int64_t rel = int64_t(a) - int64_t(pa);  // stream byte of the dword's first byte
  const bool in = rel + 4 > 0 && rel < n;
  const uint32_t x = *reinterpret_cast<const uint32_t*>(in ? a : base);
  uint32_t keep = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) keep |= (rel + k >= 0 && rel + k < n) ? (0xffu << (8 * k)) : 0u;
  return RegWin{in ? (x & keep) : 0u, int32_t(8 * (pa - base))};
}
// Window bits fit: stream bits [b, b + 32) lie below the window's end.
__device__ __forceinline__ bool regwin_has(const RegWin& r, int64_t b) {
  return r.boff + b + 32 <= 64 * 32;
}
// Stream bits [b, b + 32) (b may be negative: bits below the stream read 0).
__device__ __forceinline__ uint32_t regwin_get32(const RegWin& r, int32_t b) {
  const int32_t A = r.boff + b;
  const int32_t d = A >> 5;
  const uint32_t lo = __builtin_amdgcn_readlane(r.w, d & 63);
  const uint32_t hi = __builtin_amdgcn_readlane(r.w, (d + 1) & 63);
  return __builtin_amdgcn_alignbit(d + 1 >= 0 && d + 1 < 64 ? hi : 0u, d >= 0 && d < 64 ? lo : 0u,
                                   uint32_t(A) & 31u);
}

// ---- FSE ---------------------------------------------------------------------
// FSE_readNCount (RFC 8878 4.1.1): forward bitstream at p[0, n); fills norm[]
// (max_sym + 1 entries), returns bytes consumed or -1.
__device__ int32_t read_ncount(const uint8_t* p, int64_t n, int16_t* norm, uint32_t max_sym,
                               uint32_t max_al, uint32_t& al_out, uint32_t& nsym_out) {
  int64_t bit = 0;
  const RegWin win = regwin_load(p, n);  // the description is read from registers
  auto peek = [&](uint32_t k) -> uint32_t {  // k <= 10
    if (regwin_has(win, bit))
      return regwin_get32(win, int32_t(bit)) & ((1u << k) - 1u);
    const uint64_t v = ld64z(p, bit >> 3, n) >> (bit & 7);
    return rfl(uint32_t(v & ((uint64_t(1) << k) - 1)));  // (a flat load: uniform by fiat)
  };
  const uint32_t al = peek(4) + 5;
  bit += 4;
  if (al > max_al) return ZFAIL(-1);
  int32_t remaining = (1 << al) + 1;
  int32_t threshold = 1 << al;
  uint32_t nbits = al + 1;
  uint32_t s = 0;
  while (remaining > 1) {
    if (s > max_sym) return ZFAIL(-1);
    const int32_t max = 2 * threshold - 1 - remaining;
    int32_t count;
    const uint32_t v = peek(nbits);
    if (int32_t(v & uint32_t(threshold - 1)) < max) {
      count = int32_t(v & uint32_t(threshold - 1));
      bit += nbits - 1;
    } else {
      count = int32_t(v & uint32_t(2 * threshold - 1));
      if (count >= threshold) count -= max;
      bit += nbits;
    }
    count -= 1;  // probability; -1 = "less than 1"
    remaining -= count < 0 ? -count : count;
    norm[s++] = int16_t(count);
    if (count == 0) {  // 2-bit repeat flags of zero probabilities
      for (;;) {
        const uint32_t r = peek(2);
        bit += 2;
        for (uint32_t k = 0; k < r; ++k) {
          if (s > max_sym) return ZFAIL(-1);
          norm[s++] = 0;
        }
        if (r != 3) break;
      }
    }
    while (remaining < threshold) {
      --nbits;
      threshold >>= 1;
    }
    if ((bit >> 3) > n) return ZFAIL(-1);
  }
  if (remaining != 1) return ZFAIL(-1);
  al_out = al;
  nsym_out = s;
  return int32_t((bit + 7) >> 3);
}

// Build an FSE decoding table from normalized counts (RFC 8878 4.1.1), with
// the whole wave (called wave-uniformly by the 64 lanes of a one-wave
// workgroup; every alphabet here has <= 64 symbols: LL 36, ML 53, OF 32,
// Huffman weights 16).  The reference procedure is three serial loops; each is
// restated in parallel:
//  * low-probability symbols (count -1) take the top cells in symbol order:
//    cell size - 1 - (their rank among the low symbols);
//  * the spread visits positions (j * step) & mask for j = 0, 1, ..., skipping
//    positions above the low cells; the k-th visited valid position holds the
//    symbol s with cum[s] <= k < cum[s + 1] (counts in symbol order), so every
//    j is placed independently (a ballot counts the valid positions before it);
//  * cell u of symbol s gets state x = next[s] + (cells of s before u): the
//    cells of s in a 64-cell chunk are found by six ballots over the symbol's
//    bits, and each symbol's last cell in the chunk advances next[s].
// The serial walk returns to position 0 exactly when the positive counts fill
// the cells below the low ones; that is the check here.
__device__ bool build_fse(uint32_t* table, const int16_t* norm, uint32_t nsym, uint32_t al,
                          uint16_t* next) {
  __shared__ uint16_t s_cum[64];  // first placement of each symbol
  nsym = rfl(nsym);  // (uniform: every branch below holds a ballot, DPP or barrier)
  al = rfl(al);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t size = 1u << al, mask = size - 1;
  const uint64_t below = (uint64_t(1) << lane) - 1;
  auto mbcnt = [](uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
  };
  const bool has = lane < nsym;
  const int32_t nv = has ? int32_t(norm[lane]) : 0;
  const bool low = nv == -1;
  const uint64_t lowm = __ballot(low);
  const int32_t high = int32_t(size) - 1 - int32_t(__builtin_popcountll(lowm));
  if (low) table[size - 1 - mbcnt(lowm)] = lane;
  if (has) next[lane] = low ? uint16_t(1) : uint16_t(nv);
  const uint32_t c = nv > 0 ? uint32_t(nv) : 0u;
  const uint32_t inc = wave_scan_dpp(c);
  const uint32_t total = __builtin_amdgcn_readlane(inc, 63);
  s_cum[lane] = uint16_t(inc - c);
  __syncthreads();
  if (int32_t(total) != high + 1) return ZFAIL(false);
  const uint32_t step = (size >> 1) + (size >> 3) + 3;
  uint32_t carry = 0;
  for (uint32_t j0 = 0; j0 < size; j0 += 64) {
    const uint32_t j = j0 + lane;
    const uint32_t pos = (j * step) & mask;
    const bool valid = j < size && int32_t(pos) <= high;
    const uint64_t vm = __ballot(valid);
    if (valid) {
      const uint32_t k = carry + mbcnt(vm);
      uint32_t lo = 0, hi = nsym;  // cum[lo] <= k < cum[hi] (cum[nsym] = total)
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_cum[mid] <= k)
          lo = mid;
        else
          hi = mid;
      }
      table[pos] = lo;
    }
    carry += uint32_t(__builtin_popcountll(vm));
  }
  __syncthreads();
  for (uint32_t u0 = 0; u0 < size; u0 += 64) {
    const uint32_t u = u0 + lane;
    const bool in = u < size;
    const uint32_t s = in ? (table[u] & 0xffu) : 0u;
    uint64_t same = __ballot(in);
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const bool bit = (s >> b) & 1u;
      const uint64_t bb = __ballot(bit);
      same &= bit ? bb : ~bb;
    }
    const uint32_t x = (in ? uint32_t(next[s]) : 0u) + mbcnt(same);
    if (in) {
      const uint32_t nb = al - (31 - __builtin_clz(x));
      const uint32_t base = (x << nb) - size;
      table[u] = s | (nb << 8) | (base << 16);
      if ((same & ~below & ~(uint64_t(1) << lane)) == 0) next[s] = uint16_t(x + 1);
    }
  }
  __syncthreads();
  return true;
}

__device__ __forceinline__ void build_rle(uint32_t* table, uint32_t sym) {
  if ((threadIdx.x & 63) == 0) table[0] = sym;  // AL 0: one state, no bits
  __syncthreads();
}

// ---- Huffman -------------------------------------------------------------------
// Huffman tree description (RFC 8878 4.2.1).  Returns bytes consumed or -1;
// sets max_bits.
__device__ int32_t read_huf_tree(SmemCore& sm, const uint8_t* p, int64_t n, uint32_t& max_bits) {
  if (n < 1) return -1;
  const uint32_t hb = rfl(p[0]);
  uint32_t nw;  // weights given explicitly (the last one is implied)
  int32_t used;
  const bool w0 = (threadIdx.x & 63) == 0;
  if (hb >= 128) {  // direct 4-bit weights
    nw = hb - 127;
    used = 1 + int32_t((nw + 1) / 2);
    if (used > n) return -1;
    for (uint32_t i = threadIdx.x & 63; i < nw; i += 64) {
      const uint32_t byte = p[1 + i / 2];
      sm.wgt[i] = uint8_t((i & 1) ? (byte & 15) : (byte >> 4));
    }
  } else {  // FSE-compressed weights, two interleaved states
    const int64_t csz = hb;
    if (1 + csz > n) return -1;
    uint32_t al, nsym;
    const int32_t hlen = read_ncount(p + 1, csz, sm.norm, 15, 6, al, nsym);
    if (hlen < 0) return -1;
    __syncthreads();  // norm[] (every lane's stores) before the build reads it
    if (!build_fse(sm.hw, sm.norm, nsym, al, sm.next)) return -1;
    // The weight stream (< 128 bytes) and the table (<= 64 states, lane =
    // state) live in registers: the serial decode below reads both with
    // v_readlane, no memory round trip per weight (bits below the stream
    // read as 0, RFC 8878 4.2.1.2).
    const int64_t wn = csz - hlen;
    if (wn <= 0) return -1;
    const RegWin win = regwin_load(p + 1 + hlen, wn);
    const uint32_t last = regwin_get32(win, int32_t(8 * (wn - 1))) & 0xffu;
    if (last == 0) return -1;  // the final byte holds the end marker
    int32_t pos = int32_t(8 * (wn - 1)) + (31 - __builtin_clz(last));
    const uint32_t hwv = sm.hw[(threadIdx.x & 63) & ((1u << al) - 1u)];
    auto rd = [&](uint32_t k) -> uint32_t {  // bits [pos - k, pos), consumed (k <= 6)
      pos -= int32_t(k);
      return k ? (regwin_get32(win, pos) & ((1u << k) - 1u)) : 0u;
    };
    auto ent = [&](uint32_t st) { return uint32_t(__builtin_amdgcn_readlane(hwv, st & 63u)); };
    uint32_t s1 = rd(al), s2 = rd(al);
    nw = 0;
    for (;;) {
      if (nw >= 255) return -1;
      uint32_t e = ent(s1);
      if (w0) sm.wgt[nw] = uint8_t(fse_sym(e));
      ++nw;
      s1 = fse_base(e) + rd(fse_nb(e));
      if (pos < 0) {  // overflow: the other state's symbol ends the list
        if (w0) sm.wgt[nw] = uint8_t(fse_sym(ent(s2)));
        ++nw;
        break;
      }
      if (nw >= 255) return -1;
      e = ent(s2);
      if (w0) sm.wgt[nw] = uint8_t(fse_sym(e));
      ++nw;
      s2 = fse_base(e) + rd(fse_nb(e));
      if (pos < 0) {
        if (w0) sm.wgt[nw] = uint8_t(fse_sym(ent(s1)));
        ++nw;
        break;
      }
    }
    used = 1 + int32_t(csz);
  }
  __syncthreads();
  // From here on the whole wave works in parallel (64 symbols per chunk; the
  // reference's loops are serial over the symbols, HUF_readStats /
  // HUF_readDTableX1 in libzstd).
  const uint32_t lane = threadIdx.x & 63;
  // implied last weight: the weights' 2^(w-1) must sum to a power of two
  uint32_t part = 0;
  bool wbad = false;
  for (uint32_t i = lane; i < nw; i += 64) {
    const uint32_t w = sm.wgt[i];
    wbad |= w > uint32_t(kHufMaxBits);
    part += w ? (1u << (w - 1)) : 0u;
  }
  if (__any(wbad)) return -1;
  for (int d = 32; d; d >>= 1) part += __shfl_xor(part, d, 64);
  const uint32_t sum = part;
  if (sum == 0) return -1;
  const uint32_t mb = 32 - __builtin_clz(sum);  // highbit(sum) + 1
  if (mb > kHufMaxBits) return -1;
  const uint32_t left = (1u << mb) - sum;
  if (left == 0 || (left & (left - 1))) return -1;
  const uint32_t lastw = 31 - __builtin_clz(left) + 1;
  if (w0) sm.wgt[nw] = uint8_t(lastw);
  const uint32_t nsym = nw + 1;
  __syncthreads();
  // per weight: symbol counts, then each symbol's rank among the symbols of
  // its weight (symbol order), by ballots over 64-symbol chunks
  uint32_t cnt[kHufMaxBits + 1];
#pragma unroll
  for (int w = 0; w <= kHufMaxBits; ++w) cnt[w] = 0;
  for (uint32_t c0 = 0; c0 < nsym; c0 += 64) {
    const uint32_t i = c0 + lane;
    const uint32_t w = i < nsym ? sm.wgt[i] : 0u;
#pragma unroll
    for (int k = 0; k <= kHufMaxBits; ++k) cnt[k] += uint32_t(__builtin_popcountll(__ballot(w == uint32_t(k) && i < nsym)));
  }
  // libzstd HUF_readStats: at least two weight-1 symbols, and an even count
  if (cnt[1] < 2 || (cnt[1] & 1)) return -1;
  // decoding table: entries grouped by weight ascending, symbols ascending
  // within a weight; a symbol of weight w covers 2^(w-1) entries, nbBits = mb + 1 - w
  uint32_t wstart[kHufMaxBits + 1];
  {
    uint32_t start = 0;
#pragma unroll
    for (int w = 0; w <= kHufMaxBits; ++w) {
      wstart[w] = start;
      if (w >= 1 && uint32_t(w) <= mb) start += cnt[w] << (w - 1);
    }
  }
  uint32_t run[kHufMaxBits + 1];
#pragma unroll
  for (int w = 0; w <= kHufMaxBits; ++w) run[w] = 0;
  for (uint32_t c0 = 0; c0 < nsym; c0 += 64) {
    const uint32_t i = c0 + lane;
    const uint32_t w = i < nsym ? sm.wgt[i] : 0u;
    uint32_t st = 0;
#pragma unroll
    for (int k = 1; k <= kHufMaxBits; ++k) {
      const uint64_t m = __ballot(w == uint32_t(k) && i < nsym);
      const uint32_t before = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32),
                                                        __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
      if (w == uint32_t(k)) st = wstart[k] + ((run[k] + before) << (k - 1));
      run[k] += uint32_t(__builtin_popcountll(m));
    }
    if (i < nsym) sm.hstart[i] = uint16_t(st);
  }
  __syncthreads();
  // fill: symbols of <= 32 entries one per lane; longer ones by the whole wave
  uint64_t bigm[4] = {0, 0, 0, 0};
  for (uint32_t c0 = 0, q = 0; c0 < nsym; c0 += 64, ++q) {
    const uint32_t i = c0 + lane;
    const uint32_t w = i < nsym ? sm.wgt[i] : 0u;
    const bool small = w >= 1 && w <= 6;
    bigm[q] = __ballot(w > 6);
    if (small) {
      const uint32_t len = 1u << (w - 1), st = sm.hstart[i];
      const uint16_t ent = uint16_t(i | ((mb + 1 - w) << 8));
      for (uint32_t k = 0; k < len; ++k) sm.huf[st + k] = ent;
    }
  }
  for (uint32_t q = 0; q < 4; ++q) {
    uint64_t m = bigm[q];
    while (m) {
      const uint32_t i = 64 * q + uint32_t(__builtin_ctzll(m));
      m &= m - 1;
      const uint32_t w = sm.wgt[i];
      const uint32_t len = 1u << (w - 1), st = sm.hstart[i];
      const uint16_t ent = uint16_t(i | ((mb + 1 - w) << 8));
      for (uint32_t k = lane; k < len; k += 64) sm.huf[st + k] = ent;
    }
  }
  __syncthreads();
  max_bits = mb;
  return used;
}

// Decode one Huffman stream of `cnt` literals into out (this lane only).  The
// stream is read backward as aligned dwords: a 64-bit container plus eight
// dwords prefetched below it, so a refill rarely waits on memory (a literal
// takes <= 11 bits; a fresh load per container refill made the decode a chain
// of memory round trips).  Bits below the stream read as 0 (RFC 8878 4.2.1.2).
__device__ __forceinline__ bool huf_stream(const uint16_t* huf, uint32_t mb, const uint8_t* p, int64_t n,
                                           uint8_t* out, uint32_t cnt) {
  if (n <= 0) return cnt == 0 && n == 0;
  const uint32_t last = p[n - 1];
  if (last == 0) return false;  // the final byte holds the end marker
  // (pointer arithmetic, not an integer round trip: the address space of p
  // -- global -- then reaches the loads)
  const int32_t s0 = int32_t(reinterpret_cast<uintptr_t>(p) & 3), B0 = 8 * s0;  // bit 0, relative to ab
  const uint32_t* ab = reinterpret_cast<const uint32_t*>(p - s0);
  int32_t P = B0 + int32_t(n - 1) * 8 + (31 - __builtin_clz(last));
  int32_t cd = (P >> 5) - 1;  // the container holds dwords cd + 1 : cd
  auto raw = [&](int32_t d) { return ab[d < 0 ? 0 : d]; };
  auto fix = [&](uint32_t v, int32_t d) {  // bytes below the stream read as 0
    const int32_t cut = min(max(s0 - 4 * d, 0), 4);
    return cut >= 4 ? 0u : (v & (0xffffffffu << (8 * cut)));
  };
  uint64_t c = (uint64_t(fix(raw(cd + 1), cd + 1)) << 32) | fix(raw(cd), cd);
  uint32_t r[8];  // raw dwords cd - 1 - k
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = raw(cd - 1 - k);
  auto refill = [&](int32_t need) {  // make bits [P - need, P) available
    if (P - need < 32 * cd) {
      c = (c << 32) | fix(r[0], cd - 1);
      --cd;
#pragma unroll
      for (int k = 0; k < 7; ++k) r[k] = r[k + 1];
      r[7] = raw(cd - 8);
    }
  };
  auto literal = [&]() {
    const int32_t p0 = P - int32_t(mb);
    const uint32_t idx = uint32_t(c >> uint32_t(p0 - 32 * cd)) & ((1u << mb) - 1u);
    const uint32_t e = huf[idx];
    P -= int32_t(e >> 8);
    return e & 0xffu;
  };
  // invariant: 32 cd <= P < 32 cd + 64; a literal takes <= mb <= 11 bits, so
  // one refill check (at most one dword) covers two literals: the lanes are
  // different streams, and each check is a divergent branch.  Literals are
  // stored four to a dword store once the output is aligned (a byte store per
  // literal was a store instruction per literal).
  uint32_t i = 0;
  const uint32_t head = min(cnt, (4u - uint32_t(reinterpret_cast<uintptr_t>(out) & 3)) & 3u);
  for (; i < head; ++i) {
    refill(int32_t(mb));
    out[i] = uint8_t(literal());
  }
  for (; i + 3 < cnt; i += 4) {
    refill(2 * int32_t(mb));
    const uint32_t b0 = literal();
    const uint32_t b1 = literal();
    refill(2 * int32_t(mb));
    const uint32_t b2 = literal();
    const uint32_t b3 = literal();
    *reinterpret_cast<uint32_t*>(out + i) = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
  }
  for (; i < cnt; ++i) {
    refill(int32_t(mb));
    out[i] = uint8_t(literal());
  }
  return P == B0;
}

// ---- one zstd block -----------------------------------------------------------
struct FrameState {
  uint32_t rep0, rep1, rep2;  // repeat offsets (3.1.1.5)
  bool huf_ok;       // a Huffman table is available for treeless literals
  uint32_t huf_bits;
  bool ll_ok, of_ok, ml_ok;  // tables available for Repeat mode
  uint32_t ll_al, of_al, ml_al;
};

struct Out {
  unsigned long long* prof;  // diagnostic phase counters (OKV_ZSTD_PROF), or null
  uint8_t* base;       // this segment block's decompressed region
  uint64_t cap;
  uint64_t pos;        // bytes written
  uint64_t committed;  // bytes known visible to every lane
  uint64_t frame0;     // first output byte of the current frame
  uint32_t bmax;       // Block_Maximum_Size of the current frame (RFC 8878 3.1.1.2.4)
  bool dry;            // measuring pass: positions advance, no byte is read or written
};

// Per segment block, written by the prologue (okv_zstd_pro_kernel) for the
// sequence stage and the executor.
enum : int32_t { kKindDone = 0, kKindSeq = 1, kKindSlow = 2 };
enum : uint32_t { kFlagFcs = 1, kFlagCsum = 2, kFlagRle = 4, kFlagHuf = 8 };
// Sequence-stage tables, 16 bits per state: symbol (6 bits) | the state's
// FSE "next state" value x (10 bits; x in [count, 2 count), so < 2^(AL+1)).
// nbBits = AL - floor(log2 x) and baseline = (x << nbBits) - 2^AL follow, so
// 64 blocks' tables (160 KiB) fit one CU's LDS.
constexpr uint32_t kTabEnt = 1280;  // LL [0, 512), OF [512, 768), ML [768, 1280)
__device__ __forceinline__ uint16_t fse_pack16(uint32_t e, uint32_t al) {
  const uint32_t x = (fse_base(e) + (1u << al)) >> fse_nb(e);
  return uint16_t(fse_sym(e) | (x << 6));
}
struct ZBlk {
  const uint8_t* stream;  // sequence bitstream
  const uint8_t* lits;    // literal bytes (unused with kFlagRle)
  uint64_t fcs;           // Frame_Content_Size (kFlagFcs)
  uint32_t stream_len, nseq, lit_total, cap;
  uint32_t csum;          // stored content checksum (kFlagCsum)
  uint32_t flags;
  uint32_t ll_al, of_al, ml_al, rle_byte;
  int32_t kind;           // kKindDone / kKindSeq / kKindSlow
  int32_t st;             // kOK / kErr / kCap of the stage that owns the block
  uint32_t nseq_ok;       // sequences the sequence stage decoded (all unless the stream overflowed)
  uint32_t pfix;          // bit 31: the last one read past the stream's start: its position (bits
                          // 0-20) and offset code (21-25)
  uint32_t bmax;          // Block_Maximum_Size of the block's frame (<= 128 KiB)
  // kFlagHuf: the Huffman literal streams are left to okv_zstd_huf_kernel
  uint64_t hq_off;        // the first stream (after the jump table), from the segment's start
  uint32_t hlen[4];       // stream sizes (one stream: hlen[0], the rest 0)
  uint32_t hmb;           // the table's Max_Number_of_Bits
  uint32_t hns;           // streams: 1 or 4
};
constexpr uint32_t kHufSlot = 1u << kHufMaxBits;  // u16 decoding-table entries per deferred block

// Prologue context of one block: per-block literal scratch and table slots.
struct Pro {
  uint8_t* lit_blk;   // literal scratch of this segment block (lit_cap bytes)
  uint64_t lit_cap;
  uint16_t* tabs;     // kTabEnt packed states of this block (fse_pack16)
  ZBlk* zb;
  bool deferrable;    // the compressed block being decoded may be deferred
  uint64_t fcs;
  uint32_t fcs_on, csum_on;
  const uint8_t* seg;
  uint16_t* htab;     // kHufSlot entries: this block's Huffman decoding table for the stream stage
  const uint8_t* hq;  // deferred literal streams (huf_on)
  uint32_t hlen[4], hmb, hns, huf_on;
  uint32_t nseq;      // out: the deferred block's sequence count (lane 0)
};

__device__ __forceinline__ void prof_add(const Out& o, int k, unsigned long long v) {
  if (o.prof && (threadIdx.x & 63) == 0) atomicAdd(o.prof + k, v);
}

__device__ __forceinline__ void commit(Out& o) {
  prof_add(o, 5, 1);
  __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
  __threadfence_block();
  o.committed = o.pos;
}

// Lane-parallel byte copy of n bytes from src (global) to the output.
__device__ __forceinline__ void out_copy(Out& o, const uint8_t* src, uint64_t n) {
  const int lane = threadIdx.x & 63;
  if (!o.dry)
    for (uint64_t j = lane; j < n; j += 64) o.base[o.pos + j] = src[j];
  o.pos += n;
}

// Extra-bits count of each state's symbol into bits 25..29 of its entry, so the
// sequence loop reads one LDS word per state.  kind: 0 LL, 1 OF, 2 ML.
__device__ void seq_xbits(uint32_t* table, uint32_t al, int kind) {
  const int lane = threadIdx.x & 63;
  for (uint32_t u = lane; u < (1u << al); u += 64) {
    const uint32_t e = table[u] & 0x1ffffffu, c = fse_sym(e);
    const uint32_t bits = kind == 0 ? LL_BITS[c < 36 ? c : 0] : kind == 1 ? c : ML_BITS[c < 53 ? c : 0];
    table[u] = e | (bits << 25);
  }
  __syncthreads();
}

// ---- wave-uniform backward bit reader of the sequence stream ------------------
// The container (64 bits) and positions live in SGPRs; refills read a 256-byte
// window held in one VGPR (lane l = aligned dword wdw + l) with v_readlane, so
// the serial sequence loop touches memory once per ~256 stream bytes.  A refill
// leaves >= 57 bits in the container; a sequence reads at most 89 bits, so the
// loop refills twice per sequence and the reads themselves are shift + mask.
// Streams are < 128 KiB, so positions fit in 32 bits.
struct SeqBits {
  const uint8_t* abase;  // stream start rounded down to 4 bytes
  int32_t s0;            // stream start - abase (0..3)
  int32_t n;             // stream bytes
  int32_t pos;           // remaining bits (relative to the stream start)
  int32_t lo;            // container holds bits [lo, lo + 64)
  uint64_t c;
  int32_t wdw;           // first dword (from abase) of the window
  uint32_t win;
};

__device__ __forceinline__ void seqwin_load(SeqBits& b, int32_t top_dw) {
  const int lane = threadIdx.x & 63;
  b.wdw = top_dw - 63;
  const int32_t d = b.wdw + lane;
  const int32_t lo = 4 * d, hi = lo + 4;  // this lane's bytes, relative to abase
  uint32_t v = 0;
  if (hi > b.s0 && lo < b.s0 + b.n) {
    v = *reinterpret_cast<const uint32_t*>(b.abase + lo);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (lo + k < b.s0 || lo + k >= b.s0 + b.n) v &= ~(0xffu << (8 * k));
  }
  b.win = v;
}

__device__ __forceinline__ void seqbits_fill(SeqBits& b) {
  const int32_t lb = ((b.pos + 7) >> 3) - 8;  // container = stream bytes [lb, lb + 8)
  const int32_t A = b.s0 + lb;
  const int32_t d0 = A >> 2;
  const uint32_t sh = uint32_t(A & 3);
  if (d0 < b.wdw || d0 + 2 > b.wdw + 63) seqwin_load(b, d0 + 2);
  const int i0 = d0 - b.wdw;
  const uint32_t x0 = __builtin_amdgcn_readlane(b.win, i0);
  const uint32_t x1 = __builtin_amdgcn_readlane(b.win, i0 + 1);
  const uint32_t x2 = __builtin_amdgcn_readlane(b.win, i0 + 2);
  const uint64_t w = uint64_t(x0) | (uint64_t(x1) << 32);
  b.c = sh ? (w >> (8 * sh)) | (uint64_t(x2) << (64 - 8 * sh)) : w;
  b.lo = lb * 8;
}

// Refill when fewer than `need` (<= 57) bits are left.
__device__ __forceinline__ void seqbits_reload(SeqBits& b, int32_t need) {
  if (b.pos - b.lo < need) seqbits_fill(b);
}

__device__ __forceinline__ bool seqbits_init(SeqBits& b, const uint8_t* p, int32_t n) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  b.abase = reinterpret_cast<const uint8_t*>(a & ~uintptr_t(3));
  b.s0 = int32_t(a & 3);
  b.n = n;
  b.wdw = INT32_MIN / 8;
  b.pos = 0;
  b.lo = 0;
  b.c = 0;
  b.win = 0;
  if (n <= 0) return false;
  const uint32_t last = rfl(p[n - 1]);
  if (last == 0) return false;  // the final byte holds the end marker
  b.pos = (n - 1) * 8 + (31 - __builtin_clz(last));
  seqbits_fill(b);
  return true;
}

// Bits [pos - nb, pos) (nb <= 31, already in the container), consumed; bits
// below the stream read as 0.
__device__ __forceinline__ uint32_t seqbits_take(SeqBits& b, uint32_t nb) {
  b.pos -= int32_t(nb);
  return uint32_t(b.c >> uint32_t(b.pos - b.lo)) & uint32_t((uint64_t(1) << nb) - 1);
}
__device__ __forceinline__ uint32_t seqbits_read(SeqBits& b, uint32_t nb) {
  if (b.pos - b.lo < int32_t(nb)) seqbits_fill(b);
  return seqbits_take(b, nb);
}

// Table for one of LL / OF / ML from the symbol compression mode.
__device__ int32_t seq_table(SmemCore& sm, uint32_t* table, uint32_t mode, const int16_t* def,
                             uint32_t def_al, uint32_t def_n, uint32_t max_sym, uint32_t max_al,
                             const uint8_t* p, int64_t n, bool& ok, uint32_t& al) {
  mode = rfl(mode);  // (uniform: the table builds hold ballots, DPP and barriers)
  n = rfls64(n);
  switch (mode) {
    case 0: {  // Predefined_Mode
      for (uint32_t s = threadIdx.x & 63; s < def_n; s += 64) sm.norm[s] = def[s];
      __syncthreads();
      if (!build_fse(table, sm.norm, def_n, def_al, sm.next)) return ZFAIL(-1);
      ok = true;
      al = def_al;
      return 0;
    }
    case 1: {  // RLE_Mode
      if (n < 1 || rfl(p[0]) > max_sym) return ZFAIL(-1);
      build_rle(table, rfl(p[0]));
      ok = true;
      al = 0;
      return 1;
    }
    case 2: {  // FSE_Compressed_Mode
      uint32_t nsym;
      const int32_t used = read_ncount(p, n, sm.norm, max_sym, max_al, al, nsym);
      if (used < 0) return ZFAIL(-1);
      __syncthreads();
      if (!build_fse(table, sm.norm, nsym, al, sm.next)) return ZFAIL(-1);
      ok = true;
      return used;
    }
    default:  // Repeat_Mode
      return ok ? 0 : ZFAIL(-1);
  }
}

// Decompress one compressed zstd block (RFC 8878 3.1.1.3) into the output.
template <bool PRO, class SM>
__device__ int32_t compressed_block(SM& sm, FrameState& fs, Out& o, const uint8_t* p, int64_t n,
                                    uint8_t* lit_buf, Pro* pro) {
  p = rflp(p);
  n = rfls64(n);
  o.pos = rfl64(o.pos);
  o.cap = rfl64(o.cap);
  o.frame0 = rfl64(o.frame0);
  if (n < 1) return ZERR;
  // the block's output may not exceed Block_Maximum_Size (RFC 8878 3.1.1.2.4)
  const uint64_t blk_end = o.pos + rfl(o.bmax);
  const long long t0 = o.prof ? clock64() : 0;
  // ---- literals section header (3.1.1.3.1.1)
  const uint32_t b0 = rfl(p[0]);
  const uint32_t ltype = b0 & 3, sf = (b0 >> 2) & 3;
  uint32_t regen = 0, csize = 0, hdr = 0, nstreams = 1;
  if (ltype <= 1) {
    if (sf == 0 || sf == 2) {
      regen = b0 >> 3;
      hdr = 1;
    } else if (sf == 1) {
      if (n < 2) return ZERR;
      regen = (b0 >> 4) + (uint32_t(p[1]) << 4);
      hdr = 2;
    } else {
      if (n < 3) return ZERR;
      regen = (b0 >> 4) + (uint32_t(p[1]) << 4) + (uint32_t(p[2]) << 12);
      hdr = 3;
    }
  } else {
    if (sf <= 1) {
      if (n < 3) return ZERR;
      const uint32_t h = b0 | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16);
      regen = (h >> 4) & 0x3ff;
      csize = (h >> 14) & 0x3ff;
      hdr = 3;
      nstreams = sf == 0 ? 1 : 4;
    } else if (sf == 2) {
      if (n < 4) return ZERR;
      const uint32_t h = b0 | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
      regen = (h >> 4) & 0x3fff;
      csize = h >> 18;
      hdr = 4;
      nstreams = 4;
    } else {
      if (n < 5) return ZERR;
      const uint64_t h = uint64_t(b0) | (uint64_t(p[1]) << 8) | (uint64_t(p[2]) << 16) |
                         (uint64_t(p[3]) << 24) | (uint64_t(p[4]) << 32);
      regen = uint32_t((h >> 4) & 0x3ffff);
      csize = uint32_t((h >> 22) & 0x3ffff);
      hdr = 5;
      nstreams = 4;
    }
  }
  regen = rfl(regen);  // (flat loads: uniform by fiat, as every header field here)
  csize = rfl(csize);
  if (regen > kBlockMax) return ZERR;
  const uint8_t* lits = nullptr;  // literal source for the sequences
  uint8_t rle_byte = 0;
  bool rle = false;
  int64_t at = hdr;
  if (ltype == 0) {  // Raw_Literals_Block
    if (at + regen > n) return ZERR;
    lits = p + at;
    at += regen;
  } else if (ltype == 1) {  // RLE_Literals_Block
    if (at + 1 > n) return ZERR;
    rle_byte = p[at];
    rle = true;
    at += 1;
  } else {  // Compressed / Treeless
    if (at + csize > n) return ZERR;
    if constexpr (PRO) {
      if (regen > pro->lit_cap) return kSlow;  // per-block scratch too small: general kernel
      lit_buf = pro->lit_blk;
    }
    const uint8_t* q = p + at;
    int64_t qn = csize;
    if (ltype == 2) {
      uint32_t mb;
      const long long th = o.prof ? clock64() : 0;
      const int32_t used = read_huf_tree(sm, q, qn, mb);
      if (o.prof) prof_add(o, 12, clock64() - th);
      if (used < 0) return ZERR;
      fs.huf_ok = true;
      fs.huf_bits = mb;
      q += used;
      qn -= used;
    } else if (!fs.huf_ok) {
      return ZERR;
    }
    const int lane = threadIdx.x & 63;
    if constexpr (PRO) {
      // A block whose sequences go to the later stages leaves its streams too:
      // the table to HBM, the streams' places to zb, and okv_zstd_huf_kernel
      // decodes 16 blocks' streams per wave, one lane each (here 4 of the
      // wave's 64 lanes would).  nseq == 0 (the byte after the literals is 0)
      // emits the literals in this stage and decodes them here.
      if (pro->deferrable && at + int64_t(csize) < n && rfl(p[at + csize]) != 0) {
        const uint32_t mb = fs.huf_bits;
        if (nstreams == 4) {
          if (qn < 6) return ZERR;
          const uint32_t s1 = rfl(q[0] | (uint32_t(q[1]) << 8)),
                         s2 = rfl(q[2] | (uint32_t(q[3]) << 8)),
                         s3 = rfl(q[4] | (uint32_t(q[5]) << 8));
          const int64_t s4 = qn - 6 - int64_t(s1) - s2 - s3;
          if (s4 < 0) return ZERR;
          if (3 * ((regen + 3) / 4) > regen) return ZERR;
          pro->hq = q + 6;
          pro->hlen[0] = s1;
          pro->hlen[1] = s2;
          pro->hlen[2] = s3;
          pro->hlen[3] = uint32_t(s4);
        } else {
          pro->hq = q;
          pro->hlen[0] = uint32_t(qn);
          pro->hlen[1] = pro->hlen[2] = pro->hlen[3] = 0;
        }
        pro->hmb = mb;
        pro->hns = nstreams;
        pro->huf_on = 1;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(sm.huf);
        uint32_t* dst = reinterpret_cast<uint32_t*>(pro->htab);
        for (uint32_t u = lane; u < max(1u, (1u << mb) / 2); u += 64) dst[u] = src[u];
        lits = lit_buf;
        at += csize;
        goto sequences;
      }
    }
    bool good = true;
    if (nstreams == 1) {
      if (lane == 0) good = huf_stream(sm.huf, fs.huf_bits, q, qn, lit_buf, regen);
    } else {
      if (qn < 6) return ZERR;
      const uint32_t s1 = rfl(q[0] | (uint32_t(q[1]) << 8)), s2 = rfl(q[2] | (uint32_t(q[3]) << 8)),
                     s3 = rfl(q[4] | (uint32_t(q[5]) << 8));
      const int64_t s4 = qn - 6 - int64_t(s1) - s2 - s3;
      if (s4 < 0) return ZERR;
      const uint32_t seg = (regen + 3) / 4;
      if (3 * seg > regen) return ZERR;
      if (lane < 4) {
        const int64_t off = 6 + (lane > 0 ? s1 : 0) + (lane > 1 ? s2 : 0) + (lane > 2 ? s3 : 0);
        const int64_t len = lane == 0 ? s1 : lane == 1 ? s2 : lane == 2 ? s3 : s4;
        const uint32_t cnt = lane < 3 ? seg : regen - 3 * seg;
        good = huf_stream(sm.huf, fs.huf_bits, q + off, len, lit_buf + lane * seg, cnt);
      }
    }
    // every lane must agree the streams decoded cleanly
    if (__any(!good)) return ZERR;
    __builtin_amdgcn_s_waitcnt(0);
    __threadfence_block();
    lits = lit_buf;
    at += csize;
  }
sequences:
  const long long t1 = o.prof ? clock64() : 0;
  prof_add(o, 0, t1 - t0);
  // ---- sequences section (3.1.1.3.2)
  if (at >= n) return ZERR;
  uint32_t nseq = p[at];
  if (nseq < 128) {
    at += 1;
  } else if (nseq < 255) {
    if (at + 2 > n) return ZERR;
    nseq = ((nseq - 128) << 8) + p[at + 1];
    at += 2;
  } else {
    if (at + 3 > n) return ZERR;
    nseq = p[at + 1] + (uint32_t(p[at + 2]) << 8) + 0x7f00;
    at += 3;
  }
  uint64_t lit_left = regen;
  uint64_t lit_pos = 0;
  auto emit_lits = [&](uint64_t ll) -> bool {
    if (ll > lit_left) return false;
    if (o.pos + ll > o.cap) return false;
    if (rle) {
      const int lane = threadIdx.x & 63;
      if (!o.dry)
        for (uint64_t j = lane; j < ll; j += 64) o.base[o.pos + j] = rle_byte;
      o.pos += ll;
    } else {
      out_copy(o, lits + lit_pos, ll);
    }
    lit_pos += ll;
    lit_left -= ll;
    return true;
  };
  if (nseq == 0) {  // literals only (bytes after the header are not read, as libzstd)
    if (o.pos + lit_left > blk_end) return ZERR;
    if (o.pos + lit_left > o.cap) return kCap;
    emit_lits(lit_left);
    return kOK;
  }
  if constexpr (PRO) {
    if (!pro->deferrable) return kSlow;
  }
  if (at >= n) return ZERR;
  const uint32_t modes = rfl(p[at++]);
  if (modes & 3) return ZERR;  // reserved bits
  int32_t used;
  auto table = [&](auto&&... a) { return seq_table(sm, a...); };
  used = table(sm.ll, modes >> 6, LL_DEF, 6, 36, 35, kLLMaxAL, p + at, n - at, fs.ll_ok, fs.ll_al);
  if (used < 0) return ZERR;
  at += used;
  if ((modes >> 6) != 3) seq_xbits(sm.ll, fs.ll_al, 0);
  used = table(sm.of, (modes >> 4) & 3, OF_DEF, 5, 29, 31, kOFMaxAL, p + at, n - at, fs.of_ok,
               fs.of_al);
  if (used < 0) return ZERR;
  at += used;
  if (((modes >> 4) & 3) != 3) seq_xbits(sm.of, fs.of_al, 1);
  used = table(sm.ml, (modes >> 2) & 3, ML_DEF, 6, 53, 52, kMLMaxAL, p + at, n - at, fs.ml_ok,
               fs.ml_al);
  if (used < 0) return ZERR;
  at += used;
  if (((modes >> 2) & 3) != 3) seq_xbits(sm.ml, fs.ml_al, 2);
  if (o.prof) prof_add(o, 10, clock64() - t1);
  if constexpr (PRO) {
    // hand the sequences to the lane-per-block stage: tables to HBM, setup to zb
    const int lane = threadIdx.x & 63;
    for (uint32_t u = lane; u < (1u << fs.ll_al); u += 64) pro->tabs[u] = fse_pack16(sm.ll[u], fs.ll_al);
    for (uint32_t u = lane; u < (1u << fs.of_al); u += 64)
      pro->tabs[512 + u] = fse_pack16(sm.of[u], fs.of_al);
    for (uint32_t u = lane; u < (1u << fs.ml_al); u += 64)
      pro->tabs[768 + u] = fse_pack16(sm.ml[u], fs.ml_al);
    if (lane == 0) {
      ZBlk& z = *pro->zb;
      z.stream = p + at;
      z.stream_len = uint32_t(n - at);
      z.lits = rle ? nullptr : lits;
      z.nseq = nseq;
      pro->nseq = nseq;
      z.lit_total = regen;
      z.cap = uint32_t(min<uint64_t>(o.cap, 0x7fffffffu));
      z.fcs = pro->fcs;
      z.flags = (pro->fcs_on ? kFlagFcs : 0) | (pro->csum_on ? kFlagCsum : 0) | (rle ? kFlagRle : 0);
      z.ll_al = fs.ll_al;
      z.of_al = fs.of_al;
      z.ml_al = fs.ml_al;
      z.rle_byte = rle_byte;
      z.bmax = o.bmax;
      if (pro->huf_on) {
        z.flags |= kFlagHuf;
        z.hq_off = uint64_t(pro->hq - pro->seg);
        for (int k = 0; k < 4; ++k) z.hlen[k] = pro->hlen[k];
        z.hmb = pro->hmb;
        z.hns = pro->hns;
      }
    }
    return kDefer;
  } else {
  at = rfls64(at);
  nseq = rfl(nseq);
  lit_left = rfl64(lit_left);
  lit_pos = rfl64(lit_pos);
  fs.ll_al = rfl(fs.ll_al);
  fs.of_al = rfl(fs.of_al);
  fs.ml_al = rfl(fs.ml_al);
  fs.rep0 = rfl(fs.rep0);
  fs.rep1 = rfl(fs.rep1);
  fs.rep2 = rfl(fs.rep2);
  SeqBits br;
  if (!seqbits_init(br, p + at, n - at)) return ZERR;
  uint32_t sll = seqbits_read(br, fs.ll_al);
  uint32_t sof = seqbits_read(br, fs.of_al);
  uint32_t sml = seqbits_read(br, fs.ml_al);
  const int lane = threadIdx.x & 63;
  const bool w0 = lane == 0;
  // largest k < cnt with rec[k].x <= x (rec[0].x == 0 <= x)
  auto find = [&](uint32_t cnt, uint32_t x) {
    uint32_t lo = 0, hi = cnt;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (sm.rec[mid].x <= x)
        lo = mid;
      else
        hi = mid;
    }
    return lo;
  };
  uint32_t rep0 = fs.rep0, rep1 = fs.rep1, rep2 = fs.rep2;
  // 32-bit forms of the execution checks (blocks are < 2^31 bytes):
  // literals left, output capacity left, output since the frame start
  const uint32_t lit_lim = uint32_t(min<uint64_t>(lit_left, 0x7fffffffu));
  for (uint32_t i = 0; i < nseq;) {
    // ---- phase A: decode up to kSeqChunk sequences (wave-uniform, SALU) ----
    const long long ta = o.prof ? clock64() : 0;
    const uint32_t cap_lim = uint32_t(min<uint64_t>(o.cap - o.pos, 0x7fffffffu));
    const uint32_t bm_lim = uint32_t(blk_end - o.pos);  // <= 128 KiB
    const uint32_t back = uint32_t(min<uint64_t>(o.pos - o.frame0, 0x7fffffffu));
    const uint32_t lit_done = uint32_t(lit_pos);
    uint32_t cnt = 0, lsum = 0, osum = 0;
    for (; cnt < kSeqChunk && i < nseq && osum < kChunkClose; ++cnt, ++i) {
      if (br.pos < 0) return ZERR;  // libzstd: the stream overflowed before this sequence
      const uint32_t ell = rfl(sm.ll[sll]), eof = rfl(sm.of[sof]), eml = rfl(sm.ml[sml]);
      // extra bits: offset, then match length, then literals length
      seqbits_reload(br, 47);  // offset (<= 31) + match length (<= 16) extra bits
      const uint32_t ofs = fse_sym(eof);
      const uint32_t ofv = (1u << ofs) + seqbits_take(br, ofs);
      const uint32_t mls = fse_sym(eml), lls = fse_sym(ell);
      const uint32_t mlx = seqbits_take(br, fse_xb(eml));
      seqbits_reload(br, 42);  // literals length (<= 16) + three states (<= 26)
      const uint32_t ml = (mls < 32 ? mls + 3 : ML_BASE[mls]) + mlx;
      const uint32_t ll = (lls < 16 ? lls : LL_BASE[lls]) + seqbits_take(br, fse_xb(ell));
      // repeat offsets (3.1.1.5), as libzstd's ZSTD_decodeSequence
      // repeat offsets (RFC 8878 3.1.1.5), branch-free: ofv > 3 is a new
      // offset; else idx = ofv - 1 (+1 when ll == 0) picks rep0/rep1/rep2/rep0-1
      const bool fresh = ofv > 3;
      const uint32_t idx = ofv - 1 + (ll == 0 ? 1u : 0u);  // 0..3 when !fresh
      uint32_t t = idx == 3 ? rep0 - 1 : (idx == 1 ? rep1 : rep2);
      t += t == 0;  // libzstd: offset 0 is corrupt input, forced to 1
      const uint32_t off = fresh ? ofv - 3 : (idx == 0 ? rep0 : t);
      const bool sh1 = fresh || idx != 0, sh2 = fresh || idx >= 2;
      rep2 = sh2 ? rep1 : rep2;
      rep1 = sh1 ? rep0 : rep1;
      rep0 = sh1 ? off : rep0;
      if (i + 1 < nseq) {  // state updates: literals length, match length, offset
        sll = fse_base(ell) + seqbits_take(br, fse_nb(ell));
        sml = fse_base(eml) + seqbits_take(br, fse_nb(eml));
        sof = fse_base(eof) + seqbits_take(br, fse_nb(eof));
      }
      // execution checks (3.1.1.4): literals available, match inside the frame
      if (lsum + ll > lit_lim - lit_done) return ZERR;
      const uint32_t mstart = osum + ll;  // relative to o.pos
      if (mstart + ml > bm_lim) return ZERR;  // the block outgrows Block_Maximum_Size
      if (off > back + mstart) return ZERR;  // before the frame start (no dictionary)
      if (mstart + ml > cap_lim) return kCap;  // (the retry pass sizes the output exactly)
      if (w0) sm.rec[cnt] = make_uint4(ll, ml, uint32_t(off), 0);
      lsum += ll;
      osum += ll + ml;
    }
    if (o.dry) {  // measuring pass: the chunk's bytes are not produced
      o.pos += osum;
      lit_pos += lsum;
      lit_left -= lsum;
      continue;
    }
    const long long tb = o.prof ? clock64() : 0;
    prof_add(o, 2, tb - ta);
    commit(o);  // output before this chunk is visible to every lane
    __syncthreads();
    // ---- phase B: prefixes by a wave scan, byte -> sequence map, then every
    // literal byte and match byte of the chunk in parallel ----
    {
      uint4 r[4];
      uint32_t lt = 0, ot = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t k = 4 * lane + u;
        r[u] = k < cnt ? sm.rec[k] : make_uint4(0, 0, 0, 0);
        lt += r[u].x;
        ot += r[u].x + r[u].y;
      }
      uint32_t lp = wave_incl_scan32(lt, lane) - lt, op = wave_incl_scan32(ot, lane) - ot;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t k = 4 * lane + u;
        if (k < cnt) sm.rec[k] = make_uint4(op, r[u].x, r[u].z, lp);
        lp += r[u].x;
        op += r[u].x + r[u].y;
      }
      if (w0) sm.rec[cnt] = make_uint4(osum, 0, 0, lsum);
    }
    __syncthreads();
    const uint64_t O = o.pos;
    const bool mapped = osum <= kChunkOut;
    if (mapped) {  // map[x] = k on [opre[k], opre[k+1]): markers, then a running max
      uint4* m4 = reinterpret_cast<uint4*>(sm.map);
#pragma unroll
      for (int u = 0; u < 4; ++u) m4[4 * lane + u] = make_uint4(0, 0, 0, 0);
      __syncthreads();
      for (uint32_t k = lane + 1; k < cnt; k += 64) sm.map[sm.rec[k].x] = uint8_t(k);
      __syncthreads();
      uint4 v[4];
      uint32_t mx = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u] = m4[4 * lane + u];
        const uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int t = 0; t < 4; ++t) mx = max(mx, (w4[q] >> (8 * t)) & 0xffu);
      }
      // exclusive max-scan over lanes
      uint32_t run = mx;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(run, d, 64);
        if (lane >= d) run = max(run, y);
      }
      run = __shfl_up(run, 1, 64);
      if (lane == 0) run = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t outw = 0;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            run = max(run, (w4[q] >> (8 * t)) & 0xffu);
            outw |= run << (8 * t);
          }
          w4[q] = outw;
        }
        m4[4 * lane + u] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
      }
      __syncthreads();
    }
    const uint8_t* lsrc = rle ? nullptr : lits + lit_pos;
    const long long tr = o.prof ? clock64() : 0;
    uint32_t hops = 0;
    for (uint32_t r0 = lane; r0 < osum; r0 += 64 * 4) {
      const uint8_t* srcp[4];
      bool live[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t rel0 = r0 + 64 * u;
        live[u] = rel0 < osum;
        srcp[u] = nullptr;
        if (!live[u]) continue;
        uint32_t rel = rel0;
        // follow copies back until a literal byte or output before the chunk
        for (;;) {
          const uint32_t k = mapped ? uint32_t(sm.map[rel]) : find(cnt, rel);
          const uint4 R = sm.rec[k];
          const uint32_t in = rel - R.x;
          if (in < R.y) {
            srcp[u] = lsrc ? lsrc + R.w + in : nullptr;
            break;
          }
          const uint32_t t = in - R.y, off = R.z;
          const uint32_t mo = t < off ? t : t % off;
          const int64_t s = int64_t(R.x) + R.y + mo - int64_t(off);
          if (s < 0) {
            srcp[u] = o.base + (int64_t(O) + s);
            break;
          }
          rel = uint32_t(s);
          ++hops;
        }
      }
      uint8_t v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = srcp[u] ? *srcp[u] : rle_byte;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (live[u]) o.base[O + r0 + 64 * u] = v[u];
    }
    o.pos += osum;
    lit_pos += lsum;
    lit_left -= lsum;
    __syncthreads();  // the chunk arrays are rewritten by the next phase A
    if (o.prof) {
      prof_add(o, 6, clock64() - tb);
      prof_add(o, 8, clock64() - tr);
      unsigned long long h = hops;
      for (int d = 32; d; d >>= 1) h += __shfl_xor(h, d, 64);
      prof_add(o, 9, h);
    }
  }
  fs.rep0 = rep0;
  fs.rep1 = rep1;
  fs.rep2 = rep2;
  if (br.pos > 0) return ZERR;  // unread bits: corrupt (an over-read on the last one passes)
  if (o.prof) prof_add(o, 1, clock64() - t1);
  prof_add(o, 4, nseq);
  if (o.pos + lit_left > blk_end) return ZERR;
  if (o.pos + lit_left > o.cap) return kCap;
  emit_lits(lit_left);
  return kOK;
  }  // !PRO
}

// XXH64 of out[a, b) by lanes 0..3 (the four accumulators), result on every lane.
__device__ uint64_t xxh64_out(const uint8_t* base, uint64_t len) {
  const int lane = threadIdx.x & 63;
  const uint32_t q = lane & 3;
  uint64_t acc = (q == 0) ? XP1 + XP2 : (q == 1) ? XP2 : (q == 2) ? 0 : 0 - XP1;
  const uint64_t nstripe = len / 32;
  if (lane < 4) {
    uint64_t s = 0;
    for (; s + 8 <= nstripe; s += 8) {  // eight loads in flight ahead of the chain
      uint64_t x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = ld64u(base + (s + u) * 32 + q * 8);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = xround(acc, x[u]);
    }
    for (; s < nstripe; ++s) acc = xround(acc, ld64u(base + s * 32 + q * 8));
  }
  const uint64_t a1 = __shfl(acc, 1, 64), a2 = __shfl(acc, 2, 64), a3 = __shfl(acc, 3, 64);
  const uint64_t a0 = __shfl(acc, 0, 64);
  uint64_t h;
  if (len >= 32) {
    h = rotl64(a0, 1) + rotl64(a1, 7) + rotl64(a2, 12) + rotl64(a3, 18);
    h = (h ^ xround(0, a0)) * XP1 + XP4;
    h = (h ^ xround(0, a1)) * XP1 + XP4;
    h = (h ^ xround(0, a2)) * XP1 + XP4;
    h = (h ^ xround(0, a3)) * XP1 + XP4;
  } else {
    h = XP5;
  }
  h += len;
  uint64_t t = nstripe * 32;
  for (; t + 8 <= len; t += 8) {
    h ^= xround(0, ld64u(base + t));
    h = rotl64(h, 27) * XP1 + XP4;
  }
  if (t + 4 <= len) {
    const uint32_t v = uint32_t(base[t]) | (uint32_t(base[t + 1]) << 8) |
                       (uint32_t(base[t + 2]) << 16) | (uint32_t(base[t + 3]) << 24);
    h ^= uint64_t(v) * XP1;
    h = rotl64(h, 23) * XP2 + XP3;
    t += 4;
  }
  for (; t < len; ++t) {
    h ^= uint64_t(base[t]) * XP5;
    h = rotl64(h, 11) * XP1;
  }
  h ^= h >> 33;
  h *= XP2;
  h ^= h >> 29;
  h *= XP3;
  h ^= h >> 32;
  return h;
}

// Every frame of src[0, n) (zstd.NewReader + io.Copy semantics).
template <bool PRO, class SM>
__device__ int32_t decode_frames(SM& sm, const uint8_t* src, int64_t n, Out& o, uint8_t* lit_buf,
                                 Pro* pro) {
  int64_t at = 0;
  bool first_frame = true;
  while (at < n) {
    if (n - at < 4) return ZERR;
    const uint32_t magic = ld32z(src, at, n);
    if ((magic & 0xfffffff0u) == 0x184d2a50u) {  // skippable frame (3.1.2)
      if (n - at < 8) return ZERR;
      const uint64_t sz = ld32z(src, at + 4, n);
      if (uint64_t(n - at - 8) < sz) return ZERR;
      at += 8 + int64_t(sz);
      continue;
    }
    if (magic != 0xfd2fb528u) return ZERR;
    at += 4;
    if (at >= n) return ZERR;
    const uint32_t fhd = src[at++];
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, reserved = (fhd >> 3) & 1;
    const uint32_t has_csum = (fhd >> 2) & 1, did_flag = fhd & 3;
    if (reserved) return ZERR;
    uint64_t window = 0;
    if (!single) {  // Window_Descriptor (3.1.1.1.2)
      if (at >= n) return ZERR;
      const uint32_t wd = src[at++];
      const uint32_t wlog = 10 + (wd >> 3);
      // libzstd: windowLog above ZSTD_WINDOWLOG_MAX (31 on 64-bit hosts) is
      // frameParameter_windowTooLarge
      if (wlog > 31) return ZERR;
      window = (uint64_t(1) << wlog) + ((uint64_t(1) << wlog) / 8) * (wd & 7);
    }
    const uint32_t did_size = did_flag == 0 ? 0 : did_flag == 1 ? 1 : did_flag == 2 ? 2 : 4;
    if (at + did_size > n) return ZERR;
    uint32_t did = 0;
    for (uint32_t k = 0; k < did_size; ++k) did |= uint32_t(src[at + k]) << (8 * k);
    at += did_size;
    if (did != 0) return ZERR;  // no dictionaries are registered with the reader
    const uint32_t fcs_size = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
    if (at + fcs_size > n) return ZERR;
    uint64_t fcs = 0;
    for (uint32_t k = 0; k < fcs_size; ++k) fcs |= uint64_t(src[at + k]) << (8 * k);
    if (fcs_size == 2) fcs += 256;
    at += fcs_size;
    if (single) window = fcs;  // Single_Segment_flag: Window_Size = Frame_Content_Size
    o.bmax = uint32_t(min<uint64_t>(window, kBlockMax));  // Block_Maximum_Size
    FrameState fs;
    fs.rep0 = 1;
    fs.rep1 = 4;
    fs.rep2 = 8;
    fs.huf_ok = fs.ll_ok = fs.of_ok = fs.ml_ok = false;
    fs.huf_bits = 0;
    fs.ll_al = fs.of_al = fs.ml_al = 0;
    o.frame0 = o.pos;
    bool first_block = true;
    for (;;) {  // blocks (3.1.1.2)
      if (n - at < 3) return ZERR;
      const uint32_t bh = src[at] | (uint32_t(src[at + 1]) << 8) | (uint32_t(src[at + 2]) << 16);
      at += 3;
      const uint32_t last = bh & 1, btype = (bh >> 1) & 3, bsize = bh >> 3;
      if (btype == 0) {  // Raw_Block
        if (int64_t(bsize) > n - at) return ZERR;
        if (bsize > o.bmax) return ZERR;  // Block_Size > Block_Maximum_Size (3.1.1.2.3)
        if (o.pos + bsize > o.cap) return kCap;
        out_copy(o, src + at, bsize);
        at += bsize;
      } else if (btype == 1) {  // RLE_Block
        if (at >= n) return ZERR;
        if (bsize > o.bmax) return ZERR;
        if (o.pos + bsize > o.cap) return kCap;
        const uint8_t v = src[at];
        const int lane = threadIdx.x & 63;
        if (!o.dry)
          for (uint64_t j = lane; j < bsize; j += 64) o.base[o.pos + j] = v;
        o.pos += bsize;
        at += 1;
      } else if (btype == 2) {  // Compressed_Block (libzstd: < 128 KiB)
        if (int64_t(bsize) > n - at || bsize >= kBlockMax) return ZERR;
        if constexpr (PRO) {
          // deferrable: the input is exactly one frame holding this one block
          pro->deferrable = first_frame && first_block && last &&
                            at + int64_t(bsize) + (has_csum ? 4 : 0) == n;
          pro->fcs = fcs;
          pro->fcs_on = fcs_size != 0;
          pro->csum_on = has_csum;
          if (pro->deferrable && has_csum && (threadIdx.x & 63) == 0)
            pro->zb->csum = ld32z(src, at + bsize, n);
        }
        const int32_t r = compressed_block<PRO>(sm, fs, o, src + at, bsize, lit_buf, pro);
        if (r != kOK) return r;
        at += bsize;
      } else {
        return ZERR;  // reserved block type
      }
      first_block = false;
      if (last) break;
    }
    first_frame = false;
    if (fcs_size && o.pos - o.frame0 != fcs) return ZERR;  // Frame_Content_Size check
    if (has_csum) {
      if (n - at < 4) return ZERR;
      if (!o.dry) {  // (content-dependent: checked by the retry's producing pass)
        commit(o);
        const uint32_t want = ld32z(src, at, n);
        const uint64_t h = xxh64_out(o.base + o.frame0, o.pos - o.frame0);
        if (uint32_t(h) != want) return ZERR;
      }
      at += 4;
    }
  }
  return kOK;
}

}  // namespace zst

// Blocks whose frames outgrow their first output region are decoded again
// (zstd_run): a measuring pass sizes each one's whole output, then a producing
// pass writes it into a region of that size.  Go inflates every frame before
// its record walk (io.Copy, segment_reader.go:326), whatever OriginalSize says.
struct ZRetry {
  const uint32_t* list;  // the blocks, or null: every block the prologue handed over
  uint32_t n;
  int dry;               // 1: measuring pass (need[i]); 0: producing pass (roff)
  const uint64_t* roff;  // [n + 1] output offsets in dec (producing pass)
  uint64_t* need;        // [n] decompressed bytes (measuring pass)
  uint64_t* cap_off;     // [nblk + 1]: a produced block's region offset is stored here
};

// Raw-block outcome of ReadBlockWithStat before the decompression
// (:303-316 in Go's order, then the rawBlockBytes[:CompressedSize] slice, :321).
__device__ __forceinline__ int32_t zstd_raw_status(const Desc& d, uint64_t seg_bytes) {
  const int32_t st = go_read_status(d, seg_bytes);
  if (st != OKV_BLK_OK) return st;
  return d.compressed_size > d.block_size ? int32_t(OKV_BLK_PANIC) : int32_t(OKV_BLK_OK);
}

// One wave per segment block, persistent over the batch.  Inputs: the raw
// descriptors; outputs: decompressed bytes at dec + cap_off[b], their length,
// and a per-block status (OKV_BLK_*).  lit = per-wave literal scratch.
__global__ __launch_bounds__(64) void okv_zstd_kernel(const uint8_t* __restrict__ seg,
                                                      uint64_t seg_bytes, const Desc* __restrict__ descs,
                                                      uint32_t nblk, const uint64_t* __restrict__ cap_off,
                                                      uint8_t* __restrict__ dec, uint64_t* __restrict__ dec_len,
                                                      int32_t* __restrict__ zstatus,
                                                      uint8_t* __restrict__ lit,
                                                      unsigned long long* __restrict__ prof,
                                                      const zst::ZBlk* __restrict__ zb, ZRetry R) {
  __shared__ zst::Smem sm;
  uint8_t* lit_buf = lit + uint64_t(blockIdx.x) * zst::kBlockMax;
  const uint32_t count = R.list ? R.n : nblk;
  for (uint32_t i = blockIdx.x; i < count; i += gridDim.x) {
    const uint32_t b = R.list ? R.list[i] : i;
    if (!R.list && zb && zst::rfl(uint32_t(zb[b].kind)) != zst::kKindSlow) continue;
    // producing pass: only the blocks the measuring pass sized
    if (R.list && !R.dry && zst::rfl(uint32_t(zstatus[b])) != OKV_BLK_CAPACITY) continue;
    const Desc d = descs[b];
    int32_t st = OKV_BLK_OK;
    zst::Out o;
    o.prof = prof;
    const long long tb = prof ? clock64() : 0;
    o.dry = R.dry != 0;
    o.bmax = 0;
    if (!R.list) {
      o.base = dec + cap_off[b];
      o.cap = cap_off[b + 1] - cap_off[b];
    } else if (R.dry) {
      o.base = nullptr;
      o.cap = uint64_t(1) << 62;  // no frame set reaches it
    } else {
      o.base = dec + R.roff[i];
      o.cap = R.roff[i + 1] - R.roff[i];
    }
    o.pos = o.committed = o.frame0 = 0;
    st = zstd_raw_status(d, seg_bytes);
    if (st == OKV_BLK_OK) {
      const uint8_t* src = seg + d.offset;
      const int32_t r = zst::decode_frames<false>(sm, src, int64_t(d.compressed_size), o, lit_buf,
                                                         nullptr);
      __syncthreads();
      st = r == zst::kOK ? OKV_BLK_OK : r == zst::kCap ? OKV_BLK_CAPACITY : OKV_BLK_ZSTD_ERROR;
    }
    if ((threadIdx.x & 63) == 0) {
      if (R.list && R.dry) {
        // sized: stays OKV_BLK_CAPACITY for the producing pass
        R.need[i] = st == OKV_BLK_OK ? o.pos : 0;
        if (st != OKV_BLK_OK) {
          zstatus[b] = st;
          dec_len[b] = 0;
        }
      } else {
        zstatus[b] = st;
        dec_len[b] = st == OKV_BLK_OK ? o.pos : 0;
        if (R.list && st == OKV_BLK_OK) R.cap_off[b] = R.roff[i];
      }
    }
    if (prof) {
      zst::prof_add(o, 3, clock64() - tb);
      zst::prof_add(o, 7, 1);
    }
    __builtin_amdgcn_s_waitcnt(0);
  }
}

// The blocks the first pass left at OKV_BLK_CAPACITY (frames decompressing
// past their first region) -> list[*count].
__global__ __launch_bounds__(256) void okv_zstd_list_kernel(const int32_t* __restrict__ zstatus,
                                                            uint32_t nblk, uint32_t* __restrict__ list,
                                                            uint32_t* __restrict__ count) {
  const uint32_t b = blockIdx.x * 256 + threadIdx.x;
  const bool hit = b < nblk && zstatus[b] == OKV_BLK_CAPACITY;
  const uint64_t m = __ballot(hit);
  if (!m) return;
  const int lane = threadIdx.x & 63;
  uint32_t base = 0;
  if (lane == __ffsll(static_cast<unsigned long long>(m)) - 1)
    base = atomicAdd(count, uint32_t(__popcll(m)));
  base = __shfl(base, __ffsll(static_cast<unsigned long long>(m)) - 1, 64);
  if (hit) list[base + __popcll(m & ((uint64_t(1) << lane) - 1))] = b;
}

// roff[i] = base + sum_{j < i} round16(need[j]); roff[n] = base + total.
__global__ __launch_bounds__(1024) void okv_zstd_roff_kernel(const uint64_t* __restrict__ need,
                                                             uint32_t n, uint64_t base,
                                                             uint64_t* __restrict__ roff) {
  __shared__ uint64_t sm[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t carry = base;
  for (uint32_t i0 = 0; i0 < n; i0 += 1024) {
    const uint32_t i = i0 + threadIdx.x;
    const uint64_t v = i < n ? round16(need[i]) : 0;
    const uint64_t inc = wave_incl_scan(v, lane);
    if (lane == 63) sm[wave] = inc;
    __syncthreads();
    uint64_t before = 0, tot = 0;
    for (int w = 0; w < 16; ++w) {
      before += w < wave ? sm[w] : 0;
      tot += sm[w];
    }
    if (i < n) roff[i] = carry + before + inc - v;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) roff[n] = carry;
}

// ---- stage 1: prologue, one wave per segment block -------------------------------
// Frame / block headers, Huffman literals into the block's literal scratch, FSE
// tables into HBM.  Raw / RLE / literals-only blocks finish here; a block whose
// input is one frame holding one compressed block with sequences is deferred to
// stages 2-3; anything else goes to okv_zstd_kernel (kKindSlow).
// Registers capped for 4 waves per SIMD (128 VGPRs and a few scratch spills; uncapped:
// 140, 3 waves): prologue 755 -> 715 us at CZ (zstd_seq_chain_ab.log, r6zg).
#ifndef OKV_ZSTD_PRO_WPE
#define OKV_ZSTD_PRO_WPE 4
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(OKV_ZSTD_PRO_WPE))) void okv_zstd_pro_kernel(
    const uint8_t* __restrict__ seg, uint64_t seg_bytes, const Desc* __restrict__ descs,
    uint32_t nblk, const uint64_t* __restrict__ cap_off, uint8_t* __restrict__ dec,
    uint64_t* __restrict__ dec_len, int32_t* __restrict__ zstatus, uint8_t* __restrict__ lits,
    uint16_t* __restrict__ tabs, uint16_t* __restrict__ htab, zst::ZBlk* __restrict__ zb,
    uint64_t* __restrict__ seq_n, unsigned long long* __restrict__ prof) {
  __shared__ zst::SmemCore sm;
  const int lane = threadIdx.x & 63;
  for (uint32_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    const long long tw = prof ? clock64() : 0;
    const Desc d = descs[b];
    int32_t st = OKV_BLK_OK;
    int32_t kind = zst::kKindDone;
    uint32_t nseq = 0;
    zst::Out o;
    o.prof = prof;  // diagnostics (ablation build, OKV_ZSTD_PROF); null in the product
    o.base = dec + cap_off[b];
    o.cap = cap_off[b + 1] - cap_off[b];
    o.pos = o.committed = o.frame0 = 0;
    o.dry = false;
    o.bmax = 0;
    if ((st = zstd_raw_status(d, seg_bytes)) != OKV_BLK_OK) {
      // Seek / makeslice / EOF / short read / slice bounds (:303-321)
    } else {
      zst::Pro pro;
      pro.lit_blk = lits + cap_off[b];
      pro.lit_cap = o.cap;
      pro.tabs = tabs + uint64_t(b) * zst::kTabEnt;
      pro.zb = zb + b;
      pro.deferrable = false;
      pro.fcs = 0;
      pro.fcs_on = pro.csum_on = 0;
      pro.htab = htab + uint64_t(b) * zst::kHufSlot;
      pro.seg = seg;
      pro.huf_on = 0;
      pro.nseq = 0;
      const int32_t r = zst::decode_frames<true>(sm, seg + d.offset, int64_t(d.compressed_size), o,
                                                 nullptr, &pro);
      __syncthreads();
      if (r == zst::kDefer) {
        kind = zst::kKindSeq;
        nseq = pro.nseq;
      } else if (r == zst::kSlow) {
        kind = zst::kKindSlow;
      } else {
        st = r == zst::kOK ? OKV_BLK_OK : r == zst::kCap ? OKV_BLK_CAPACITY : OKV_BLK_ZSTD_ERROR;
      }
    }
    if (lane == 0) {
      zb[b].kind = kind;
      zb[b].st = zst::kOK;
      seq_n[b] = nseq;  // (scanned in place by okv_zstd_seqoff_kernel)
      if (kind == zst::kKindDone) {
        zstatus[b] = st;
        dec_len[b] = st == OKV_BLK_OK ? o.pos : 0;
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    if (prof && lane == 0) {
      atomicAdd(prof + 11, (unsigned long long)(clock64() - tw));
      atomicAdd(prof + 13, 1ull);
    }
  }
}

// ---- stage 1b: Huffman literal streams, 16 blocks per wave -----------------------
// One lane per stream (4 per block), each block's decoding table in LDS: the
// streams of a deferred block (kFlagHuf) decode here into its literal scratch,
// where the executor reads them.  A stream that fails its checks (no end
// marker, bits left over; RFC 8878 4.2.2) fails the block: zb.st = kErr,
// which the sequence stage keeps and the executor reports (the literals come
// before the sequences, as in the general kernel).
// (The streams and the scratch are addressed from the kernel's arguments, not
// through zb's pointers: a pointer read from memory is flat, and a flat load
// counts against the LDS counter too, so every table lookup's wait would also
// wait for the stream prefetch.)
// kHB blocks per wave (kHB * 4 KiB of LDS): fewer blocks per wave put more
// waves on each CU's four SIMDs (the stream chains are latency-bound).
template <uint32_t kHB>
__global__ __launch_bounds__(64) void okv_zstd_huf_kernel(zst::ZBlk* __restrict__ zb, uint32_t nblk,
                                                          const uint16_t* __restrict__ htab,
                                                          const uint8_t* __restrict__ seg,
                                                          uint8_t* __restrict__ blit,
                                                          const uint64_t* __restrict__ cap_off) {
  __shared__ uint16_t ht[kHB * zst::kHufSlot];
  const int lane = threadIdx.x & 63;
  const uint32_t j = uint32_t(lane) >> 2, sidx = uint32_t(lane) & 3;
  const uint32_t b0 = blockIdx.x * kHB, b = b0 + j;
  bool mine = false;
  uint32_t mb = 0;
  if (j < kHB && b < nblk) {
    mine = zb[b].kind == zst::kKindSeq && (zb[b].flags & zst::kFlagHuf);
    mb = mine ? zb[b].hmb : 0u;
  }
  // the tables: 2^(mb+1) bytes each (at least one 1 KiB piece), LDS DMA
  const uint8_t* src = reinterpret_cast<const uint8_t*>(htab);
  for (uint32_t jj = 0; jj < kHB; ++jj) {
    const uint32_t mj = __builtin_amdgcn_readlane(mine ? mb + 1 : 0u, int(4 * jj));
    if (!mj) continue;
    const uint32_t pieces = mj > 10 ? 1u << (mj - 10) : 1u;
    for (uint32_t k = 0; k < pieces; ++k)
      __builtin_amdgcn_global_load_lds(src + (uint64_t(b0 + jj) * zst::kHufSlot * 2 + k * 1024 + 16 * lane),
                                       OKV_LDS_PTR(reinterpret_cast<uint4*>(ht) + jj * (zst::kHufSlot / 8) + k * 64),
                                       16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bool good = true;
  if (mine) {
    const uint32_t regen = zb[b].lit_total, ns = zb[b].hns;
    if (sidx < ns) {
      const uint32_t sl = (regen + 3) / 4;  // (4 streams: 3 sl <= regen, checked by the prologue)
      const uint32_t cnt = ns == 1 ? regen : sidx < 3 ? sl : regen - 3 * sl;
      uint32_t off = 0;
      for (uint32_t k = 0; k < sidx; ++k) off += zb[b].hlen[k];
      uint8_t* lits = blit + cap_off[b] + sidx * sl;  // == zb[b].lits + sidx * seg
      good = zst::huf_stream(ht + j * zst::kHufSlot, mb, seg + zb[b].hq_off + off,
                             int64_t(zb[b].hlen[sidx]), lits, cnt);
    }
  }
  const uint64_t bad = __ballot(!good);
  if (mine && sidx == 0 && ((bad >> (4 * j)) & 0xfull)) zb[b].st = zst::kErr;
}

#ifndef OKV_ZSTD_HUF_BLOCKS
#define OKV_ZSTD_HUF_BLOCKS 8  // 0.392 vs 0.439 ms at 16, 0.391 at 4 (CZ, profiles/r4/session)
#endif
constexpr uint32_t kHufBlocks = OKV_ZSTD_HUF_BLOCKS;  // blocks per wave of the stream stage

namespace zst {
// One-workgroup exclusive scan of v(i), i < n -> out[i], out[n] = total: each
// thread owns kScanPer consecutive elements of a tile, their loads all in
// flight before one block scan per tile (an element per thread per round
// left a chain of dependent HBM trips: 80 us for CZ's 16 384 blocks).
constexpr uint32_t kScanPer = 16;
template <class V>
__device__ __forceinline__ void block_excl_scan(uint32_t n, V v_of, uint64_t* __restrict__ out) {
  __shared__ uint64_t sm[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t carry = 0;
  for (uint32_t t0 = 0; t0 < n; t0 += 1024 * kScanPer) {
    const uint32_t base = t0 + threadIdx.x * kScanPer;
    uint64_t v[kScanPer];
    uint64_t sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) v[k] = base + k < n ? v_of(base + k) : 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) sum += v[k];
    const uint64_t inc = wave_incl_scan(sum, lane);
    if (lane == 63) sm[wave] = inc;
    __syncthreads();
    uint64_t before = 0, tot = 0;
    for (int w = 0; w < 16; ++w) {
      before += w < wave ? sm[w] : 0;
      tot += sm[w];
    }
    uint64_t run = carry + before + inc - sum;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
      if (base + k < n) out[base + k] = run;
      run += v[k];
    }
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) out[n] = carry;
}
}  // namespace zst

// Exclusive scan of the deferred blocks' sequence counts, in place: seq_off[b]
// holds block b's count (okv_zstd_pro_kernel: 0 unless deferred) -> its offset,
// seq_off[nblk] the total.  (A compact array: the ZBlk fields are a line per
// block, and one workgroup reading 16 384 lines took 80 us.)
__global__ __launch_bounds__(1024) void okv_zstd_seqoff_kernel(uint32_t nblk,
                                                               uint64_t* __restrict__ seq_off) {
  zst::block_excl_scan(nblk, [&](uint32_t i) -> uint64_t { return seq_off[i]; }, seq_off);
}

namespace zst {
// Per-lane backward bit reader over aligned dwords, two dwords prefetched, so a
// lane's serial decode rarely waits on memory.  Bit positions are relative to
// the aligned base ab; stream bytes outside [s0, s0 + n) read as 0.
struct LaneBits {
  const uint8_t* ab;
  int32_t s0, n;
  int32_t P;       // remaining bits, as ab-relative position
  int32_t acc_lo;  // acc holds bits [acc_lo, acc_lo + 64)
  uint64_t acc;
  uint32_t nx0, nx1;  // raw dwords acc_lo / 32 - 1 and - 2 (masked when shifted in)
  int32_t nd;         // dword index loaded into nx1 next
};
// Raw aligned dword d (clamped into the buffer): an unconditional load whose
// value is only used when it is shifted in, so prefetches do not stall.
__device__ __forceinline__ uint32_t lb_raw(const LaneBits& b, int32_t d) {
  const int32_t lim = (b.s0 + b.n - 1) >> 2;
  const int32_t dc = d < 0 ? 0 : (d > lim ? lim : d);
  // a global (not flat) load: it counts in vmcnt only, so LDS waits do not drain it
  return *(const __attribute__((address_space(1))) uint32_t*)(b.ab + 4 * dc);
}
// Bytes of dword d outside the stream [s0, s0 + n) read as 0 (branch-free:
// lanes are different blocks, so branches would diverge).
__device__ __forceinline__ uint32_t lb_fix(const LaneBits& b, uint32_t v, int32_t d) {
  const int32_t lo = 4 * d;
  const int32_t cut = min(max(b.s0 - lo, 0), 4);        // bytes below the stream
  const int32_t keep = min(max(b.s0 + b.n - lo, 0), 4);  // bytes up to the stream end
  const uint32_t mlo = cut >= 4 ? 0u : (0xffffffffu << (8 * cut));
  const uint32_t mhi = keep >= 4 ? 0xffffffffu : ((1u << (8 * keep)) - 1u);
  return v & mlo & mhi;
}
__device__ __forceinline__ uint32_t lb_dw(const LaneBits& b, int32_t d) {
  return lb_fix(b, lb_raw(b, d), d);
}
// Ensure k (<= 32) bits are in the container.
__device__ __forceinline__ void lb_ensure(LaneBits& b, int32_t k) {
  if (b.P - b.acc_lo < k) {
    const int32_t d = (b.acc_lo >> 5) - 1;  // the dword held in nx0
    b.acc = (b.acc << 32) | lb_fix(b, b.nx0, d);
    b.acc_lo -= 32;
    b.nx0 = b.nx1;
    b.nx1 = lb_raw(b, b.nd);
    --b.nd;
  }
}
__device__ __forceinline__ uint32_t lb_take(LaneBits& b, uint32_t k) {
  b.P -= int32_t(k);
  return uint32_t(b.acc >> uint32_t(b.P - b.acc_lo)) & uint32_t((uint64_t(1) << k) - 1);
}

// 128-bit window reader for the sequence stage.  The window holds aligned
// dwords [wd, wd + 4); the three dwords below it are loaded (one 12-byte load)
// unconditionally at the end of every sequence and only read at the end of the
// next one, after the next table gathers have drained the load queue -- so the
// stream never stalls the lane chain.  One sequence reads <= 89 bits; the
// window always holds > 96.  Bits below the stream's start are not masked: the
// chain reads them only as the state bits of a sequence that starts past the
// stream (libzstd's overflow), which is not stored; the extra bits are read
// by the executor (bits_below), which masks them.
typedef uint32_t Dw3 __attribute__((ext_vector_type(3)));
struct WinBits {
  LaneBits f;             // ab / s0 / n (masking), P
  int32_t wd;
  uint64_t lo, hi;        // dwords wd+1:wd, wd+3:wd+2 (masked)
  Dw3 nx;                 // raw dwords from max(wd - 3, 0) (in flight)
};
__device__ __forceinline__ void wb_issue(WinBits& w) {
  // (clamped at the stream's first dword: a window that reaches below it
  // takes its dwords from the clamped load, wb_slide)
  w.nx = *(const __attribute__((address_space(1))) Dw3*)(w.f.ab + 4 * max(w.wd - 3, 0));
}
// k <= 31 bits at window bit pos: the two dwords around it (selects, no
// branches) and one funnel shift.
__device__ __forceinline__ uint32_t wb_take(WinBits& w, uint32_t k) {
  w.f.P -= int32_t(k);
  const uint32_t pos = uint32_t(w.f.P - 32 * w.wd);  // 0 .. 128 - k
  const uint32_t i = pos >> 5;
  const uint32_t w0 = uint32_t(w.lo), w1 = uint32_t(w.lo >> 32), w2 = uint32_t(w.hi),
                 w3 = uint32_t(w.hi >> 32);
  const uint32_t a = i == 0 ? w0 : i == 1 ? w1 : i == 2 ? w2 : w3;
  const uint32_t c = i == 0 ? w1 : i == 1 ? w2 : i == 2 ? w3 : 0u;
  const uint32_t v = __builtin_amdgcn_alignbit(c, a, pos & 31u);
  return v & ((1u << k) - 1u);
}
// Bits [pos, pos + 64) / [pos, pos + 32) of the window (window-relative pos,
// 0 <= pos < 128; bits above the window read as 0): selects and funnel shifts,
// no change to the read position (the sequence loop sets P itself).
__device__ __forceinline__ uint64_t wb_get64(const WinBits& w, uint32_t pos) {
  const uint32_t i = pos >> 5, s = pos & 31u;
  const uint32_t w0 = uint32_t(w.lo), w1 = uint32_t(w.lo >> 32), w2 = uint32_t(w.hi),
                 w3 = uint32_t(w.hi >> 32);
  const uint32_t a = i == 0 ? w0 : i == 1 ? w1 : i == 2 ? w2 : w3;
  const uint32_t b = i == 0 ? w1 : i == 1 ? w2 : i == 2 ? w3 : 0u;
  const uint32_t c = i == 0 ? w2 : i == 1 ? w3 : 0u;
  return uint64_t(__builtin_amdgcn_alignbit(b, a, s)) |
         (uint64_t(__builtin_amdgcn_alignbit(c, b, s)) << 32);
}
__device__ __forceinline__ uint32_t wb_get32(const WinBits& w, uint32_t pos) {
  const uint32_t i = pos >> 5;
  const uint32_t w0 = uint32_t(w.lo), w1 = uint32_t(w.lo >> 32), w2 = uint32_t(w.hi),
                 w3 = uint32_t(w.hi >> 32);
  const uint32_t a = i == 0 ? w0 : i == 1 ? w1 : i == 2 ? w2 : w3;
  const uint32_t c = i == 0 ? w1 : i == 1 ? w2 : i == 2 ? w3 : 0u;
  return __builtin_amdgcn_alignbit(c, a, pos & 31u);
}
__device__ __forceinline__ uint32_t lowmask(uint32_t k) { return (1u << k) - 1u; }  // k <= 31

// Slide the window down so its top dword holds bit P - 1; by 0..3 dwords.
__device__ __forceinline__ void wb_slide(WinBits& w) {
  const int32_t dtop = ((w.f.P + 31) >> 5) - 1;
  int32_t sft = w.wd + 3 - dtop;
  sft = sft < 0 ? 0 : (sft > 3 ? 3 : sft);
  // dwords wd - 3, wd - 2, wd - 1 (a load clamped at dword 0, wd < 3: dwords
  // 0 and 1 from their places in it; the dwords before the stream are garbage)
  const bool full = w.wd >= 3;
  const uint32_t c0 = w.nx.x, c1 = full ? w.nx.y : w.nx.x,
                 c2 = full ? w.nx.z : (w.wd == 2 ? w.nx.y : w.nx.x);
  // the last reads of the dwords in flight before the next loads: those then
  // reuse their registers (a load hoisted above these reads needs other
  // registers and a loop-carried copy, which waits for it)
  asm volatile("" ::"v"(c0), "v"(c1), "v"(c2) : "memory");
  const uint32_t w0 = uint32_t(w.lo), w1 = uint32_t(w.lo >> 32), w2 = uint32_t(w.hi),
                 w3 = uint32_t(w.hi >> 32);
  // C = [c0 c1 c2 w0 w1 w2 w3]; new window k = C[k + 3 - sft]
  const uint32_t n0 = sft == 0 ? w0 : sft == 1 ? c2 : sft == 2 ? c1 : c0;
  const uint32_t n1 = sft == 0 ? w1 : sft == 1 ? w0 : sft == 2 ? c2 : c1;
  const uint32_t n2 = sft == 0 ? w2 : sft == 1 ? w1 : sft == 2 ? w0 : c2;
  const uint32_t n3 = sft == 0 ? w3 : sft == 1 ? w2 : sft == 2 ? w1 : w0;
  w.lo = uint64_t(n0) | (uint64_t(n1) << 32);
  w.hi = uint64_t(n2) | (uint64_t(n3) << 32);
  w.wd -= sft;
  wb_issue(w);
}

// The same slide in two halves, for a window whose dwords below arrive two
// sequences after their load (okv_zstd_seq_kernel): the shift for the position
// Pn after the sequence, known early in it; the load of the dwords below the
// window at wd (issued as soon as wd is known); the shift itself, with the
// dwords of the load issued a sequence earlier.
__device__ __forceinline__ int32_t wb_sft(const WinBits& w, int32_t Pn) {
  const int32_t sft = w.wd + 3 - (((Pn + 31) >> 5) - 1);
  return sft < 0 ? 0 : (sft > 3 ? 3 : sft);
}
__device__ __forceinline__ Dw3 wb_load(const WinBits& w, int32_t wd) {
  return *(const __attribute__((address_space(1))) Dw3*)(w.f.ab + 4 * max(wd - 3, 0));
}
__device__ __forceinline__ void wb_shift(WinBits& w, const Dw3& nx, int32_t sft) {
  // (the load's first use here, after the sequence's other memory operations:
  // selects on it hoisted to the sequence's top would wait for it there)
  uint32_t x = nx.x, y = nx.y, z = nx.z;
  asm volatile("" : "+v"(x), "+v"(y), "+v"(z)::"memory");
  const bool full = w.wd >= 3;  // (as wb_slide)
  const uint32_t c0 = x, c1 = full ? y : x, c2 = full ? z : (w.wd == 2 ? y : x);
  const uint32_t w0 = uint32_t(w.lo), w1 = uint32_t(w.lo >> 32), w2 = uint32_t(w.hi),
                 w3 = uint32_t(w.hi >> 32);
  const uint32_t n0 = sft == 0 ? w0 : sft == 1 ? c2 : sft == 2 ? c1 : c0;
  const uint32_t n1 = sft == 0 ? w1 : sft == 1 ? w0 : sft == 2 ? c2 : c1;
  const uint32_t n2 = sft == 0 ? w2 : sft == 1 ? w1 : sft == 2 ? w0 : c2;
  const uint32_t n3 = sft == 0 ? w3 : sft == 1 ? w2 : sft == 2 ? w1 : w0;
  w.lo = uint64_t(n0) | (uint64_t(n1) << 32);
  w.hi = uint64_t(n2) | (uint64_t(n3) << 32);
  w.wd -= sft;
}

// A sequence as the sequence stage leaves it: literal-length code (6 bits) |
// its extra bits (16) << 6 | match-length code (6) << 22 | extra bits (16) << 28
// | the offset value (ofv = 2^code + extra bits, saturated at 2^20 - 1) << 44.
// The executor resolves repeat offsets (a scan over its window of sequences),
// turns codes into lengths and makes the execution checks (RFC 8878 3.1.1.4)
// in sequence order.  An offset past 2^20 - 4 is past any single-block frame's
// output, which the executor holds to Block_Maximum_Size (<= 128 KiB, ZBlk::bmax)
// before the offset check, so the saturated value (and any repeat of it)
// fails the same check.
__device__ __forceinline__ uint64_t seq_pack(uint32_t llc, uint32_t llx, uint32_t mlc, uint32_t mlx,
                                             uint32_t ofv) {
  return uint64_t(llc | (llx << 6) | (mlc << 22)) | (uint64_t(mlx) << 28) |
         (uint64_t(min(ofv, 0xfffffu)) << 44);
}
}  // namespace zst

// ---- stage 2: sequences, one lane per segment block --------------------------------
// RFC 8878 3.1.1.3.2 / libzstd ZSTD_decodeSequence for every deferred block at
// once: each lane owns a block's FSE states and bitstream, checks the stream
// as the general kernel does and writes each sequence's codes, extra bits and
// raw offset value (seq_pack; the repeat offsets are the executor's scan).
// 64 blocks advance per wave instruction.  The lane chain is one table lookup per state
// per sequence: the 64 blocks' tables live in LDS (16-bit states, 160 KiB: one
// workgroup per CU), so a step costs its instructions plus an LDS trip, not an
// HBM / L2 trip (the round-2/3 form gathered 32-bit states from HBM:
// ~1900 cycles per sequence, most of it the gather's latency).
namespace zst {
// Extra-bits count and baseline of literal-length / match-length codes (RFC
// 8878 3.1.1.3.2.1.1, the LL_BITS / LL_BASE / ML_BITS / ML_BASE tables above)
// without a memory lookup.
// All branch-free (bsel masks): the lanes are different blocks, and these
// feed the state chain.
__device__ __forceinline__ uint32_t msk(bool c) { return 0u - uint32_t(c); }
__device__ __forceinline__ uint32_t ll_xbits(uint32_t c) {
  const uint32_t mid = max(1u, (c - min(c, 16u)) >> 1);
  return bsel(msk(c < 16), 0u, bsel(msk(c < 25), mid, c - 19));
}
__device__ __forceinline__ uint32_t ml_xbits(uint32_t c) {
  const uint32_t mid = max(1u, (c - min(c, 32u)) >> 1);
  return bsel(msk(c < 32), 0u, bsel(msk(c < 43), mid, c - 36));
}
// LL_BASE[16..24] - 16 and ML_BASE[32..40] - 35, 6 bits each (the same list)
constexpr uint64_t kLLB = 0ull | (2ull << 6) | (4ull << 12) | (6ull << 18) | (8ull << 24) |
                          (12ull << 30) | (16ull << 36) | (24ull << 42) | (32ull << 48);
__device__ __forceinline__ uint32_t ll_base(uint32_t c) {
  const uint32_t j = min(c - min(c, 16u), 8u), k = (c - min(c, 25u)) & 31u;
  const uint32_t mid = 16u + uint32_t(kLLB >> (6 * j)) % 64u;
  return bsel(msk(c < 16), c, bsel(msk(c < 25), mid, 64u << k));
}
__device__ __forceinline__ uint32_t ml_base(uint32_t c) {
  const uint32_t j = min(c - min(c, 32u), 8u), k = (c - min(c, 43u)) & 31u;
  const uint32_t mid = 35u + uint32_t(kLLB >> (6 * j)) % 64u;
  const uint32_t hi = bsel(msk(c < 41), mid, bsel(msk(c < 42), 83u, 99u));
  return bsel(msk(c < 32), c + 3, bsel(msk(c < 43), hi, (128u << k) + 3u));
}
// One packed state: symbol, nbBits and baseline (al = the table's accuracy log).
struct St16 {
  uint32_t sym, nb, base;
};
__device__ __forceinline__ St16 st16(uint32_t e, uint32_t al) {
  const uint32_t x = e >> 6;  // >= 1 in every built table (x | 1: clz defined on garbage)
  const uint32_t nb = al + __builtin_clz(x | 1u) - 31u;
  return St16{e & 63u, nb, (x << nb) - (1u << al)};
}
}  // namespace zst

__global__ __launch_bounds__(64) void okv_zstd_seq_kernel(zst::ZBlk* __restrict__ zb, uint32_t nblk,
                                                          const uint16_t* __restrict__ tabs,
                                                          const uint64_t* __restrict__ seq_off,
                                                          uint64_t* __restrict__ seqs) {
  __shared__ uint16_t tl[64 * zst::kTabEnt];  // 163 840 B: this workgroup's 64 blocks' tables
  const int lane = threadIdx.x & 63;
  const uint32_t b0 = blockIdx.x * 64;
  const uint32_t nb_wg = min(64u, nblk - b0);
  {  // the tables of blocks [b0, b0 + nb_wg): LDS DMA, 1 KiB per wave instruction
    const uint8_t* src = reinterpret_cast<const uint8_t*>(tabs + uint64_t(b0) * zst::kTabEnt);
    const uint32_t n16 = nb_wg * zst::kTabEnt * 2 / 16;  // 160 pieces of 16 B per block
    for (uint32_t k0 = 0; k0 < n16; k0 += 64) {
      const uint32_t k = min(k0 + uint32_t(lane), n16 - 1);  // a tail lane reloads the last piece
      __builtin_amdgcn_global_load_lds(src + 16ull * k, OKV_LDS_PTR(reinterpret_cast<uint4*>(tl) + k0),
                                       16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const uint32_t b = b0 + lane;
  if (b >= nblk || zb[b].kind != zst::kKindSeq) return;
  const zst::ZBlk z = zb[b];
  if (z.st != zst::kOK) {  // the literal streams failed (okv_zstd_huf_kernel): nothing to decode
    zb[b].nseq_ok = 0;
    zb[b].pfix = 0;
    return;
  }
  const uint16_t* T = tl + lane * zst::kTabEnt;
  uint64_t* S = seqs + seq_off[b];
  int32_t st = zst::kOK;
  uint32_t nok = 0;  // sequences decoded before any overflow
  uint32_t fix = 0;  // bit 31: the last stored sequence needs its extras masked (ZBlk::pfix)
  zst::WinBits br;
  {
    const uintptr_t a = reinterpret_cast<uintptr_t>(z.stream);
    br.f.ab = reinterpret_cast<const uint8_t*>(a & ~uintptr_t(3));
    br.f.s0 = int32_t(a & 3);
    br.f.n = int32_t(z.stream_len);
  }
  const uint32_t last = br.f.n > 0 ? z.stream[br.f.n - 1] : 0;
  if (last == 0) {
    st = zst::kErr;  // no end marker
  } else {
    br.f.P = 8 * br.f.s0 + (br.f.n - 1) * 8 + (31 - __builtin_clz(last));
    const int32_t dtop = (br.f.s0 + br.f.n - 1) >> 2;
    br.wd = dtop - 3;
    br.lo = uint64_t(zst::lb_dw(br.f, dtop - 3)) | (uint64_t(zst::lb_dw(br.f, dtop - 2)) << 32);
    br.hi = uint64_t(zst::lb_dw(br.f, dtop - 1)) | (uint64_t(zst::lb_dw(br.f, dtop)) << 32);
    zst::wb_issue(br);
    const uint32_t lla = z.ll_al, ofa = z.of_al, mla = z.ml_al;
    uint32_t sll = zst::wb_take(br, lla);
    uint32_t sof = zst::wb_take(br, ofa);
    uint32_t sml = zst::wb_take(br, mla);
    zst::wb_slide(br);
    const int32_t P0 = 8 * br.f.s0;
    int32_t pl = 0, pfix = 0;
    // software-pipelined: sequence i + 1's three state lookups are issued as
    // soon as its states are known, before the window slide
    uint32_t ell = T[sll & 511], eof = T[512 + (sof & 255)], eml = T[768 + (sml & 511)];
    // No breaks: a failed check sets st and the loop ends at its head.  An
    // early exit would make the window loads in flight at the latch
    // loop-carried copies, i.e. a full wait for them (and the store) every
    // sequence.
    // The previous sequence's packed form is stored at the top of the next
    // iteration: every wait for the window loads also waits for older stores
    // (vmcnt), so the store is issued a whole sequence before that wait.
    uint64_t pend_seq = 0;
    // One sequence.  The dwords below the window are loaded as soon as the
    // sequence's length in bits is known and shifted in at the end of the NEXT
    // sequence (two load sets, alternating: the loop runs two sequences per
    // trip), so a load has about two sequences to arrive -- an L2 hit, which
    // a lane whose window enters a new 64-byte piece takes about every 50
    // sequences, no longer stalls the wave (profiles/r6/session/zstd_seq_chain_ab.log).
    // act: the lane still decodes (the second sequence of a trip runs on every
    // lane of the trip; a lane that ended with the first keeps its state)
    auto step = [&](uint32_t i, const zst::Dw3& cur, zst::Dw3& nxt, bool act) {
      if (i && act) S[i - 1] = pend_seq;
      // libzstd: the stream overflowed before this sequence
      const bool over = br.f.P < P0;
      // Every field's position follows from the three states: offset extra
      // bits, then ML, then LL extra bits, then the LL / ML / OF state bits
      // (read high to low).  The state bits and both length extras come out
      // of one 64-bit window read (<= 26 + 16 + 16 bits), the offset extras of
      // one 32-bit read; the repeat offsets are the executor's (a scan).
      const zst::St16 L = zst::st16(ell, lla), O = zst::st16(eof, ofa), M = zst::st16(eml, mla);
      const uint32_t ofs = O.sym, xml = zst::ml_xbits(M.sym), xll = zst::ll_xbits(L.sym);
      const uint32_t nsb = i + 1 < z.nseq ? L.nb + M.nb + O.nb : 0u;
      const int32_t Pn = br.f.P - int32_t(ofs + xml + xll + nsb);
      const int32_t sft = zst::wb_sft(br, Pn);
      nxt = zst::wb_load(br, br.wd - sft);  // for the next sequence's shift
      const uint32_t p1 = uint32_t(br.f.P - 32 * br.wd) - ofs;  // offset extras at [p1, p1 + ofs)
      const uint32_t p4 = p1 - xml - xll - nsb;                 // state bits at [p4, p4 + nsb)
      const uint64_t e = zst::wb_get64(br, p4);
      const uint32_t ofx = zst::wb_get32(br, p1) & zst::lowmask(ofs);
      const uint32_t sbits = uint32_t(e) & zst::lowmask(nsb);
      const uint32_t llx = uint32_t(e >> nsb) & zst::lowmask(xll);
      const uint32_t mlx = uint32_t(e >> (nsb + xll)) & zst::lowmask(xml);
      // next states (an unused last update reads nothing: nsb = 0) and their
      // entries, in flight during the window shift
      sll = L.base + (sbits >> (M.nb + O.nb));
      sml = M.base + ((sbits >> O.nb) & zst::lowmask(M.nb));
      sof = O.base + (sbits & zst::lowmask(O.nb));
      const uint32_t e0 = T[sll & 511], e1 = T[512 + (sof & 255)], e2 = T[768 + (sml & 511)];
      ell = act ? e0 : ell;
      eof = act ? e1 : eof;
      eml = act ? e2 : eml;
      pend_seq = act ? zst::seq_pack(L.sym, llx, M.sym, mlx, (1u << ofs) + ofx) : pend_seq;
      // the start (< 2^21) and offset code of the sequence stored at the top
      // of this iteration, kept for the one that reads past the stream's
      // start (below)
      pfix = (act && over) ? pl : pfix;
      pl = act ? (br.f.P | int32_t(ofs << 21)) : pl;
      br.f.P = act ? Pn : br.f.P;
      zst::wb_shift(br, cur, act ? sft : 0);
      // the stream overflowed before this sequence: it is not stored; the
      // execution checks of the sequences before it come first (executor)
      st = act ? (over ? zst::kErr : zst::kOK) : st;
      nok += (act && !over) ? 1u : 0u;
    };
    zst::Dw3 nb2;
    // (the first window loads complete before the loop: a load pending at its
    // head would make the head wait on the loop's own loads every trip)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // (no exit between a trip's two sequences: a trip that could end after the
    // first would leave that one's load pending at the loop's head, and the
    // head would wait on the loop's own loads every trip)
    for (uint32_t i = 0; i < z.nseq && st == zst::kOK; i += 2) {
      step(i, br.nx, nb2, true);
      step(i + 1, nb2, br.nx, i + 1 < z.nseq && st == zst::kOK);
    }
    if (st == zst::kOK && z.nseq) S[z.nseq - 1] = pend_seq;
    // The last stored sequence may read extra bits past the stream's start
    // (libzstd's overflow: the next sequence, if any, is not stored), which
    // the window does not mask: the executor reads that one's extra bits
    // again from the stream, those bits as 0 (bits_below).
    if (st != zst::kOK) fix = uint32_t(pfix) | 0x80000000u;  // overflow before the next sequence
    else if (z.nseq && br.f.P < P0) fix = uint32_t(pl) | 0x80000000u;
    if (st == zst::kOK && br.f.P > P0) st = zst::kErr;  // unread bits
  }
  zb[b].st = st;  // the executor ranks it after the sequences' own checks
  zb[b].nseq_ok = nok;
  zb[b].pfix = fix;
}

// ---- stage 3: execution, one wave per segment block --------------------------------
// Sequences in chunks of <= 256 sequences / 4 KiB of output.  For each output
// byte of a chunk the wave records its source -- a literal, output before the
// chunk, or an earlier byte of the chunk -- then resolves in-chunk chains by
// pointer jumping in LDS (sources always lie before the byte, so there are no
// cycles), and gathers every byte independently.
// Diagnostics (OKV_ZSTD_PROF): per-phase cycles accumulated in registers and
// added to this workgroup's own slot, so profiling adds no shared atomics.
#define PMARK(k)                  \
  do {                            \
    if (prof) {                   \
      const long long tq = clock64(); \
      pacc[(k)] += tq - tp0;      \
      tp0 = tq;                   \
    }                             \
  } while (0)
namespace zst {
// Wave64 inclusive max-scan by DPP (wave_scan_dpp's pattern; 0 is the
// identity: unsigned values).  All 64 lanes active.
__device__ __forceinline__ uint32_t wave_max_scan_dpp(uint32_t x) {
  x = max(x, uint32_t(__builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, true)));   // row_shr:1
  x = max(x, uint32_t(__builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, true)));   // row_shr:2
  x = max(x, uint32_t(__builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, true)));   // row_shr:4
  x = max(x, uint32_t(__builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, true)));   // row_shr:8
  x = max(x, uint32_t(__builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false)));  // row_bcast:15
  x = max(x, uint32_t(__builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false)));  // row_bcast:31
  return x;
}
// Bits [P - 64, P) of a sequence stream (bytes outside it read as 0, as the
// sequence stage reads them): bit 63 is stream bit P - 1.
__device__ __forceinline__ uint64_t bits_below(const LaneBits& f, int32_t P) {
  const int32_t a = P - 64;
  const int32_t d0 = a >> 5;  // (arithmetic: a < 0 reads zero dwords)
  const uint32_t s = uint32_t(a) & 31u;
  const uint32_t w0 = lb_dw(f, d0), w1 = lb_dw(f, d0 + 1), w2 = lb_dw(f, d0 + 2);
  return uint64_t(__builtin_amdgcn_alignbit(w1, w0, s)) |
         (uint64_t(__builtin_amdgcn_alignbit(w2, w1, s)) << 32);
}
// The next k (<= 31) bits from the top of g.
__device__ __forceinline__ uint32_t take_top(uint64_t& g, uint32_t k) {
  const uint32_t v = k ? uint32_t(g >> (64u - k)) : 0u;
  g <<= k;
  return v;
}

// Repeat offsets (RFC 8878 3.1.1.5) as maps of the state (rep0, rep1, rep2),
// so a wave resolves 256 sequences' offsets with one scan instead of a lane
// chain.  Slot j of the new state is a constant, or max(r_src - k, 1) of the
// old state; maps of that form compose into that form (max(max(x - a, 1) - b,
// 1) = max(x - a - b, 1)), and every state value is >= 1.  A slot is one
// dword: the constant or k (bits 0-23: offsets are saturated at 2^20 - 1, k
// counts sequences of one window) | src << 24 | const << 26.
struct RepMap {
  uint32_t s0, s1, s2;
};
constexpr uint32_t kRepConst = 1u << 26;
__device__ __forceinline__ RepMap rep_id() { return RepMap{0u, 1u << 24, 2u << 24}; }
// One sequence's map: a new offset (ofv > 3) -> (ofv - 3, r0, r1); else idx =
// ofv - 1 (+1 when the literal length is 0): 0 -> unchanged, 1 -> (r1, r0, r2),
// 2 -> (r2, r0, r1), 3 -> (r0 - 1, r0, r1), where a 0 offset becomes 1 (libzstd).
__device__ __forceinline__ RepMap rep_map(uint32_t ofv, bool ll0) {
  const bool fresh = ofv > 3;
  const uint32_t idx = ofv - 1 + (ll0 ? 1u : 0u);
  const uint32_t a = fresh ? (kRepConst | (ofv - 3)) : idx == 1 ? (1u << 24) : idx == 2 ? (2u << 24)
                                                                             : idx == 3 ? 1u : 0u;
  return RepMap{a, (!fresh && idx == 0) ? (1u << 24) : 0u, (fresh || idx >= 2) ? (1u << 24) : (2u << 24)};
}
__device__ __forceinline__ uint32_t rep_sel(uint32_t j, uint32_t a, uint32_t b, uint32_t c) {
  return j == 0 ? a : j == 1 ? b : c;
}
// slot j of (a, then b)
__device__ __forceinline__ uint32_t rep_slot(const RepMap& a, uint32_t sb) {
  const uint32_t sa = rep_sel((sb >> 24) & 3u, a.s0, a.s1, a.s2);
  const uint32_t vb = sb & 0xffffffu, va = sa & 0xffffffu;
  return (sb & kRepConst) ? sb : (sa & kRepConst) ? (kRepConst | (va > vb ? va - vb : 1u)) : sa + vb;
}
__device__ __forceinline__ RepMap rep_compose(const RepMap& a, const RepMap& b) {
  return RepMap{rep_slot(a, b.s0), rep_slot(a, b.s1), rep_slot(a, b.s2)};
}
__device__ __forceinline__ uint32_t rep_val(uint32_t s, uint32_t r0, uint32_t r1, uint32_t r2) {
  const uint32_t x = rep_sel((s >> 24) & 3u, r0, r1, r2), v = s & 0xffffffu;
  return (s & kRepConst) ? v : (x > v ? x - v : 1u);
}
__device__ __forceinline__ void rep_apply(const RepMap& m, uint32_t& r0, uint32_t& r1, uint32_t& r2) {
  const uint32_t n0 = rep_val(m.s0, r0, r1, r2), n1 = rep_val(m.s1, r0, r1, r2),
                 n2 = rep_val(m.s2, r0, r1, r2);
  r0 = n0;
  r1 = n1;
  r2 = n2;
}
// One DPP step of the wave scan of maps: lanes without a source keep the
// identity (bound_ctrl off), so every lane composes.
template <int kCtrl, int kRows>
__device__ __forceinline__ RepMap rep_dpp(const RepMap& m) {
  const RepMap id = rep_id();
  const RepMap y{uint32_t(__builtin_amdgcn_update_dpp(int(id.s0), int(m.s0), kCtrl, kRows, 0xf, false)),
                 uint32_t(__builtin_amdgcn_update_dpp(int(id.s1), int(m.s1), kCtrl, kRows, 0xf, false)),
                 uint32_t(__builtin_amdgcn_update_dpp(int(id.s2), int(m.s2), kCtrl, kRows, 0xf, false))};
  return rep_compose(y, m);
}
// Inclusive scan of the lanes' maps (lane order = sequence order), DPP as
// wave_scan_dpp.  All 64 lanes active.
__device__ __forceinline__ RepMap rep_scan(RepMap m) {
  m = rep_dpp<0x111, 0xf>(m);  // row_shr:1
  m = rep_dpp<0x112, 0xf>(m);  // row_shr:2
  m = rep_dpp<0x114, 0xf>(m);  // row_shr:4
  m = rep_dpp<0x118, 0xf>(m);  // row_shr:8
  m = rep_dpp<0x142, 0xa>(m);  // row_bcast:15
  m = rep_dpp<0x143, 0xc>(m);  // row_bcast:31
  return m;
}

constexpr uint32_t kTerm = 0x80000000u, kLit = 0x40000000u, kIdx = 0x3fffffffu;
// a global (not flat) byte load: the literal pointer comes from a ZBlk field, so
// the compiler cannot tell its address space; flat loads would count in lgkmcnt
// too and make every LDS wait of the gather drain them
__device__ __forceinline__ uint32_t gload_u8(const uint8_t* p) {
  return *(const __attribute__((address_space(1))) uint8_t*)p;
}
}

// Executor chunk: output bytes covered by one byte map (kEU 16-byte map
// pieces per lane).  1 KiB keeps the workgroup at 9 KiB of LDS: with the
// gather's 128 registers, 16 workgroups per CU (2 KiB: 14 KiB, 11 per CU;
// executor 2.95 -> 2.70 ms, profiles/r3/r3w).
#ifndef OKV_ZSTD_EXEC_OUT
#define OKV_ZSTD_EXEC_OUT 1024
#endif
constexpr uint32_t kExecOut = OKV_ZSTD_EXEC_OUT;
constexpr int kEU = int(kExecOut / 1024);
#ifndef OKV_ZSTD_GQ
#define OKV_ZSTD_GQ 2
#endif
#ifndef OKV_ZSTD_GB
#define OKV_ZSTD_GB 4
#endif
#ifndef OKV_ZSTD_SU
#define OKV_ZSTD_SU 2
#endif
// sequences loaded per chunk: kSU per lane (each chunk loads, scans and records its whole
// window, and a 1 KiB chunk executes far fewer than 256 of them)
constexpr int kSU = OKV_ZSTD_SU;
constexpr uint32_t kSW = 64u * kSU;
static_assert(kSW <= zst::kSeqChunk, "sequence window (byte map entries are 8-bit)");
constexpr int kGQ = OKV_ZSTD_GQ;  // gather: output dwords per lane per step (2 since round 6: at
                                  // the 5-wave cap with 12 B of scratch, executor -2 % against 1,
                                  // profiles/r6/session/zstd_seq_chain_ab.log; round 3 uncapped:
                                  // 2: 128 registers, 4: 163 -- slower, profiles/r3/r3v, r3z)
constexpr int kGB = OKV_ZSTD_GB;  // source resolution: 64-byte groups per batch
static_assert(kExecOut <= zst::kChunkOut && kExecOut % 1024 == 0 && (kExecOut & (kExecOut - 1)) == 0,
              "exec chunk");
// Executor grid (blocks are strided over it); the profiling slots are sized
// for the largest grid.
constexpr uint32_t kExecGridMax = 16384;
// Registers capped for 5 waves per SIMD (with one output dword per lane and
// 4-group batches: 96 registers + 52 B of spills, executor 2.35-2.38 vs
// 2.43-2.51 ms for 2 dwords / 8 groups uncapped, profiles/r3/r3z).  A build
// with -DOKV_ZSTD_EXEC_WPE=0 drops the cap (A/B).
#ifndef OKV_ZSTD_EXEC_WPE
#define OKV_ZSTD_EXEC_WPE 5
#endif
#if OKV_ZSTD_EXEC_WPE > 0
#define OKV_ZSTD_EXEC_ATTR __attribute__((amdgpu_waves_per_eu(OKV_ZSTD_EXEC_WPE)))
#else
#define OKV_ZSTD_EXEC_ATTR
#endif
__global__ __launch_bounds__(64) OKV_ZSTD_EXEC_ATTR void okv_zstd_exec_kernel(
    const zst::ZBlk* __restrict__ zb, uint32_t nblk, const uint64_t* __restrict__ seq_off,
    uint64_t* __restrict__ seqs, const uint64_t* __restrict__ cap_off,
    uint8_t* __restrict__ dec, uint64_t* __restrict__ dec_len, int32_t* __restrict__ zstatus,
    unsigned long long* __restrict__ prof) {
  __shared__ uint4 rec[kSW + 1];
  __shared__ uint32_t srcx[kExecOut];
  __shared__ uint8_t map[kExecOut];
  const int lane = threadIdx.x & 63;
  unsigned long long pacc[10] = {};
  for (uint32_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    const int32_t kind = zst::rfl(uint32_t(zb[b].kind));
    if (kind != zst::kKindSeq) continue;
    // the sequence stage's outcome (stream overflow, unread bits) ranks after
    // the execution checks of the sequences it decoded: those run here, in
    // sequence order, before any sequence is executed (RFC 8878 3.1.1.4; the
    // general kernel's order).  A failed block executes nothing more.
    const int32_t st0 = zst::rfl(uint32_t(zb[b].st));
    const bool exec = st0 == zst::kOK;
    int32_t bst = zst::kOK;
    const uint32_t nseq = zst::rfl(zb[b].nseq_ok), lit_total = zst::rfl(zb[b].lit_total);
    const uint32_t zcap = zst::rfl(zb[b].cap);
    const uint32_t bmax = zst::rfl(zb[b].bmax);  // Block_Maximum_Size (<= 128 KiB)
    const uint32_t flags = zst::rfl(zb[b].flags);
    const bool rle = flags & zst::kFlagRle;
    const uint8_t rle_byte = uint8_t(zst::rfl(zb[b].rle_byte));
    const uint8_t* lits = zst::rflp(zb[b].lits);
    uint8_t* out = dec + zst::rfl64(cap_off[b]);
    uint64_t* S = seqs + zst::rfl64(seq_off[b]);
    // execution checks (3.1.1.4) in sequence order, before anything runs; the
    // block's totals for the end checks.  A failed block executes nothing.
    uint32_t O = 0, lp = 0;
    // the last sequence's extra bits when it read past the stream's start
    // (okv_zstd_seq_kernel leaves those unmasked): read again, masked
    const uint32_t pfix = zst::rfl(zb[b].pfix);
    zst::LaneBits sb;
    {
      const uintptr_t a = reinterpret_cast<uintptr_t>(zst::rflp(zb[b].stream));
      sb.ab = reinterpret_cast<const uint8_t*>(a & ~uintptr_t(3));
      sb.s0 = int32_t(a & 3);
      sb.n = int32_t(zst::rfl(zb[b].stream_len));
    }
    uint32_t rep0 = 1, rep1 = 4, rep2 = 8;  // repeat offsets before the window
    // (the next window's sequences are loaded while this one is checked: the
    // pass is a chain of windows per block)
    uint64_t nx[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) nx[u] = nseq ? S[min(4u * lane + u, nseq - 1)] : 0;
    for (uint32_t i0 = 0; i0 < nseq; i0 += 256) {
      const uint32_t nrem = nseq - i0;
      uint64_t cur[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        cur[u] = nx[u];
        nx[u] = S[min(i0 + 256 + 4u * lane + u, nseq - 1)];
      }
      uint32_t lt = 0, ot = 0, ll[4], ml[4], of[4], ofv[4];
      bool ll0[4];
      zst::RepMap m = zst::rep_id();
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t k = 4 * lane + u;
        const uint64_t vr = cur[u];
        const uint32_t lo = uint32_t(vr), hi = uint32_t(vr >> 32);
        const bool live = k < nrem;
        const uint32_t lc = lo & 63u, mc = (lo >> 22) & 63u;
        uint32_t llx = (lo >> 6) & 0xffffu, mlx = ((lo >> 28) | (hi << 4)) & 0xffffu, ov = hi >> 12;
        if ((pfix >> 31) && i0 + k == nseq - 1) {  // (one lane of one block, rarely)
          const uint32_t oc = (pfix >> 21) & 31u;
          uint64_t g = zst::bits_below(sb, int32_t(pfix & 0x1fffffu));
          const uint32_t ofx = zst::take_top(g, oc);
          mlx = zst::take_top(g, zst::ml_xbits(mc));
          llx = zst::take_top(g, zst::ll_xbits(lc));
          ov = min((1u << oc) + ofx, 0xfffffu);
        }
        // (baselines computed, not looked up: an LDS table would cost this
        // kernel a workgroup per CU, 11 -> 10)
        ll[u] = live ? zst::ll_base(lc) + llx : 0u;
        ml[u] = live ? zst::ml_base(mc) + mlx : 0u;
        ofv[u] = live ? ov : 1u;  // a dead sequence: the identity map
        ll0[u] = live && lc == 0;
        m = zst::rep_compose(m, zst::rep_map(ofv[u], ll0[u]));
        lt += ll[u];
        ot += ll[u] + ml[u];
      }
      // repeat offsets: the maps of the lanes before this one, applied to the
      // state before the window, then this lane's sequences in order
      m = zst::rep_scan(m);
      {
        zst::RepMap ex{uint32_t(__shfl_up(int(m.s0), 1, 64)), uint32_t(__shfl_up(int(m.s1), 1, 64)),
                       uint32_t(__shfl_up(int(m.s2), 1, 64))};
        if (lane == 0) ex = zst::rep_id();
        uint32_t r0 = rep0, r1 = rep1, r2 = rep2;
        zst::rep_apply(ex, r0, r1, r2);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          zst::rep_apply(zst::rep_map(ofv[u], ll0[u]), r0, r1, r2);
          // (an offset past 2^20 - 1 is past any single-block frame's output,
          // which is held to Block_Maximum_Size (<= 128 KiB) before the offset
          // check below, so the saturated value fails the same check)
          of[u] = 4 * lane + u < nrem ? min(r0, 0xfffffu) : 0u;
        }
        rep0 = __builtin_amdgcn_readlane(r0, 63);
        rep1 = __builtin_amdgcn_readlane(r1, 63);
        rep2 = __builtin_amdgcn_readlane(r2, 63);
      }
      uint32_t lpx = wave_scan_dpp(lt) - lt, opx = wave_scan_dpp(ot) - ot;
      // the lengths back in place for the execution pass: ll (18 bits) | ml (18)
      // << 18 | offset (28) << 36 (lengths < 2^18; a block that fails a check
      // below is never executed)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t k = 4 * lane + u;
        if (k < nrem)
          S[i0 + k] = uint64_t(ll[u]) | (uint64_t(ml[u]) << 18) | (uint64_t(of[u]) << 36);
      }
      uint32_t fcode = 0;  // the lane's first failing sequence: 1 / 3 / 4 kErr, 2 kCap
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        // (32-bit: lengths < 2^18, 256 per window, totals <= cap < 2^31)
        const uint32_t mst = O + opx + ll[u];  // match start in the block output
        // (the general kernel's order; a block past Block_Maximum_Size is
        // corrupt whatever its region, so that check precedes the capacity)
        const uint32_t code = 4 * lane + u >= nrem            ? 0u
                              : lp + lpx + ll[u] > lit_total  ? 1u
                              : mst + ml[u] > bmax            ? 4u
                              : of[u] > mst                   ? 3u
                              : mst + ml[u] > zcap            ? 2u
                                                              : 0u;
        fcode = fcode ? fcode : code;
        lpx += ll[u];
        opx += ll[u] + ml[u];
      }
      const uint64_t fm = __ballot(fcode != 0);
      if (fm) {
        const uint32_t c = __builtin_amdgcn_readlane(fcode, __ffsll(static_cast<unsigned long long>(fm)) - 1);
        bst = c == 2 ? zst::kCap : zst::kErr;
        break;
      }
      O += __builtin_amdgcn_readlane(opx, 63);
      lp += __builtin_amdgcn_readlane(lpx, 63);
    }
    if (bst == zst::kOK && !exec) bst = st0;
    if (bst == zst::kOK && uint64_t(O) + (lit_total - lp) > bmax) bst = zst::kErr;
    if (bst == zst::kOK && uint64_t(O) + (lit_total - lp) > zcap) bst = zst::kCap;
    if (bst == zst::kOK && (flags & zst::kFlagFcs) && uint64_t(O) + (lit_total - lp) != zb[b].fcs)
      bst = zst::kErr;  // Frame_Content_Size check
    if (bst != zst::kOK) {
      if (lane == 0) {
        zstatus[b] = bst == zst::kCap ? OKV_BLK_CAPACITY : OKV_BLK_ZSTD_ERROR;
        dec_len[b] = 0;
      }
      continue;
    }
    O = 0;
    lp = 0;
    // (each window's records are loaded as soon as the window before it knows
    // its length, so the load runs under that window's execution)
    uint64_t nxr[kSU];
#pragma unroll
    for (int u = 0; u < kSU; ++u) nxr[u] = nseq ? S[min(uint32_t(kSU * lane + u), nseq - 1)] : 0;
    for (uint32_t i0 = 0; i0 < nseq;) {
      long long tp0 = prof ? clock64() : 0;
      const uint32_t nrem = nseq - i0;
      // up to kSW sequences: lane holds sequences kSU lane .. kSU lane + kSU - 1
      uint32_t ll[kSU], ml[kSU], of[kSU];
      uint32_t lt = 0, ot = 0;
#pragma unroll
      for (int u = 0; u < kSU; ++u) {
        const uint32_t k = kSU * lane + u;
        const uint64_t v = k < nrem ? nxr[u] : 0;
        ll[u] = uint32_t(v) & 0x3ffff;
        ml[u] = uint32_t(v >> 18) & 0x3ffff;
        of[u] = uint32_t(v >> 36);
        lt += ll[u];
        ot += ll[u] + ml[u];
      }
      uint32_t lpx = wave_scan_dpp(lt) - lt, opx = wave_scan_dpp(ot) - ot;
      uint32_t fit = 0;  // sequences that end within the byte map (a prefix: ballots)
#pragma unroll
      for (int u = 0; u < kSU; ++u) {
        const uint32_t k = kSU * lane + u;
        rec[k] = make_uint4(opx, ll[u], of[u], lpx);
        lpx += ll[u];
        opx += ll[u] + ml[u];
        fit += uint32_t(__builtin_popcountll(__ballot(k < nrem && opx <= kExecOut)));
      }
      if (lane == 63) rec[kSW] = make_uint4(opx, 0, 0, lpx);
      const uint32_t cnt = fit ? fit : 1;  // a single long sequence when none fits
#pragma unroll
      for (int u = 0; u < kSU; ++u) nxr[u] = S[min(i0 + cnt + uint32_t(kSU * lane + u), nseq - 1)];
      __syncthreads();
      const uint32_t osum = zst::rfl(rec[cnt].x), lsum = zst::rfl(rec[cnt].w);
      PMARK(0);
      if (fit) {
        // byte -> sequence map: markers, then a running max
        uint4* m4 = reinterpret_cast<uint4*>(map);
#pragma unroll
        for (int u = 0; u < kEU; ++u) m4[kEU * lane + u] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        for (uint32_t k = lane + 1; k < cnt; k += 64) map[rec[k].x] = uint8_t(k);
        __syncthreads();
        uint4 v[kEU];
        uint32_t mx = 0;
#pragma unroll
        for (int u = 0; u < kEU; ++u) {
          v[u] = m4[kEU * lane + u];
          const uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int t = 0; t < 4; ++t) mx = max(mx, (w4[q] >> (8 * t)) & 0xffu);
        }
        uint32_t run = zst::wave_max_scan_dpp(mx);
        run = __shfl_up(run, 1, 64);
        if (lane == 0) run = 0;
#pragma unroll
        for (int u = 0; u < kEU; ++u) {
          uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            uint32_t outw = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              run = max(run, (w4[q] >> (8 * t)) & 0xffu);
              outw |= run << (8 * t);
            }
            w4[q] = outw;
          }
          m4[kEU * lane + u] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
        __syncthreads();
        PMARK(1);
        // each byte's source, resolved to a terminal (a literal or output before
        // the chunk) a batch of kGB 64-byte groups at a time: the batch's
        // immediate sources are computed and stored (map and record reads all in
        // flight), then followed by pointer jumping over the whole batch.  A
        // source before the batch is already terminal (one read); chains inside
        // the batch halve each round.  Every entry always holds a source of its
        // byte (its own, or one further along its chain), and LDS operations of
        // one wave complete in order, so the rounds' reads and writes need no
        // other ordering.
        uint32_t rounds = 0;
        for (uint32_t x0 = 0; x0 < osum; x0 += 64 * kGB) {
          uint32_t kk[kGB];
#pragma unroll
          for (int u = 0; u < kGB; ++u) {
            const uint32_t x = x0 + 64 * u + lane;
            kk[u] = map[x];  // (x < x0 + 64 kGB <= kExecOut; past osum: ignored below)
          }
          uint4 R[kGB];
#pragma unroll
          for (int u = 0; u < kGB; ++u) R[u] = rec[kk[u]];
          uint32_t sv[kGB];
#pragma unroll
          for (int u = 0; u < kGB; ++u) {
            // branch-free: a literal byte, or a match byte whose source is
            // before the chunk (terminal) or inside it.  A byte past the first
            // period of an overlapping match (offset < match length) points at
            // the byte one period earlier, which the pointer jumping resolves (a
            // modulo here cost more than the extra rounds: 8.3K -> 5.3K cycles
            // per chunk, profiles/r3/r3t)
            const uint32_t x = x0 + 64 * u + lane;
            const uint32_t in = x - R[u].x;
            const bool lit = in < R[u].y;
            const int32_t sx = int32_t(x) - int32_t(R[u].z);
            const uint32_t vm = sx < 0 ? (zst::kTerm | uint32_t(int32_t(O) + sx)) : uint32_t(sx);
            const uint32_t vl = zst::kTerm | zst::kLit | (lp + R[u].w + in);
            sv[u] = x >= osum ? zst::kTerm : lit ? vl : vm;
          }
          PMARK(2);
          // (reads and writes unconditional and branch-free: x < x0 + 64 kGB <=
          // kExecOut, and a terminal entry's index bits read some entry of the
          // map, whose value is dropped; entries past osum are never used)
          bool pend = false;
#pragma unroll
          for (int u = 0; u < kGB; ++u) {
            srcx[x0 + 64 * u + lane] = sv[u];
            pend |= !(sv[u] & zst::kTerm);
          }
          while (__any(pend)) {
            uint32_t r[kGB];
#pragma unroll
            for (int u = 0; u < kGB; ++u) r[u] = srcx[sv[u] & (kExecOut - 1)];
            pend = false;
#pragma unroll
            for (int u = 0; u < kGB; ++u) {
              sv[u] = (sv[u] & zst::kTerm) ? sv[u] : r[u];
              srcx[x0 + 64 * u + lane] = sv[u];
              pend |= !(sv[u] & zst::kTerm);
            }
            ++rounds;
          }
          PMARK(3);
        }
        __syncthreads();
        PMARK(3);
        pacc[8] += rounds;
        // gather: lanes own aligned output dwords (kGQ per lane per step, 4 kGQ
        // byte loads in flight, one dword store each).  A head byte before O is
        // re-read from the previous chunk's output; tail bytes past the chunk
        // are written as 0 and overwritten by the next chunk the same way.
        // Branch-free: every source entry is read first (the index clamped into
        // the map: a head byte's wraps, a tail byte's is stale, both ignored),
        // then every byte is loaded from a valid address (an RLE literal or a
        // zero byte reads the block's first output byte) and selected.
        // the previous chunk's stores visible to this gather's loads (waited
        // here, not at that chunk's end: they complete under this chunk's
        // source resolution)
        __builtin_amdgcn_s_waitcnt(0);
        __threadfence_block();
        const uint32_t g0 = O >> 2, g1 = (O + osum + 3) >> 2;
        const uint64_t out_a = reinterpret_cast<uint64_t>(out);
        const uint64_t lit_a = reinterpret_cast<uint64_t>(lits);
        for (uint32_t gb = g0 + lane; gb < g1; gb += 64 * kGQ) {
          uint32_t sv[4 * kGQ];
#pragma unroll
          for (int u = 0; u < 4 * kGQ; ++u) {
            const uint32_t a = 4 * (gb + 64 * (u >> 2)) + (u & 3);
            sv[u] = srcx[min(a - O, kExecOut - 1)];
          }
          uint32_t bv[4 * kGQ], sel[4 * kGQ];  // sel: 0 zero, 1 RLE literal, 2 loaded
#pragma unroll
          for (int u = 0; u < 4 * kGQ; ++u) {
            const uint32_t g = gb + 64 * (u >> 2);
            const uint32_t a = 4 * g + (u & 3);
            const bool in = g < g1 && a - O < osum;  // (a < O wraps)
            const bool head = g < g1 && a < O;
            const bool lit = in && (sv[u] & zst::kLit);
            const bool rl = lit && rle;
            const uint64_t base = lit && !rle ? lit_a : out_a;
            const uint32_t idx = in && !rl ? (sv[u] & zst::kIdx) : head ? a : 0u;
            bv[u] = zst::gload_u8(reinterpret_cast<const uint8_t*>(base + idx));
            sel[u] = in || head ? (rl ? 1u : 2u) : 0u;
          }
#pragma unroll
          for (int q = 0; q < kGQ; ++q) {
            const uint32_t g = gb + 64 * q;
            uint32_t w = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int u = 4 * q + j;
              const uint32_t v = sel[u] == 2 ? (bv[u] & 0xffu) : sel[u] == 1 ? rle_byte : 0u;
              w |= v << (8 * j);
            }
            if (g < g1) reinterpret_cast<uint32_t*>(out)[g] = w;
          }
        }
      } else {
        // one sequence longer than the map: every match byte lands on this
        // sequence's literals or on output before it; stored as aligned dwords
        const uint4 R = rec[0];
        __builtin_amdgcn_s_waitcnt(0);  // (the previous chunk's stores, as above)
        __threadfence_block();
        const uint32_t g0 = O >> 2, g1 = (O + osum + 3) >> 2;
        for (uint32_t gb = g0 + lane; gb < g1; gb += 64 * kGQ) {
          const uint8_t* ptr[4 * kGQ];
          uint32_t spec[4 * kGQ];
#pragma unroll
          for (int u = 0; u < 4 * kGQ; ++u) {
            const uint32_t g = gb + 64 * (u >> 2);
            const uint32_t a = 4 * g + (u & 3);
            const uint32_t x = a - O;
            const bool in = g < g1 && a >= O && x < osum;
            int32_t sx;  // literal index (>= 0) of this sequence, or output offset from O
            if (x < R.y) {
              sx = int32_t(x);
            } else {
              const uint32_t t = x - R.y, off = R.z;
              const uint32_t mo = t < off ? t : t % off;
              sx = int32_t(R.y + mo) - int32_t(off);
            }
            spec[u] = (g >= g1 || (a >= O && !in)) ? 2u : ((in && sx >= 0 && rle) ? 1u : 0u);
            ptr[u] = spec[u] ? out
                             : (!in ? out + a
                                    : (sx >= 0 ? lits + lp + uint32_t(sx) : out + (int32_t(O) + sx)));
          }
          uint32_t bv[4 * kGQ];
#pragma unroll
          for (int u = 0; u < 4 * kGQ; ++u) bv[u] = zst::gload_u8(ptr[u]);
#pragma unroll
          for (int q = 0; q < kGQ; ++q) {
            const uint32_t g = gb + 64 * q;
            uint32_t w = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int u = 4 * q + j;
              const uint32_t v = spec[u] == 2 ? 0u : spec[u] == 1 ? rle_byte : (bv[u] & 0xffu);
              w |= v << (8 * j);
            }
            if (g < g1) reinterpret_cast<uint32_t*>(out)[g] = w;
          }
        }
      }
      PMARK(4);
      __syncthreads();
      PMARK(5);
      pacc[9] += 1;
      O += osum;
      lp += lsum;
      i0 += cnt;
    }
    // literals after the last sequence
    {
      __builtin_amdgcn_s_waitcnt(0);  // (the last chunk's stores)
      __threadfence_block();
      const uint32_t tl = lit_total - lp;
      const uint32_t g0 = O >> 2, g1 = (O + tl + 3) >> 2;
      for (uint32_t gb = g0 + lane; gb < g1; gb += 64 * kGQ) {
        uint32_t bv[4 * kGQ];
        uint32_t spec[4 * kGQ];
#pragma unroll
        for (int u = 0; u < 4 * kGQ; ++u) {
          const uint32_t g = gb + 64 * (u >> 2);
          const uint32_t a = 4 * g + (u & 3);
          const bool in = g < g1 && a >= O && a - O < tl;
          spec[u] = (g >= g1 || (a >= O && !in)) ? 2u : ((in && rle) ? 1u : 0u);
          const uint8_t* ptr = spec[u] ? out : (!in ? out + a : lits + lp + (a - O));
          bv[u] = zst::gload_u8(ptr);
        }
#pragma unroll
        for (int q = 0; q < kGQ; ++q) {
          const uint32_t g = gb + 64 * q;
          uint32_t w = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int u = 4 * q + j;
            const uint32_t v = spec[u] == 2 ? 0u : spec[u] == 1 ? rle_byte : (bv[u] & 0xffu);
            w |= v << (8 * j);
          }
          if (g < g1) reinterpret_cast<uint32_t*>(out)[g] = w;
        }
      }
      O += tl;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __threadfence_block();
    int32_t st = OKV_BLK_OK;
    if (flags & zst::kFlagCsum) {
      const uint64_t h = zst::xxh64_out(out, O);
      if (uint32_t(h) != zst::rfl(zb[b].csum)) st = OKV_BLK_ZSTD_ERROR;
    }
    if (lane == 0) {
      zstatus[b] = st;
      dec_len[b] = st == OKV_BLK_OK ? O : 0;
    }
  }
  if (prof && lane == 0)
    for (int k = 0; k < 10; ++k) prof[blockIdx.x * 16 + k] = pacc[k];
}

// First output region of a block: round16(OriginalSize), which is exactly the
// frame's output for Go-written blocks -- bounded, so a descriptor claiming a
// huge OriginalSize does not size the scratch (int(OriginalSize) < 0 walks no
// record at all, :340).  Frames that decompress past the region are decoded
// again into a region of their measured size (zstd_run).
__device__ __forceinline__ uint64_t first_region(const Desc& d) {
  const uint64_t bound = (uint64_t(1) << 20) + 32 * min(d.compressed_size, uint64_t(1) << 32);
  return round16(min(d.original_size, bound));
}

// Exclusive scan of per-block first regions (first_region).
__global__ __launch_bounds__(1024) void okv_zstd_cap_kernel(const Desc* __restrict__ descs,
                                                            uint32_t nblk,
                                                            uint64_t* __restrict__ cap_off) {
  zst::block_excl_scan(nblk, [&](uint32_t i) -> uint64_t { return first_region(descs[i]); }, cap_off);
}

// Descriptors of the decompressed blocks for the record walk (passes 1-3):
// offset into the scratch, BlockSize = decompressed length.
__global__ void okv_zstd_desc_kernel(const Desc* __restrict__ descs, uint32_t nblk,
                                     const uint64_t* __restrict__ cap_off,
                                     const uint64_t* __restrict__ dec_len,
                                     Desc* __restrict__ out) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  Desc d;
  d.offset = cap_off[b];
  d.block_size = dec_len[b];
  d.original_size = descs[b].original_size;
  d.compressed_size = 0;
  out[b] = d;
}

// Frames that decompress past their first region (first_region): the general
// kernel measures each one's whole output (a pass that reads and writes no
// byte), then decodes it into a region of that size appended to the scratch
// (kept: the other blocks' bytes are already there).  Go's io.Copy inflates
// the whole frame set before the record walk (segment_reader.go:320-330), so
// these blocks decode and walk like any other; no OKV_BLK_CAPACITY status
// leaves the zstd stage.  One extra host round trip per zstd decode (the
// retry count); Go-written blocks never need the retry.
int zstd_regrow(okv_ctx* ctx, const uint8_t* seg, uint64_t seg_bytes, const Desc* descs,
                uint32_t nblk, uint64_t* total_io) {
  hipStream_t s = ctx->stream;
  int rc;
  if ((rc = grow(ctx, reinterpret_cast<void**>(&ctx->z_list), &ctx->z_cap_list,
                 (size_t(nblk) + 1) * 4 + 64)))
    return rc;
  uint32_t* d_count = ctx->z_list + nblk;
  OKV_HIP(hipMemsetAsync(d_count, 0, 4, s));
  hipLaunchKernelGGL(okv_zstd_list_kernel, dim3((nblk + 255) / 256), dim3(256), 0, s, ctx->z_status,
                     nblk, ctx->z_list, d_count);
  uint32_t n = 0;
  OKV_HIP(hipMemcpyAsync(&n, d_count, 4, hipMemcpyDeviceToHost, s));
  OKV_HIP(hipStreamSynchronize(s));
  ctx->z_retried = n;
  if (n == 0) return OKV_OK;
  if ((rc = grow(ctx, reinterpret_cast<void**>(&ctx->z_need), &ctx->z_cap_need,
                 (size_t(n) * 2 + 2) * 8)))
    return rc;
  uint64_t* need = ctx->z_need;
  uint64_t* roff = ctx->z_need + n;
  const uint32_t grid = std::min<uint32_t>(n, 2048);
  // the literal scratch is sized for the first pass's grid (>= this one)
  hipLaunchKernelGGL(okv_zstd_kernel, dim3(grid), dim3(64), 0, s, seg, seg_bytes, descs, nblk,
                     ctx->z_cap_off, ctx->z_dec, ctx->z_dec_len, ctx->z_status, ctx->z_lit, nullptr,
                     nullptr, ZRetry{ctx->z_list, n, 1, nullptr, need, nullptr});
  const uint64_t base = (*total_io + 15) & ~uint64_t(15);
  hipLaunchKernelGGL(okv_zstd_roff_kernel, dim3(1), dim3(1024), 0, s, need, n, base, roff);
  OKV_HIP(hipGetLastError());
  uint64_t end = 0;
  OKV_HIP(hipMemcpyAsync(&end, roff + n, 8, hipMemcpyDeviceToHost, s));
  OKV_HIP(hipStreamSynchronize(s));
  if (end + 64 > ctx->z_cap_dec) {  // grow the scratch, keeping the first pass's bytes
    uint8_t* nd = nullptr;
    const size_t c = (size_t(end) + 64 + 4095) & ~size_t(4095);
    OKV_HIP(hipMalloc(&nd, c));
    OKV_HIP(hipMemcpyAsync(nd, ctx->z_dec, *total_io, hipMemcpyDeviceToDevice, s));
    OKV_HIP(hipStreamSynchronize(s));
    (void)hipFree(ctx->z_dec);
    ctx->z_dec = nd;
    ctx->z_cap_dec = c;
  }
  hipLaunchKernelGGL(okv_zstd_kernel, dim3(grid), dim3(64), 0, s, seg, seg_bytes, descs, nblk,
                     ctx->z_cap_off, ctx->z_dec, ctx->z_dec_len, ctx->z_status, ctx->z_lit, nullptr,
                     nullptr, ZRetry{ctx->z_list, n, 0, roff, nullptr, ctx->z_cap_off});
  OKV_HIP(hipGetLastError());
  *total_io = end;
  return OKV_OK;
}

// Decompress every block into dec + cap_off[b] (capacities already scanned;
// total = cap_off[nblk]).  Stages: prologue -> sequence offsets -> sequences ->
// executor -> general kernel for the blocks the prologue handed over.
// OKV_ZSTD_GENERAL=1 sends every block through the general kernel (A/B);
// OKV_ZSTD_PROF=1 prints per-stage milliseconds to stderr (diagnostics only).
int zstd_run(okv_ctx* ctx, const uint8_t* seg, uint64_t seg_bytes, const Desc* descs,
             uint32_t nblk, uint64_t* total_io) {
  hipStream_t s = ctx->stream;
  int rc;
  const uint64_t total = *total_io;
  const bool general = ctx->zstd_one_pass || okv::knob("OKV_ZSTD_GENERAL") != nullptr;
  const bool prof = okv::knob("OKV_ZSTD_PROF") != nullptr;
  hipEvent_t ev[6] = {};
  if (prof)
    for (auto& e : ev) (void)hipEventCreate(&e);
  if (prof) (void)hipEventRecord(ev[0], s);
  zst::ZBlk* zb = nullptr;
  static unsigned long long* eprof_buf = nullptr;
  unsigned long long* eprof = nullptr;
  if (prof) {
    if (!eprof_buf) (void)hipMalloc(&eprof_buf, 16 * 8 * kExecGridMax);
    eprof = eprof_buf;
    (void)hipMemsetAsync(eprof, 0, 16 * 8 * kExecGridMax, s);
  }
  static unsigned long long* pprof_buf = nullptr;  // prologue phase cycles (diagnostics)
  unsigned long long* pprof = nullptr;
  if (prof) {
    if (!pprof_buf) (void)hipMalloc(&pprof_buf, 16 * 8);
    pprof = pprof_buf;
    (void)hipMemsetAsync(pprof, 0, 16 * 8, s);
  }
  if (!general) {
    if ((rc = grow(ctx, reinterpret_cast<void**>(&ctx->z_zb), &ctx->z_cap_zb,
                   size_t(nblk) * sizeof(zst::ZBlk))))
      return rc;
    if ((rc = grow(ctx, reinterpret_cast<void**>(&ctx->z_tabs), &ctx->z_cap_tabs,
                   size_t(nblk) * (zst::kTabEnt + zst::kHufSlot) * 2 + 16)))
      return rc;
    if ((rc = grow(ctx, reinterpret_cast<void**>(&ctx->z_blit), &ctx->z_cap_blit, total + 64)))
      return rc;
    if ((rc = grow(ctx, reinterpret_cast<void**>(&ctx->z_seq_off), &ctx->z_cap_seq_off,
                   (size_t(nblk) + 1) * 8)))
      return rc;
    zb = reinterpret_cast<zst::ZBlk*>(ctx->z_zb);
    uint16_t* htab = reinterpret_cast<uint16_t*>(ctx->z_tabs) + size_t(nblk) * zst::kTabEnt;
    // one workgroup per block (no per-workgroup scratch; OKV_ZSTD_PRO_GRID: A/B)
    const uint32_t pgrid = okv::knob("OKV_ZSTD_PRO_GRID") ? uint32_t(atoi(okv::knob("OKV_ZSTD_PRO_GRID")))
                                                       : nblk;
    hipLaunchKernelGGL(okv_zstd_pro_kernel, dim3(std::max(1u, std::min(nblk, pgrid))), dim3(64), 0, s,
                       seg, seg_bytes, descs, nblk, ctx->z_cap_off, ctx->z_dec, ctx->z_dec_len,
                       ctx->z_status, ctx->z_blit, reinterpret_cast<uint16_t*>(ctx->z_tabs), htab, zb,
                       ctx->z_seq_off, pprof);
    hipLaunchKernelGGL(okv_zstd_seqoff_kernel, dim3(1), dim3(1024), 0, s, nblk, ctx->z_seq_off);
    uint64_t nseq_total = 0;
    OKV_HIP(hipMemcpyAsync(&nseq_total, ctx->z_seq_off + nblk, 8, hipMemcpyDeviceToHost, s));
    if (!ctx->z_ev) OKV_HIP(hipEventCreateWithFlags(&ctx->z_ev, hipEventDisableTiming));
    OKV_HIP(hipEventRecord(ctx->z_ev, s));
    // the literal streams decode while the host reads the sequence count
#ifdef OKV_ABLATE
    const uint32_t hb = okv::knob("OKV_ZSTD_HUF_BLOCKS") ? uint32_t(atoi(okv::knob("OKV_ZSTD_HUF_BLOCKS")))
                                                        : kHufBlocks;
    if (hb == 16)
      hipLaunchKernelGGL(okv_zstd_huf_kernel<16>, dim3((nblk + 15) / 16), dim3(64), 0, s, zb, nblk,
                         htab, seg, ctx->z_blit, ctx->z_cap_off);
    else if (hb == 8)
      hipLaunchKernelGGL(okv_zstd_huf_kernel<8>, dim3((nblk + 7) / 8), dim3(64), 0, s, zb, nblk,
                         htab, seg, ctx->z_blit, ctx->z_cap_off);
    else if (hb == 2)
      hipLaunchKernelGGL(okv_zstd_huf_kernel<2>, dim3((nblk + 1) / 2), dim3(64), 0, s, zb, nblk,
                         htab, seg, ctx->z_blit, ctx->z_cap_off);
    else
#endif
    hipLaunchKernelGGL(okv_zstd_huf_kernel<kHufBlocks>, dim3((nblk + kHufBlocks - 1) / kHufBlocks),
                       dim3(64), 0, s, zb, nblk, htab, seg, ctx->z_blit, ctx->z_cap_off);
    OKV_HIP(hipEventSynchronize(ctx->z_ev));
    if (prof) (void)hipEventRecord(ev[1], s);
    if ((rc = grow(ctx, reinterpret_cast<void**>(&ctx->z_seqs), &ctx->z_cap_seqs,
                   nseq_total * 8 + 64)))
      return rc;
    hipLaunchKernelGGL(okv_zstd_seq_kernel, dim3((nblk + 63) / 64), dim3(64), 0, s, zb, nblk,
                       reinterpret_cast<const uint16_t*>(ctx->z_tabs), ctx->z_seq_off, ctx->z_seqs);
    if (prof) (void)hipEventRecord(ev[2], s);
    // one workgroup per block by default: the dispatcher balances blocks of
    // unequal work better than a grid-stride loop (16 384 x 64 KiB: 3.8 ms vs
    // 4.6 ms at 4096 workgroups, 5.6 at 2816); profiling caps it at its slots
    uint32_t egrid = okv::knob("OKV_ZSTD_EXEC_GRID") ? uint32_t(atoi(okv::knob("OKV_ZSTD_EXEC_GRID")))
                                                  : nblk;
    if (prof) egrid = std::min(egrid, kExecGridMax);
    egrid = std::max(egrid, 1u);
#ifndef OKV_ZSTD_EXEC_PAD  // A/B builds: dynamic LDS per workgroup to lower the executor's occupancy
#define OKV_ZSTD_EXEC_PAD 0  // (18 / 16 / 11 per CU: slower, zstd_seq_chain_ab.log)
#endif
    hipLaunchKernelGGL(okv_zstd_exec_kernel, dim3(std::min<uint32_t>(nblk, egrid)), dim3(64),
                       OKV_ZSTD_EXEC_PAD, s,
                       zb, nblk, ctx->z_seq_off, ctx->z_seqs, ctx->z_cap_off, ctx->z_dec,
                       ctx->z_dec_len, ctx->z_status, eprof);
  }
  if (prof) (void)hipEventRecord(ev[3], s);
  const uint32_t grid = std::min<uint32_t>(nblk, 2048);
  if ((rc = grow(ctx, reinterpret_cast<void**>(&ctx->z_lit), &ctx->z_cap_lit,
                 size_t(grid) * kZstdLitBytes)))
    return rc;
  hipLaunchKernelGGL(okv_zstd_kernel, dim3(grid), dim3(64), 0, s, seg, seg_bytes, descs, nblk,
                     ctx->z_cap_off, ctx->z_dec, ctx->z_dec_len, ctx->z_status, ctx->z_lit,
                     nullptr, zb, ZRetry{nullptr, 0, 0, nullptr, nullptr, nullptr});
  OKV_HIP(hipGetLastError());
  if ((rc = zstd_regrow(ctx, seg, seg_bytes, descs, nblk, total_io))) return rc;
  if (prof) {
    (void)hipEventRecord(ev[4], s);
    (void)hipStreamSynchronize(s);
    float t[4] = {};
    for (int k = 0; k < 4; ++k) (void)hipEventElapsedTime(&t[k], ev[k], ev[k + 1]);
    fprintf(stderr,
            "[zstd prof] %u blocks: prologue+seqoff %.3f ms, sequences %.3f ms, executor %.3f ms, "
            "general %.3f ms\n",
            nblk, t[0], t[1], t[2], t[3]);
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    static unsigned long long hs[16 * kExecGridMax];
    (void)hipMemcpy(hs, eprof, sizeof(hs), hipMemcpyDeviceToHost);
    unsigned long long h[16] = {};
    for (uint32_t w = 0; w < kExecGridMax; ++w)
      for (int k = 0; k < 16; ++k) h[k] += hs[w * 16 + k];
    const double c = h[9] ? double(h[9]) : 1.0;
    fprintf(stderr,
            "[zstd exec] chunks %llu, cycles/chunk: load+scan %.0f map %.0f sources %.0f jump %.0f "
            "(rounds %.2f) gather %.0f commit %.0f\n",
            h[9], h[0] / c, h[1] / c, h[2] / c, h[3] / c, h[8] / c, h[4] / c, h[5] / c);
    unsigned long long pp[16] = {};
    (void)hipMemcpy(pp, pprof, sizeof(pp), hipMemcpyDeviceToHost);
    const double nb = pp[13] ? double(pp[13]) : 1.0;
    fprintf(stderr,
            "[zstd pro] blocks %llu, cycles/block: whole %.0f literals %.0f (huffman tree %.0f) "
            "sequence tables %.0f\n",
            pp[13], pp[11] / nb, pp[0] / nb, pp[12] / nb, pp[10] / nb);
  }
  return OKV_OK;
}
void launch_zstd_cap(hipStream_t s, const Desc* descs, uint32_t nblk, uint64_t* cap_off) {
  hipLaunchKernelGGL(okv_zstd_cap_kernel, dim3(1), dim3(1024), 0, s, descs, nblk, cap_off);
}
void launch_zstd_desc(hipStream_t s, const Desc* descs, uint32_t nblk, const uint64_t* cap_off,
                      const uint64_t* dec_len, Desc* out) {
  hipLaunchKernelGGL(okv_zstd_desc_kernel, dim3((nblk + 255) / 256), dim3(256), 0, s, descs, nblk,
                     cap_off, dec_len, out);
}

}  // namespace okv

#ifdef OKV_ZSTD_TRACE
// Diagnostic: the last corrupt-input exit's source line and the exit count
// since the previous call (then reset).
extern "C" int okv_debug_zstd_err(int* out2) {
  int h[4] = {};
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(okv::zst::g_zerr), sizeof(h)) != hipSuccess) return -1;
  out2[0] = h[0];
  out2[1] = h[1];
  out2[2] = h[2];
  out2[3] = h[3];
  int z[4] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(okv::zst::g_zerr), z, sizeof(z));
  return 0;
}
#endif
