// okv_decode.hip -- MI355X (gfx950) batched SST data-block decode.
//
// Replaces the record loop of sst.SegmentReader.ReadBlockWithStat
// (/root/reference/sst/segment_reader.go:295-355) for many blocks at once.
// Launches per call:
//   1. okv_count_kernel  -- one lane per block walks the record headers in
//      HBM, validating exactly what the Go loop validates; per block it emits
//      (status, rows, key bytes, value bytes, end position), the positions and
//      key lengths of its first kRCap records (block-major table, written
//      through LDS in whole 16-byte pieces) and a 256-block exclusive scan.
//      Blocks with more rows go on the "big block" list.  Pass 2 runs in the
//      same launch: the workgroup that arrives last scans the tile totals
//      (sc1 hand-off), so a decode needs no memset and no scan launch.
//   2. pass 3, by the call's average block span:
//      okv_tile_kernel (> 16 KiB, the C3/C5 kernel) -- one workgroup per
//        16 KiB source tile of a block: the tile's bytes are DMA'd into LDS
//        while wave 0 rebuilds the row table from pass 1's record table; whole
//        value chunks go out as wave-uniform runs, keys and the chunks that
//        mix rows by a per-lane lookup; tile 0 writes the SoA row index.
//      okv_gather_small_kernel (<= 16 KiB blocks) -- one wave per block, the
//        whole block staged in LDS.
//      okv_decode_fused_kernel (<= 512 small blocks) -- passes 1-3 in one
//        launch (replaces 1 and 2 as well).
//   3. okv_copy_kernel   -- persistent, over the big-block list only: stages
//      the block in LDS and chases its headers there (rare: > kRCap rows).
// OKV_F_INDEX_ONLY writes spans into seg instead of arenas (+ okv_index_kernel).
// Measured alternatives to pass 3 are in DESIGN.md §4 and the ablation build
// (-DOKV_ABLATE).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "okv_ctx.hpp"
#include "okv_kernels.hpp"
#include "okv_sst.h"

namespace okv {

// Record table from pass 1, block-major: record r < kRCap of block b at
// rt_pos[b * kRCap + r] (u32 position in the block) and rt_kl[b * kRCap + r]
// (u16 key length).  A consumer wave reads a block's table with one
// coalesced 256-B (128-B) load.  Pass 1 buffers kRecChunk records per lane
// in LDS and writes them out as whole 16-byte pieces (see okv_count_kernel).
__device__ __forceinline__ uint64_t rec_index(uint32_t /*nblk*/, uint32_t b, uint32_t r) {
  return uint64_t(b) * kRCap + r;
}
constexpr uint32_t kRecChunk = 16;  // records per lane between two LDS flushes

// ---------------------------------------------------------------------------
// Pass 1: header walk in HBM, one lane per block.
// ---------------------------------------------------------------------------
// Small segments (prefetch = 1): each lane first touches one dword per 128-B
// line of its block's record bytes -- independent loads, all in flight at
// once -- so the dependent header chase then hits the caches instead of HBM.
// A single-tile launch (one workgroup) also zeroes the big-block counter and
// writes the totals itself (no memset, no scan launch): single_* non-null.
//
// Record table: every kRecChunk steps of the walk the workgroup stops at a
// barrier and writes the slots its lanes recorded since the last stop, as
// whole 16-byte pieces of the block-major table (4 consecutive lanes write
// one block's 64 bytes of positions).  Lockstep per-lane stores into a
// strided table (round 2: [r/16][block][r%16], u32 positions + u64 headers)
// left partial lines that the walk's own reads evicted between steps: 136 MB
// written per C3 launch for 50 MB of slots.
//
// Big blocks (okv_copy_kernel): more than kRCap rows, a walk ending at or past
// 4 GiB, or past span_cap (the tile pass's span: okv_tile_kernel).
__global__ __launch_bounds__(kThreads) void okv_count_kernel(
    const uint8_t* __restrict__ seg, uint64_t seg_bytes, const Desc* __restrict__ descs,
    uint32_t nblk, int comp, BlockCount* __restrict__ cnt, Prefix* __restrict__ lp,
    Prefix* __restrict__ tile_tot, uint32_t* __restrict__ rt_pos, uint16_t* __restrict__ rt_kl,
    uint32_t* __restrict__ big_list, uint32_t* __restrict__ big_count,
    const int32_t* __restrict__ pre_status, int prefetch, uint64_t span_cap,
    Prefix* __restrict__ tile_pre, Totals* __restrict__ tot, uint64_t* __restrict__ row_start,
    uint32_t* __restrict__ arrive, uint32_t* __restrict__ big_zero,
    const Totals* __restrict__ base, uint32_t bidx0, unsigned long long* __restrict__ span_max) {
  // slots of the current chunk: positions [lane][kRecChunk + 1] (odd stride:
  // the walking lanes' stores hit distinct banks), key lengths [lane][kRecChunk]
  __shared__ uint32_t s_pos[kThreads * (kRecChunk + 1)];
  __shared__ __align__(16) uint16_t s_kl[kThreads * kRecChunk];
  __shared__ uint32_t s_rows[kThreads];
  const uint32_t tid = threadIdx.x;
  const uint32_t b = blockIdx.x * kTile + tid;
  uint64_t rows = 0, kb = 0, vb = 0, p = 0;
  int32_t st = OKV_BLK_OK;
  // the other big-block counter slot, for the next launch (its readers, the
  // previous decode's kernels, have completed: stream order)
  if (blockIdx.x == 0 && tid == 0 && big_zero) *big_zero = 0;
  uint64_t len = 0, orig = 0, off = 0;
  bool walking = false;
  if (b < nblk) {
    const Desc d = descs[b];
    const int32_t pre = pre_status ? pre_status[b] : int32_t(OKV_BLK_OK);
    if (pre != OKV_BLK_OK) {
      st = pre;  // outcome of the zstd stage (raw-block bounds, decoder error)
    } else if ((st = go_read_status(d, seg_bytes)) != OKV_BLK_OK) {
      // Seek error / makeslice panic / io.EOF / ErrUnexpectedBytesRead (:303-316)
    } else if (comp == OKV_COMP_ZSTD) {
      st = OKV_BLK_UNSUPPORTED;  // index-only spans cannot point into decompressed bytes
    } else {
      len = (comp == OKV_COMP_LZ4) ? 0 : d.block_size;  // Q7 (:331-333)
      orig = go_walk_bound(d.original_size);  // int(OriginalSize) < 0: no iteration (:340)
      off = d.offset;
      walking = true;
      if (prefetch && orig && len) {
        // up to 32 lines (4 KiB), all issued before any is waited on;
        // addresses clamped into [offset, offset + min(orig, len))
        const uint64_t first = off & ~uint64_t(3);
        const uint64_t last = (off + (orig < len ? orig : len) - 1) & ~uint64_t(3);
        uint32_t v[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) {
          uint64_t a = (off & ~uint64_t(127)) + 128ull * u;
          a = a < first ? first : (a > last ? last : a);
          v[u] = *reinterpret_cast<const uint32_t*>(seg + a);
        }
        uint32_t acc = 0;
#pragma unroll
        for (int u = 0; u < 32; ++u) acc ^= v[u];
        asm volatile("" ::"v"(acc));  // keep the loads; their values are unused
      }
    }
  }
  // The walk is a dependent chain (record i+1 starts where i ends), so this
  // kernel is bound by HBM latency x the longest block's row count.
  const uint32_t b0 = blockIdx.x * kTile;
  for (uint32_t c = 0; c < uint32_t(kRCap) / kRecChunk; ++c) {
    const uint64_t cap = uint64_t(c + 1) * kRecChunk;
    if (walking) {
      while (p < orig && rows < cap) {  // :340
        if (len - p < 6) { st = OKV_BLK_PANIC; break; }  // u16/u32 reads (:342-345)
        uint32_t kl, vl;
        header_global(seg, off + p, kl, vl);
        const uint64_t room = len - p - 6;
        if (kl > room || vl > room - kl) {  // zero-length reads always succeed (:490-493)
          st = OKV_BLK_PANIC;                // key/value reads (:346-349)
          break;
        }
        const uint32_t slot = uint32_t(rows) & (kRecChunk - 1);
        s_pos[tid * (kRecChunk + 1) + slot] = uint32_t(p);
        s_kl[tid * kRecChunk + slot] = uint16_t(kl);
        rows++;
        kb += kl;
        vb += vl;
        p += 6 + uint64_t(kl) + uint64_t(vl);
      }
      if (st != OKV_BLK_OK) walking = false;
    }
    s_rows[tid] = st == OKV_BLK_OK ? uint32_t(rows) : 0u;
    __syncthreads();
    // slots [c * 16, c * 16 + 16) of the workgroup's blocks, live ones only
    for (uint32_t q = tid; q < uint32_t(kTile) * 4; q += kThreads) {
      const uint32_t lb = q >> 2, sub = q & 3, slot = c * kRecChunk + sub * 4;
      if (b0 + lb < nblk && slot < s_rows[lb]) {
        const uint32_t* s = &s_pos[lb * (kRecChunk + 1) + sub * 4];
        *reinterpret_cast<uint4*>(rt_pos + rec_index(nblk, b0 + lb, slot)) =
            make_uint4(s[0], s[1], s[2], s[3]);
      }
    }
    if (rt_kl) {
      for (uint32_t q = tid; q < uint32_t(kTile) * 2; q += kThreads) {
        const uint32_t lb = q >> 1, sub = q & 1, slot = c * kRecChunk + sub * 8;
        if (b0 + lb < nblk && slot < s_rows[lb])
          *reinterpret_cast<uint4*>(rt_kl + rec_index(nblk, b0 + lb, slot)) =
              *reinterpret_cast<const uint4*>(&s_kl[lb * kRecChunk + sub * 8]);
      }
    }
    walking = walking && p < orig;  // (then rows == cap)
    if (!__syncthreads_or(walking)) break;  // also the barrier before the slots are reused
  }
  // blocks with more than kRCap rows: finish the walk without recording
  if (walking) {
    while (p < orig) {
      if (len - p < 6) { st = OKV_BLK_PANIC; break; }
      uint32_t kl, vl;
      header_global(seg, off + p, kl, vl);
      const uint64_t room = len - p - 6;
      if (kl > room || vl > room - kl) { st = OKV_BLK_PANIC; break; }
      rows++;
      kb += kl;
      vb += vl;
      p += 6 + uint64_t(kl) + uint64_t(vl);
    }
  }
  if (b < nblk) {
    if (st != OKV_BLK_OK) rows = kb = vb = 0;
    if (st == OKV_BLK_OK && (rows > kRCap || p >= (uint64_t(1) << 32) || p > span_cap))
      big_list[atomicAdd(big_count, 1u)] = bidx0 + b;  // staged path (okv_copy_kernel)
    BlockCount c;
    c.rows = rows;
    c.kbytes = kb;
    c.vbytes = vb;
    c.pend = p;
    c.status = st;
    c.pad = 0;
    cnt[b] = c;
  }
  if (span_max) {  // the longest walk (okv_decode_plan: the tile pass's span hint)
    unsigned long long m = b < nblk && st == OKV_BLK_OK ? p : 0ull;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const unsigned long long o = __shfl_xor(m, d, 64);
      m = o > m ? o : m;
    }
    if ((tid & 63) == 0 && m) atomicMax(span_max, m);
  }
  // workgroup exclusive scan of (rows, padded kb, padded vb, bad)
  __shared__ uint64_t s_w[4][kThreads / 64];
  const int lane = tid & 63, wave = tid >> 6;
  uint64_t v[4] = {rows, round16(kb), round16(vb), uint64_t(b < nblk && st != OKV_BLK_OK)};
  uint64_t inc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    inc[k] = wave_incl_scan(v[k], lane);
    if (lane == 63) s_w[k][wave] = inc[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint64_t off2 = 0;
    for (int w = 0; w < wave; ++w) off2 += s_w[k][w];
    inc[k] += off2 - v[k];  // exclusive
  }
  if (b < nblk) {
    Prefix e;
    e.rows = inc[0];
    e.kb = inc[1];
    e.vb = inc[2];
    e.bad = inc[3];
    lp[b] = e;
  }
  // Pass 2 in the same launch: the workgroup whose arrival is counted last
  // scans the tile totals.  Hand-off (MI355X_MICROARCH.md, inter-workgroup
  // hand-off table, row 1): one lane per workgroup stores its totals with sc1
  // stores, drains them (vmcnt(0)), then adds to one unsharded agent-scope
  // counter; the workgroup whose add came last (told by the value it returns)
  // reads every total with sc1 loads.  Round 4 made the add a release and
  // the last adder acquire: an L2 write-back per workgroup of the ~66 KB of
  // record table each has just written -- 6.5 us more per C3 count (A/B,
  // profiles/r5/session/ab_count_arrival.log).  The totals travel write-
  // through (sc1 stores, drained before the add), so no producer needs a
  // release; the last adder still takes an agent-scope acquire before its
  // loads (one L1 invalidate, in one workgroup), so the loads are ordered
  // after the add by the memory model, not only by the sc1 load path.
  __shared__ uint32_t s_last;
  if (tid == kThreads - 1) {
    const Prefix t{inc[0] + v[0], inc[1] + v[1], inc[2] + v[2], inc[3] + v[3]};
    if (gridDim.x == 1) {
      const Totals b0 = base ? *base : Totals{0, 0, 0, 0};
      *tile_pre = Prefix{b0.rows, b0.kb, b0.vb, b0.bad};
      *tot = Totals{b0.rows + t.rows, b0.kb + t.kb, b0.vb + t.vb, b0.bad + t.bad};
      if (row_start) row_start[nblk] = b0.rows + t.rows;
      s_last = 0;
    } else {
      Prefix* q = tile_tot + blockIdx.x;
      __hip_atomic_store(&q->rows, t.rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&q->kb, t.kb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&q->vb, t.vb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&q->bad, t.bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t a =
          __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = a == gridDim.x - 1;
    }
  }
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  // the last workgroup: exclusive scan of gridDim.x tile totals, 256 at a time
  // (from the totals of the blocks before this launch's, for a decode in pieces)
  uint64_t carry[4] = {0, 0, 0, 0};
  if (base) {
    carry[0] = base->rows;
    carry[1] = base->kb;
    carry[2] = base->vb;
    carry[3] = base->bad;
  }
  for (uint32_t base = 0; base < gridDim.x; base += kThreads) {
    const uint32_t i = base + tid;
    uint64_t x[4] = {0, 0, 0, 0};
    if (i < gridDim.x) {
      const Prefix* q = tile_tot + i;
      x[0] = __hip_atomic_load(&q->rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      x[1] = __hip_atomic_load(&q->kb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      x[2] = __hip_atomic_load(&q->vb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      x[3] = __hip_atomic_load(&q->bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    uint64_t in[4];
    __syncthreads();  // s_w reuse
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      in[k] = wave_incl_scan(x[k], lane);
      if (lane == 63) s_w[k][wave] = in[k];
    }
    __syncthreads();
    uint64_t sum[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint64_t o = carry[k];
      for (int w = 0; w < wave; ++w) o += s_w[k][w];
      in[k] += o - x[k];  // exclusive
      sum[k] = s_w[k][0] + s_w[k][1] + s_w[k][2] + s_w[k][3];
    }
    if (i < gridDim.x) tile_pre[i] = Prefix{in[0], in[1], in[2], in[3]};
#pragma unroll
    for (int k = 0; k < 4; ++k) carry[k] += sum[k];
  }
  if (tid == 0) {
    *tot = Totals{carry[0], carry[1], carry[2], carry[3]};
    if (row_start) row_start[nblk] = carry[0];
    // every workgroup has added: reset the counter for the next launch
    __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------------------
// Pass 3: per-block materialisation.
// ---------------------------------------------------------------------------
struct CopyParams {
  const uint8_t* seg;
  uint64_t seg_bytes;
  const Desc* descs;
  uint32_t nblk;
  int comp;
  int index_only;
  const BlockCount* cnt;
  const Prefix* lp;
  const Prefix* tile_pre;
  const uint32_t* rt_pos;     // pass-1 record table: positions (block-major, rec_index)
  const uint16_t* rt_kl;      // ... and key lengths (null unless the pass needs them)
  uint32_t* big_list;         // blocks with > kRCap rows (or >= 4 GiB walks)
  uint32_t* big_count;
  uint64_t* row_start;
  uint64_t* key_base;
  uint64_t* val_base;
  int32_t* blk_status;
  uint64_t* key_off;
  uint16_t* key_len;
  uint64_t* val_off;
  uint32_t* val_len;
  uint8_t* key_arena;
  uint8_t* val_arena;
  uint64_t row_cap, key_cap, val_cap;
  // value sweep hand-off (okv_value_sweep_kernel; null: pass 3 gathers values itself)
  uint64_t* vsrc;             // [row] segment position of the row's value
  uint32_t* vtile;            // [value-arena tile] row owning the tile's first byte
  uint4* bchunk;              // [row] the chunk holding the end of the row's value
  const Totals* tot;          // call totals (pass 1 / pass 2)
  uint64_t span_cap;          // okv_tile_kernel: blocks whose walk ends past it are big
};

// The value sweep runs when every row's index is written by the per-block
// pass 3 and the value arena is gap-free: no big block (okv_copy_kernel's
// rows) and no capacity failure.  Every workgroup of both kernels reads the
// same scalars, so they agree.
constexpr uint32_t kSwTile = 4096;  // value-arena bytes per sweep tile
__device__ __forceinline__ bool sweep_safe(const Totals& T, uint32_t nbig, uint64_t row_cap,
                                           uint64_t key_cap, uint64_t val_cap) {
  return nbig == 0 && T.rows <= row_cap && T.kb <= key_cap && T.vb <= val_cap;
}

// Global row / arena bases of block b and its final status (capacity check).
struct BlockBase {
  uint64_t row0, kb0, vb0;
  int32_t st;
};
__device__ __forceinline__ BlockBase block_base_of(const CopyParams& P, const BlockCount& c,
                                                   const Prefix& l, const Prefix& t) {
  BlockBase r;
  r.row0 = t.rows + l.rows;
  r.kb0 = t.kb + l.kb;
  r.vb0 = t.vb + l.vb;
  r.st = c.status;
  if (r.st == OKV_BLK_OK &&
      (r.row0 + c.rows > P.row_cap ||
       (!P.index_only && (r.kb0 + round16(c.kbytes) > P.key_cap ||
                          r.vb0 + round16(c.vbytes) > P.val_cap))))
    r.st = OKV_BLK_CAPACITY;
  return r;
}
__device__ __forceinline__ BlockBase block_base(const CopyParams& P, uint32_t b,
                                                const BlockCount& c) {
  return block_base_of(P, c, P.lp[b], P.tile_pre[b / kTile]);
}

// Lanes per row for a region whose rows average `avg` bytes.
__device__ __forceinline__ uint32_t group_size(uint64_t avg) {
  const uint64_t chunks = avg / 16 + 2;
  uint32_t g = 1;
  while (g < 64 && g < chunks) g <<= 1;
  return g;
}

struct GatherSmem {
  uint32_t rec[kRCap + 1];   // record position within the block
  uint32_t kpre[kRCap + 1];  // exclusive prefix of key lengths (kpre[rows] = total)
  uint32_t vpre[kRCap + 1];  // exclusive prefix of value lengths
  uint32_t ksb[kRCap];       // source of key-region byte x of row r = off + ksb[r] + x
  uint32_t vsb[kRCap];       // likewise for values
};

// Byte source for the gather: the segment in HBM (two aligned 16-byte loads +
// funnel).  rel = position relative to the block start (may be a few bytes
// negative for windows that begin before a row: those bytes are masked off).
struct GlobalWin {
  const uint8_t* seg;
  uint64_t seg_bytes;
  uint64_t off;
  __device__ __forceinline__ uint4 at(int64_t rel) const {
    return window16(seg, seg_bytes, int64_t(off) + rel);
  }
  __device__ __forceinline__ void header(uint32_t pos, uint32_t& kl, uint32_t& vl) const {
    header_global(seg, off + pos, kl, vl);
  }
};
// Gather one arena region (keys or values) of a block.  Each wave streams
// contiguous 1 KiB destination tiles: lane l of tile t writes chunk 64t + l
// (16 bytes, dwordx4).  The row holding the chunk's first byte is found by
// binary search on the lane's first chunk and by linear advance after
// (chunks only move forward).  A chunk that spills past its row is completed
// in registers from the following rows; past the region end it is zero (the
// 16-byte padding).  kU tiles per iteration keep kU windows in flight per lane.
// Tiles t0, t0 + ts, ... (< t1) of a region.
template <bool kVal, class Src, uint32_t kU = 4>
__device__ __forceinline__ void gather_tiles(const Src& src, const GatherSmem& sm, int rows,
                                             uint8_t* __restrict__ arena, uint64_t dbase,
                                             uint32_t t0, uint32_t t1, uint32_t ts) {
  const uint32_t* pre = kVal ? sm.vpre : sm.kpre;
  const uint32_t* sb = kVal ? sm.vsb : sm.ksb;
  const uint32_t total = pre[rows];
  const uint32_t N = (total + 15) >> 4;  // chunks, including the padded tail
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t last = uint32_t(rows) - 1;
  const uint32_t cmax = (N < t1 * 64 ? N : t1 * 64) - 1;  // last chunk of the range (ts == 1)
  for (uint32_t t = t0; t < t1; t += kU * ts) {
    uint4 v[kU];
    uint32_t rr[kU];
    // phase 1: rows and addresses; issue every load before any data is used
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint32_t c = (t + u * ts) * 64 + lane;
      const bool ok = (t + u * ts) < t1 && c < N;
      // lanes past the range reload the range's last chunk (an address a
      // valid lane loads in this iteration).  Pointing them at the range's
      // first tile with the current row's bias re-fetched ~40 evicted lines
      // per block (0.32 GB at C3).
      const uint32_t x = (ok ? c : cmax) << 4;
      // the row holding byte x: r = #{k in [1, rows) : pre[k] <= x}, a binary
      // search per chunk (pre[rows] = total > x ends every probe past the
      // last row).  The kU searches are independent, so their LDS reads
      // overlap; advancing linearly from the previous chunk's row cost one
      // dependent read per row passed (16 per tile for 64-byte rows).
      uint32_t r = 0;
#pragma unroll
      for (uint32_t st = 64; st; st >>= 1) {
        const uint32_t j = r + st;
        r = pre[min(j, last + 1)] <= x ? j : r;
      }
      rr[u] = r;
      v[u] = src.at(int64_t(sb[r]) + int64_t(x));
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint32_t c = (t + u * ts) * 64 + lane;
      if ((t + u * ts) < t1 && c < N) {
        const uint32_t x = c << 4, xe = x + 16;
        uint4 out = v[u];
        const uint32_t ri = rr[u];
        if (xe > pre[ri + 1]) {  // spills past row ri (or past the region end)
          out = merge_bytes(make_uint4(0, 0, 0, 0), out, 0, int32_t(pre[ri + 1] - x));
          for (uint32_t j = ri + 1; j <= last && pre[j] < xe; ++j) {
            const uint32_t q0 = pre[j], q1 = pre[j + 1];
            if (q1 == q0) continue;
            const uint4 w = src.at(int64_t(sb[j]) + int64_t(x));
            out = merge_bytes(out, w, int32_t(q0 - x), int32_t((q1 < xe ? q1 : xe) - x));
          }
        }
        *reinterpret_cast<uint4*>(arena + dbase + uint64_t(x)) = out;
      }
    }
  }
}

// Tiles of a region split over nw waves in contiguous ranges.  Measured (C3,
// DESIGN.md §4): interleaving the tiles over the waves, 2 or 8 tiles per
// iteration, prefetching a spilling chunk's next-row window with the first
// (+11 VGPRs: 4 waves/SIMD instead of 5) and forcing 6-8 waves/SIMD (spills)
// are all slower.
template <bool kVal, class Src>
__device__ __forceinline__ void gather_region(const Src& src, const GatherSmem& sm, int rows,
                                              uint8_t* __restrict__ arena, uint64_t dbase,
                                              uint32_t wave, uint32_t nw) {
  const uint32_t T = ((kVal ? sm.vpre : sm.kpre)[rows] + 1023) >> 10;  // 1 KiB tiles
  gather_tiles<kVal, Src>(src, sm, rows, arena, dbase, uint32_t(uint64_t(T) * wave / nw),
                          uint32_t(uint64_t(T) * (wave + 1) / nw), 1);
}

// Per-block metadata every gather kernel starts from.
struct BlockMeta {
  BlockCount c;
  BlockBase B;
  uint64_t off;
};
__device__ __forceinline__ BlockMeta block_meta(const CopyParams& P, uint32_t b) {
  BlockMeta m;
  m.c = P.cnt[b];
  m.B = block_base(P, b, m.c);
  m.off = P.descs[b].offset;
  return m;
}
// Block outcome (tid 0) and whether the gather kernels handle its rows
// (else: nothing to do, or a big block for okv_copy_kernel / okv_index_kernel).
__device__ __forceinline__ bool block_head(const CopyParams& P, uint32_t b, const BlockMeta& m) {
  if (threadIdx.x == 0) {
    P.row_start[b] = m.B.row0;
    if (P.key_base) P.key_base[b] = m.B.kb0;
    if (P.val_base) P.val_base[b] = m.B.vb0;
    P.blk_status[b] = m.B.st;
  }
  return m.B.st == OKV_BLK_OK && m.c.rows != 0 && m.c.rows <= uint64_t(kRCap) &&
         m.c.pend < (uint64_t(1) << 32);
}

// Row table (wave 0, lane r = row r): wave scans give each row's key/value
// prefix and its source bias.
__device__ __forceinline__ void fill_row_table(GatherSmem& sm, int rows, uint32_t rec,
                                               uint32_t kl, uint32_t vl) {
  const uint32_t tid = threadIdx.x & 63;
  const uint32_t ki = wave_incl_scan32(kl, tid), vi = wave_incl_scan32(vl, tid);
  if (int(tid) < rows) {
    sm.rec[tid] = rec;
    sm.kpre[tid] = ki - kl;
    sm.vpre[tid] = vi - vl;
    sm.ksb[tid] = rec + 6 - (ki - kl);       // >= 0: earlier keys precede rec
    sm.vsb[tid] = rec + 6 + kl - (vi - vl);  // >= 0: earlier values precede rec
    if (int(tid) == rows - 1) {
      sm.rec[rows] = rec + 6 + kl + vl;
      sm.kpre[rows] = ki;
      sm.vpre[rows] = vi;
    }
  }
}
// ... from headers read at the pass-1 positions
template <class Src>
__device__ __forceinline__ void build_row_table(const Src& src, GatherSmem& sm, int rows,
                                                uint32_t rec) {
  uint32_t kl = 0, vl = 0;
  if (int(threadIdx.x & 63) < rows) src.header(rec, kl, vl);
  fill_row_table(sm, rows, rec, kl, vl);
}
// SoA row index of a block (lane r = row r).
__device__ __forceinline__ void write_row_index(const CopyParams& P, const GatherSmem& sm,
                                                const BlockMeta& m, int rows) {
  const uint32_t tid = threadIdx.x;
  if (int(tid) >= rows) return;
  const uint64_t g = m.B.row0 + tid;
  const uint32_t kl = sm.kpre[tid + 1] - sm.kpre[tid], vl = sm.vpre[tid + 1] - sm.vpre[tid];
  P.key_len[g] = uint16_t(kl);
  P.val_len[g] = vl;
  if (P.index_only) {
    P.key_off[g] = m.off + sm.rec[tid] + 6;
    P.val_off[g] = m.off + sm.rec[tid] + 6 + kl;
  } else {
    P.key_off[g] = m.B.kb0 + sm.kpre[tid];
    P.val_off[g] = m.B.vb0 + sm.vpre[tid];
  }
}

// Value-sweep hand-off (lane r = row r): each row's value source, the row
// owning each value-arena tile that starts inside its value, and the row's
// boundary chunk.  A 16-byte chunk holding the end of row r's value (end not
// 16-aligned) mixes rows (or the block's zero padding); the lane of the row
// owning its first byte assembles it from the block's row table into
// bchunk[row], and the sweep stores it with its tile (whole lines).  The
// loads are issued first (with the key loads in flight: see okv_rows_kernel).
__device__ __forceinline__ uint4 boundary_chunk(const CopyParams& P, const GatherSmem& sm,
                                                const BlockMeta& m, int rows) {
  const uint32_t t = threadIdx.x;
  uint4 out = make_uint4(0, 0, 0, 0);
  if (int(t) >= rows) return out;
  const uint32_t v0 = sm.vpre[t], e = sm.vpre[t + 1];
  const uint32_t C = e & ~15u;
  if (e == v0 || (e & 15) == 0 || v0 > C) return out;  // no chunk of mine to assemble
  out = merge_bytes(out, window16(P.seg, P.seg_bytes, int64_t(m.off + sm.vsb[t] + C)), 0,
                    int32_t(e - C));
  for (uint32_t j = t + 1; int(j) < rows && sm.vpre[j] < C + 16; ++j) {
    const uint32_t q0 = sm.vpre[j], q1 = sm.vpre[j + 1];
    if (q1 == q0) continue;
    const uint4 w = window16(P.seg, P.seg_bytes, int64_t(m.off + sm.vsb[j] + C));
    out = merge_bytes(out, w, int32_t(q0 - C), int32_t(min(q1, C + 16) - C));
  }
  return out;
}
__device__ __forceinline__ void sweep_handoff(const CopyParams& P, const GatherSmem& sm,
                                              const BlockMeta& m, int rows, const uint4& bc) {
  const uint32_t t = threadIdx.x;
  if (int(t) >= rows) return;
  const uint64_t g = m.B.row0 + t;
  const uint32_t kl = sm.kpre[t + 1] - sm.kpre[t];
  const uint32_t v0 = sm.vpre[t], e = sm.vpre[t + 1];
  P.vsrc[g] = m.off + sm.rec[t] + 6 + kl;
  P.bchunk[g] = bc;
  for (uint64_t x = (m.B.vb0 + v0 + kSwTile - 1) & ~uint64_t(kSwTile - 1); x < m.B.vb0 + e;
       x += kSwTile)
    P.vtile[x / kSwTile] = uint32_t(g);
}

// ---------------------------------------------------------------------------
// Pass 3, source tiles (large blocks).  Block b is cut into
// tiles of kT source bytes, tile t = block bytes [t kT, (t + 1) kT), one
// short-lived 256-thread workgroup each, dispatched in address order: the
// whole chip's loads and stores stay in one compact window of the segment
// and the arenas (the one-shot copy shape).  A workgroup
//   1. loads the block's metadata and its pass-1 record table (one trip),
//   2. DMAs its tile (plus a 16-byte lead-in and a guard line) into LDS with
//      global_load_lds_dwordx4 -- the only read of the record bytes,
//   3. writes every key and value byte whose SOURCE lies in its tile: the
//      destination ranges are contiguous (rows are packed in record order),
//      each 16-byte destination chunk is assembled from the stage (one LDS
//      window per row piece) and stored whole; the two chunks at a range's
//      ends that the neighbouring tile shares are stored byte-exactly
//      (store_partial: disjoint bytes, no read-modify-write).
// The value-range cut between two tiles of a block moves up to the next
// 128-byte line of the arena when the bytes it adds lie in the tile's staged
// extension (kLineExt source bytes past its end): stores from two workgroups
// never share that line.  (Every store instruction that covers part of a
// 64-byte sector costs the HBM a whole 64-byte write request -- the L2 does
// not merge separate stores into one; PMC by output class)
// Tile 0 also writes the block's row index (SoA) and its block outputs.  The
// last tile writes the zero padding of the block's arena regions.  Each
// source byte is read once and each arena byte written once, so the pass
// moves its algorithmic bytes: the round-2 row pass + value sweep read the
// lines values share with headers and keys twice (1.11x).
// kXcd: consecutive tiles run on one XCD (hardware deals workgroups to the 8
// XCDs round-robin), so a block's metadata and the chunks two tiles share
// meet in one L2.
// ---------------------------------------------------------------------------
template <uint32_t kUnits>
struct TileRowsT {
  uint32_t pre[2][kRCap + 1];  // [key, value] exclusive prefix of lengths (pre[rows] = total)
  uint32_t sb[2][kRCap];       // block position of region byte x of row r = sb[r] + x
  uint32_t x[4];               // owned key range [x0, x1), value range [x2, x3)
  // value runs (kRuns): whole value chunks in units of <= 64 inside one
  // row piece {dest chunk, stage byte of its first chunk, count}, and the
  // value chunks that mix rows, padding or a neighbouring tile's bytes
  uint32_t unit[3][kUnits];
  uint32_t bnd[2 * kRCap + 4];  // (sector form: up to two mixed sectors per row)
  uint32_t nunit, nbnd;
};
// value runs of a kT-byte tile: at most one partial run per row plus kT / 1 KiB
// whole ones (16 KiB tiles: 96 entries, as before)
template <uint32_t kT>
using TileRows = TileRowsT<(kT / 1024 + kRCap + 16 + 15) & ~15u>;

// 16 bytes at byte s (0..15, wave-uniform) of the 32-byte window (x, y): a
// scalar branch picks the dwords, then 4 v_alignbyte.
__device__ __forceinline__ uint4 funnel_u(const uint4& x, const uint4& y, uint32_t s) {
  const uint32_t r = s & 3;
  switch (s >> 2) {
    case 0:
      return make_uint4(funnel(x.y, x.x, r), funnel(x.z, x.y, r), funnel(x.w, x.z, r),
                        funnel(y.x, x.w, r));
    case 1:
      return make_uint4(funnel(x.z, x.y, r), funnel(x.w, x.z, r), funnel(y.x, x.w, r),
                        funnel(y.y, y.x, r));
    case 2:
      return make_uint4(funnel(x.w, x.z, r), funnel(y.x, x.w, r), funnel(y.y, y.x, r),
                        funnel(y.z, y.y, r));
    default:
      return make_uint4(funnel(y.x, x.w, r), funnel(y.y, y.x, r), funnel(y.z, y.y, r),
                        funnel(y.w, y.z, r));
  }
}

// A destination chunk of a tile whose owned bytes [lo, hi) span rows or
// padding: each row's piece from a global window (rare; kept out of line).
__device__ __noinline__ uint4 tile_chunk_pieces(const uint8_t* seg, uint64_t seg_bytes, uint64_t off,
                                                const uint32_t* pre, const uint32_t* sb,
                                                uint32_t rows, uint32_t r, uint32_t x,
                                                uint32_t lo, uint32_t hi) {
  const uint32_t dend = min(hi, pre[rows]);
  uint4 out = make_uint4(0, 0, 0, 0);
  for (uint32_t d = lo; d < dend; ++r) {
    const uint32_t e = min(dend, pre[r + 1]);
    if (e > d) {  // bytes [d, e) of the chunk from row r
      out = merge_bytes(out, window16(seg, seg_bytes, int64_t(off + sb[r] + x)), int32_t(d - x),
                        int32_t(e - x));
      d = e;
    }
  }
  return out;
}

// (The measured alternatives -- other tile sizes and widths, phase probes,
// per-chunk lookups, direct global loads -- are tile_pass_diag in
// okv_decode_ablate.inc, ablation build only.)
// kSkip (ablation build only, okv_tile_kernel_skip): output classes left
// unwritten, to attribute the pass's HBM write traffic -- 1 the SoA row index,
// 2 value runs, 4 key chunks, 8 boundary value chunks, 16 partial chunks;
// forms: 64 the round-5 cuts (no line cut, below); 128 whole 64-byte sectors
// per store (+ 256 key cuts unrounded, + 512 the stage extension).
template <uint32_t kT, uint32_t kNT, bool kXcd, uint32_t kSkip = 0>
__device__ __forceinline__ void tile_pass(const CopyParams& P, uint32_t tpb, uint32_t ntile) {
  constexpr uint32_t kG = kT / 64 + 8;  // 64-byte destination granules of the key range
  constexpr bool kSector = (kSkip & 128) != 0;       // whole 64-byte sectors per store
  constexpr bool kLineCut = !(kSkip & 64) && !kSector;  // the product: value cuts on lines
  constexpr bool kKeyRound = kSector && !(kSkip & 256);  // (256: key cuts left as they are)
  constexpr uint32_t kLineExt = (kLineCut || (kSkip & 512)) ? 512 : 0;  // (512: stage extension)
  __shared__ TileRows<kT> R;
  __shared__ uint8_t gt[1][kG];         // row holding key byte max(64 g, range start)
  __shared__ uint4 stage[(kT + kLineExt) / 16 + 4];
  uint32_t L = blockIdx.x;
  if constexpr (kXcd) L = (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  if (L >= ntile) return;
  // uniform block index (an SGPR: the loads below are scalar, all in one trip)
  const uint32_t b = __builtin_amdgcn_readfirstlane(L / tpb);
  const uint32_t t = L - b * tpb;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  // one trip: the block's scalars and (wave 0) its record table
  uint32_t rec = 0, kl = 0;
  if (tid < 64) {
    rec = P.rt_pos[rec_index(P.nblk, b, lane)];
    kl = P.rt_kl[rec_index(P.nblk, b, lane)];
  }
  const uint64_t off = P.descs[b].offset;
  const BlockCount c = P.cnt[b];
  const Prefix lpre = P.lp[b], tpre = P.tile_pre[b / kTile];
  // consume every scalar here: the scheduler otherwise sinks each load to its
  // first use, one dependent trip after another
  asm volatile("" ::"s"(off), "s"(c.rows), "s"(c.kbytes), "s"(c.vbytes), "s"(c.pend),
               "s"(c.status), "s"(lpre.rows), "s"(lpre.kb), "s"(lpre.vb), "s"(tpre.rows),
               "s"(tpre.kb), "s"(tpre.vb));
  const uint64_t row0 = tpre.rows + lpre.rows, kb0 = tpre.kb + lpre.kb, vb0 = tpre.vb + lpre.vb;
  const bool fits = row0 + c.rows <= P.row_cap &&
                    (P.index_only ||
                     (kb0 + round16(c.kbytes) <= P.key_cap && vb0 + round16(c.vbytes) <= P.val_cap));
  const int32_t st = (c.status == OKV_BLK_OK && !fits) ? int32_t(OKV_BLK_CAPACITY) : c.status;
  // Tile 0 writes the block outputs and the SoA row index.  Stores wait
  // until the LDS tables are built: the compiler makes wave 0's LDS writes
  // wait for the wave's outstanding memory operations (it cannot tell them
  // from the DMA's LDS target).
  auto block_outputs = [&]() {
    if (t == 0 && tid == 0) {
      P.row_start[b] = row0;
      if (P.key_base) P.key_base[b] = kb0;
      if (P.val_base) P.val_base[b] = vb0;
      P.blk_status[b] = st;
    }
  };
  const uint64_t pend = c.pend;
  const uint32_t P0 = t * kT;
  // big blocks are okv_copy_kernel's (the same test as okv_count_kernel's)
  if (st != OKV_BLK_OK || c.rows == 0 || c.rows > uint64_t(kRCap) || pend > P.span_cap ||
      pend >= (uint64_t(1) << 32) || P0 >= pend) {
    block_outputs();
    return;
  }
  const uint32_t rows = uint32_t(c.rows), lastr = rows - 1;
  const uint32_t P1 = uint32_t(min<uint64_t>(uint64_t(P0) + kT, pend));
  const bool last_tile = P1 == pend;
  // stage = segment lines [A, E): the line before the one holding the tile's
  // first byte (a chunk's window begins up to 15 bytes before its first owned
  // byte) through the line after the one holding its last byte + 15
  const int64_t A = int64_t((off + P0) & ~uint64_t(15)) - 16;
  const int64_t E = int64_t((off + P1 + 15) & ~uint64_t(15)) + 16 + (last_tile ? 0 : kLineExt);
  const uint32_t np = uint32_t((E - A) >> 4);
  // Waves 1.. issue the DMA; wave 0 builds the row table meanwhile.  (With a
  // share of the DMA in flight, wave 0's LDS row-table writes would wait for
  // it: the compiler cannot tell them apart from the DMA's LDS target.)
  if (!P.index_only && tid >= 64) {
    const int64_t lim = int64_t(round16(P.seg_bytes));
    const uint32_t u = tid - 64;
    for (uint32_t k0 = 0; k0 < np; k0 += kNT - 64) {
      const uint32_t i = k0 + u;
      if (i < np) {
        int64_t a = A + (int64_t(i) << 4);
        if (a < 0 || a + 16 > lim) a = int64_t(off) & ~int64_t(15);  // bytes never used
        __builtin_amdgcn_global_load_lds(P.seg + a, OKV_LDS_PTR(stage + k0 + (u & ~63u)), 16,
                                         0, 0);
      }
    }
  }
  // row table (wave 0, lane r = row r) while the tile is in flight
  if (tid < 64) {
    const bool live = lane < rows;
    uint32_t nxt = __builtin_amdgcn_update_dpp(0u, rec, 0x130, 0xf, 0xf, false);  // rec[lane + 1]
    if (lane == lastr) nxt = uint32_t(pend);
    const uint32_t k = live ? kl : 0u, v = live ? nxt - rec - 6 - kl : 0u;
    const uint32_t ki = wave_scan_dpp(k), vi = wave_scan_dpp(v);
    const uint32_t kp = ki - k, vp = vi - v;
    const uint32_t ks = rec + 6, vs = rec + 6 + k;  // block positions of the key / value
    if (live) {
      R.pre[0][lane] = kp;
      R.pre[1][lane] = vp;
      R.sb[0][lane] = ks - kp;
      R.sb[1][lane] = vs - vp;
      if (lane == lastr) {
        R.pre[0][rows] = ki;
        R.pre[1][rows] = vi;
      }
    }
    if (!P.index_only) {
      // the owned ranges: [first byte whose source is >= P0, same for P1); the
      // last tile also owns the 16-byte padding after the region
      const uint32_t KT = __builtin_amdgcn_readlane(ki, lastr);
      const uint32_t VT = __builtin_amdgcn_readlane(vi, lastr);
      // (row: the lane holding that byte; lastr when none does)
      auto first_at = [&](uint32_t len, uint32_t src, uint32_t pr, uint32_t tot, uint32_t Q,
                          uint32_t& row) {
        const uint64_t mk = __ballot(live && len && src + len > Q);
        row = lastr;
        if (!mk) return tot;
        const uint32_t j = uint32_t(__ffsll(static_cast<unsigned long long>(mk)) - 1);
        row = j;
        const uint32_t s0 = __builtin_amdgcn_readlane(src, j), p0 = __builtin_amdgcn_readlane(pr, j);
        return Q > s0 ? p0 + (Q - s0) : p0;
      };
      uint32_t X[4], jx, jv;
      X[0] = first_at(k, ks, kp, KT, P0, jx);
      X[1] = last_tile ? uint32_t(round16(KT)) : first_at(k, ks, kp, KT, P1, jx);
      X[2] = first_at(v, vs, vp, VT, P0, jv);
      X[3] = last_tile ? uint32_t(round16(VT)) : first_at(v, vs, vp, VT, P1, jx);
      if constexpr (kLineCut) {
        // a cut Y at source Q moves up to the next 128-byte line of the arena
        // when the bytes it adds have their sources within kLineExt - 32 of Q
        // (the tile before the cut stages that far); both tiles of a cut
        // decide from the same row table, so they agree
        auto line_cut = [&](uint32_t Y, uint32_t Q) -> uint32_t {
          const uint32_t end = uint32_t(round16(VT));
          uint32_t Yl = uint32_t(((vb0 + Y + 127) & ~uint64_t(127)) - vb0);
          Yl = Yl > end ? end : Yl;
          if (Yl <= Y || Y >= VT) return Yl <= Y ? Y : Yl;
          const uint32_t y = min(Yl, VT) - 1;  // the last real byte the tile would add
          const uint64_t mk = __ballot(live && v && vp <= y && y < vp + v);
          if (!mk) return Y;
          const uint32_t j = uint32_t(__ffsll(static_cast<unsigned long long>(mk)) - 1);
          const uint32_t sy = __builtin_amdgcn_readlane(vs, j) + (y - __builtin_amdgcn_readlane(vp, j));
          return sy + 32 <= Q + kLineExt ? Yl : Y;
        };
        if (t != 0) X[2] = line_cut(X[2], P0);
        if (!last_tile) X[3] = line_cut(X[3], P1);
        if (X[2] > X[3]) X[2] = X[3];
        // the row holding X2 (head chunk: none when X2 is line-aligned)
        const uint64_t mh = __ballot(live && v && vp <= X[2] && X[2] < vp + v);
        jv = mh ? uint32_t(__ffsll(static_cast<unsigned long long>(mh)) - 1) : lastr;
      }
      // (sector form) the unrounded value cut at P1: value bytes before it
      // have their sources in this tile's stage
      const uint32_t Yv1 = X[3];
      if constexpr (kSector) {
        // every cut between two tiles of a block moves up to a 64-byte sector
        // of the arena, so no destination sector is shared by two tiles; the
        // few bytes this adds to the tile before the cut come from global
        // windows when they lie past its stage
        auto sector_up = [](uint32_t Y, uint64_t base, uint32_t tot) -> uint32_t {
          const uint32_t end = uint32_t(round16(tot));
          const uint32_t Ys = uint32_t(((base + Y + 63) & ~uint64_t(63)) - base);
          return Ys > end ? end : Ys;
        };
        if (t != 0) {
          if (kKeyRound) X[0] = sector_up(X[0], kb0, KT);
          X[2] = sector_up(X[2], vb0, VT);
        }
        if (!last_tile) {
          if (kKeyRound) X[1] = sector_up(X[1], kb0, KT);
          X[3] = sector_up(X[3], vb0, VT);
        }
        X[0] = min(X[0], X[1]);
        X[2] = min(X[2], X[3]);
      }
      if (lane == 0) {
        R.x[0] = X[0];
        R.x[1] = X[1];
        R.x[2] = X[2];
        R.x[3] = X[3];
      }
      // granule table of the key range: gt[0][g - (X0 >> 6)] = row holding byte
      // max(64 g, X0); granules past the last row's bytes (padding) keep the
      // preset lastr.  Values need none: their boundary chunks carry their row.
#pragma unroll
      for (uint32_t reg = 0; reg < 1u; ++reg) {
        const uint32_t X0 = X[2 * reg], X1 = X[2 * reg + 1];
        if (X1 <= X0) continue;
        const uint32_t g0 = X0 >> 6, gl = (X1 - 1) >> 6;
        for (uint32_t g = g0 + lane; g <= gl; g += 64) gt[reg][g - g0] = uint8_t(lastr);
        const uint32_t pr = reg ? vp : kp, ln = reg ? v : k;
        if (live && ln) {
          const uint32_t e = pr + ln;
          if (pr <= X0 && X0 < e) gt[reg][0] = uint8_t(lane);
          const uint32_t gs = max(g0 + 1, (pr + 63) >> 6), ge = min(gl, ((e + 63) >> 6) - 1);
          for (uint32_t g = gs; g <= ge; ++g) gt[reg][g - g0] = uint8_t(lane);
        }
      }
      if constexpr (kSector) {
        // row pieces of the owned value range: [a, e) = row r's bytes in [X2, X3).
        // Runs: the whole 64-byte sectors inside a piece (and before Yv1), in
        // units of <= 64 chunks -- one wave store writes whole sectors.  Every
        // other sector a piece touches is a mixed sector: its four chunks are
        // assembled by four adjacent lanes and stored by one instruction.
        const uint32_t X2 = X[2], X3 = X[3];
        const uint32_t a = max(vp, X2), e = min(vp + v, X3);
        const bool piece = live && v && a < e;
        const uint64_t va = vb0 + a, ve = vb0 + min(e, Yv1);
        const uint64_t s0 = (va + 63) & ~uint64_t(63), s1 = ve & ~uint64_t(63);
        const bool run = piece && s1 > s0;
        const uint32_t cs = run ? uint32_t((s0 - vb0) >> 4) : 0u;
        const uint32_t wc = run ? uint32_t((s1 - s0) >> 4) : 0u;
        const uint32_t nu = (wc + 63) >> 6;
        const uint32_t ui = wave_scan_dpp(nu);
        const uint32_t sbias0 = uint32_t(int64_t(off) - A);
        for (uint32_t q = 0; q < nu; ++q) {
          const uint32_t u = ui - nu + q;
          R.unit[0][u] = cs + 64 * q;
          R.unit[1][u] = vs - vp + 16 * (cs + 64 * q) + sbias0;
          R.unit[2][u] = min(64u, wc - 64 * q);
        }
        // mixed sectors, as (sector - the region's first sector) << 8 | the
        // lowest row with bytes in it (rows in order, head before tail; equal
        // neighbours skipped by the consumer)
        const uint64_t vs0 = vb0 >> 6;
        const uint32_t hsec = uint32_t(((vb0 + a) >> 6) - vs0);
        const uint32_t tsec = uint32_t(((vb0 + e - 1) >> 6) - vs0);
        const bool need_h = piece && (!run || s0 > va);
        const bool need_t = piece && (run ? s1 < vb0 + e : tsec != hsec);
        const uint32_t nme = uint32_t(need_h) + uint32_t(need_t);
        const uint32_t mi = wave_scan_dpp(nme) - nme;
        if (need_h) R.bnd[mi] = (hsec << 8) | lane;
        if (need_t) R.bnd[mi + uint32_t(need_h)] = (tsec << 8) | lane;
        const uint32_t nunit = __builtin_amdgcn_readlane(ui, 63);
        const uint32_t nmix = __builtin_amdgcn_readlane(mi + nme, 63);
        if (lane == 0) {
          R.nbnd = nmix;
          R.nunit = nunit;
        }
      } else {
        // row pieces of the owned value range: [a, e) = row r's bytes in [X2, X3)
        const uint32_t X2 = X[2], X3 = X[3];
        const uint32_t a = max(vp, X2), e = min(vp + v, X3);
        const bool piece = live && v && a < e;
        const uint32_t cs = piece ? (a + 15) >> 4 : 0u, ce = piece ? e >> 4 : 0u;
        const uint32_t wc = ce > cs ? ce - cs : 0u;
        const uint32_t nu = (wc + 63) >> 6;
        const uint32_t ui = wave_scan_dpp(nu);
        const uint32_t sbias0 = uint32_t(int64_t(off) - A);
        for (uint32_t q = 0; q < nu; ++q) {
          const uint32_t u = ui - nu + q;
          R.unit[0][u] = cs + 64 * q;
          R.unit[1][u] = vs - vp + 16 * (cs + 64 * q) + sbias0;
          R.unit[2][u] = min(64u, wc - 64 * q);
        }
        // boundary chunks: where a piece ends inside a chunk, and the range's
        // first chunk when it starts inside one (in order; equal neighbours
        // skipped), as chunk << 8 | the row holding the chunk's first owned
        // byte: the lowest row whose piece ends in the chunk (a row before it
        // holding that byte would end in the chunk too), or for the head chunk
        // the row holding X2
        const bool eb = piece && (e & 15);
        const uint64_t m = __ballot(eb);
        const uint32_t head = (X2 < X3 && (X2 & 15)) ? 1u : 0u;
        const uint32_t idx = head + uint32_t(__builtin_amdgcn_mbcnt_hi(
                                        uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u)));
        if (eb) R.bnd[idx] = ((e >> 4) << 8) | lane;
        // read lane 63 with the whole wave active (inside the lane-0 branch the
        // compiler may compute ui for lane 0 only)
        const uint32_t nunit = __builtin_amdgcn_readlane(ui, 63);
        if (lane == 0) {
          if (head) R.bnd[0] = ((X2 >> 4) << 8) | jv;
          R.nbnd = head + uint32_t(__builtin_popcountll(m));
          R.nunit = nunit;
        }
      }
    }
    if (P.index_only && t == 0 && live) {  // the SoA row index (spans into seg)
      const uint64_t g = row0 + lane;
      P.key_len[g] = uint16_t(k);
      P.val_len[g] = v;
      P.key_off[g] = off + ks;
      P.val_off[g] = off + vs;
    }
  }
  if (P.index_only) {
    block_outputs();
    return;
  }
  // the DMA waves wait for their loads (wave 0 has none: its SoA stores drain
  // on their own)
  if (tid >= 64) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0 && tid < 64) {  // the block outputs and SoA row index (from the LDS tables)
    block_outputs();
    if (!(kSkip & 1) && lane < rows) {
      const uint64_t g = row0 + lane;
      const uint32_t kp = R.pre[0][lane], vp = R.pre[1][lane];
      P.key_len[g] = uint16_t(R.pre[0][lane + 1] - kp);
      P.val_len[g] = R.pre[1][lane + 1] - vp;
      P.key_off[g] = kb0 + kp;
      P.val_off[g] = vb0 + vp;
    }
  }
  const uint32_t kx0 = R.x[0], kx1 = R.x[1], vx0 = R.x[2], vx1 = R.x[3];
  const uint32_t nk = kx1 > kx0 ? ((kx1 + 15) >> 4) - (kx0 >> 4) : 0u;
  const uint32_t sbias = uint32_t(int64_t(off) - A);  // stage byte of block position s: s + sbias
  {
    // value runs: one unit of <= 64 whole chunks of one row per wave iteration
    const uint32_t nunit = R.nunit, nbnd = R.nbnd;
    uint8_t* const varena = P.val_arena + vb0;
    for (uint32_t u = tid >> 6; u < ((kSkip & 2) ? 0u : nunit); u += kNT / 64) {
      const uint32_t c0 = __builtin_amdgcn_readfirstlane(R.unit[0][u]);
      const uint32_t sbyte = __builtin_amdgcn_readfirstlane(R.unit[1][u]);
      const uint32_t cnt = __builtin_amdgcn_readfirstlane(R.unit[2][u]);
      if (lane < cnt) {
        const uint32_t line = (sbyte >> 4) + lane;
        const uint4 w = funnel_u(stage[line], stage[line + 1], sbyte & 15);
        *reinterpret_cast<uint4*>(varena + (uint64_t(c0 + lane) << 4)) = w;
      }
    }
    if constexpr (kSector) {
      // keys (from the first chunk of the range's first sector, so each wave
      // store covers whole sectors) and the mixed value sectors, four lanes
      // each: per-lane lookup; sources past the stage from global windows
      const uint32_t kc0 = kx0 >> 4;
      const uint32_t kph = uint32_t(((kb0 >> 4) + kc0) & 3u);
      const uint32_t nk4 = nk ? (kph + nk + 3) & ~3u : 0u;
      const uint32_t vph = uint32_t(vb0 & 63);
      for (uint32_t j = tid; j < nk4 + 4 * nbnd; j += kNT) {
        const uint32_t reg = j >= nk4;
        if ((kSkip & 4) && !reg) continue;
        uint32_t r;
        int32_t xs;
        if (reg) {
          const uint32_t ei = (j - nk4) >> 2;
          const uint32_t bv = R.bnd[ei];
          if (ei && (bv >> 8) == (R.bnd[ei - 1] >> 8)) continue;
          xs = int32_t((bv >> 8) * 64u) - int32_t(vph) + int32_t(16 * ((j - nk4) & 3u));
          r = bv & 255u;
        } else {
          xs = int32_t(16 * (kc0 + j)) - int32_t(16 * kph);
          r = 0;
        }
        const uint32_t X0 = reg ? vx0 : kx0, X1 = reg ? vx1 : kx1;
        if (xs + 16 <= int32_t(X0) || xs >= int32_t(X1)) continue;
        const uint32_t x = uint32_t(xs);
        const uint32_t lo = max(x, X0), hi = min(x + 16, X1);
        const uint32_t* pre = R.pre[reg];
        const uint32_t* sb = R.sb[reg];
        if (!reg) r = uint32_t(gt[0][(lo >> 6) - (X0 >> 6)]);
        while (r < lastr && pre[r + 1] <= lo) ++r;
        uint8_t* dst = (reg ? P.val_arena + vb0 : P.key_arena + kb0) + x;
        const uint32_t dend = min(hi, pre[rows]);
        uint4 out = make_uint4(0, 0, 0, 0);
        for (uint32_t d = lo; d < dend; ++r) {
          const uint32_t e = min(dend, pre[r + 1]);
          if (e > d) {
            const uint32_t bi = sb[r] + x + sbias;
            const uint4 w = ((bi >> 4) + 1 < np)
                                ? load16_lds_b128(stage, bi)
                                : window16(P.seg, P.seg_bytes, int64_t(off) + sb[r] + x);
            out = merge_bytes(out, w, int32_t(d - x), int32_t(e - x));
            d = e;
          }
        }
        if (lo == x && hi == x + 16)
          *reinterpret_cast<uint4*>(dst) = out;
        else
          store_partial(dst, out, lo - x, hi - x);
      }
      return;
    }
    // keys and the boundary value chunks: per-lane lookup
    for (uint32_t j = tid; j < nk + nbnd; j += kNT) {
      const uint32_t reg = j >= nk;
      if ((kSkip & 4) && !reg) continue;
      if ((kSkip & 8) && reg) continue;
      const uint32_t bv = reg ? R.bnd[j - nk] : 0u;
      if (reg && j > nk && (bv >> 8) == (R.bnd[j - nk - 1] >> 8)) continue;
      const uint32_t X0 = reg ? vx0 : kx0, X1 = reg ? vx1 : kx1;
      const uint32_t x = reg ? (bv >> 8) << 4 : ((kx0 >> 4) + j) << 4;
      const uint32_t lo = max(x, X0), hi = min(x + 16, X1);
      const uint32_t* pre = R.pre[reg];
      const uint32_t* sb = R.sb[reg];
      uint32_t r = reg ? (bv & 255u) : uint32_t(gt[0][(lo >> 6) - (X0 >> 6)]);
      while (r < lastr && pre[r + 1] <= lo) ++r;
      uint8_t* dst = (reg ? P.val_arena + vb0 : P.key_arena + kb0) + x;
      const uint32_t dend = min(hi, pre[rows]);
      uint4 out = make_uint4(0, 0, 0, 0);
      for (uint32_t d = lo; d < dend; ++r) {
        const uint32_t e = min(dend, pre[r + 1]);
        if (e > d) {
          out = merge_bytes(out, load16_lds_b128(stage, sb[r] + x + sbias), int32_t(d - x),
                            int32_t(e - x));
          d = e;
        }
      }
      if (lo == x && hi == x + 16)
        *reinterpret_cast<uint4*>(dst) = out;
      else if (!(kSkip & 16))
        store_partial(dst, out, lo - x, hi - x);
    }
  }
}

// 8 waves per SIMD (8 workgroups per CU: the LDS bound; registers capped at
// 64 per lane, no spills; the uncapped form measured equal).
template <uint32_t kT, uint32_t kNT, bool kXcd>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(kT <= 16384 || kNT == 1024 ? 8 : 4))) void okv_tile_kernel(
    CopyParams P, uint32_t tpb, uint32_t ntile) {
  tile_pass<kT, kNT, kXcd>(P, tpb, ntile);
}

#ifdef OKV_ABLATE  // the measured alternative pass-3 forms (ablation build only)
#include "okv_decode_ablate.inc"
#endif


// Pass 3, small-block staged form (blocks averaging <= 16 KiB, e.g. 4 KiB
// blocks): one wave per block DMAs the whole block into its LDS stage right
// after the metadata arrives, then reads the record headers and assembles
// every key and value chunk from the stage: two dependent HBM trips per block
// (metadata + record positions, then the block) instead of four (metadata,
// positions, headers, key tiles, value tiles).  Blocks that do not fit the
// stage take the global-window gather (same workgroup, same row table code).
constexpr uint32_t kSmallStage = 5 * 1024;  // staged bytes per block (DMA pieces of 1 KiB)

// Byte source: a block's LDS stage; block byte x at stage byte bias + x.
struct StageWin {
  const uint4* s4;
  uint32_t bias;
  __device__ __forceinline__ uint4 at(int64_t rel) const {
    return load16_lds_b128(s4, uint32_t(int64_t(bias) + rel));
  }
  __device__ __forceinline__ void header(uint32_t pos, uint32_t& kl, uint32_t& vl) const {
    header_lds(reinterpret_cast<const uint32_t*>(s4), bias + pos, kl, vl);
  }
};

__global__ __launch_bounds__(64) void okv_gather_small_kernel(CopyParams P) {
  __shared__ GatherSmem sm;
  __shared__ uint4 stage[kSmallStage / 16 + 4];
  const uint32_t lane = threadIdx.x;
  for (uint32_t b = blockIdx.x; b < P.nblk; b += gridDim.x) {
    // record positions ride with the metadata (slots exist for every r < kRCap)
    const uint32_t rec0 = P.rt_pos[rec_index(P.nblk, b, lane)];
    const BlockMeta m = block_meta(P, b);
    if (block_head(P, b, m)) {
      const int rows = int(m.c.rows);
      const uint32_t rec = int(lane) < rows ? rec0 : 0u;
      const uint32_t shift = uint32_t(m.off & 15);
      // stage byte 0 = block byte -(16 + shift): a 16-byte lead-in for
      // windows that begin before a row, and 32 bytes of slack at the end
      const uint32_t need = 16 + shift + uint32_t(m.c.pend) + 32;
      if (need <= kSmallStage && !P.index_only) {
        const int64_t D = int64_t(m.off) - int64_t(shift) - 16;
        const int64_t lim = int64_t(round16(P.seg_bytes));
        const uint32_t np = (need + 1023) >> 10;
        for (uint32_t p = 0; p < np; ++p) {
          int64_t a = D + (int64_t(p) << 10) + int64_t(lane << 4);
          if (a < 0 || a + 16 > lim) a = int64_t(m.off) & ~int64_t(15);  // bytes never used
          __builtin_amdgcn_global_load_lds(P.seg + a, OKV_LDS_PTR(stage + p * 64), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const StageWin src{stage, 16 + shift};
        build_row_table(src, sm, rows, rec);
        write_row_index(P, sm, m, rows);
        gather_region<false>(src, sm, rows, P.key_arena, m.B.kb0, 0, 1);
        gather_region<true>(src, sm, rows, P.val_arena, m.B.vb0, 0, 1);
      } else {
        const GlobalWin src{P.seg, P.seg_bytes, m.off};
        build_row_table(src, sm, rows, rec);
        write_row_index(P, sm, m, rows);
        if (!P.index_only) {
          gather_region<false>(src, sm, rows, P.key_arena, m.B.kb0, 0, 1);
          gather_region<true>(src, sm, rows, P.val_arena, m.B.vb0, 0, 1);
        }
      }
    }
  }
}

// Single-pass decode for small batches of small blocks (<= kFusedMaxBlocks
// blocks averaging <= 16 KiB): passes 1-3 in ONE launch.  One wave per block
// takes the next block index from a counter, DMAs the whole block into LDS,
// walks its record headers there exactly as the Go loop does (lane 0;
// statuses as in okv_count_kernel) and publishes the block's (rows, key
// bytes, value bytes, bad); the block whose arrival is counted last scans all
// of them and publishes every block's exclusive prefix (sc1 stores and loads,
// flags tagged with the call's epoch so nothing is reset between calls);
// every block then gathers its rows from its stage.  (A decoupled look-back
// measured slower: its chain deepens with the blocks in flight.)  Blocks with more than kRCap rows, or too
// large to stage, get their counts the same way (a global-memory walk) and go
// to okv_copy_kernel through the big-block list, with cnt / lp / tile_pre
// written as passes 1-2 would.
constexpr uint32_t kFusedMaxBlocks = 512;  // every block of the grid resident at once
struct FusedParams {
  const int32_t* pre;     // zstd-stage statuses or null
  BlockCount* cnt;        // what passes 1-2 write, for okv_copy_kernel
  Prefix* lp;
  Prefix* tile_pre;
  uint32_t* flag;         // [nblk] (epoch << 2) | 1 aggregate, | 2 inclusive
  Prefix* agg;            // [nblk]
  Prefix* incl;           // [nblk]
  unsigned long long* ctr;  // block-index counter (monotone across calls)
  unsigned long long* arr;  // arrival counter (monotone across calls, same base)
  unsigned long long base;  // its value at this call's start
  uint32_t epoch;
  Totals* tot;
  uint32_t* big_zero;  // the other big-block counter slot: zeroed for the next launch
};

// Hand-off without release/acquire fences (an agent-scope release writes back
// the whole L2, an acquire invalidates it -- per block, that swamps the
// kernel): payload and flag go through coherent (sc1) stores, the payload
// drained before the flag, and the reader polls and reads with sc1 loads
// (cdna_hip_programming.md G16, valid forms).
__device__ __forceinline__ void publish(uint32_t* f, Prefix* slot, const Prefix& v, uint32_t tag) {
  __hip_atomic_store(&slot->rows, v.rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&slot->kb, v.kb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&slot->vb, v.vb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&slot->bad, v.bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(f, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void publish_payload(Prefix* slot, const Prefix& v) {
  __hip_atomic_store(&slot->rows, v.rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&slot->kb, v.kb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&slot->vb, v.vb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&slot->bad, v.bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ uint32_t flag_peek(const uint32_t* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ Prefix prefix_peek(const Prefix* slot) {
  Prefix v;
  v.rows = __hip_atomic_load(&slot->rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  v.kb = __hip_atomic_load(&slot->kb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  v.vb = __hip_atomic_load(&slot->vb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  v.bad = __hip_atomic_load(&slot->bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return v;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// kLB: the form for batches of any size (okv_decode_stream_kernel below):
// the exclusive prefix by a decoupled look-back instead of the last arrival's
// scan, so no block waits for blocks that may not be resident.
// The exclusive prefix by a decoupled look-back: the ablation build's stream
// kernel (okv_decode_ablate_lb.inc); declared here, defined only there.
__device__ Prefix fused_prefix_lookback(const CopyParams& P, const FusedParams& F, uint32_t b,
                                        uint32_t lane, uint32_t tag, const Prefix& mine);
#ifdef OKV_ABLATE
// (ablation build: wall-clock stamps of the fused kernel's phases per block --
// start, staged, walked, prefix known, done; okv_debug_fused_times)
__device__ uint64_t g_fused_t[kFusedMaxBlocks * 8];
#define OKV_FUSED_STAMP(i) \
  if (lane == 0 && b < kFusedMaxBlocks) g_fused_t[b * 8 + (i)] = wall_clock64()
#else
#define OKV_FUSED_STAMP(i)
#endif

// The fused kernel's look-back word per block: (epoch | 1 << 31) << 32 | its
// counts packed in 30 bits -- rows (10), padded key bytes / 16 (9), padded
// value bytes / 16 (9), failed (1), overflow (1: the counts do not fit and
// are in F.agg[b], published before the word).  One 8-byte write-through
// store is the payload and the flag at once.
__device__ __forceinline__ bool fused_pack(const Prefix& v, uint32_t& w) {
  if (v.rows >= 1024 || v.kb >= (512u << 4) || v.vb >= (512u << 4)) return false;
  w = uint32_t(v.rows) | uint32_t(v.kb >> 4) << 10 | uint32_t(v.vb >> 4) << 19 |
      uint32_t(v.bad) << 28;
  return true;
}

// A small block's header walk (okv_count_kernel's checks in Go's order,
// segment_reader.go:338-352) from its LDS stage, by the whole wave on a
// wave-uniform position, run-length speculated (okv_point_kernel's walk):
// from a record at p of length rl, lane j reads the header at p + j rl -- a
// record start if every record before it had the same header; the first lane
// that breaks the run (past OriginalSize, a failed check, another header) is
// itself a true record start.  A round of two dependent LDS reads confirms 2
// to 64 records (C2's fixed 86-byte records: all 42 in one round); lane 0
// alone paid one dependent header decode per record.  Record positions of
// rows < kRCap go to rec[].  A failed block has no rows (rows = kb = vb = 0)
// and p at the failing record.
template <class Src>
__device__ __forceinline__ void walk_staged(const Src& lsrc, uint32_t L, uint64_t original_size,
                                            uint32_t* rec, uint32_t lane, int32_t& st,
                                            uint64_t& rows, uint64_t& kb, uint64_t& vb,
                                            uint64_t& p) {
  const uint32_t o32 = __builtin_amdgcn_readfirstlane(
      uint32_t(min<uint64_t>(go_walk_bound(original_size), 0xffffffffull)));  // (:340)
  uint32_t pp = 0, nr = 0;
  kb = vb = 0;
  while (pp < o32) {  // :340
    uint32_t kl, vl;
    lsrc.header(min(pp, L), kl, vl);  // (one address: a broadcast)
    kl = __builtin_amdgcn_readfirstlane(kl);
    vl = __builtin_amdgcn_readfirstlane(vl);
    const uint32_t room = L - pp - 6;
    // u16/u32 reads (:342-345), key/value reads (:346-349)
    if (!((L - pp >= 6) & (kl <= room) & (vl <= room - kl))) {
      st = OKV_BLK_PANIC;
      break;
    }
    const uint32_t rl = 6 + kl + vl;
    const uint32_t q = pp + lane * rl;  // (< 64 * 64 KiB)
    uint32_t kj, vj;
    lsrc.header(min(q, L), kj, vj);
    const uint32_t rj = L - q - 6;
    const bool okj = (q <= L) & (L - q >= 6) & (kj <= rj) & (vj <= rj - kj);
    // (the run is of equal headers, not only equal lengths: the counts add
    // m key and value lengths)
    const bool brk = lane >= 1 && (q >= o32 || !okj || kj != kl || vj != vl);
    const uint64_t bm = __ballot(brk);
    const uint32_t m = bm ? uint32_t(__builtin_ctzll(bm)) : 64u;  // (>= 1)
    if (lane < m && nr + lane < uint32_t(kRCap)) rec[nr + lane] = q;
    nr += m;
    kb += uint64_t(m) * kl;
    vb += uint64_t(m) * vl;
    pp += m * rl;  // the breaking lane's position: a true record start
    if (m == 64 || pp >= o32) continue;
    const uint32_t okm = __builtin_amdgcn_readlane(uint32_t(okj), m);
    const uint32_t km = __builtin_amdgcn_readlane(kj, m), vm = __builtin_amdgcn_readlane(vj, m);
    if (!okm) {
      st = OKV_BLK_PANIC;
      break;
    }
    if (lane == 0 && nr < uint32_t(kRCap)) rec[nr] = pp;
    ++nr;
    kb += km;
    vb += vm;
    pp += 6 + km + vm;
  }
  rows = nr;
  p = pp;
  if (st != OKV_BLK_OK) rows = kb = vb = 0;
}
// The same walk in HBM by lane 0 (a block too large for the stage); the
// results are broadcast to the wave.
__device__ __forceinline__ void walk_global(const uint8_t* seg, uint64_t off, uint64_t len,
                                            uint64_t original_size, uint32_t* rec, uint32_t lane,
                                            int32_t& st, uint64_t& rows, uint64_t& kb,
                                            uint64_t& vb, uint64_t& p) {
  rows = kb = vb = p = 0;
  if (lane == 0) {
    const uint64_t orig = go_walk_bound(original_size);
    while (p < orig) {  // :340
      if (len - p < 6) { st = OKV_BLK_PANIC; break; }  // :342-345
      uint32_t kl, vl;
      header_global(seg, off + p, kl, vl);
      const uint64_t room = len - p - 6;
      if (kl > room || vl > room - kl) { st = OKV_BLK_PANIC; break; }  // :346-349
      if (rows < kRCap) rec[rows] = uint32_t(p);
      rows++;
      kb += kl;
      vb += vl;
      p += 6 + uint64_t(kl) + uint64_t(vl);
    }
    if (st != OKV_BLK_OK) rows = kb = vb = 0;
  }
  st = __shfl(st, 0, 64);
  rows = __shfl(rows, 0, 64);
  kb = __shfl(kb, 0, 64);
  vb = __shfl(vb, 0, 64);
  p = __shfl(p, 0, 64);
}

template <bool kLB>  // (kLB: the ablation build's stream kernel only)
__device__ __forceinline__ void fused_pass(const CopyParams& P, const FusedParams& F) {
  __shared__ GatherSmem sm;
  __shared__ uint4 stage[kSmallStage / 16 + 4];
  const uint32_t lane = threadIdx.x;
  uint32_t b = blockIdx.x;
  if constexpr (kLB) {  // blocks by arrival (the stream kernel's grid is not resident)
    __shared__ uint32_t s_b;
    if (lane == 0) s_b = uint32_t(atomicAdd(F.ctr, 1ull) - F.base);
    __syncthreads();
    b = s_b;
    if (b >= P.nblk) return;
  }
  // (the product grid is all resident -- a quarter of the device's capacity
  // -- and dispatched in index order, so a block waits only on lower indices
  // that have started: no block-index counter)
  const uint32_t tag = F.epoch << 2;
  OKV_FUSED_STAMP(0);
  if (b == 0 && lane == 0) *F.big_zero = 0;
  // ---- pass 1 for this block (okv_count_kernel's rules) ----
  const Desc d = P.descs[b];
  const uint64_t len = (P.comp == OKV_COMP_LZ4) ? 0 : d.block_size;  // Q7 (:331-333)
  const uint32_t shift = uint32_t(d.offset & 15);
  int32_t st = OKV_BLK_OK;
  {
    const int32_t pre = F.pre ? F.pre[b] : int32_t(OKV_BLK_OK);
    if (pre != OKV_BLK_OK) st = pre;  // outcome of the zstd stage
    else if ((st = go_read_status(d, P.seg_bytes)) != OKV_BLK_OK) {}  // :303-316
    else if (P.comp == OKV_COMP_ZSTD) st = OKV_BLK_UNSUPPORTED;
  }
  const uint32_t need = 16 + shift + uint32_t(len < kSmallStage ? len : kSmallStage) + 32;
  const bool staged = st == OKV_BLK_OK && len + 16 + shift + 32 <= kSmallStage;
  if (staged && len) {  // the whole block (BlockSize bytes) into the stage
    const int64_t D = int64_t(d.offset) - int64_t(shift) - 16;
    const int64_t lim = int64_t(round16(P.seg_bytes));
    const uint32_t np = (need + 1023) >> 10;
    for (uint32_t p = 0; p < np; ++p) {
      int64_t a = D + (int64_t(p) << 10) + int64_t(lane << 4);
      if (a < 0 || a + 16 > lim) a = int64_t(d.offset) & ~int64_t(15);  // bytes never used
      __builtin_amdgcn_global_load_lds(P.seg + a, OKV_LDS_PTR(stage + p * 64), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  OKV_FUSED_STAMP(1);
  const StageWin lsrc{stage, 16 + shift};
  uint64_t rows = 0, kb = 0, vb = 0, p = 0;
  if (st == OKV_BLK_OK && staged)
    walk_staged(lsrc, uint32_t(len), d.original_size, sm.rec, lane, st, rows, kb, vb, p);
  else if (st == OKV_BLK_OK)  // not stageable: lane 0 walks the headers in HBM
    walk_global(P.seg, d.offset, len, d.original_size, sm.rec, lane, st, rows, kb, vb, p);
  __syncthreads();  // the walk's record positions (sm.rec) are read by every lane below
  OKV_FUSED_STAMP(2);
  const Prefix mine{rows, round16(kb), round16(vb), uint64_t(st != OKV_BLK_OK)};
  Prefix ex{0, 0, 0, 0};
  // ---- pass 2: each block sums its predecessors' published counts ----
  // One write-through 8-byte word per block carries its counts and the
  // call's tag (fused_pack); every lane loads the words of up to
  // kFusedMaxBlocks / 64 predecessors at once and re-polls only those not
  // yet published.  (Round 5: the last block to arrive scanned every
  // block's counts and published the prefixes behind a second flag -- a
  // chain of dependent cross-XCD trips that every block waited out.)
  uint64_t* word = reinterpret_cast<uint64_t*>(F.flag);
  const uint32_t want = F.epoch | 0x80000000u;
  if (!kLB && lane == 0) {
    uint32_t w = 0;
    if (!fused_pack(mine, w)) {
      publish_payload(&F.agg[b], mine);  // sc1 stores, drained
      w = 1u << 29;
    }
    __hip_atomic_store(&word[b], uint64_t(want) << 32 | w, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  // Pass 3 up to the stores, while the predecessors' counts arrive: a staged
  // block's key and value regions are assembled into an LDS image (block-
  // local offsets); only the row index and the image's copy-out wait for the
  // prefix.  (C2: the gather after the wait took 3.0 us of a 14 us kernel.)
  __shared__ uint4 img[kSmallStage / 16 + 2];
  const int nr = int(rows);
  const bool pre_asm = !kLB && staged && st == OKV_BLK_OK && nr > 0 && rows <= uint64_t(kRCap) &&
                       !P.index_only;
  const uint32_t kreg = uint32_t(round16(kb)), vreg = uint32_t(round16(vb));
  if (pre_asm) {
    static_assert(sizeof(img) >= kSmallStage, "both regions fit the image");
    const uint32_t rec = int(lane) < nr ? sm.rec[lane] : 0u;
    build_row_table(lsrc, sm, nr, rec);
    uint8_t* const im = reinterpret_cast<uint8_t*>(img);
    gather_region<false>(lsrc, sm, nr, im, 0, 0, 1);
    gather_region<true>(lsrc, sm, nr, im, kreg, 0, 1);
  }
  if constexpr (kLB) {
    ex = fused_prefix_lookback(P, F, b, lane, tag, mine);  // ablation build only
  } else {
    constexpr uint32_t kU = kFusedMaxBlocks / 64;
    uint64_t wv[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint32_t k = lane + 64 * u;
      wv[u] = k < b ? __hip_atomic_load(&word[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                    : uint64_t(want) << 32;
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint32_t k = lane + 64 * u;
      while (uint32_t(wv[u] >> 32) != want) {
        __builtin_amdgcn_s_sleep(1);
        wv[u] = __hip_atomic_load(&word[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const uint32_t w = uint32_t(wv[u]);
      if (w >> 29 & 1u) {
        const Prefix o = prefix_peek(&F.agg[k]);
        ex.rows += o.rows;
        ex.kb += o.kb;
        ex.vb += o.vb;
        ex.bad += o.bad;
      } else {
        ex.rows += w & 1023u;
        ex.kb += uint64_t(w >> 10 & 511u) << 4;
        ex.vb += uint64_t(w >> 19 & 511u) << 4;
        ex.bad += w >> 28 & 1u;
      }
    }
    ex.rows = wave_sum64(ex.rows);
    ex.kb = wave_sum64(ex.kb);
    ex.vb = wave_sum64(ex.vb);
    ex.bad = wave_sum64(ex.bad);
    if (b == P.nblk - 1 && lane == 0) {  // the totals
      *F.tot = Totals{ex.rows + mine.rows, ex.kb + mine.kb, ex.vb + mine.vb, ex.bad + mine.bad};
      P.row_start[P.nblk] = ex.rows + mine.rows;
    }
  }
  OKV_FUSED_STAMP(3);
  // ---- what passes 1-2 leave for okv_copy_kernel, and the totals ----
  if (lane == 0) {
    BlockCount c;
    c.rows = rows;
    c.kbytes = kb;
    c.vbytes = vb;
    c.pend = p;
    c.status = st;
    c.pad = 0;
    F.cnt[b] = c;
    F.lp[b] = ex;
    if (b % kTile == 0) F.tile_pre[b / kTile] = Prefix{0, 0, 0, 0};
    if (st == OKV_BLK_OK && (rows > kRCap || p >= (uint64_t(1) << 32)))
      P.big_list[atomicAdd(P.big_count, 1u)] = b;
  }
  // ---- pass 3 ----
  BlockMeta m;
  m.c = BlockCount{rows, kb, vb, p, st, 0};
  m.B = block_base_of(P, m.c, ex, Prefix{0, 0, 0, 0});
  m.off = d.offset;
  if (!block_head(P, b, m)) {
    OKV_FUSED_STAMP(4);
    return;
  }
  if (pre_asm) {  // the row index, then the image out in whole 16-byte chunks
    write_row_index(P, sm, m, nr);
    for (uint32_t c = lane; c < kreg / 16; c += 64)
      *reinterpret_cast<uint4*>(P.key_arena + m.B.kb0 + 16ull * c) = img[c];
    for (uint32_t c = lane; c < vreg / 16; c += 64)
      *reinterpret_cast<uint4*>(P.val_arena + m.B.vb0 + 16ull * c) = img[kreg / 16 + c];
    OKV_FUSED_STAMP(4);
    return;
  }
  const uint32_t rec = int(lane) < nr ? sm.rec[lane] : 0u;
  if (staged) {
    build_row_table(lsrc, sm, nr, rec);
    write_row_index(P, sm, m, nr);
    if (!P.index_only) {
      gather_region<false>(lsrc, sm, nr, P.key_arena, m.B.kb0, 0, 1);
      gather_region<true>(lsrc, sm, nr, P.val_arena, m.B.vb0, 0, 1);
    }
  } else {
    const GlobalWin gsrc{P.seg, P.seg_bytes, m.off};
    build_row_table(gsrc, sm, nr, rec);
    write_row_index(P, sm, m, nr);
    if (!P.index_only) {
      gather_region<false>(gsrc, sm, nr, P.key_arena, m.B.kb0, 0, 1);
      gather_region<true>(gsrc, sm, nr, P.val_arena, m.B.vb0, 0, 1);
    }
  }
  OKV_FUSED_STAMP(4);
}

__global__ __launch_bounds__(64) void okv_decode_fused_kernel(CopyParams P, FusedParams F) {
  fused_pass<false>(P, F);
}

// ---------------------------------------------------------------------------
// Pass 4 (big blocks only): LDS-staged decode with a serial header chase.
// ---------------------------------------------------------------------------
struct SlowRows {               // general path: 64-bit positions, batched rows
  uint64_t rec[kRowBatch];        // record position within the block
  uint64_t kpre[kRowBatch + 1];   // key-byte prefix within the block
  uint64_t vpre[kRowBatch + 1];   // value-byte prefix within the block
  uint32_t klen[kRowBatch];
  uint32_t vlen[kRowBatch];
};
struct FastRows {               // fast path: block staged in LDS, <= kFastRows rows
  uint32_t rec[kFastRows + 1];    // record position; rec[rows] = end of the walk
  uint32_t kpre[kFastRows + 1];   // exclusive prefix of key lengths
  uint32_t vpre[kFastRows + 1];   // exclusive prefix of value lengths
};
// okv_point_get's probe key (<= 8 KiB): over the fast row table's prefix
// arrays, which its search does not use (the record positions stay live).
struct FindRows {
  uint32_t rec[kFastRows + 1];
  uint32_t key[8192 / 4];
};
static_assert(offsetof(FindRows, key) == offsetof(FastRows, kpre), "key starts at kpre");
static_assert(sizeof(FindRows) <= sizeof(FastRows), "the key adds no LDS");
struct __align__(16) CopySmem {
  uint4 stage[(kStage + kStagePad) / 16];  // [16 B guard][block image][guard]
  union {
    SlowRows s;
    FastRows f;
    FindRows k;
  };
};

// Byte source: the LDS image of the block (byte index = 16 + shift + pos).
struct LdsSrc {
  const uint32_t* sw;
  uint32_t bias;
  __device__ __forceinline__ void header(uint64_t pos, uint32_t& kl, uint32_t& vl) const {
    header_lds(sw, bias + uint32_t(pos), kl, vl);
  }
  __device__ __forceinline__ uint4 load16(int64_t pos) const {
    return load16_lds(sw, uint32_t(int64_t(bias) + pos));
  }
};

// Byte source: the block in HBM (blocks too large to stage).
struct GlobalSrc {
  const uint8_t* seg;
  uint64_t seg_bytes;
  uint64_t off;
  __device__ __forceinline__ void header(uint64_t pos, uint32_t& kl, uint32_t& vl) const {
    header_global(seg, off + pos, kl, vl);
  }
  __device__ __forceinline__ uint4 load16(int64_t pos) const {
    return load16_global(seg, seg_bytes, int64_t(off) + pos);
  }
};


// Copy rows [0, nb) of one region (keys or values) into `arena`:
//   row i bytes = src[spos_i, spos_i + len_i) -> arena[dbase + pre_i, ...).
// Lane groups of G lanes own one row; each lane writes 16-byte aligned
// destination chunks (dwordx4), masked head/tail chunks with narrow stores.
template <int V, class Src>
__device__ __forceinline__ void copy_region(const Src& src, uint8_t* __restrict__ arena,
                                            uint64_t dbase, const uint64_t* pre,
                                            const uint64_t* rec, const uint32_t* klen,
                                            const uint32_t* len, bool is_val, int nb,
                                            uint32_t G) {
  const uint32_t tid = threadIdx.x;
  const uint32_t grp = tid / G, sub = tid % G, ngrp = blockDim.x / G;
  for (uint32_t i = grp; i < uint32_t(nb); i += ngrp) {
    const uint64_t L = len[i];
    if (L == 0) continue;
    const uint64_t d0 = dbase + pre[i];
    const int64_t s0 = int64_t(rec[i] + 6 + (is_val ? klen[i] : 0));
    const uint64_t c0 = d0 & ~uint64_t(15), c1 = (d0 + L + 15) & ~uint64_t(15);
    for (uint64_t ca = c0 + 16ull * sub; ca < c1; ca += 16ull * G) {
      const int64_t rel = int64_t(ca) - int64_t(d0);
      const uint4 v = (V == 5) ? make_uint4(uint32_t(ca), 0, 0, 0) : src.load16(s0 + rel);
      const uint32_t lo = ca < d0 ? uint32_t(d0 - ca) : 0u;
      const uint64_t end = d0 + L - ca;
      const uint32_t hi = end < 16 ? uint32_t(end) : 16u;
      if (lo == 0 && hi == 16) {
        *reinterpret_cast<uint4*>(arena + ca) = v;
      } else if (V != 4) {
        store_partial(arena + ca, v, lo, hi);
      }
    }
  }
}

template <int V, class Src>
__device__ __forceinline__ void materialise(const Src& src, const CopyParams& P,
                                           CopySmem& sm, uint64_t rows, uint64_t kbytes,
                                           uint64_t vbytes, uint64_t row0, uint64_t kb0,
                                           uint64_t vb0, uint64_t pend) {
  const uint32_t tid = threadIdx.x;
  const uint32_t Gk = group_size(kbytes / rows), Gv = group_size(vbytes / rows);
  uint64_t p = 0, kacc = 0, vacc = 0;  // chase state (lane 0)
  for (uint64_t r0 = 0; r0 < rows; r0 += kRowBatch) {
    const int nb = int(rows - r0 < kRowBatch ? rows - r0 : kRowBatch);
    if (tid == 0) {
      // serial header chase: record i+1 starts at rec_i + 6 + klen_i + vlen_i
      // (lengths and positions clamped to pass 1's totals and walk end: if the
      // segment changed under the decode, reads stay inside the block's walk
      // and writes inside its regions)
      for (int i = 0; i < nb; ++i) {
        uint32_t kl, vl;
        src.header(p, kl, vl);
        kl = uint32_t(min<uint64_t>(kl, kbytes - kacc));
        vl = uint32_t(min<uint64_t>(vl, vbytes - vacc));
        sm.s.rec[i] = p;
        sm.s.klen[i] = kl;
        sm.s.vlen[i] = vl;
        sm.s.kpre[i] = kacc;
        sm.s.vpre[i] = vacc;
        kacc += kl;
        vacc += vl;
        p = min<uint64_t>(p + 6 + uint64_t(kl) + uint64_t(vl), pend - 6);
      }
      sm.s.kpre[nb] = kacc;
      sm.s.vpre[nb] = vacc;
    }
    __syncthreads();
    // SoA row index (coalesced over rows)
    for (int i = tid; i < nb; i += blockDim.x) {
      const uint64_t g = row0 + r0 + i;
      P.key_off[g] = kb0 + sm.s.kpre[i];
      P.key_len[g] = uint16_t(sm.s.klen[i]);
      P.val_off[g] = vb0 + sm.s.vpre[i];
      P.val_len[g] = sm.s.vlen[i];
    }
    copy_region<V>(src, P.key_arena, kb0, sm.s.kpre, sm.s.rec, sm.s.klen, sm.s.klen, false, nb, Gk);
    copy_region<V>(src, P.val_arena, vb0, sm.s.vpre, sm.s.rec, sm.s.klen, sm.s.vlen, true, nb, Gv);
    __syncthreads();
  }
  // zero the 16-byte padding tail of each arena region
  if (tid == 0) {
    const uint64_t ke = kb0 + kbytes, ve = vb0 + vbytes;
    const uint4 z = make_uint4(0, 0, 0, 0);
    if (ke & 15) store_partial(P.key_arena + (ke & ~uint64_t(15)), z, uint32_t(ke & 15), 16);
    if (ve & 15) store_partial(P.val_arena + (ve & ~uint64_t(15)), z, uint32_t(ve & 15), 16);
  }
}

// ---- fast path: the block is staged in LDS and has <= kFastRows rows ------
// Every arena store is a full, aligned 16-byte chunk.  A chunk is owned by
// the row containing its first byte; its owner lane assembles it in
// registers, merging bytes of the following rows when the chunk spills past
// its row (no partial stores, so neighbouring chunks never race).  The last
// chunk of a region is zero-filled past the region end (16-byte padding).
template <bool kVal, int V = 3>
__device__ __forceinline__ void copy_region_fast(const uint4* __restrict__ s4, uint32_t bias,
                                                 uint8_t* __restrict__ arena, uint64_t dbase,
                                                 const FastRows& t, int rows, uint32_t G) {
  const uint32_t* pre = kVal ? t.vpre : t.kpre;
  const uint32_t tid = threadIdx.x;
  const uint32_t grp = tid / G, sub = tid % G, ngrp = blockDim.x / G;
  for (uint32_t i = grp; i < uint32_t(rows); i += ngrp) {
    const uint32_t p0 = pre[i], p1 = pre[i + 1];
    if (p1 == p0) continue;
    const uint32_t cfirst = (p0 + 15) >> 4, clast = (p1 - 1) >> 4;
    const uint32_t si = bias + t.rec[i] + 6 + (kVal ? t.kpre[i + 1] - t.kpre[i] : 0u);
    for (uint32_t c = cfirst + sub; c <= clast; c += G) {
      const uint32_t cs = c << 4, ce = cs + 16;
      if (V == 6) {  // diagnostic: stores only
        *reinterpret_cast<uint4*>(arena + dbase + cs) = make_uint4(cs, i, 0, 0);
        continue;
      }
      uint4 out = load16_lds_b128(s4, si + (cs - p0));
      if (ce > p1) {  // spills past row i: keep [0, p1-cs), gather the rest
        out = merge_bytes(make_uint4(0, 0, 0, 0), out, 0, int32_t(p1 - cs));
        for (uint32_t j = i + 1; j < uint32_t(rows) && pre[j] < ce; ++j) {
          const uint32_t q0 = pre[j], q1 = pre[j + 1];
          if (q1 == q0) continue;
          const uint32_t sj = bias + t.rec[j] + 6 + (kVal ? t.kpre[j + 1] - t.kpre[j] : 0u);
          const uint4 v = load16_lds_b128(s4, sj - (q0 - cs));
          out = merge_bytes(out, v, int32_t(q0 - cs), int32_t((q1 < ce ? q1 : ce) - cs));
        }
      }
      if (V == 7) {  // diagnostic: no stores
        asm volatile("" ::"v"(out.x), "v"(out.y), "v"(out.z), "v"(out.w));
        continue;
      }
      *reinterpret_cast<uint4*>(arena + dbase + cs) = out;
    }
  }
}

// SoA rows and both arena regions of a block staged in LDS whose row table
// (rec / kpre / vpre, <= kFastRows rows) is built.
template <int V>
__device__ __forceinline__ void emit_fast(const CopyParams& P, CopySmem& sm, uint32_t bias,
                                          int rows, uint64_t kbytes, uint64_t vbytes,
                                          uint64_t row0, uint64_t kb0, uint64_t vb0) {
  const uint32_t tid = threadIdx.x;
  FastRows& t = sm.f;
  for (int i = tid; i < rows; i += blockDim.x) {
    const uint64_t g = row0 + i;
    P.key_off[g] = kb0 + t.kpre[i];
    P.key_len[g] = uint16_t(t.kpre[i + 1] - t.kpre[i]);
    P.val_off[g] = vb0 + t.vpre[i];
    P.val_len[g] = t.vpre[i + 1] - t.vpre[i];
  }
  if (V < 3) return;
  const uint32_t Gk = group_size(kbytes / rows), Gv = group_size(vbytes / rows);
  copy_region_fast<false, V>(sm.stage, bias, P.key_arena, kb0, t, rows, Gk);
  copy_region_fast<true, V>(sm.stage, bias, P.val_arena, vb0, t, rows, Gv);
}

template <int V>
__device__ __forceinline__ void materialise_fast(const CopyParams& P, CopySmem& sm,
                                                uint32_t bias, int rows, uint64_t kbytes,
                                                uint64_t vbytes, uint64_t row0, uint64_t kb0,
                                                uint64_t vb0) {
  const uint32_t tid = threadIdx.x;
  FastRows& t = sm.f;
  if (tid == 0) {
    // serial header chase in LDS: record i+1 starts at rec_i + 6 + klen_i + vlen_i
    // (lengths clamped to pass 1's totals: if the segment changed under the
    // decode, the walk still writes only inside this block's regions)
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(sm.stage);
    uint32_t p = 0, ka = 0, va = 0;
    for (int i = 0; i < rows; ++i) {
      uint32_t kl, vl;
      header_lds(sw, bias + p, kl, vl);
      kl = min(kl, uint32_t(kbytes) - ka);
      vl = min(vl, uint32_t(vbytes) - va);
      t.rec[i] = p;
      t.kpre[i] = ka;
      t.vpre[i] = va;
      ka += kl;
      va += vl;
      p = min(p + 6 + kl + vl, uint32_t(kStage));
    }
    t.rec[rows] = p;
    t.kpre[rows] = ka;
    t.vpre[rows] = va;
  }
  __syncthreads();
  if (V < 2) return;  // diagnostic ablation (okv_copy_kernel<V>)
  emit_fast<V>(P, sm, bias, rows, kbytes, vbytes, row0, kb0, vb0);
}

__global__ __launch_bounds__(kThreads) void okv_copy_kernel(CopyParams P) {
  __shared__ CopySmem sm;
  const uint32_t tid = threadIdx.x;
  const uint32_t nbig = *P.big_count;
  for (uint32_t k = blockIdx.x; k < nbig; k += gridDim.x) {
    const uint32_t b = P.big_list[k];
    const BlockCount c = P.cnt[b];
    const BlockBase B = block_base(P, b, c);
    if (B.st != OKV_BLK_OK) continue;  // status written by okv_gather_kernel
    const Desc d = P.descs[b];
    if (c.pend <= uint64_t(kStage)) {
      // stage [offset - shift, offset + pend) with aligned 16-byte loads
      const uint32_t shift = uint32_t(d.offset & 15);
      const uint32_t nch = uint32_t((shift + c.pend + 15) / 16);
      const uint4* g = reinterpret_cast<const uint4*>(P.seg + (d.offset - shift));
      for (uint32_t ci = tid; ci < nch; ci += kThreads) sm.stage[1 + ci] = load_nt16(g + ci);
      __syncthreads();
      if (c.rows <= uint64_t(kFastRows)) {
        materialise_fast<3>(P, sm, 16u + shift, int(c.rows), c.kbytes, c.vbytes, B.row0, B.kb0,
                            B.vb0);
      } else {
        LdsSrc src{reinterpret_cast<const uint32_t*>(sm.stage), 16u + shift};
        materialise<3>(src, P, sm, c.rows, c.kbytes, c.vbytes, B.row0, B.kb0, B.vb0, c.pend);
      }
    } else {
      GlobalSrc src{P.seg, P.seg_bytes, d.offset};
      materialise<3>(src, P, sm, c.rows, c.kbytes, c.vbytes, B.row0, B.kb0, B.vb0, c.pend);
    }
    __syncthreads();  // LDS is reused by the next big block
  }
}

// ---------------------------------------------------------------------------
// Point reads: a host-mode call of a few small uncompressed blocks (GetRow's
// one block, GetRange's few; segment_reader.go:362-404, :410-475).  One
// workgroup decodes the batch block after block, reading the staged bytes
// straight from the context's pinned slab and writing every output into it,
// so the call is one launch and one synchronisation (no H2D / D2H copies,
// no plan, no totals read-back).  Per block: the block's
// bytes into LDS (one trip over PCIe), the header walk in LDS by lane 0 with
// okv_count_kernel's checks in Go's order (:338-352), recording the row table
// as it goes, then the SoA rows and both arena regions from LDS (emit_fast;
// blocks of more than kFastRows rows re-walk in batches, materialise).  The
// host admits only batches whose OK blocks stage (BlockSize <= kStage).
// ---------------------------------------------------------------------------
#ifdef OKV_ABLATE
// (ablation build: wall-clock stamps of the point kernel's phases for the
// last block of the last call -- start, staged, walked, prefixes, emitted;
// okv_debug_point_times, tools/point_phases.py)
__device__ uint64_t g_point_t[8];
#define OKV_POINT_STAMP(i) \
  if (tid == 0) g_point_t[i] = wall_clock64()
#else
#define OKV_POINT_STAMP(i)
#endif
// okv_point_get's search (GetRow :395-403): the key (<= kFindKey bytes, host
// memory, 4-byte aligned) and the answer: found = 1 (the row's key and value
// at key_arena / val_arena, lengths at key_len[0] / val_len[0]), 0, or -1
// (more rows than the row table: the caller decodes the block in full).
struct PointFind {
  const uint8_t* key;
  uint32_t klen;
  int32_t* found;
  uint32_t* done;  // non-null: the call's completion word in the pinned slab (point_wait)
  uint32_t seq;    // ... the value the kernel writes there last
};
// The kernel's last act: every wave's slab writes pushed to system scope,
// then one store of the call's sequence number, for which the host spins
// (point_wait) instead of waiting in hipStreamSynchronize.
__device__ __forceinline__ void point_done(const PointFind& F) {
  if (!F.done) return;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(F.done, F.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
constexpr uint32_t kFindKey = 8192;  // (held in the row table's prefix arrays)

template <bool kFind>
__global__ __launch_bounds__(kThreads) void okv_point_kernel(CopyParams P, Totals* tot,
                                                             PointFind F) {
  __shared__ CopySmem sm;
  __shared__ uint64_t s_walk[4];  // rows, key bytes, value bytes, walk end
  __shared__ uint32_t s_wsum[2][kThreads / 64];
  __shared__ int32_t s_st, s_pst;
  __shared__ uint32_t s_pw[2];
  const uint32_t tid = threadIdx.x;
  const uint32_t* sw = reinterpret_cast<const uint32_t*>(sm.stage);
  uint64_t row0 = 0, kb0 = 0, vb0 = 0, bad = 0;  // exclusive prefixes (uniform)
  if constexpr (kFind) {  // the key into LDS (the prefix arrays: unused by the search)
    static_assert(sizeof(sm.k.key) >= kFindKey, "the key fits its LDS array");
    const uint32_t* k4 = reinterpret_cast<const uint32_t*>(F.key);
    for (uint32_t i = tid; i < (F.klen + 3) / 4; i += kThreads) sm.k.key[i] = k4[i];
  }
  for (uint32_t b = 0; b < P.nblk; ++b) {
    OKV_POINT_STAMP(0);
    const Desc d = P.descs[b];
    const int32_t st0 = go_read_status(d, P.seg_bytes);  // :303-316
    const uint64_t len = P.comp == OKV_COMP_LZ4 ? 0 : d.block_size;  // Q7 (:331-333)
    const uint32_t shift = uint32_t(d.offset & 15);
    if (st0 == OKV_BLK_OK && len) {  // stage [offset - shift, offset + len): one trip
      // (LDS DMA: every 16-byte piece in flight at once -- a load/store loop
      // paid one PCIe round trip per iteration, ~16 for a 64 KiB block)
      const uint32_t nch = uint32_t((shift + len + 15) >> 4);
      const uint8_t* g = P.seg + (d.offset - shift);
      const uint32_t lane = tid & 63, wave = tid >> 6;
      for (uint32_t c0 = wave * 64; c0 < nch; c0 += kThreads) {
        if (c0 + lane < nch)  // (an inactive lane writes no LDS)
          __builtin_amdgcn_global_load_lds(g + 16ull * (c0 + lane), OKV_LDS_PTR(sm.stage + 1 + c0),
                                           16, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    OKV_POINT_STAMP(1);
    const uint32_t bias = 16u + shift;
    // The header walk (Go's checks in its order) by wave 0 on a wave-uniform
    // position, run-length speculated: from a record at p of length len, lane
    // j reads the header at p + j * len -- a record start if every record
    // before it was len long.  The first lane that breaks the run (past
    // OriginalSize, a failed check, another length) ends the round; its
    // position is a true record start, so a round confirms at least two
    // records (the one at p and the next) and up to 64 when lengths repeat,
    // for two dependent LDS reads.  (Lane 0 alone, one dependent header
    // decode per record: 120 ns a record, 80 us of a 64 KiB block's GetRow.)
    const uint32_t L = st0 == OKV_BLK_OK ? uint32_t(len) : 0u;  // <= kStage
    const uint64_t orig = go_walk_bound(d.original_size);       // int(OriginalSize) (:340)
    if (tid < 64) {
      const uint32_t lane = tid;
      const uint32_t o32 =
          __builtin_amdgcn_readfirstlane(uint32_t(min<uint64_t>(orig, 0xffffffffull)));
      uint32_t p = 0, rows = 0;
      int32_t pst = st0;
      if (st0 == OKV_BLK_OK) {
        while (p < o32) {  // :340
          uint32_t kl, vl;
          header_lds(sw, bias + min(p, L), kl, vl);  // (one address: a broadcast)
          kl = __builtin_amdgcn_readfirstlane(kl);
          vl = __builtin_amdgcn_readfirstlane(vl);
          const uint32_t room = L - p - 6;
          // u16/u32 reads (:342-345), key/value reads (:346-349)
          if (!((L - p >= 6) & (kl <= room) & (vl <= room - kl))) {
            pst = OKV_BLK_PANIC;
            break;
          }
          const uint32_t rl = 6 + kl + vl;
          const uint32_t q = p + lane * rl;  // (< 64 * 64 KiB)
          uint32_t kj, vj;
          header_lds(sw, bias + min(q, L), kj, vj);
          const uint32_t rj = L - q - 6;
          const bool okj = (q <= L) & (L - q >= 6) & (kj <= rj) & (vj <= rj - kj);
          const bool brk = lane >= 1 && (q >= o32 || !okj || 6 + kj + vj != rl);
          const uint64_t bm = __ballot(brk);
          const uint32_t m = bm ? uint32_t(__builtin_ctzll(bm)) : 64u;  // (>= 1)
          if (lane < m) sm.f.rec[min(rows + lane, uint32_t(kFastRows))] = q;
          rows += m;
          p += m * rl;  // the breaking lane's position: a true record start
          if (m == 64 || p >= o32) continue;
          const uint32_t okm = __builtin_amdgcn_readlane(uint32_t(okj), m);
          const uint32_t lm = __builtin_amdgcn_readlane(6 + kj + vj, m);
          if (!okm) {
            pst = OKV_BLK_PANIC;
            break;
          }
          if (lane == 0) sm.f.rec[min(rows, uint32_t(kFastRows))] = p;
          ++rows;
          p += lm;
        }
      }
      if (tid == 0) {
        s_pw[0] = p;
        s_pw[1] = rows;
        s_pst = pst;
      }
    }
    __syncthreads();
    if (tid == 0) {
      int32_t st = s_pst;
      uint32_t rows = s_pw[1], p = s_pw[0];
      // a walk that reached the block end short of OriginalSize: the header read (:342-345)
      if (st == OKV_BLK_OK && p < orig) st = OKV_BLK_PANIC;
      if (st != OKV_BLK_OK) rows = p = 0;  // a failed block has no rows
      s_walk[0] = rows;
      s_walk[3] = p;
      s_st = st;
      P.row_start[b] = row0;
      P.key_base[b] = kb0;
      P.val_base[b] = vb0;
      P.blk_status[b] = st;
    }
    __syncthreads();
    OKV_POINT_STAMP(2);
    const uint64_t rows = s_walk[0], pend = s_walk[3];
    const int32_t st = s_st;
    uint64_t kb = 0, vb = 0;
    if constexpr (kFind) {
      // the first row whose key equals F.key: one lane per row compares in
      // LDS, the lowest index wins; only that row's bytes go back
      __shared__ uint32_t s_hit;
      if (tid == 0) s_hit = ~0u;
      __syncthreads();
      const bool listed = rows <= uint64_t(kFastRows);
      if (st == OKV_BLK_OK && listed) {
        const uint32_t* tk = sm.k.key;
        for (uint32_t i = tid; i < uint32_t(rows); i += kThreads) {
          uint32_t kl, vl;
          header_lds(sw, bias + sm.f.rec[i], kl, vl);
          if (kl != F.klen) continue;
          const uint32_t kp = bias + sm.f.rec[i] + 6;
          bool eq = true;
          for (uint32_t j = 0; j < kl && eq; j += 4) {
            const uint32_t bi = kp + j, sh = bi & 3;
            const uint32_t a = funnel(sw[(bi >> 2) + 1], sw[bi >> 2], sh);
            const uint32_t n = min(4u, kl - j);
            const uint32_t m = n == 4 ? ~0u : (1u << (8 * n)) - 1u;
            eq = ((a ^ tk[j >> 2]) & m) == 0;
          }
          if (eq) atomicMin(&s_hit, i);
        }
      }
      __syncthreads();
      OKV_POINT_STAMP(3);
      const uint32_t hit = s_hit;
      uint32_t kl = 0, vl = 0;
      if (hit != ~0u) {
        const uint32_t r0 = bias + sm.f.rec[hit];
        header_lds(sw, r0, kl, vl);
        uint4* ka = reinterpret_cast<uint4*>(P.key_arena);
        uint4* va = reinterpret_cast<uint4*>(P.val_arena);
        for (uint32_t c = tid; c < (kl + 15) / 16; c += kThreads) ka[c] = load16_lds(sw, r0 + 6 + 16 * c);
        for (uint32_t c = tid; c < (vl + 15) / 16; c += kThreads)
          va[c] = load16_lds(sw, r0 + 6 + kl + 16 * c);
      }
      if (tid == 0) {
        *F.found = st != OKV_BLK_OK ? 0 : !listed ? -1 : hit != ~0u ? 1 : 0;
        P.key_len[0] = uint16_t(kl);
        P.val_len[0] = vl;
        *tot = Totals{hit != ~0u ? 1u : 0u, kl, vl, uint64_t(st != OKV_BLK_OK)};
      }
      OKV_POINT_STAMP(4);
      point_done(F);
      return;  // (one block)
    }
    if (st == OKV_BLK_OK && rows) {
      if (rows <= uint64_t(kFastRows)) {
        // key / value lengths of the recorded rows, exclusive prefixes (4 rows a lane)
        constexpr int kPer = kFastRows / kThreads;
        uint32_t kls[kPer], vls[kPer], ks = 0, vs = 0;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          const uint32_t i = tid * kPer + j;
          kls[j] = vls[j] = 0;
          if (i < rows) header_lds(sw, bias + sm.f.rec[i], kls[j], vls[j]);
          ks += kls[j];
          vs += vls[j];
        }
        const uint32_t ki = wave_scan_dpp(ks), vi = wave_scan_dpp(vs);
        const uint32_t wave = tid >> 6;
        if ((tid & 63) == 63) {
          s_wsum[0][wave] = ki;
          s_wsum[1][wave] = vi;
        }
        __syncthreads();
        uint32_t kx = ki - ks, vx = vi - vs;
        uint32_t ktot = 0, vtot = 0;
#pragma unroll
        for (uint32_t w = 0; w < kThreads / 64; ++w) {
          kx += w < wave ? s_wsum[0][w] : 0u;
          vx += w < wave ? s_wsum[1][w] : 0u;
          ktot += s_wsum[0][w];
          vtot += s_wsum[1][w];
        }
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          const uint32_t i = tid * kPer + j;
          if (i < rows) {
            sm.f.kpre[i] = kx;
            sm.f.vpre[i] = vx;
          }
          kx += kls[j];
          vx += vls[j];
        }
        if (tid == 0) {
          sm.f.rec[rows] = uint32_t(pend);
          sm.f.kpre[rows] = ktot;
          sm.f.vpre[rows] = vtot;
        }
        kb = ktot;
        vb = vtot;
        __syncthreads();
        OKV_POINT_STAMP(3);
        emit_fast<3>(P, sm, bias, int(rows), kb, vb, row0, kb0, vb0);
      } else {
        // more rows than the row table holds: the byte totals by a second
        // walk (the block passed its checks), then the batched row tables
        if (tid == 0) {
          uint64_t k = 0, v = 0;
          for (uint32_t q = 0; q < uint32_t(pend);) {
            uint32_t kl, vl;
            header_lds(sw, bias + q, kl, vl);
            k += kl;
            v += vl;
            q += 6 + kl + vl;
          }
          s_walk[1] = k;
          s_walk[2] = v;
        }
        __syncthreads();
        kb = s_walk[1];
        vb = s_walk[2];
        LdsSrc src{sw, bias};
        materialise<3>(src, P, sm, rows, kb, vb, row0, kb0, vb0, pend);
      }
    }
    row0 += rows;
    kb0 += round16(kb);
    vb0 += round16(vb);
    bad += st != OKV_BLK_OK;
    __syncthreads();  // the stage and the row table are reused by the next block
    OKV_POINT_STAMP(4);
  }
  if (tid == 0) {
    P.row_start[P.nblk] = row0;
    *tot = Totals{row0, kb0, vb0, bad};
  }
  point_done(F);
}

// ---------------------------------------------------------------------------
// OKV_F_INDEX_ONLY for big blocks: one lane per block re-walks the headers.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void okv_index_kernel(CopyParams P) {
  const uint32_t nbig = *P.big_count;
  for (uint32_t k = blockIdx.x * kThreads + threadIdx.x; k < nbig; k += gridDim.x * kThreads) {
    const uint32_t b = P.big_list[k];
    const BlockCount c = P.cnt[b];
    const BlockBase B = block_base(P, b, c);
    if (B.st != OKV_BLK_OK) continue;
    const uint64_t off = P.descs[b].offset;
    uint64_t p = 0;
    for (uint64_t r = 0; r < c.rows; ++r) {
      uint32_t kl, vl;
      header_global(P.seg, off + p, kl, vl);
      const uint64_t g = B.row0 + r;
      P.key_off[g] = off + p + 6;
      P.key_len[g] = uint16_t(kl);
      P.val_off[g] = off + p + 6 + kl;
      P.val_len[g] = vl;
      // (clamped to pass 1's walk end: reads stay in the block if the segment
      // changed under the decode)
      p = min<uint64_t>(p + 6 + uint64_t(kl) + uint64_t(vl), c.pend - 6);
    }
  }
}

// ---------------------------------------------------------------------------
// XXH64 of each block's BlockSize bytes (BlockStat.Hash, segment_writer.go:185).
// XXH64 has four independent accumulators, so four lanes share one block
// (lane q owns stripe word q); the merge and tail run on lane q == 0.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void okv_hash_kernel(const uint8_t* __restrict__ seg,
                                                            uint64_t seg_bytes,
                                                            const Desc* __restrict__ descs,
                                                            uint32_t nblk,
                                                            uint64_t* __restrict__ out) {
  const uint32_t gid = blockIdx.x * kThreads + threadIdx.x;
  const uint32_t b = gid >> 2, q = gid & 3;
  const bool live = b < nblk;
  Desc d = {0, 0, 0, 0};
  if (live) d = descs[b];
  const bool ok = live && d.offset < seg_bytes && seg_bytes - d.offset >= d.block_size;
  const uint8_t* p = seg + (ok ? d.offset : 0);
  const uint64_t len = ok ? d.block_size : 0;
  const uint64_t nstripe = len / 32;
  const uint64_t seed = 0;
  uint64_t acc = (q == 0) ? seed + XP1 + XP2 : (q == 1) ? seed + XP2 : (q == 2) ? seed : seed - XP1;
  const bool aligned = ((reinterpret_cast<uintptr_t>(p)) & 7) == 0;
  for (uint64_t s = 0; s < nstripe; ++s) {
    const uint8_t* w = p + s * 32 + q * 8;
    const uint64_t x = aligned ? *reinterpret_cast<const uint64_t*>(w) : ld64u(w);
    acc = xround(acc, x);
  }
  // gather the four accumulators onto lane q == 0 of the quad
  const int lane = threadIdx.x & 63;
  const uint64_t a1 = __shfl(acc, (lane & ~3) + 1, 64);
  const uint64_t a2 = __shfl(acc, (lane & ~3) + 2, 64);
  const uint64_t a3 = __shfl(acc, (lane & ~3) + 3, 64);
  if (!live || q != 0) return;
  if (!ok) {
    out[b] = 0;
    return;
  }
  uint64_t h;
  if (len >= 32) {
    const uint64_t v1 = acc, v2 = a1, v3 = a2, v4 = a3;
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = (h ^ xround(0, v1)) * XP1 + XP4;
    h = (h ^ xround(0, v2)) * XP1 + XP4;
    h = (h ^ xround(0, v3)) * XP1 + XP4;
    h = (h ^ xround(0, v4)) * XP1 + XP4;
  } else {
    h = seed + XP5;
  }
  h += len;
  const uint8_t* t = p + nstripe * 32;
  const uint8_t* end = p + len;
  while (t + 8 <= end) {
    h ^= xround(0, ld64u(t));
    h = rotl64(h, 27) * XP1 + XP4;
    t += 8;
  }
  if (t + 4 <= end) {
    const uint32_t v = uint32_t(t[0]) | (uint32_t(t[1]) << 8) | (uint32_t(t[2]) << 16) |
                       (uint32_t(t[3]) << 24);
    h ^= uint64_t(v) * XP1;
    h = rotl64(h, 23) * XP2 + XP3;
    t += 4;
  }
  while (t < end) {
    h ^= uint64_t(*t) * XP5;
    h = rotl64(h, 11) * XP1;
    ++t;
  }
  h ^= h >> 33;
  h *= XP2;
  h ^= h >> 29;
  h *= XP3;
  h ^= h >> 32;
  out[b] = h;
}

void launch_hash(hipStream_t stream, const uint8_t* seg, uint64_t seg_bytes, const Desc* descs,
                 uint32_t nblk, uint64_t* out) {
  if (!nblk) return;
  const uint64_t threads = uint64_t(nblk) * 4;
  hipLaunchKernelGGL(okv_hash_kernel, dim3(uint32_t((threads + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, stream, seg, seg_bytes, descs, nblk, out);
}

#ifdef OKV_ABLATE  // the look-back stream kernel (ablation build only)
#include "okv_decode_ablate_lb.inc"
#endif
}  // namespace okv

// ===========================================================================
// C-ABI (include/okv_sst.h)
// ===========================================================================
using namespace okv;

namespace {

int ensure_blocks(okv_ctx* ctx, uint32_t nblk) {
  const size_t n = std::max<size_t>(nblk, 1);
  if (n <= ctx->cap_blocks && ctx->d_cnt) return OKV_OK;
  const size_t ntiles = (n + kTile - 1) / kTile;
  if (ctx->d_cnt) {
    OKV_HIP(hipStreamSynchronize(ctx->stream));
    (void)hipFree(ctx->d_cnt);
    (void)hipFree(ctx->d_lp);
    (void)hipFree(ctx->d_tile_tot);
    (void)hipFree(ctx->d_tile_pre);
    (void)hipFree(ctx->d_rec);
    (void)hipFree(ctx->d_big);
  }
  if (!ctx->d_ctr) {
    OKV_HIP(hipMalloc(&ctx->d_ctr, 64));
    OKV_HIP(hipMemsetAsync(ctx->d_ctr, 0, 64, ctx->stream));
    ctx->big_slot = 0;
  }
  OKV_HIP(hipMalloc(&ctx->d_rec, n * kRCap * sizeof(uint32_t)));
  OKV_HIP(hipMalloc(&ctx->d_big, (n + 1) * sizeof(uint32_t)));
  OKV_HIP(hipMalloc(&ctx->d_cnt, n * sizeof(BlockCount)));
  OKV_HIP(hipMalloc(&ctx->d_lp, n * sizeof(Prefix)));
  OKV_HIP(hipMalloc(&ctx->d_tile_tot, (ntiles + 1) * sizeof(Prefix)));
  OKV_HIP(hipMalloc(&ctx->d_tile_pre, (ntiles + 1) * sizeof(Prefix)));
  ctx->cap_blocks = n;
  return OKV_OK;
}

// Counters kept across calls (zeroed once): the count kernel's arrival
// counter (reset by its last workgroup) and two big-block counter slots.  A
// launch uses slot big_slot and zeroes the other one, which the next launch
// uses: its previous readers (the kernels of the decode before) have completed
// by then, so no memset launch is needed per decode.
constexpr uint32_t kCtrArrive = 0, kCtrBig = 1;
uint32_t* big_counter(okv_ctx* ctx, uint32_t other = 0) {
  return ctx->d_ctr + kCtrBig + (ctx->big_slot ^ other);
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// Event slot k (0..kProfEv-1) of the current timed call, or nullptr when not
// profiling: 0 start, 1 zstd stage done, 2 pass 1 done, 3 pass 2 done, 4 end.
constexpr int kProfEv = 5;
hipEvent_t prof_event(okv_ctx* ctx, int k) {
  if (!ctx->prof) return nullptr;
  const size_t need = ctx->ev_used + kProfEv;
  while (ctx->ev.size() < need) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    ctx->ev.push_back(e);
  }
  return ctx->ev[ctx->ev_used + k];
}

void prof_mark(okv_ctx* ctx, int k) {
  hipEvent_t e = prof_event(ctx, k);
  if (e) (void)hipEventRecord(e, ctx->stream);
  if (e && k == kProfEv - 1) ctx->ev_used += kProfEv;
}

// Working inputs of passes 1-3: the segment itself, or for zstd blocks the
// decompressed bytes (okv_zstd.hip) with per-block statuses from that stage.
struct Work {
  const uint8_t* seg;
  uint64_t seg_bytes;
  const Desc* descs;
  int comp;
  const int32_t* pre;
};

int prepare(okv_ctx* ctx, const uint8_t* d_seg, uint64_t seg_bytes, const Desc* d_desc,
            uint32_t nblk, int comp, bool index_only, Work* w) {
  *w = Work{d_seg, seg_bytes, d_desc, comp, nullptr};
  ctx->z_retried = 0;
  if (comp != OKV_COMP_ZSTD || index_only || nblk == 0) return OKV_OK;
  int rc;
  if (nblk + 1 > ctx->z_cap_blocks || !ctx->z_cap_off) {
    OKV_HIP(hipStreamSynchronize(ctx->stream));
    (void)hipFree(ctx->z_cap_off);
    (void)hipFree(ctx->z_dec_len);
    (void)hipFree(ctx->z_status);
    (void)hipFree(ctx->z_desc);
    const size_t n = size_t(nblk) + 1;
    OKV_HIP(hipMalloc(&ctx->z_cap_off, n * 8));
    OKV_HIP(hipMalloc(&ctx->z_dec_len, n * 8));
    OKV_HIP(hipMalloc(&ctx->z_status, n * 4));
    OKV_HIP(hipMalloc(&ctx->z_desc, n * sizeof(Desc)));
    ctx->z_cap_blocks = n;
  }
  launch_zstd_cap(ctx->stream, d_desc, nblk, ctx->z_cap_off);
  uint64_t total = 0;
  OKV_HIP(hipMemcpyAsync(&total, ctx->z_cap_off + nblk, 8, hipMemcpyDeviceToHost, ctx->stream));
  OKV_HIP(hipStreamSynchronize(ctx->stream));
  if ((rc = grow(ctx, reinterpret_cast<void**>(&ctx->z_dec), &ctx->z_cap_dec, total + 64)))
    return rc;
  if ((rc = zstd_run(ctx, d_seg, seg_bytes, d_desc, nblk, &total))) return rc;
  launch_zstd_desc(ctx->stream, d_desc, nblk, ctx->z_cap_off, ctx->z_dec_len, ctx->z_desc);
  OKV_HIP(hipGetLastError());
  // offsets <= total < seg_bytes, so no decompressed block reads as EOF
  *w = Work{ctx->z_dec, total + 16, ctx->z_desc, OKV_COMP_NONE, ctx->z_status};
  return OKV_OK;
}

// Pass-3 workgroup width from the call's average block span (seg_bytes /
// nblk: it assumes the blocks tile the segment, which holds for whole-segment
// decodes; a caller decoding a few blocks of a large segment gets the
// 256-thread form, which is correct for any block size).
uint32_t gather_threads(const okv_ctx* ctx, const Work& w, uint32_t nblk) {
  if (ctx->gather_threads) return ctx->gather_threads;
  return nblk && w.seg_bytes / nblk <= 16384 ? 64u : 256u;
}

// Launch passes 1 and 2 on device inputs.  rt_kl: record key lengths for the
// tile pass (null: positions only); span_cap: blocks whose walk ends past it
// go to the big-block list.
int launch_plan(okv_ctx* ctx, const Work& w, uint32_t nblk, uint64_t* d_row_start,
                bool timed = false, uint16_t* rt_kl = nullptr, uint64_t span_cap = ~0ull,
                unsigned long long* span_max = nullptr) {
  int rc = ensure_blocks(ctx, nblk);
  if (rc) return rc;
  // one launch: the count walk, and the tile-total scan by its last workgroup
  // (an empty batch still runs one workgroup: it writes the zero totals)
  const uint32_t ntiles = std::max<uint32_t>(1, (nblk + kTile - 1) / kTile);
  // prefetch block lines before the chase when the segment fits in the caches
  // and blocks are small (dense headers); 64 KiB blocks touch ~5 % of their lines
  int prefetch = nblk && w.seg_bytes <= (64ull << 20) && w.seg_bytes / nblk <= 16384;
#ifdef OKV_ABLATE
  if (const char* v = getenv("OKV_COUNT_PREFETCH")) prefetch = atoi(v) && nblk;  // A/B
#endif
  hipLaunchKernelGGL(okv_count_kernel, dim3(ntiles), dim3(kThreads), 0, ctx->stream, w.seg,
                     w.seg_bytes, w.descs, nblk, w.comp, ctx->d_cnt, ctx->d_lp, ctx->d_tile_tot,
                     ctx->d_rec, rt_kl, ctx->d_big, big_counter(ctx), w.pre, prefetch, span_cap,
                     ctx->d_tile_pre, ctx->d_tot, d_row_start, ctx->d_ctr + kCtrArrive,
                     big_counter(ctx, 1), nullptr, 0u, span_max);
  OKV_HIP(hipGetLastError());
  ctx->big_slot ^= 1u;  // the launch zeroes the other slot: the next launch's counter
  if (timed) prof_mark(ctx, 2);  // (the caller marks 3: after the big-block kernel)
  return OKV_OK;
}

// Tile-pass geometry (okv_tile_kernel): tiles per block from the call's
// average block span, rounded down to 4 KiB (a segment's meta block and
// trailer add far less than that per block); blocks whose walk ends past
// tpb tiles are big blocks (okv_copy_kernel).  Index-only decodes write only
// the row index: one workgroup per block, no span limit.
struct TileGeo {
  uint32_t tpb;
  uint64_t span_cap;
};
// Tiles per block from the average block span, or from the longest walk the
// last okv_decode_plan of the same batch measured (blocks longer than the span
// go to okv_copy_kernel: with bimodal block sizes most bytes would).
TileGeo tile_geo(const okv_ctx* ctx, const Work& w, uint32_t nblk, bool index_only) {
  if (index_only || !nblk) return {1, ~0ull};
  const uint64_t kT = uint64_t(ctx->tile_kib) << 10;
  uint64_t span = (w.seg_bytes / nblk) & ~uint64_t(4095);
  if (span < 4096) span = 4096;
  const SpanHint& h = ctx->span_hint;
  if (h.nblk == nblk && h.seg == w.seg && h.descs == w.descs && h.seg_bytes == w.seg_bytes)
    span = std::max<uint64_t>(span, (h.span + 4095) & ~uint64_t(4095));
  // (the hint is consumed by the decode that uses it -- decode_device clears
  // it -- so a later batch staged into the same buffers is not sized by it)
  uint64_t tpb = std::min<uint64_t>(64, (span + kT - 1) / kT);
  while (tpb > 1 && uint64_t(nblk) * tpb >= (uint64_t(1) << 31)) tpb >>= 1;
  return {uint32_t(tpb), tpb * kT};
}

template <uint32_t kT, uint32_t kNT, bool kXcd, int kDiag>
void launch_tile_t(hipStream_t s, const CopyParams& P, uint32_t tpb, uint32_t ntile) {
  const uint32_t grid = kXcd ? ((ntile + 7u) & ~7u) : ntile;
#ifdef OKV_ABLATE
  if constexpr (kDiag == 9) {
    hipLaunchKernelGGL((okv_tile_kernel_w7<kT, kNT, kXcd>), dim3(grid), dim3(kNT), 0, s, P, tpb,
                       ntile);
    return;
  } else if constexpr (kDiag >= 32) {
    hipLaunchKernelGGL((okv_tile_kernel_skip<kT, kNT, kXcd, uint32_t(kDiag - 32)>), dim3(grid),
                       dim3(kNT), 0, s, P, tpb, ntile);
  } else {
    hipLaunchKernelGGL((okv_tile_kernel_diag<kT, kNT, kXcd, kDiag>), dim3(grid), dim3(kNT), 0, s,
                       P, tpb, ntile);
  }
#else
  static_assert(kDiag == 0, "the product library has no diagnostic arms");
  hipLaunchKernelGGL((okv_tile_kernel<kT, kNT, kXcd>), dim3(grid), dim3(kNT), 0, s, P, tpb, ntile);
#endif
}
typedef void (*TileLaunch)(hipStream_t, const CopyParams&, uint32_t, uint32_t);
struct TileForm {
  uint32_t kib, threads, diag;
  TileLaunch x, plain;
};
#define OKV_TILE_FORM(K, N, D)                                                              \
  TileForm {                                                                                \
    K, N, D, launch_tile_t<K * 1024, N, true, D>, launch_tile_t<K * 1024, N, false, D>      \
  }
#ifdef OKV_ABLATE
const TileForm kTileForms[] = {OKV_TILE_FORM(16, 256, 0), OKV_TILE_FORM(8, 256, 0),
                               OKV_TILE_FORM(32, 256, 0), OKV_TILE_FORM(16, 512, 0),
                               OKV_TILE_FORM(32, 512, 0), OKV_TILE_FORM(4, 256, 0),
                               OKV_TILE_FORM(16, 256, 1), OKV_TILE_FORM(16, 256, 2),
                               OKV_TILE_FORM(16, 256, 3), OKV_TILE_FORM(16, 256, 4),
                               OKV_TILE_FORM(16, 256, 5), OKV_TILE_FORM(16, 256, 6),
                               OKV_TILE_FORM(16, 256, 7), OKV_TILE_FORM(16, 256, 8),
                               OKV_TILE_FORM(8, 256, 8), OKV_TILE_FORM(32, 512, 8),
                               OKV_TILE_FORM(16, 256, 9), OKV_TILE_FORM(64, 1024, 0),
                               OKV_TILE_FORM(64, 512, 0),
                               // write attribution (okv_tile_kernel_skip): d32 + kSkip
                               OKV_TILE_FORM(16, 256, 32), OKV_TILE_FORM(16, 256, 33),
                               OKV_TILE_FORM(16, 256, 34), OKV_TILE_FORM(16, 256, 36),
                               OKV_TILE_FORM(16, 256, 40), OKV_TILE_FORM(16, 256, 48),
                               OKV_TILE_FORM(16, 256, 63),
                               // value cuts on 128-byte lines (tile_pass kSkip 64)
                               OKV_TILE_FORM(16, 256, 96),
                               // whole 64-byte sectors per store (tile_pass kSkip 128)
                               OKV_TILE_FORM(16, 256, 160), OKV_TILE_FORM(16, 256, 672),
                               OKV_TILE_FORM(16, 256, 928)};
const TileForm* tile_form(uint32_t kib, uint32_t threads, uint32_t diag) {
  for (const TileForm& f : kTileForms)
    if (f.kib == kib && f.threads == threads && f.diag == diag) return &f;
  return nullptr;
}
#endif
void launch_tile(okv_ctx* ctx, const CopyParams& P, const TileGeo& g) {
#ifdef OKV_ABLATE
  const TileForm* f = tile_form(ctx->tile_kib, ctx->tile_threads, ctx->tile_diag);
  (ctx->tile_xcd ? f->x : f->plain)(ctx->stream, P, g.tpb, P.nblk * g.tpb);
#else
  // the product form: 16 KiB source tiles, 256 threads, XCD-grouped, value runs
  launch_tile_t<16384, 256, true, 0>(ctx->stream, P, g.tpb, P.nblk * g.tpb);
#endif
}

int read_totals(okv_ctx* ctx, Totals* out) {
  OKV_HIP(hipMemcpyAsync(ctx->h_tot, ctx->d_tot, sizeof(Totals), hipMemcpyDeviceToHost,
                         ctx->stream));
  OKV_HIP(hipStreamSynchronize(ctx->stream));
  *out = *ctx->h_tot;
  return OKV_OK;
}

// Scratch of the single-pass small-block decode (flags zeroed once; the epoch
// tag makes every call's flags fresh).
int ensure_fused(okv_ctx* ctx, uint32_t nblk) {
  const size_t n = std::max<size_t>(nblk, 1);
  if (n <= ctx->f_cap && ctx->f_flag) return OKV_OK;
  if (ctx->f_flag) {
    OKV_HIP(hipStreamSynchronize(ctx->stream));
    (void)hipFree(ctx->f_flag);
    (void)hipFree(ctx->f_agg);
    (void)hipFree(ctx->f_incl);
  }
  // (8 bytes per block: the fused kernel's look-back words; the ablation
  // stream kernel uses the first 4 bytes per block as its flags)
  OKV_HIP(hipMalloc(&ctx->f_flag, n * sizeof(uint64_t)));
  OKV_HIP(hipMemsetAsync(ctx->f_flag, 0, n * sizeof(uint64_t), ctx->stream));
  OKV_HIP(hipMalloc(&ctx->f_agg, n * sizeof(Prefix)));
  OKV_HIP(hipMalloc(&ctx->f_incl, n * sizeof(Prefix)));
  if (!ctx->f_ctr) {
    OKV_HIP(hipMalloc(&ctx->f_ctr, 2 * sizeof(unsigned long long)));  // blocks, arrivals
    OKV_HIP(hipMemsetAsync(ctx->f_ctr, 0, 2 * sizeof(unsigned long long), ctx->stream));
    ctx->f_base = 0;
  }
  ctx->f_cap = n;
  return OKV_OK;
}

#ifdef OKV_ABLATE  // the measured alternative forms of round 4 (ablation build only)
#include "okv_decode_ablate_host.inc"
#endif

int decode_device(okv_ctx* ctx, const uint8_t* seg, uint64_t seg_bytes, const Desc* descs,
                  uint32_t nblk, int comp, okv_decode_out* o, uint32_t flags) {
  const bool index_only = flags & OKV_F_INDEX_ONLY;
  if (!o->row_start || !o->blk_status) return set_err(ctx, OKV_E_ARG, "row_start/blk_status");
  if (!aligned16(seg)) return set_err(ctx, OKV_E_ARG, "device seg must be 16-byte aligned");
  if (!index_only && (!aligned16(o->key_arena) || !aligned16(o->val_arena)))
    return set_err(ctx, OKV_E_ARG, "device arenas must be 16-byte aligned");
  prof_mark(ctx, 0);
  Work w;
  int rc = prepare(ctx, seg, seg_bytes, descs, nblk, comp, index_only, &w);
  if (rc) return rc;
  prof_mark(ctx, 1);
  // small blocks: passes 1-3 in one launch (okv_decode_fused_kernel)
  const bool fused =
      ctx->fused && nblk && nblk <= ctx->fused_max && gather_threads(ctx, w, nblk) == 64;
  // (ablation build, OKV_DECODE_STREAM=1: larger batches of small blocks in
  // the same single pass with the prefix by decoupled look-back,
  // okv_decode_stream_kernel -- measured 9.2 vs 1.38 ms per CM segment of
  // 386 K blocks: every block's look-back walks back to an inclusive frontier
  // that lags by the blocks in flight; the product runs passes 1-3)
#ifdef OKV_ABLATE
  const bool stream = ctx->stream_lb && ctx->fused && nblk > ctx->fused_max &&
                      gather_threads(ctx, w, nblk) == 64;
#else
  constexpr bool stream = false;
#endif
  // large blocks: the source-tile pass (okv_tile_kernel); value_sweep 1-7 are
  // the round-2 forms (row pass + address-ordered value sweep)
  const bool large = nblk && !fused && !stream && gather_threads(ctx, w, nblk) == 256;
  // (ablation build, OKV_DECODE_GROUP=1: small blocks past the fused batch in
  // the grouped single pass, okv_group_kernel -- measured slower than passes
  // 1-3: CM decode stage 5.9-6.8 vs 4.1 ms)
#ifdef OKV_ABLATE
  const bool group = ctx->group && nblk && !fused && !stream && !large && !index_only;
#else
  constexpr bool group = false;
#endif
#ifdef OKV_ABLATE
  // OKV_VALUE_SWEEP=9: the one-launch per-block decode (okv_block_kernel)
  // (10: the same with 512-thread workgroups; 11: diagnostic, the prefix from
  // okv_count_kernel instead of the look-back)
  const bool block = large && ctx->value_sweep >= 9 && !index_only && !w.pre;
  const bool block_diag = block && ctx->value_sweep == 11;
  const bool tile = large && !block && ctx->value_sweep >= 8;
  const bool sweep = large && !tile && !block && ctx->value_sweep && !index_only &&
                     ctx->gather_staged && o->row_cap < (uint64_t(1) << 32);
#else
  const bool tile = large;  // the product: okv_tile_kernel for every large-block decode
  constexpr bool sweep = false, block = false, block_diag = false;
#endif
  const TileGeo geo = tile ? tile_geo(ctx, w, nblk, index_only) : TileGeo{1, ~0ull};
  ctx->span_hint = SpanHint{};  // a plan's hint sizes the one decode that follows it
  uint16_t* rt_kl = nullptr;
  if (tile || sweep) {
    if ((rc = ensure_blocks(ctx, nblk)) ||
        (rc = grow(ctx, &ctx->d_hdr, &ctx->cap_hdr, size_t(nblk) * kRCap * 2)))
      return rc;
    rt_kl = static_cast<uint16_t*>(ctx->d_hdr);
  }
  if ((rc = ensure_blocks(ctx, nblk))) return rc;
  uint32_t* const big_count = big_counter(ctx);  // this decode's slot (launch_plan flips it)
#ifdef OKV_ABLATE
  const uint32_t b0 = tile && ctx->pieces ? piece_split(nblk) : 0u;
  // small blocks in pieces of ~small_piece bytes (OKV_SMALL_PIECE_MB): count
  // then gather per piece, the gather reading what the count just read
  uint32_t spn = 0;
  if (!fused && !stream && !large && !group && nblk && ctx->small_piece &&
      w.seg_bytes > ctx->small_piece)
    spn = std::max<uint32_t>(kTile, uint32_t(uint64_t(nblk) * ctx->small_piece / w.seg_bytes) &
                                        ~uint32_t(kTile - 1));
  if (spn >= nblk) spn = 0;
#endif
  // the big-block kernel (okv_copy_kernel, okv_index_kernel) runs right after
  // passes 1-2 when they are one count launch: before the chained context's
  // pass-3 wait, so with decodes in flight it runs under the other decode's
  // pass 3 (the list is empty on C1-C5: an empty launch cost 4.6 us + a
  // kernel boundary in front of each pass 3), and before the pass-3 mark, so
  // the pass-3 interval times the tile / gather kernel alone
  bool early_big = false;
  if (fused || stream || (block && !block_diag)) {
    if ((rc = ensure_fused(ctx, nblk))) return rc;
    prof_mark(ctx, 2);
    prof_mark(ctx, 3);
#ifdef OKV_ABLATE
  } else if (group) {
    if ((rc = ensure_group(ctx, (nblk + kGroup - 1) / kGroup))) return rc;
    prof_mark(ctx, 2);
    prof_mark(ctx, 3);
#endif
#ifdef OKV_ABLATE
  } else if (b0) {
    rc = launch_plan_pieces(ctx, w, nblk, b0, o->row_start, rt_kl, geo.span_cap);
    if (rc) return rc;
  } else if (spn) {  // the counts run piece by piece with the gathers below
    if (!ctx->d_ptot) OKV_HIP(hipMalloc(&ctx->d_ptot, 2 * sizeof(Totals)));
    prof_mark(ctx, 2);
    prof_mark(ctx, 3);
#endif
  } else {
    rc = launch_plan(ctx, w, nblk, o->row_start, true, rt_kl, geo.span_cap);
    if (rc) return rc;
    early_big = nblk != 0;
    if (!early_big) prof_mark(ctx, 3);
  }
  CopyParams P;
  P.seg = w.seg;
  P.seg_bytes = w.seg_bytes;
  P.descs = w.descs;
  P.nblk = nblk;
  P.comp = w.comp;
  P.index_only = index_only ? 1 : 0;
  P.rt_pos = ctx->d_rec;
  P.rt_kl = rt_kl;
  P.span_cap = geo.span_cap;
  P.big_list = ctx->d_big;
  P.big_count = big_count;
  P.cnt = ctx->d_cnt;
  P.lp = ctx->d_lp;
  P.tile_pre = ctx->d_tile_pre;
  P.row_start = o->row_start;
  P.key_base = o->key_base;
  P.val_base = o->val_base;
  P.blk_status = o->blk_status;
  P.key_off = o->key_off;
  P.key_len = o->key_len;
  P.val_off = o->val_off;
  P.val_len = o->val_len;
  P.key_arena = o->key_arena;
  P.val_arena = o->val_arena;
  P.row_cap = o->row_cap;
  P.key_cap = index_only ? 0 : o->key_cap;
  P.val_cap = index_only ? 0 : o->val_cap;
  P.vsrc = nullptr;
  P.vtile = nullptr;
  P.bchunk = nullptr;
  P.tot = ctx->d_tot;
  uint64_t sw_tiles = 0;
  if (sweep) {
    sw_tiles = (o->val_cap + kSwTile - 1) / kSwTile;
    if ((rc = grow(ctx, &ctx->d_vsrc, &ctx->cap_vsrc, std::max<uint64_t>(o->row_cap, 1) * 24 + 256)) ||
        (rc = grow(ctx, &ctx->d_vtile, &ctx->cap_vtile, (sw_tiles + 4) * 4)))
      return rc;
    // [row] u64 sources, then [row] 16-byte boundary chunks
    P.vsrc = static_cast<uint64_t*>(ctx->d_vsrc);
    P.bchunk = reinterpret_cast<uint4*>(static_cast<uint8_t*>(ctx->d_vsrc) +
                                        ((std::max<uint64_t>(o->row_cap, 1) * 8 + 255) & ~255ull));
    P.vtile = static_cast<uint32_t*>(ctx->d_vtile);
  }
  const uint32_t gt = nblk ? gather_threads(ctx, w, nblk) : 0;
  ctx->last_path = (comp ? OKV_PATH_ZSTD : 0u) |
                   (comp == OKV_COMP_ZSTD && !index_only && ctx->z_retried ? OKV_PATH_ZSTD_REGROW : 0u) |
                   (!nblk ? 0u
                    : fused ? OKV_PATH_FUSED
                    : stream ? OKV_PATH_STREAM
                    : group ? OKV_PATH_GROUP | OKV_PATH_BIG  // (ablation builds only)
                    : OKV_PATH_BIG | (tile ? OKV_PATH_TILE
                                      : sweep ? OKV_PATH_SWEEP | OKV_PATH_STAGED
                                      : gt == 256 && ctx->gather_staged && !index_only
                                          ? OKV_PATH_STAGED
                                      : gt == 64 && ctx->gather_staged ? OKV_PATH_SMALL
                                                                       : OKV_PATH_GATHER));
  const uint32_t nbig_grid = std::min<uint32_t>(nblk, 512);
  auto launch_big = [&]() {
    if (index_only)
      hipLaunchKernelGGL(okv_index_kernel, dim3((nbig_grid + kThreads - 1) / kThreads),
                         dim3(kThreads), 0, ctx->stream, P);
    else
      hipLaunchKernelGGL(okv_copy_kernel, dim3(nbig_grid), dim3(kThreads), 0, ctx->stream, P);
  };
  if (early_big) {
    launch_big();
    OKV_HIP(hipGetLastError());
    prof_mark(ctx, 3);
  }
  // okv_decode_chain: pass 3 after the chained context's last pass 3.  (A
  // shared pass-3 stream for chained contexts instead of this event wait
  // measured slower: C5 0.407 vs 0.396 ms, C3 1.465 vs 1.449 ms per step with
  // decodes in flight, profiles/r6/session/pass3_queue_ab.log.)
  if (ctx->chain && ctx->chain->p3_rec)
    OKV_HIP(hipStreamWaitEvent(ctx->stream, ctx->chain->p3_done, 0));
  if (nblk) {
    const dim3 g(ctx->gather_grid ? std::min<uint32_t>(nblk, ctx->gather_grid) : nblk);
#ifdef OKV_ABLATE
    if (block_diag) {
      hipLaunchKernelGGL((okv_block_kernel<1024, false>), dim3(nblk), dim3(1024), 0, ctx->stream, P,
                         FusedParams{});
    } else
#endif
    if (fused || stream || block) {
      FusedParams F;
      F.pre = w.pre;
      F.cnt = ctx->d_cnt;
      F.lp = ctx->d_lp;
      F.tile_pre = ctx->d_tile_pre;
      F.flag = ctx->f_flag;
      F.agg = ctx->f_agg;
      F.incl = ctx->f_incl;
      F.ctr = ctx->f_ctr;
      F.arr = ctx->f_ctr + 1;
      F.base = ctx->f_base;
      ctx->f_epoch = (ctx->f_epoch + 1) & 0x3fffffffu;
      F.epoch = ctx->f_epoch;
      F.tot = ctx->d_tot;
      F.big_zero = big_counter(ctx, 1);
#ifdef OKV_ABLATE
      if (block && ctx->value_sweep == 10)
        hipLaunchKernelGGL(okv_block_kernel<512>, dim3(nblk), dim3(512), 0, ctx->stream, P, F);
      else if (block)
        hipLaunchKernelGGL(okv_block_kernel<1024>, dim3(nblk), dim3(1024), 0, ctx->stream, P, F);
      else if (stream)
        hipLaunchKernelGGL(okv_decode_stream_kernel, dim3(nblk), dim3(64), 0, ctx->stream, P, F);
      else
#endif
        hipLaunchKernelGGL(okv_decode_fused_kernel, dim3(nblk), dim3(64), 0, ctx->stream, P, F);
      const hipError_t le = hipGetLastError();
      if (le != hipSuccess) {
        // nothing ran: the counters keep their value, so f_base must too
        return set_err(ctx, OKV_E_HIP, "okv_decode_fused_kernel launch", le);
      }
      // (the stream / block arms advance both counters by nblk once the grid
      // completes; the product fused kernel uses none)
      if (stream || block) ctx->f_base += nblk;
      if (!block) ctx->big_slot ^= 1u;  // the kernel zeroed the other slot (see big_counter)
    }
#ifdef OKV_ABLATE
    else if (group) {
      GroupParams G;
      G.pre = w.pre;
      G.cnt = ctx->d_cnt;
      G.lp = ctx->d_lp;
      G.tile_pre = ctx->d_tile_pre;
      G.flag = ctx->g_flag;
      G.agg = ctx->g_agg;
      G.incl = ctx->g_incl;
      ctx->g_epoch = (ctx->g_epoch + 1) & 0x3fffffffu;
      if (!ctx->g_epoch) ctx->g_epoch = 1;  // (a zero tag would match the zeroed flags)
      G.epoch = ctx->g_epoch;
      G.tot = ctx->d_tot;
      G.big_zero = big_counter(ctx, 1);
      hipLaunchKernelGGL(okv_group_kernel, dim3((nblk + kGroup - 1) / kGroup), dim3(kThreads), 0,
                         ctx->stream, P, G);
      OKV_HIP(hipGetLastError());
      ctx->big_slot ^= 1u;  // the kernel zeroed the other slot (see big_counter)
    }
#endif
    else if (tile) {
      if ((ctx->tile_diag >= 3 && ctx->tile_diag <= 5) || ctx->tile_diag == 7) {
        // phase probe: 8 timestamps per 256th workgroup
        const size_t n = (size_t(nblk) * geo.tpb / 256 + 1) * 64;
        if ((rc = grow(ctx, &ctx->d_vsrc, &ctx->cap_vsrc, n))) return rc;
        P.vsrc = static_cast<uint64_t*>(ctx->d_vsrc);
      }
#ifdef OKV_ABLATE
      if (b0) {  // the first piece's tile pass, then the second's after its walk
        launch_tile(ctx, piece_params(P, 0, b0), geo);
        OKV_HIP(hipStreamWaitEvent(ctx->stream, ctx->ev_piece[1], 0));
        launch_tile(ctx, piece_params(P, b0, nblk - b0), geo);
      } else
#endif
        launch_tile(ctx, P, geo);
    }
#ifdef OKV_ABLATE
    else if (sweep) {
      // per-block rows + keys (one wave per block), then the value sweep
      hipLaunchKernelGGL(okv_rows_kernel, g, dim3(64), 0, ctx->stream, P);
      if (sw_tiles) {
        SweepParams S{w.seg, w.seg_bytes, o->val_off, o->val_len, P.vsrc, P.vtile, P.bchunk,
                      o->val_arena,
                      ctx->d_tot, P.big_count, o->row_cap, o->key_cap, o->val_cap};
        if (ctx->value_sweep == 5)
          hipLaunchKernelGGL((okv_value_sweep_kernel<4, true>), dim3(uint32_t((sw_tiles + 3) / 4)),
                             dim3(256), 0, ctx->stream, S);
        else if (ctx->value_sweep == 7)
          hipLaunchKernelGGL((okv_value_sweep_kernel<3, true>), dim3(uint32_t((sw_tiles + 2) / 3)),
                             dim3(256), 0, ctx->stream, S);
        else if (ctx->value_sweep == 6)
          hipLaunchKernelGGL((okv_value_sweep_kernel<2, true>), dim3(uint32_t((sw_tiles + 1) / 2)),
                             dim3(256), 0, ctx->stream, S);
        else if (ctx->value_sweep == 4)
          hipLaunchKernelGGL(okv_value_sweep_kernel<4>, dim3(uint32_t((sw_tiles + 3) / 4)),
                             dim3(256), 0, ctx->stream, S);
        else if (ctx->value_sweep == 2)
          hipLaunchKernelGGL(okv_value_sweep_kernel<2>, dim3(uint32_t((sw_tiles + 1) / 2)),
                             dim3(256), 0, ctx->stream, S);
        else
          hipLaunchKernelGGL(okv_value_sweep_kernel<1>, dim3(uint32_t(sw_tiles)), dim3(256), 0,
                             ctx->stream, S);
      }
      // the whole pass when the sweep is unsafe on device (big blocks,
      // capacity); otherwise every workgroup returns at once (small grid)
      hipLaunchKernelGGL((okv_gather_staged_kernel<kThreads>), dim3(std::min<uint32_t>(nblk, 2048)),
                         dim3(kThreads), 0, ctx->stream, P);
    } else if (gather_threads(ctx, w, nblk) == 256 && ctx->gather_staged && !index_only) {
      hipLaunchKernelGGL((okv_gather_staged_kernel<kThreads>), g, dim3(kThreads), 0, ctx->stream, P);
    } else if (spn && ctx->gather_staged) {
      Totals* pt = static_cast<Totals*>(ctx->d_ptot);
      const Totals* base = nullptr;
      for (uint32_t p0 = 0, k = 0; p0 < nblk; p0 += spn, ++k) {
        const uint32_t n = std::min(spn, nblk - p0);
        Totals* tot = p0 + n == nblk ? ctx->d_tot : pt + (k & 1);
        launch_count_piece(ctx, w, p0, n, o->row_start, base, tot, k == 0);
        hipLaunchKernelGGL(okv_gather_small_kernel, dim3(n), dim3(64), 0, ctx->stream,
                           piece_params(P, p0, n));
        base = tot;
      }
      ctx->big_slot ^= 1u;  // the first count launch zeroed the other slot
    } else if (gather_threads(ctx, w, nblk) == 64 && ctx->gather_staged)
      hipLaunchKernelGGL(okv_gather_small_kernel, g, dim3(64), 0, ctx->stream, P);
    else if (gather_threads(ctx, w, nblk) == 64)
      hipLaunchKernelGGL(okv_gather_kernel<64>, g, dim3(64), 0, ctx->stream, P);
    else
      hipLaunchKernelGGL(okv_gather_kernel<kThreads>, g, dim3(kThreads), 0, ctx->stream, P);
#else
    else if (gather_threads(ctx, w, nblk) == 64) {
      hipLaunchKernelGGL(okv_gather_small_kernel, g, dim3(64), 0, ctx->stream, P);
    } else {
      return set_err(ctx, OKV_E_ARG, "decode path");  // unreachable: large => tile
    }
#endif
    if (!block && !early_big) launch_big();  // (the block kernel decodes every block itself)
    OKV_HIP(hipGetLastError());
  }
  if (ctx->p3_done) {
    OKV_HIP(hipEventRecord(ctx->p3_done, ctx->stream));
    ctx->p3_rec = true;
  }
  prof_mark(ctx, 4);
  if (flags & OKV_F_ASYNC) return OKV_OK;
  Totals T;
  rc = read_totals(ctx, &T);
  if (rc) return rc;
  o->n_rows = T.rows;
  o->key_bytes = index_only ? 0 : T.kb;
  o->val_bytes = index_only ? 0 : T.vb;
  o->n_bad_blocks = T.bad;
  if (T.rows > o->row_cap || (!index_only && (T.kb > o->key_cap || T.vb > o->val_cap)))
    return set_err(ctx, OKV_E_CAPACITY, "output capacity too small (totals set)");
  return OKV_OK;
}

// Host pointers: stage inputs to device scratch, decode, copy results back.
// Upper bounds of a host-mode decode's outputs from the host descriptors
// (uncompressed blocks: a block's records lie in its BlockSize bytes inside
// the segment, each >= 6 bytes; every block region pads to 16 bytes), or
// false when they do not exist (zstd: decompressed sizes) or exceed `limit`.
bool output_bounds(const uint8_t* /*seg*/, uint64_t seg_bytes, const okv_block_desc* descs,
                   uint32_t nblk, int comp, uint64_t limit, uint64_t* rows, uint64_t* bytes) {
  if (comp == OKV_COMP_ZSTD) return false;
  uint64_t r = 0, by = 0;
  for (uint32_t b = 0; b < nblk; ++b) {
    const okv_block_desc& d = descs[b];
    uint64_t span = 0;
    if (comp != OKV_COMP_LZ4 && int64_t(d.offset) >= 0 && d.offset < seg_bytes)
      span = std::min<uint64_t>(d.block_size, seg_bytes - d.offset);
    r += span / 6;
    by += span + 16;
    if (by > limit) return false;
  }
  *rows = r;
  *bytes = by;
  return true;
}

// ---- point reads (okv_point_kernel) -----------------------------------------
// A host-mode call goes through the point path when it is a few uncompressed
// (or LZ4-flagged) blocks whose readable blocks each fit the LDS stage: the
// shim's GetRow reads one block, GetRange the few its btree walks select.
constexpr uint32_t kPointMaxBlocks = 16;
constexpr uint64_t kPointMaxBytes = uint64_t(512) << 10;  // (1 MiB of 64 KiB blocks: 409 vs 309 us
// for the staged device path; 256 KiB: 111 vs 233 us, profiles/r6/session/point_batch_ab.log)

bool point_eligible(uint64_t seg_bytes, const okv_block_desc* descs, uint32_t nblk, int comp,
                    uint32_t flags) {
  if (comp == OKV_COMP_ZSTD || (flags & OKV_F_INDEX_ONLY) || nblk == 0 ||
      nblk > kPointMaxBlocks || seg_bytes > kPointMaxBytes)
    return false;
  for (uint32_t b = 0; b < nblk; ++b) {
    const Desc& d = reinterpret_cast<const Desc*>(descs)[b];
    if (comp != OKV_COMP_LZ4 && go_read_status(d, seg_bytes) == OKV_BLK_OK &&
        d.block_size > uint64_t(kStage))
      return false;
  }
  return true;
}

int grow_host(okv_ctx* ctx, uint8_t** p, size_t* cap, size_t need) {
  if (need <= *cap && *p) return OKV_OK;
  if (*p) {
    OKV_HIP(hipStreamSynchronize(ctx->stream));
    OKV_HIP(hipHostFree(*p));
    *p = nullptr;
    *cap = 0;
  }
  const size_t c = (std::max<size_t>(need, size_t(1) << 20) + 4095) & ~size_t(4095);
  OKV_HIP(hipHostMalloc(reinterpret_cast<void**>(p), c, hipHostMallocDefault));
  *cap = c;
  return OKV_OK;
}

// Wait for a point-kernel call by spinning on its completion word in the
// pinned slab (point_done), polling the stream every 1 024 spins so that a
// failed launch ends the wait; hipStreamSynchronize then reports the error.
// (A GetRow is one launch plus this wait; hipStreamSynchronize alone sleeps
// through several microseconds after the kernel's last store.)
int point_wait(okv_ctx* ctx, const volatile uint32_t* done, uint32_t seq) {
  for (uint32_t n = 1; *done != seq; ++n) {
    if ((n & 1023u) == 0 && hipStreamQuery(ctx->stream) != hipErrorNotReady) break;
    __builtin_ia32_pause();
  }
  if (*done != seq) OKV_HIP(hipStreamSynchronize(ctx->stream));
  std::atomic_thread_fence(std::memory_order_acquire);
  return OKV_OK;
}


// One launch, one synchronisation: the blocks and descriptors are copied into
// the pinned slab, the kernel reads them there and writes every output there
// (both over PCIe), and the outputs are copied into the caller's arrays.
int decode_point(okv_ctx* ctx, const uint8_t* seg, uint64_t seg_bytes, const okv_block_desc* descs,
                 uint32_t nblk, int comp, okv_decode_out* o) {
  // output bounds from the descriptors: a readable block's records lie in its
  // BlockSize bytes (>= 6 bytes each); each arena region pads to 16 bytes
  uint64_t R = 0, A = 0;
  for (uint32_t b = 0; b < nblk; ++b) {
    const Desc& d = reinterpret_cast<const Desc*>(descs)[b];
    if (comp == OKV_COMP_LZ4 || go_read_status(d, seg_bytes) != OKV_BLK_OK) continue;
    R += d.block_size / 6;
    A += round16(d.block_size);
  }
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t n1 = size_t(nblk) + 1;
  const size_t o_desc = al(seg_bytes + 64), o_rs = al(o_desc + nblk * sizeof(Desc)),
               o_kb = al(o_rs + n1 * 8), o_vb = al(o_kb + n1 * 8), o_st = al(o_vb + n1 * 8),
               o_tot = al(o_st + n1 * 4), o_ko = al(o_tot + sizeof(Totals) + 16),
               o_kl = al(o_ko + R * 8), o_vo = al(o_kl + R * 2), o_vl = al(o_vo + R * 8),
               o_ka = al(o_vl + R * 4), o_va = al(o_ka + A + 16), total = al(o_va + A + 16);
  int rc = grow_host(ctx, &ctx->h_slab, &ctx->cap_slab, total);
  if (rc) return rc;
  uint8_t* S = ctx->h_slab;
  if (seg_bytes) std::memcpy(S, seg, seg_bytes);
  std::memcpy(S + o_desc, descs, nblk * sizeof(Desc));
  CopyParams P;
  std::memset(&P, 0, sizeof(P));
  P.seg = S;
  P.seg_bytes = seg_bytes;
  P.descs = reinterpret_cast<const Desc*>(S + o_desc);
  P.nblk = nblk;
  P.comp = comp;
  P.row_start = reinterpret_cast<uint64_t*>(S + o_rs);
  P.key_base = reinterpret_cast<uint64_t*>(S + o_kb);
  P.val_base = reinterpret_cast<uint64_t*>(S + o_vb);
  P.blk_status = reinterpret_cast<int32_t*>(S + o_st);
  P.key_off = reinterpret_cast<uint64_t*>(S + o_ko);
  P.key_len = reinterpret_cast<uint16_t*>(S + o_kl);
  P.val_off = reinterpret_cast<uint64_t*>(S + o_vo);
  P.val_len = reinterpret_cast<uint32_t*>(S + o_vl);
  P.key_arena = S + o_ka;
  P.val_arena = S + o_va;
  P.row_cap = R;
  P.key_cap = A + 16;
  P.val_cap = A + 16;
  Totals* tot = reinterpret_cast<Totals*>(S + o_tot);
  ctx->last_path = OKV_PATH_POINT;
  uint32_t* done = reinterpret_cast<uint32_t*>(S + o_tot + sizeof(Totals));
  *done = 0;
  const uint32_t seq = ++ctx->point_seq ? ctx->point_seq : ++ctx->point_seq;  // (never 0)
  hipLaunchKernelGGL(okv_point_kernel<false>, dim3(1), dim3(kThreads), 0, ctx->stream, P, tot,
                     PointFind{nullptr, 0, nullptr, done, seq});
  OKV_HIP(hipGetLastError());
  if ((rc = point_wait(ctx, done, seq))) return rc;
  const Totals T = *tot;
  o->n_rows = T.rows;
  o->key_bytes = T.kb;
  o->val_bytes = T.vb;
  o->n_bad_blocks = T.bad;
  if (T.rows > o->row_cap || T.kb > o->key_cap || T.vb > o->val_cap)
    return set_err(ctx, OKV_E_CAPACITY, "output capacity too small (totals set)");
  auto out = [](void* dst, const void* src, size_t n) {
    if (dst && n) std::memcpy(dst, src, n);
  };
  out(o->row_start, P.row_start, n1 * 8);
  out(o->blk_status, P.blk_status, size_t(nblk) * 4);
  out(o->key_base, P.key_base, size_t(nblk) * 8);
  out(o->val_base, P.val_base, size_t(nblk) * 8);
  out(o->key_off, P.key_off, T.rows * 8);
  out(o->key_len, P.key_len, T.rows * 2);
  out(o->val_off, P.val_off, T.rows * 8);
  out(o->val_len, P.val_len, T.rows * 4);
  out(o->key_arena, P.key_arena, T.kb);
  out(o->val_arena, P.val_arena, T.vb);
  return OKV_OK;
}

// okv_point_get: GetRow's block step on one block in one launch (the block,
// its descriptor and the key in the pinned slab; the row, if any, back).
int point_get(okv_ctx* ctx, const uint8_t* seg, uint64_t seg_bytes, const okv_block_desc* desc,
              int comp, const uint8_t* key, uint64_t klen, okv_point_row* out) {
  out->status = OKV_BLK_OK;
  out->found = -1;
  out->key = out->val = nullptr;
  out->key_len = out->val_len = 0;
  ctx->last_path = 0;  // (OKV_PATH_POINT once the kernel is launched: okv_last_path)
  if (!ctx->point || klen > kFindKey || !point_eligible(seg_bytes, desc, 1, comp, 0))
    return OKV_OK;  // not a point-path block: the caller decodes it in full
  const Desc& d = *reinterpret_cast<const Desc*>(desc);
  const uint64_t A = go_read_status(d, seg_bytes) == OKV_BLK_OK ? round16(d.block_size) : 0;
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t o_desc = al(seg_bytes + 64), o_key = al(o_desc + sizeof(Desc)),
               o_misc = al(o_key + klen + 16), o_tot = al(o_misc + 72), o_ka = al(o_tot + 64),
               o_va = al(o_ka + A + 16), total = al(o_va + A + 16);
  int rc = grow_host(ctx, &ctx->h_slab, &ctx->cap_slab, total);
  if (rc) return rc;
  uint8_t* S = ctx->h_slab;
  if (seg_bytes) std::memcpy(S, seg, seg_bytes);
  std::memcpy(S + o_desc, desc, sizeof(Desc));
  if (klen) std::memcpy(S + o_key, key, klen);
  CopyParams P;
  std::memset(&P, 0, sizeof(P));
  P.seg = S;
  P.seg_bytes = seg_bytes;
  P.descs = reinterpret_cast<const Desc*>(S + o_desc);
  P.nblk = 1;
  P.comp = comp;
  uint64_t* misc = reinterpret_cast<uint64_t*>(S + o_misc);  // row_start[2], bases, status, lens
  P.row_start = misc;
  P.key_base = misc + 2;
  P.val_base = misc + 3;
  P.blk_status = reinterpret_cast<int32_t*>(misc + 4);
  P.key_len = reinterpret_cast<uint16_t*>(misc + 5);
  P.val_len = reinterpret_cast<uint32_t*>(misc + 6);
  int32_t* found = reinterpret_cast<int32_t*>(misc + 7);
  P.key_arena = S + o_ka;
  P.val_arena = S + o_va;
  Totals* tot = reinterpret_cast<Totals*>(S + o_tot);
  ctx->last_path = OKV_PATH_POINT;
  uint32_t* done = reinterpret_cast<uint32_t*>(misc + 8);
  *done = 0;
  const uint32_t seq = ++ctx->point_seq ? ctx->point_seq : ++ctx->point_seq;  // (never 0)
  hipLaunchKernelGGL(okv_point_kernel<true>, dim3(1), dim3(kThreads), 0, ctx->stream, P, tot,
                     PointFind{S + o_key, uint32_t(klen), found, done, seq});
  OKV_HIP(hipGetLastError());
  if ((rc = point_wait(ctx, done, seq))) return rc;
  out->status = *P.blk_status;
  out->found = *found;
  if (out->found == 1) {
    out->key = P.key_arena;
    out->key_len = *P.key_len;
    out->val = P.val_arena;
    out->val_len = *P.val_len;
  }
  return OKV_OK;
}

// Host pointers: stage inputs to device scratch, decode, copy results back.
// The device outputs are sized from the host descriptors' bounds when those
// exist (one pass-1 walk per call); otherwise from a pass-1 plan first.
int decode_host(okv_ctx* ctx, const uint8_t* seg, uint64_t seg_bytes, const okv_block_desc* descs,
                uint32_t nblk, int comp, okv_decode_out* o, uint32_t flags) {
  if (ctx->point && point_eligible(seg_bytes, descs, nblk, comp, flags))
    return decode_point(ctx, seg, seg_bytes, descs, nblk, comp, o);
  const bool index_only = flags & OKV_F_INDEX_ONLY;
  int rc = grow(ctx, reinterpret_cast<void**>(&ctx->d_seg), &ctx->cap_seg, seg_bytes + 64);
  if (rc) return rc;
  rc = grow(ctx, reinterpret_cast<void**>(&ctx->d_desc), &ctx->cap_desc,
            size_t(nblk) * sizeof(Desc) + 64);
  if (rc) return rc;
  if (seg_bytes)
    OKV_HIP(hipMemcpyAsync(ctx->d_seg, seg, seg_bytes, hipMemcpyHostToDevice, ctx->stream));
  if (nblk)
    OKV_HIP(hipMemcpyAsync(ctx->d_desc, descs, size_t(nblk) * sizeof(Desc),
                           hipMemcpyHostToDevice, ctx->stream));
  rc = ensure_blocks(ctx, nblk);
  if (rc) return rc;
  // device output layout inside one scratch allocation
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t n1 = size_t(nblk) + 1;
  size_t off_rs = 0, off_kb = al(off_rs + n1 * 8), off_vb = al(off_kb + n1 * 8),
         off_st = al(off_vb + n1 * 8), off_rows = al(off_st + n1 * 4);
  uint64_t brows = 0, bbytes = 0;
  const bool bounded = output_bounds(seg, seg_bytes, descs, nblk, comp, uint64_t(1) << 30, &brows,
                                     &bbytes);
  uint64_t R, KB, VB;  // device capacities
  if (bounded) {
    R = std::min<uint64_t>(brows, o->row_cap);
    KB = index_only ? 0 : std::min<uint64_t>(bbytes, o->key_cap);
    VB = index_only ? 0 : std::min<uint64_t>(bbytes, o->val_cap);
  } else {
    rc = grow(ctx, &ctx->d_out, &ctx->cap_out, off_rows + 256);
    if (rc) return rc;
    uint8_t* base = static_cast<uint8_t*>(ctx->d_out);
    Work w;
    rc = prepare(ctx, ctx->d_seg, seg_bytes, ctx->d_desc, nblk, comp, index_only, &w);
    if (rc) return rc;
    rc = launch_plan(ctx, w, nblk, reinterpret_cast<uint64_t*>(base + off_rs));
    if (rc) return rc;
    Totals T;
    rc = read_totals(ctx, &T);
    if (rc) return rc;
    o->n_rows = T.rows;
    o->key_bytes = index_only ? 0 : T.kb;
    o->val_bytes = index_only ? 0 : T.vb;
    o->n_bad_blocks = T.bad;
    if (T.rows > o->row_cap || (!index_only && (T.kb > o->key_cap || T.vb > o->val_cap)))
      return set_err(ctx, OKV_E_CAPACITY, "output capacity too small (totals set)");
    R = T.rows;
    KB = index_only ? 0 : T.kb;
    VB = index_only ? 0 : T.vb;
  }
  size_t off_ko = al(off_rows), off_kl = al(off_ko + R * 8), off_vo = al(off_kl + R * 2),
         off_vl = al(off_vo + R * 8), off_ka = al(off_vl + R * 4), off_va = al(off_ka + KB),
         total = al(off_va + VB) + 256;
  // grow (keeps nothing: plan results live in ctx scratch, row_start[nblk] is rewritten)
  rc = grow(ctx, &ctx->d_out, &ctx->cap_out, total);
  if (rc) return rc;
  uint8_t* base = static_cast<uint8_t*>(ctx->d_out);
  okv_decode_out d = *o;
  d.row_start = reinterpret_cast<uint64_t*>(base + off_rs);
  d.key_base = reinterpret_cast<uint64_t*>(base + off_kb);
  d.val_base = reinterpret_cast<uint64_t*>(base + off_vb);
  d.blk_status = reinterpret_cast<int32_t*>(base + off_st);
  d.key_off = reinterpret_cast<uint64_t*>(base + off_ko);
  d.key_len = reinterpret_cast<uint16_t*>(base + off_kl);
  d.val_off = reinterpret_cast<uint64_t*>(base + off_vo);
  d.val_len = reinterpret_cast<uint32_t*>(base + off_vl);
  d.key_arena = index_only ? nullptr : base + off_ka;
  d.val_arena = index_only ? nullptr : base + off_va;
  d.row_cap = R;
  d.key_cap = KB;
  d.val_cap = VB;
  rc = decode_device(ctx, ctx->d_seg, seg_bytes, ctx->d_desc, nblk, comp, &d,
                     (flags & ~OKV_F_ASYNC) | OKV_F_DEVICE_PTRS);
  o->n_rows = d.n_rows;
  o->key_bytes = d.key_bytes;
  o->val_bytes = d.val_bytes;
  o->n_bad_blocks = d.n_bad_blocks;
  if (rc == OKV_E_CAPACITY) {  // the caller's capacity (a bounded decode: totals are set)
    return set_err(ctx, OKV_E_CAPACITY, "output capacity too small (totals set)");
  }
  if (rc) return rc;
  const uint64_t nR = d.n_rows, nK = index_only ? 0 : d.key_bytes, nV = index_only ? 0 : d.val_bytes;
  auto d2h = [&](void* dst, const void* src, size_t n) -> int {
    if (dst && n) OKV_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, ctx->stream));
    return OKV_OK;
  };
  if ((rc = d2h(o->row_start, d.row_start, n1 * 8))) return rc;
  if ((rc = d2h(o->blk_status, d.blk_status, size_t(nblk) * 4))) return rc;
  if (!index_only) {
    if ((rc = d2h(o->key_base, d.key_base, size_t(nblk) * 8))) return rc;
    if ((rc = d2h(o->val_base, d.val_base, size_t(nblk) * 8))) return rc;
    if ((rc = d2h(o->key_arena, d.key_arena, nK))) return rc;
    if ((rc = d2h(o->val_arena, d.val_arena, nV))) return rc;
  }
  if ((rc = d2h(o->key_off, d.key_off, nR * 8))) return rc;
  if ((rc = d2h(o->key_len, d.key_len, nR * 2))) return rc;
  if ((rc = d2h(o->val_off, d.val_off, nR * 8))) return rc;
  if ((rc = d2h(o->val_len, d.val_len, nR * 4))) return rc;
  OKV_HIP(hipStreamSynchronize(ctx->stream));
  return OKV_OK;
}

}  // namespace

extern "C" {

int okv_abi_version(void) { return OKV_ABI_VERSION; }

okv_ctx* okv_open_ex(int device, void* stream, const okv_open_opts* opts) {
  if (opts && opts->size < sizeof(okv_open_opts)) return nullptr;
  okv_ctx* ctx = okv_open_on_stream(device, stream);
  if (ctx && opts) {
    if (opts->flags & OKV_OPEN_NO_FUSED) ctx->fused = false;
    ctx->zstd_one_pass = (opts->flags & OKV_OPEN_ZSTD_ONE_PASS) != 0;
    ctx->point = (opts->flags & OKV_OPEN_NO_POINT) == 0;
  }
  return ctx;
}

okv_ctx* okv_open_on_stream(int device, void* stream) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  okv_ctx* ctx = new okv_ctx();
  ctx->device = device;
  // The fused kernel's blocks wait for the last-arriving block of their grid,
  // so every block must be resident at once: cap the batch at a quarter of
  // the device's resident capacity for it (room for other contexts' grids on
  // the same device), and at kFusedMaxBlocks.
  {
    int ncu = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, okv_decode_fused_kernel, 64, 0) !=
            hipSuccess)
      ncu = per_cu = 0;
    ctx->fused_max = std::min<uint32_t>(kFusedMaxBlocks, uint32_t(ncu) * uint32_t(per_cu) / 4);
    if (ctx->fused_max == 0) ctx->fused = false;
  }
#ifdef OKV_ABLATE
  // ablation build only: the measured alternative forms (tools/ablate*.py)
  // A/B knobs of the pass-3 launch (both bit-exact): OKV_GATHER_THREADS=64|256
  // (workgroup width), OKV_GATHER_GRID=<workgroups> (persistent grid)
  if (const char* v = getenv("OKV_GATHER_THREADS")) {
    ctx->gather_threads = uint32_t(atoi(v));
    if (ctx->gather_threads != 64 && ctx->gather_threads != 256) {
      delete ctx;
      return nullptr;
    }
  }
  if (const char* v = getenv("OKV_GATHER_GRID")) ctx->gather_grid = uint32_t(atoi(v));
  if (const char* v = getenv("OKV_DECODE_FUSED")) ctx->fused = atoi(v) != 0;
  if (const char* v = getenv("OKV_DECODE_GROUP")) ctx->group = atoi(v) != 0;
  if (const char* v = getenv("OKV_DECODE_PIECES")) ctx->pieces = atoi(v) != 0;
  if (const char* v = getenv("OKV_DECODE_STREAM")) ctx->stream_lb = atoi(v) != 0;
  if (const char* v = getenv("OKV_SMALL_PIECE_MB")) ctx->small_piece = uint64_t(atoi(v)) << 20;
  if (const char* v = getenv("OKV_GATHER_STAGED")) ctx->gather_staged = atoi(v) != 0;
  if (const char* v = getenv("OKV_VALUE_SWEEP")) {
    ctx->value_sweep = uint32_t(atoi(v));
    if (ctx->value_sweep > 11 || ctx->value_sweep == 3) {
      delete ctx;
      return nullptr;
    }
  }
  if (const char* v = getenv("OKV_TILE")) {  // <KiB>[x][w<threads>]
    ctx->tile_kib = uint32_t(atoi(v));
    ctx->tile_xcd = strchr(v, 'x') != nullptr;
    const char* w = strchr(v, 'w');
    ctx->tile_threads = w ? uint32_t(atoi(w + 1)) : 256u;
    const char* dg = strchr(v, 'd');
    ctx->tile_diag = dg ? uint32_t(atoi(dg + 1)) : 0u;
    if (!tile_form(ctx->tile_kib, ctx->tile_threads, ctx->tile_diag)) {
      delete ctx;
      return nullptr;
    }
  }
#endif
  if (stream) {
    ctx->stream = static_cast<hipStream_t>(stream);
  } else {
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
      delete ctx;
      return nullptr;
    }
    ctx->own_stream = true;
  }
  if (hipMalloc(&ctx->d_tot, sizeof(Totals)) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&ctx->h_tot), sizeof(Totals), 0) != hipSuccess ||
      hipMalloc(&ctx->d_span, sizeof(unsigned long long)) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&ctx->h_span), sizeof(unsigned long long), 0) !=
          hipSuccess) {
    okv_close(ctx);
    return nullptr;
  }
  return ctx;
}

okv_ctx* okv_open(int device) { return okv_open_on_stream(device, nullptr); }

void okv_close(okv_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  // unchain: contexts that wait on this one, and the one this one waits on
  for (okv_ctx* c : ctx->chained_by)
    if (c->chain == ctx) c->chain = nullptr;
  if (ctx->chain) {
    auto& v = ctx->chain->chained_by;
    v.erase(std::remove(v.begin(), v.end(), ctx), v.end());
  }
  (void)hipFree(ctx->d_cnt);
  (void)hipFree(ctx->d_lp);
  (void)hipFree(ctx->d_tile_tot);
  (void)hipFree(ctx->d_tile_pre);
  (void)hipFree(ctx->d_rec);
  (void)hipFree(ctx->d_big);
  (void)hipFree(ctx->d_ctr);
  if (ctx->p3_done) (void)hipEventDestroy(ctx->p3_done);
  (void)hipFree(ctx->f_flag);
  (void)hipFree(ctx->f_agg);
  (void)hipFree(ctx->f_incl);
  (void)hipFree(ctx->g_flag);
  (void)hipFree(ctx->g_agg);
  (void)hipFree(ctx->g_incl);
  (void)hipFree(ctx->f_ctr);
  (void)hipFree(ctx->d_tot);
  if (ctx->h_tot) (void)hipHostFree(ctx->h_tot);
  if (ctx->h_span) (void)hipHostFree(ctx->h_span);
  (void)hipFree(ctx->d_span);
  (void)hipFree(ctx->d_seg);
  (void)hipFree(ctx->d_desc);
  (void)hipFree(ctx->d_out);
  (void)hipFree(ctx->d_hash);
  if (ctx->h_slab) (void)hipHostFree(ctx->h_slab);
  (void)hipFree(ctx->d_vsrc);
  (void)hipFree(ctx->d_hdr);
  (void)hipFree(ctx->d_vtile);
  (void)hipFree(ctx->z_cap_off);
  (void)hipFree(ctx->z_dec_len);
  (void)hipFree(ctx->z_status);
  (void)hipFree(ctx->z_desc);
  (void)hipFree(ctx->z_dec);
  (void)hipFree(ctx->z_lit);
  (void)hipFree(ctx->z_blit);
  (void)hipFree(ctx->z_tabs);
  (void)hipFree(ctx->d_ptot);
  if (ctx->z_ev) (void)hipEventDestroy(ctx->z_ev);
  (void)hipFree(ctx->z_zb);
  (void)hipFree(ctx->z_seq_off);
  (void)hipFree(ctx->z_seqs);
  (void)hipFree(ctx->z_list);
  (void)hipFree(ctx->z_need);
  if (ctx->stream2) {
    (void)hipStreamSynchronize(ctx->stream2);
    (void)hipStreamDestroy(ctx->stream2);
  }
  for (hipEvent_t& ev : ctx->ev_piece)
    if (ev) (void)hipEventDestroy(ev);
  (void)hipFree(ctx->d_tot2);
  okv::enc_release(ctx);
  okv::merge_release(ctx);
  if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* okv_last_error(const okv_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }
void* okv_stream(const okv_ctx* ctx) { return ctx ? ctx->stream : nullptr; }

// Chained contexts are driven from one host thread (as every okv_ctx: not
// thread safe); okv_close unchains both directions, so neither context keeps
// a pointer to a closed one.
int okv_decode_chain(okv_ctx* ctx, okv_ctx* after) {
  if (!ctx || after == ctx || (after && after->device != ctx->device))
    return set_err(ctx, OKV_E_ARG, "okv_decode_chain: contexts");
  int prev = -1;
  OKV_HIP(hipGetDevice(&prev));
  for (okv_ctx* c : {ctx, after}) {
    if (c && !c->p3_done) {
      OKV_HIP(hipSetDevice(c->device));
      const hipError_t e = hipEventCreateWithFlags(&c->p3_done, hipEventDisableTiming);
      if (e != hipSuccess) {
        (void)hipSetDevice(prev);
        return set_err(ctx, OKV_E_HIP, "okv_decode_chain: event", e);
      }
    }
  }
  OKV_HIP(hipSetDevice(prev));  // the caller's current device is left as it was
  if (ctx->chain) {
    auto& v = ctx->chain->chained_by;
    v.erase(std::remove(v.begin(), v.end(), ctx), v.end());
  }
  ctx->chain = after;
  if (after) after->chained_by.push_back(ctx);
  return OKV_OK;
}

int okv_sync(okv_ctx* ctx) {
  if (!ctx) return OKV_E_ARG;
  OKV_HIP(hipStreamSynchronize(ctx->stream));
  return OKV_OK;
}

int okv_decode_plan(okv_ctx* ctx, const uint8_t* seg, uint64_t seg_bytes,
                    const okv_block_desc* descs, uint32_t nblk, int compression, uint32_t flags,
                    uint64_t* n_rows, uint64_t* key_bytes, uint64_t* val_bytes) {
  if (!ctx || (!seg && seg_bytes) || (!descs && nblk)) return set_err(ctx, OKV_E_ARG, "args");
  OKV_HIP(hipSetDevice(ctx->device));
  const uint8_t* d_seg = seg;
  const Desc* d_desc = reinterpret_cast<const Desc*>(descs);
  int rc;
  if (!(flags & OKV_F_DEVICE_PTRS)) {
    if ((rc = grow(ctx, reinterpret_cast<void**>(&ctx->d_seg), &ctx->cap_seg, seg_bytes + 64)))
      return rc;
    if ((rc = grow(ctx, reinterpret_cast<void**>(&ctx->d_desc), &ctx->cap_desc,
                   size_t(nblk) * sizeof(Desc) + 64)))
      return rc;
    if (seg_bytes)
      OKV_HIP(hipMemcpyAsync(ctx->d_seg, seg, seg_bytes, hipMemcpyHostToDevice, ctx->stream));
    if (nblk)
      OKV_HIP(hipMemcpyAsync(ctx->d_desc, descs, size_t(nblk) * sizeof(Desc),
                             hipMemcpyHostToDevice, ctx->stream));
    d_seg = ctx->d_seg;
    d_desc = ctx->d_desc;
  } else if (!aligned16(seg)) {
    return set_err(ctx, OKV_E_ARG, "device seg must be 16-byte aligned");
  }
  Work w;
  if ((rc = prepare(ctx, d_seg, seg_bytes, d_desc, nblk, compression,
                    (flags & OKV_F_INDEX_ONLY) != 0, &w)))
    return rc;
  OKV_HIP(hipMemsetAsync(ctx->d_span, 0, sizeof(unsigned long long), ctx->stream));
  if ((rc = launch_plan(ctx, w, nblk, nullptr, false, nullptr, ~0ull, ctx->d_span))) return rc;
  OKV_HIP(hipMemcpyAsync(ctx->h_span, ctx->d_span, sizeof(unsigned long long),
                         hipMemcpyDeviceToHost, ctx->stream));
  Totals T;
  if ((rc = read_totals(ctx, &T))) return rc;  // (synchronises: h_span is valid too)
  ctx->span_hint = SpanHint{w.seg, w.descs, w.seg_bytes, nblk, *ctx->h_span};
  if (n_rows) *n_rows = T.rows;
  if (key_bytes) *key_bytes = (flags & OKV_F_INDEX_ONLY) ? 0 : T.kb;
  if (val_bytes) *val_bytes = (flags & OKV_F_INDEX_ONLY) ? 0 : T.vb;
  return OKV_OK;
}

int okv_decode_blocks(okv_ctx* ctx, const uint8_t* seg, uint64_t seg_bytes,
                      const okv_block_desc* descs, uint32_t nblk, int compression,
                      okv_decode_out* out, uint32_t flags) {
  if (!ctx || !out || (!seg && seg_bytes) || (!descs && nblk))
    return set_err(ctx, OKV_E_ARG, "null argument");
  if (compression < 0 || compression > 2) return set_err(ctx, OKV_E_ARG, "compression");
  OKV_HIP(hipSetDevice(ctx->device));
  if (flags & OKV_F_DEVICE_PTRS)
    return decode_device(ctx, seg, seg_bytes, reinterpret_cast<const Desc*>(descs), nblk,
                         compression, out, flags);
  return decode_host(ctx, seg, seg_bytes, descs, nblk, compression, out, flags);
}

int okv_point_get(okv_ctx* ctx, const uint8_t* seg, uint64_t seg_bytes,
                  const okv_block_desc* desc, int compression, const uint8_t* key,
                  uint64_t key_len, okv_point_row* out) {
  if (!ctx || !out || !desc || (!seg && seg_bytes) || (!key && key_len))
    return set_err(ctx, OKV_E_ARG, "null argument");
  if (compression < 0 || compression > 2) return set_err(ctx, OKV_E_ARG, "compression");
  OKV_HIP(hipSetDevice(ctx->device));
  return point_get(ctx, seg, seg_bytes, desc, compression, key, key_len, out);
}

int okv_decode_totals(okv_ctx* ctx, okv_decode_out* out) {
  if (!ctx || !out) return OKV_E_ARG;
  Totals T;
  int rc = read_totals(ctx, &T);
  if (rc) return rc;
  out->n_rows = T.rows;
  out->key_bytes = T.kb;
  out->val_bytes = T.vb;
  out->n_bad_blocks = T.bad;
  if (T.rows > out->row_cap || T.kb > out->key_cap || T.vb > out->val_cap)
    return OKV_E_CAPACITY;
  return OKV_OK;
}

int okv_hash_blocks(okv_ctx* ctx, const uint8_t* seg, uint64_t seg_bytes,
                    const okv_block_desc* descs, uint32_t nblk, uint64_t* hashes,
                    uint32_t flags) {
  if (!ctx || !hashes || (!seg && seg_bytes) || (!descs && nblk)) return OKV_E_ARG;
  OKV_HIP(hipSetDevice(ctx->device));
  const uint8_t* d_seg = seg;
  const Desc* d_desc = reinterpret_cast<const Desc*>(descs);
  uint64_t* d_h = hashes;
  int rc;
  if (!(flags & OKV_F_DEVICE_PTRS)) {
    if ((rc = grow(ctx, reinterpret_cast<void**>(&ctx->d_seg), &ctx->cap_seg, seg_bytes + 64)))
      return rc;
    if ((rc = grow(ctx, reinterpret_cast<void**>(&ctx->d_desc), &ctx->cap_desc,
                   size_t(nblk) * sizeof(Desc) + 64)))
      return rc;
    if ((rc = grow(ctx, reinterpret_cast<void**>(&ctx->d_hash), &ctx->cap_hash,
                   size_t(nblk) * 8 + 64)))
      return rc;
    if (seg_bytes)
      OKV_HIP(hipMemcpyAsync(ctx->d_seg, seg, seg_bytes, hipMemcpyHostToDevice, ctx->stream));
    if (nblk)
      OKV_HIP(hipMemcpyAsync(ctx->d_desc, descs, size_t(nblk) * sizeof(Desc),
                             hipMemcpyHostToDevice, ctx->stream));
    d_seg = ctx->d_seg;
    d_desc = ctx->d_desc;
    d_h = ctx->d_hash;
  }
  if (nblk) {
    launch_hash(ctx->stream, d_seg, seg_bytes, d_desc, nblk, d_h);
    OKV_HIP(hipGetLastError());
  }
  if (!(flags & OKV_F_DEVICE_PTRS)) {
    if (nblk)
      OKV_HIP(hipMemcpyAsync(hashes, d_h, size_t(nblk) * 8, hipMemcpyDeviceToHost, ctx->stream));
  }
  if (!(flags & OKV_F_ASYNC)) OKV_HIP(hipStreamSynchronize(ctx->stream));
  return OKV_OK;
}

#ifdef OKV_ABLATE
// Diagnostic (tile-pass phase probe, OKV_TILE=...d3 / d7): copy the probe buffer to host.
int okv_debug_probe(okv_ctx* ctx, void* host, size_t bytes) {
  if (!ctx || !ctx->d_vsrc) return OKV_E_ARG;
  OKV_HIP(hipMemcpy(host, ctx->d_vsrc, std::min(bytes, ctx->cap_vsrc), hipMemcpyDeviceToHost));
  return OKV_OK;
}
#endif

uint32_t okv_last_path(const okv_ctx* ctx) { return ctx ? ctx->last_path : 0u; }

int okv_profile(okv_ctx* ctx, int enable) {
  if (!ctx) return OKV_E_ARG;
  OKV_HIP(hipStreamSynchronize(ctx->stream));
  ctx->prof = enable != 0;
  ctx->ev_used = 0;
  for (double& m : ctx->prof_ms) m = 0;
  ctx->prof_calls = 0;
  return OKV_OK;
}

int okv_profile_read(okv_ctx* ctx, double* ms, uint64_t* calls) {
  if (!ctx) return OKV_E_ARG;
  OKV_HIP(hipStreamSynchronize(ctx->stream));
  // intervals: [0,1] zstd stage, [1,2] pass 1, [2,3] pass 2, [3,4] pass 3
  static const int slot[4] = {3, 0, 1, 2};  // -> ms {count, scan, gather, zstd}
  for (size_t i = 0; i + kProfEv <= ctx->ev_used; i += kProfEv) {
    for (int k = 0; k < 4; ++k) {
      float t = 0.f;
      OKV_HIP(hipEventElapsedTime(&t, ctx->ev[i + k], ctx->ev[i + k + 1]));
      ctx->prof_ms[slot[k]] += t;
    }
    ctx->prof_calls++;
  }
  ctx->ev_used = 0;
  if (ms)
    for (int k = 0; k < 4; ++k) ms[k] = ctx->prof_ms[k];
  if (calls) *calls = ctx->prof_calls;
  return OKV_OK;
}

void* okv_device_alloc(okv_ctx* ctx, size_t bytes) {
  void* p = nullptr;
  if (ctx) (void)hipSetDevice(ctx->device);
  if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) return nullptr;
  return p;
}
void okv_device_free(okv_ctx* ctx, void* p) {
  if (ctx) (void)hipSetDevice(ctx->device);
  if (p) (void)hipFree(p);
}
void* okv_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 1, 0) != hipSuccess) return nullptr;
  return p;
}
void okv_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}
int okv_memcpy(okv_ctx* ctx, void* dst, const void* src, size_t bytes, int kind) {
  if (!ctx) return OKV_E_ARG;
  hipMemcpyKind k = kind == 0   ? hipMemcpyHostToDevice
                    : kind == 1 ? hipMemcpyDeviceToHost
                                : hipMemcpyDeviceToDevice;
  OKV_HIP(hipMemcpyAsync(dst, src, bytes, k, ctx->stream));
  OKV_HIP(hipStreamSynchronize(ctx->stream));
  return OKV_OK;
}

}  // extern "C"
