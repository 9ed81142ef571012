// okv_encode.hip -- MI355X (gfx950) segment encode: SegmentWriter.WriteRow x n
// followed by Close, for a batch of rows already in HBM.
//
// The reference writer (/root/reference/sst/segment_writer.go:80-328) appends
// each framed row [u16 LE klen][u32 LE vlen][key][value] to the open block and
// flushes it once its length reaches DataBlockThresholdBytes (:138-143); the
// flush pads it to (len/DataBlockSize + 1) * DataBlockSize bytes (Q2,
// :171-182), hashes the padded block with XXH64 (:185) and appends a BlockStat
// (block_stat.go:9-42).  Close writes the meta block (:284-328) and the
// 25-byte trailer (:226-276).
//
// The greedy cut is a chain: the block starting at row a ends at the first
// row b with P(b) - P(a-1) >= T (P = inclusive prefix of record sizes), and
// the next block starts at b+1.  Launches (DESIGN.md "Encode"):
//   E1 okv_enc_size_next_kernel  record sizes, 2048-row tile scans, empty-key
//                            check, and next(a) from a 256-row lookahead (E3 below
//                            only when a block is longer than that)
//   E2 okv_enc_scan_kernel   tile totals -> tile prefixes (one workgroup)
//   E3 okv_enc_next_kernel   next(a) - a for every row: 2048-row tiles stage
//                            P over the tile + 2048 rows of lookahead in LDS and
//                            merge targets P(a-1)+T against it (global
//                            galloping search past the window)
//   E4 okv_enc_jump0_kernel  per chunk of C rows and entry offset j < W (W =
//                            longest block in rows): walk next() to the chunk
//                            end -> (exit offset, blocks started)
//   E5 okv_enc_jump_kernel   pointer doubling of those tables over chunks
//   E6 okv_enc_resolve_kernel the chain's entry and block count per chunk
//   E7 okv_enc_emit_kernel   block first rows
//   E8 okv_enc_stat_kernel   OriginalSize, BlockSize, meta entry sizes + scans
//   E9 okv_enc_offset_kernel BlockStat.Offset and meta entry offsets
//   E10 okv_enc_pack_kernel  one workgroup per block: every lane assembles
//                            aligned 16-byte chunks of the padded block
//                            (header bytes synthesised, key/value bytes from
//                            two aligned loads + funnel) and stores them whole
//   E11 okv_hash_kernel      XXH64 per block (shared with the decode)
//   E12 okv_enc_meta_kernel  block index entries + meta head
// The meta block's XXH64 is one sequential hash; it runs on the host
// (okv_encode_close).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "okv_ctx.hpp"
#include "okv_kernels.hpp"
#include "okv_sst.h"

extern "C" uint64_t okv_xxh64(const void* data, size_t len, uint64_t seed);

namespace okv {

constexpr int kEItems = 8;
constexpr uint32_t kETile = kThreads * kEItems;  // rows (or blocks) per scan tile
constexpr uint32_t kLook = 2048;                 // lookahead rows staged by E3
constexpr uint32_t kPackRows = 512;              // rows per LDS batch in E10
constexpr uint64_t kNone = ~uint64_t(0);

// Per block, the pack kernel keeps the first kFkStride bytes of the block
// (u16 key length, u32 value length, then the FirstKey) for the meta kernel:
// one whole 64-byte line per block (four chunk stores of consecutive lanes;
// 48-byte entries, partial lines, cost the pack kernel 0.17 ms at C4).
constexpr uint32_t kFkStride = 64;
constexpr uint32_t kFkCap = kFkStride - 6;  // FirstKey bytes so kept

struct EncTotals {
  unsigned long long min_size;    // smallest record (6 + k + v)
  unsigned long long bad_row;     // first row with an empty key (kNone: none)
  unsigned long long wmax;        // max over rows of next(a) - a
  unsigned long long total_raw;   // P(n-1)
  unsigned long long nb;          // blocks
  unsigned long long data_bytes;  // sum of BlockSize
  unsigned long long meta_ent;    // sum of meta index entry sizes
  unsigned long long last_raw;    // OriginalSize of the last block (Q1)
  unsigned long long head;        // meta head bytes (keys, bloom, compression, count)
  unsigned long long fault;       // a chain-table invariant failed (never expected)
  unsigned long long bmax;        // largest BlockSize
  unsigned long long far;         // a block longer than the fused lookahead
  unsigned long long pad[4];
};

struct EncScratch {
  uint64_t* pl = nullptr;        // [n] tile-local inclusive prefix of record sizes
  uint32_t* nx = nullptr;        // [n] next(a) - a
  size_t cap_rows = 0;
  uint64_t* tile_tot = nullptr;  // [ntiles]
  uint64_t* tile_pre = nullptr;  // [ntiles]
  size_t cap_tiles = 0;
  uint32_t* jt = nullptr;        // [levels][nch][W] exit offsets
  uint32_t* jb = nullptr;        // [levels][nch][W] blocks started
  size_t cap_jump = 0;
  uint32_t* entry = nullptr;     // [nch]
  uint64_t* kbase = nullptr;     // [nch]
  size_t cap_chunks = 0;
  uint64_t* first = nullptr;     // [nb+1]
  Desc* desc = nullptr;          // [nb]
  uint64_t* hash = nullptr;      // [nb]
  uint64_t* bsl = nullptr;       // [nb] tile-local inclusive BlockSize scan
  uint64_t* esl = nullptr;       // [nb] tile-local inclusive meta entry size scan
  uint64_t* moff = nullptr;      // [nb] meta entry offsets (relative to the meta block)
  uint64_t* orig = nullptr;      // [nb] OriginalSize (the rows' record bytes) of each block
  uint16_t* fkl = nullptr;       // [nb] key length of each block's first row (its FirstKey)
  uint8_t* fk = nullptr;         // [nb][kFkStride] the block's first bytes (the LDS pack kernel)
  size_t cap_blocks = 0;
  uint16_t* jts = nullptr;       // [ntiles][kCutS] level-0 chain table of the tile cut
  uint16_t* jbs = nullptr;       // (exit offsets <= 256, blocks <= 2 048: 16 bits each)
  uint32_t* tentry = nullptr;    // [ntiles] the tile's entry row, blocks before it
  uint64_t* tkbase = nullptr;
  size_t cap_cut = 0;
  uint64_t* btile = nullptr;     // [4][nbtiles]: BlockSize tot/pre, entry tot/pre
  size_t cap_btiles = 0;
  // single-pass plan (okv_enc_plan_kernel): per-chunk look-back state
  uint32_t* p_flag = nullptr;    // [nch], zeroed once; tags carry p_epoch
  void* p_inc = nullptr;         // [nch] PlanChunk
  uint4* p_tab = nullptr;        // [nch][kFuseLook]
  uint32_t* p_jlim = nullptr;    // [nch]
  size_t cap_pch = 0;
  unsigned long long* p_ctr = nullptr;  // chunk claim counter (monotone across calls)
  unsigned long long p_base = 0;
  uint32_t p_epoch = 0;
  bool have_pl = false;          // pl / tile_pre hold the row prefix (E1-E2 ran)
  EncTotals* d_tot = nullptr;
  EncTotals* h_tot = nullptr;    // pinned
  // host-mode staging
  uint8_t* d_in = nullptr;
  size_t cap_in = 0;
  uint8_t* d_outseg = nullptr;
  size_t cap_outseg = 0;
  uint8_t* close_buf[2] = {nullptr, nullptr};  // pinned D2H chunks of the meta block (Close)
  hipEvent_t close_ev[2] = {nullptr, nullptr};
  // profiling (okv_encode_profile_read): cut, pack, hash, meta
  std::vector<hipEvent_t> ev;
  size_t ev_used = 0;
  double ms[4] = {0, 0, 0, 0};
  uint64_t calls = 0;
};

void enc_release(okv_ctx* ctx) {
  EncScratch* e = ctx->enc;
  if (!e) return;
  void* ps[] = {e->pl, e->nx, e->tile_tot, e->tile_pre, e->jt, e->jb, e->entry, e->kbase,
                e->first, e->desc, e->hash, e->bsl, e->esl, e->moff, e->orig, e->fkl, e->fk, e->jts,
                e->jbs, e->tentry, e->tkbase, e->btile,
                e->d_tot, e->d_in, e->d_outseg, e->p_flag, e->p_inc, e->p_tab, e->p_jlim,
                e->p_ctr};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  if (e->h_tot) (void)hipHostFree(e->h_tot);
  for (int i = 0; i < 2; ++i) {
    if (e->close_buf[i]) (void)hipHostFree(e->close_buf[i]);
    if (e->close_ev[i]) (void)hipEventDestroy(e->close_ev[i]);
  }
  for (hipEvent_t v : e->ev) (void)hipEventDestroy(v);
  delete e;
  ctx->enc = nullptr;
}

// ---------------------------------------------------------------------------
// Shared device helpers
// ---------------------------------------------------------------------------
// P(i) = sum of record sizes of rows 0..i (P(-1) = 0).
// Branch-free (the loads of index 0 stand in for P(-1)), so a caller's other
// independent loads are not held behind a divergent block's wait.
__device__ __forceinline__ uint64_t Pg(const uint64_t* __restrict__ pl,
                                       const uint64_t* __restrict__ tile_pre, int64_t i) {
  const uint64_t j = i < 0 ? 0 : uint64_t(i);
  const uint64_t v = pl[j] + tile_pre[j / kETile];
  return i < 0 ? 0 : v;
}

// v from the lane the DPP control names (id where there is none), 64 bits as
// two v_mov_dpp: a reduction or scan step without an LDS round trip.
template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ uint64_t dpp64(uint64_t v, uint64_t id) {
  const uint32_t lo = __builtin_amdgcn_update_dpp(uint32_t(id), uint32_t(v), kCtrl, kRowMask, 0xf,
                                                  false);
  const uint32_t hi = __builtin_amdgcn_update_dpp(uint32_t(id >> 32), uint32_t(v >> 32), kCtrl,
                                                  kRowMask, 0xf, false);
  return uint64_t(lo) | (uint64_t(hi) << 32);
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  return uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v)), l))) |
         (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v >> 32)), l))) << 32);
}
// Wave64 min / max (all lanes active; the result is wave-uniform): row_shr
// 1, 2, 4, 8 leave each 16-lane row's result in its lane 15.
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
  v = std::min(v, dpp64<0x111>(v, ~0ull));
  v = std::min(v, dpp64<0x112>(v, ~0ull));
  v = std::min(v, dpp64<0x114>(v, ~0ull));
  v = std::min(v, dpp64<0x118>(v, ~0ull));
  return std::min(std::min(readlane64(v, 15), readlane64(v, 31)),
                  std::min(readlane64(v, 47), readlane64(v, 63)));
}
__device__ __forceinline__ uint64_t wave_max64(uint64_t v) {
  v = std::max(v, dpp64<0x111>(v, 0));
  v = std::max(v, dpp64<0x112>(v, 0));
  v = std::max(v, dpp64<0x114>(v, 0));
  v = std::max(v, dpp64<0x118>(v, 0));
  return std::max(std::max(readlane64(v, 15), readlane64(v, 31)),
                  std::max(readlane64(v, 47), readlane64(v, 63)));
}
// Wave64 inclusive scan of a 64-bit value by DPP (wave_scan_dpp's steps).
__device__ __forceinline__ uint64_t wave_scan_dpp64(uint64_t x) {
  x += dpp64<0x111>(x, 0);
  x += dpp64<0x112>(x, 0);
  x += dpp64<0x114>(x, 0);
  x += dpp64<0x118>(x, 0);
  x += dpp64<0x142, 0xa>(x, 0);  // row_bcast:15
  x += dpp64<0x143, 0xc>(x, 0);  // row_bcast:31
  return x;
}

// Workgroup exclusive scan of one u64 per thread (kThreads threads); also
// returns the workgroup total.  `sm` holds kThreads/64 + 1 entries.
__device__ __forceinline__ uint64_t wg_excl_scan(uint64_t v, uint64_t* sm, uint64_t& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t inc = wave_scan_dpp64(v);  // (all lanes active)
  if (lane == 63) sm[wave] = inc;
  __syncthreads();
  uint64_t before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; ++w) {
    const uint64_t t = sm[w];
    before += (w < wave) ? t : 0;
    tot += t;
  }
  __syncthreads();
  total = tot;
  return before + inc - v;
}

// rotl64(x, 31) as two independent alignbit ops (the shift/or form is two deep)
__device__ __forceinline__ uint64_t rotl31(uint64_t x) {
  const uint32_t lo = uint32_t(x), hi = uint32_t(x >> 32);
  return uint64_t(__builtin_amdgcn_alignbit(lo, hi, 1)) |
         (uint64_t(__builtin_amdgcn_alignbit(hi, lo, 1)) << 32);
}
// XXH64 round with its input already multiplied by PRIME64_2 (xp = in * XP2):
// the accumulator chain is add, rotate, multiply.
__device__ __forceinline__ uint64_t xround_pre(uint64_t acc, uint64_t xp) {
  return rotl31(acc + xp) * XP1;
}

__device__ __forceinline__ uint64_t wave_sum64_u(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

__global__ void okv_enc_init_wmax_kernel(EncTotals* t) { t->wmax = 0; }

__global__ void okv_enc_init_kernel(EncTotals* t) {
  t->min_size = kNone;
  t->bad_row = kNone;
  t->wmax = 0;
  t->total_raw = 0;
  t->nb = 0;
  t->data_bytes = 0;
  t->meta_ent = 0;
  t->last_raw = 0;
  t->head = 0;
  t->fault = 0;
  t->bmax = 0;
  t->far = 0;
  t->pad[0] = 0;  // EP: per-block capacity exceeded
}

// ---------------------------------------------------------------------------
// E1 (with E3 fused): record sizes (WriteRow :121-125 frames 6 + len(key) +
// len(val) bytes), empty-key check (:89-91), tile-local prefix AND next(a).  next(a) only
// depends on differences of P, so a tile that stages the record sizes of its
// rows plus kFuseLook lookahead rows computes it without the global prefix.
// A block longer than the lookahead sets tot->far; the host then reruns E3
// (okv_enc_next_kernel) over global P for every row.
// ---------------------------------------------------------------------------
constexpr uint32_t kFuseLook = 256;
constexpr uint32_t kFuseWin = kETile + kFuseLook;  // staged rows
constexpr int kFuseItems = kFuseWin / kThreads;    // 9

__global__ __launch_bounds__(kThreads) void okv_enc_size_next_kernel(
    const uint16_t* __restrict__ key_len, const uint32_t* __restrict__ val_len, uint64_t n,
    uint64_t T, uint64_t* __restrict__ pl, uint64_t* __restrict__ tile_tot,
    uint32_t* __restrict__ nx, EncTotals* __restrict__ tot) {
  __shared__ uint64_t W[kFuseWin + 1];  // W[m] = sum of sizes of window rows [0, m)
  __shared__ uint64_t sm[kThreads / 64 + 1];
  const uint64_t cs = uint64_t(blockIdx.x) * kETile;
  const uint64_t nwin = std::min<uint64_t>(n - cs, kFuseWin);
  uint64_t mn = kNone, bad = kNone;
  uint32_t klv[kFuseItems], vlv[kFuseItems];  // (all loads in flight together)
#pragma unroll
  for (int i = 0; i < kFuseItems; ++i) {
    const uint64_t r = cs + std::min<uint64_t>(i * kThreads + threadIdx.x, nwin - 1);
    klv[i] = key_len[r];
    vlv[i] = val_len[r];
  }
#pragma unroll
  for (int i = 0; i < kFuseItems; ++i) {  // coalesced loads
    const uint32_t j = i * kThreads + threadIdx.x;
    uint64_t sz = 0;
    if (j < nwin) {
      const uint64_t r = cs + j;
      const uint32_t kl = klv[i];
      sz = 6u + uint64_t(kl) + uint64_t(vlv[i]);
      if (j < kETile) {
        if (kl == 0 && r < bad) bad = r;
        mn = sz < mn ? sz : mn;
      }
    }
    W[j + 1] = sz;
  }
  __syncthreads();
  uint64_t loc[kFuseItems], sum = 0;
#pragma unroll
  for (int i = 0; i < kFuseItems; ++i) {
    sum += W[1 + threadIdx.x * kFuseItems + i];
    loc[i] = sum;
  }
  uint64_t total;
  const uint64_t ex = wg_excl_scan(sum, sm, total);
#pragma unroll
  for (int i = 0; i < kFuseItems; ++i) W[1 + threadIdx.x * kFuseItems + i] = ex + loc[i];
  if (threadIdx.x == 0) W[0] = 0;
  __syncthreads();
  const uint32_t rows = uint32_t(std::min<uint64_t>(n - cs, kETile));
  for (int i = 0; i < kEItems; ++i) {  // tile-local inclusive prefix, coalesced stores
    const uint32_t j = i * kThreads + threadIdx.x;
    if (j < rows) pl[cs + j] = W[j + 1];
  }
  if (threadIdx.x == 0) tile_tot[blockIdx.x] = W[rows];
  // next(a): first m > a - cs with W[m] >= W[a - cs] + T  (b = cs + m - 1)
  const uint32_t M = uint32_t(nwin) + 1;
  const bool complete = cs + nwin == n;
  const uint32_t a0 = threadIdx.x * kEItems;
  uint64_t wmax = 0;
  bool far = false;
  uint32_t mb = 0;
  uint32_t dv[kEItems];
#pragma unroll
  for (int i = 0; i < kEItems; ++i) dv[i] = 0;
  for (int i = 0; i < kEItems; ++i) {
    const uint32_t ar = a0 + i;
    if (ar >= rows) break;
    const uint64_t target = W[ar] + T;
    if (i == 0) {
      uint32_t L = ar + 1, H = M;
      while (L < H) {
        const uint32_t m = (L + H) >> 1;
        if (W[m] >= target)
          H = m;
        else
          L = m + 1;
      }
      mb = L;
    } else {
      mb = std::max(mb, ar + 1);
      while (mb < M && W[mb] < target) ++mb;
    }
    uint64_t next;
    if (mb < M)
      next = cs + mb;
    else if (complete)
      next = n;
    else {
      far = true;
      next = cs + ar + 1;
    }
    const uint64_t d = next - (cs + ar);
    dv[i] = uint32_t(d);
    wmax = d > wmax ? d : wmax;
  }
  if (cs + a0 + kEItems <= n) {
    uint4* q = reinterpret_cast<uint4*>(nx + cs + a0);
    q[0] = make_uint4(dv[0], dv[1], dv[2], dv[3]);
    q[1] = make_uint4(dv[4], dv[5], dv[6], dv[7]);
  } else {
    for (int i = 0; i < kEItems; ++i)
      if (cs + a0 + i < n) nx[cs + a0 + i] = dv[i];
  }
  mn = wave_min64(mn);
  bad = wave_min64(bad);
  wmax = wave_max64(wmax);
  const bool anyfar = __any(far);
  if ((threadIdx.x & 63) == 0) {
    if (mn < __atomic_load_n(&tot->min_size, __ATOMIC_RELAXED))
      atomicMin(&tot->min_size, (unsigned long long)mn);
    if (bad != kNone) atomicMin(&tot->bad_row, (unsigned long long)bad);
    if (wmax > __atomic_load_n(&tot->wmax, __ATOMIC_RELAXED))
      atomicMax(&tot->wmax, (unsigned long long)wmax);
    if (anyfar) atomicOr(&tot->far, 1ull);
  }
}

// ---------------------------------------------------------------------------
// E2: one workgroup of 1024 threads: exclusive scan of n u64 values.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void okv_enc_scan_kernel(const uint64_t* __restrict__ in,
                                                            uint64_t n,
                                                            uint64_t* __restrict__ out,
                                                            unsigned long long* __restrict__ total) {
  __shared__ uint64_t sm[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t carry = 0;
  for (uint64_t b = 0; b < n; b += 1024) {
    const uint64_t i = b + threadIdx.x;
    const uint64_t v = i < n ? in[i] : 0;
    const uint64_t inc = wave_incl_scan(v, lane);
    if (lane == 63) sm[wave] = inc;
    __syncthreads();
    uint64_t before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      const uint64_t t = sm[w];
      before += (w < wave) ? t : 0;
      tot += t;
    }
    if (i < n) out[i] = carry + before + inc - v;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0 && total) *total = carry;
}

// The sum of n u64 values (one workgroup; loads unrolled so they overlap --
// okv_enc_scan_kernel's carried chunks took 88 us over C4's 48 828 tiles).
__global__ __launch_bounds__(1024) void okv_enc_sum_kernel(const uint64_t* __restrict__ in,
                                                           uint64_t n,
                                                           unsigned long long* __restrict__ total) {
  __shared__ uint64_t sm[16];
  uint64_t acc = 0;
  for (uint64_t b = 0; b < n; b += 8 * 1024) {
    uint64_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint64_t i = b + u * 1024 + threadIdx.x;
      v[u] = i < n ? in[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  acc = wave_sum64_u(acc);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += sm[w];
    *total = t;
  }
}

// ---------------------------------------------------------------------------
// E3: next(a) = 1 + min{b >= a : P(b) >= P(a-1) + T}, or n if none
// (WriteRow's `blockBuffer.Len() >= DataBlockThresholdBytes`, :138).
// ---------------------------------------------------------------------------
__device__ uint64_t next_far(const uint64_t* __restrict__ pl, const uint64_t* __restrict__ tp,
                             uint64_t n, uint64_t lo, uint64_t target) {
  // all rows < lo have P < target; galloping then binary search on HBM
  uint64_t step = 1, hi;
  for (;;) {
    hi = lo + step - 1;
    if (hi >= n) {
      hi = n;
      break;
    }
    if (Pg(pl, tp, int64_t(hi)) >= target) break;
    lo = hi + 1;
    step <<= 1;
  }
  uint64_t L = lo, H = hi;
  while (L < H) {
    const uint64_t m = L + (H - L) / 2;
    if (Pg(pl, tp, int64_t(m)) >= target)
      H = m;
    else
      L = m + 1;
  }
  return L >= n ? n : L + 1;
}

__global__ __launch_bounds__(kThreads) void okv_enc_next_kernel(
    const uint64_t* __restrict__ pl, const uint64_t* __restrict__ tp, uint64_t n, uint64_t T,
    uint32_t* __restrict__ nx, EncTotals* __restrict__ tot) {
  __shared__ uint64_t W[kETile + kLook + 1];
  const uint64_t cs = uint64_t(blockIdx.x) * kETile;
  // a block holds at most ceil(T / smallest record) + 1 rows: stage only that
  // much lookahead.  W[m] = P(cs - 1 + m), m < M
  const uint64_t msz = std::max<uint64_t>(tot->min_size, 1);
  const uint64_t look = std::min<uint64_t>(kLook, T / msz + 2);
  const uint64_t M = std::min<uint64_t>(n - cs + 1, kETile + look + 1);
  for (uint32_t m = threadIdx.x; m < M; m += kThreads) W[m] = Pg(pl, tp, int64_t(cs + m) - 1);
  __syncthreads();
  const bool complete = cs - 1 + M == n;  // the window reaches the last row
  const uint32_t a0 = threadIdx.x * kEItems;  // tile-relative first row
  uint64_t wmax = 0;
  uint32_t mb = 0;
  uint32_t dv[kEItems];
#pragma unroll
  for (int i = 0; i < kEItems; ++i) dv[i] = 0;
  for (int i = 0; i < kEItems; ++i) {
    const uint32_t ar = a0 + i;
    if (cs + ar >= n) break;
    const uint64_t target = W[ar] + T;
    uint64_t next;
    if (i == 0) {  // binary search in W[ar+1, M)
      uint32_t L = ar + 1, H = uint32_t(M);
      while (L < H) {
        const uint32_t m = (L + H) >> 1;
        if (W[m] >= target)
          H = m;
        else
          L = m + 1;
      }
      mb = L;
    } else {  // targets only grow: advance linearly
      mb = std::max(mb, ar + 1);
      while (mb < M && W[mb] < target) ++mb;
    }
    if (mb < M)
      next = cs + mb;  // b = cs - 1 + mb, next = b + 1
    else if (complete)
      next = n;
    else
      next = next_far(pl, tp, n, cs - 1 + M, target);
    const uint64_t d = next - (cs + ar);
    dv[i] = uint32_t(d);
    wmax = d > wmax ? d : wmax;
  }
  if (cs + a0 + kEItems <= n) {  // 32 contiguous bytes per lane
    uint4* q = reinterpret_cast<uint4*>(nx + cs + a0);
    q[0] = make_uint4(dv[0], dv[1], dv[2], dv[3]);
    q[1] = make_uint4(dv[4], dv[5], dv[6], dv[7]);
  } else {
    for (int i = 0; i < kEItems; ++i)
      if (cs + a0 + i < n) nx[cs + a0 + i] = dv[i];
  }
  wmax = wave_max64(wmax);
  if ((threadIdx.x & 63) == 0 && wmax > __atomic_load_n(&tot->wmax, __ATOMIC_RELAXED))
    atomicMax(&tot->wmax, (unsigned long long)wmax);
}

// ---------------------------------------------------------------------------
// E4-E7: the block-start chain.  Chunk c = rows [cC, cC + C), C >= W, so a
// chain leaving chunk c enters chunk c+1 at offset < W.  Level-k tables give,
// for entry offset j of chunk c, the entry offset after 2^k chunks and the
// number of blocks started on the way.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void okv_enc_jump0_kernel(const uint32_t* __restrict__ nx,
                                                                 uint64_t n, uint64_t C,
                                                                 uint32_t W, uint64_t nch,
                                                                 uint32_t* __restrict__ jt,
                                                                 uint32_t* __restrict__ jb) {
  const uint64_t gid = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  const uint64_t c = gid / W, j = gid % W;
  if (c >= nch) return;
  const uint64_t ce = std::min<uint64_t>(n, (c + 1) * C);
  uint64_t pos = c * C + j;
  uint32_t cnt = 0;
  while (pos < ce) {
    ++cnt;
    pos += nx[pos];
  }
  jt[gid] = uint32_t(pos - ce);
  jb[gid] = cnt;
}

__global__ __launch_bounds__(kThreads) void okv_enc_jump_kernel(
    const uint32_t* __restrict__ jt0, const uint32_t* __restrict__ jb0, uint32_t* __restrict__ jt1,
    uint32_t* __restrict__ jb1, uint32_t W, uint64_t nch, uint64_t h, EncTotals* tot) {
  // (the tables hold nch * W < 2^32 entries: 32-bit index arithmetic -- a
  // 64-bit division by W was most of this kernel's instructions)
  const uint32_t gid = blockIdx.x * kThreads + threadIdx.x;
  const uint64_t c = gid / W;
  if (c >= nch) return;
  uint32_t e = jt0[gid];
  const uint32_t b = jb0[gid];
  if (e >= W) {  // exits land below W by construction (C >= W); guard the gather
    tot->fault = 1;
    e = W - 1;
  }
  if (c + h < nch) {
    const uint32_t g2 = uint32_t(c + h) * W + e;
    jt1[gid] = jt0[g2];
    jb1[gid] = b + jb0[g2];
  } else {
    jt1[gid] = e;
    jb1[gid] = b;
  }
}

__global__ __launch_bounds__(kThreads) void okv_enc_resolve_kernel(
    const uint32_t* __restrict__ jt, const uint32_t* __restrict__ jb, uint32_t levels, uint32_t W,
    uint64_t nch, uint32_t* __restrict__ entry, uint64_t* __restrict__ kbase,
    EncTotals* __restrict__ tot) {
  const uint64_t c = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (c >= nch) return;
  const uint64_t lv = nch * W;
  uint64_t cur = 0, cnt = 0;
  uint32_t pos = 0;
  for (int k = int(levels) - 1; k >= 0; --k) {
    if ((c >> k) & 1) {
      const uint64_t idx = uint64_t(k) * lv + cur * W + pos;
      cnt += jb[idx];
      pos = jt[idx];
      cur += uint64_t(1) << k;
      if (pos >= W) {
        tot->fault = 1;
        pos = W - 1;
      }
    }
  }
  entry[c] = pos;
  kbase[c] = cnt;
  if (c == nch - 1) tot->nb = cnt + jb[c * W + pos];
}

// (the general path, after E3 over global P: a block longer than the fused
// lookahead; okv_enc_emit_tile_kernel is the usual one)
__global__ __launch_bounds__(kThreads) void okv_enc_emit_kernel(
    const uint32_t* __restrict__ nx, uint64_t n, uint64_t C, uint64_t nch,
    const uint32_t* __restrict__ entry, const uint64_t* __restrict__ kbase,
    uint64_t* __restrict__ first, uint64_t nb, const uint64_t* __restrict__ pl,
    const uint64_t* __restrict__ tp, const uint16_t* __restrict__ key_len,
    uint64_t* __restrict__ orig, uint16_t* __restrict__ fkl, EncTotals* __restrict__ tot) {
  const uint64_t c = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (c >= nch) return;
  const uint64_t ce = std::min<uint64_t>(n, (c + 1) * C);
  uint64_t pos = c * C + entry[c], k = kbase[c];
  while (pos < ce) {
    if (k >= nb) {
      tot->fault = 1;
      return;
    }
    const uint64_t nxt = pos + nx[pos];
    first[k] = pos;
    orig[k] = Pg(pl, tp, int64_t(nxt) - 1) - Pg(pl, tp, int64_t(pos) - 1);
    fkl[k] = key_len[pos];
    ++k;
    pos = nxt;
  }
  if (c == nch - 1) {
    if (k != nb) tot->fault = 1;
    first[nb] = n;
  }
}

// ---------------------------------------------------------------------------
// The tile cut: E1 + E3 + E4 per kETile-row tile in LDS --
// record sizes, next(a) and the tile's level-0 chain table -- and, after the
// pointer doubling (E5-E6), E7 per tile in LDS again with each block's
// OriginalSize and FirstKey length for E8.  No per-row array is written
// (round 4 wrote the record prefix and next(a), 12 B per row, and read them
// back in scattered chain walks and the stat kernel); each tile reads its
// rows' lengths (6 B per row) twice instead.  A block longer than the
// lookahead (tot->far) takes the general kernels above.
// ---------------------------------------------------------------------------
constexpr uint32_t kCutS = kFuseLook + 1;  // entry offsets into a tile: chains enter at <= kFuseLook

struct CutSmem {
  union {
    uint32_t W[kFuseWin + 1];  // W[m] = record bytes of window rows [0, m) (a window of
                               // 2^32 bytes or more: tot->far, the general kernels)
    struct {                   // okv_enc_cut_kernel, once next(a) is known
      uint32_t ex[kCutS];      // per entry: exit offset, blocks started
      uint32_t nb[kCutS];
    } c;
  };
  uint16_t nx[kETile];  // next(a) - a of the tile's rows
  uint16_t kl[kETile];  // their key lengths (okv_enc_emit_tile_kernel)
  uint64_t sm[kThreads / 64 + 1];
};
static_assert(8 * kCutS <= sizeof(uint32_t) * (kFuseWin + 1), "cut tables fit the prefix's LDS");

// The tile's window (its rows + kFuseLook lookahead rows): sizes, prefix and
// next(a) for the tile's rows into S (okv_enc_size_next_kernel's rules).
// Returns the tile's row count.
__device__ uint32_t cut_stage(const uint16_t* __restrict__ key_len,
                              const uint32_t* __restrict__ val_len, uint64_t n, uint64_t T,
                              uint64_t cs, CutSmem& S, uint64_t& mn, uint64_t& bad, uint64_t& wmax,
                              bool& far) {
  const uint64_t nwin = std::min<uint64_t>(n - cs, kFuseWin);
  mn = kNone;
  bad = kNone;
  bool wide = false;
  // coalesced loads, all issued before the first is used (clamped addresses:
  // a conditional load per item compiled to nine serial HBM round trips)
  uint32_t klv[kFuseItems], vlv[kFuseItems];
#pragma unroll
  for (int i = 0; i < kFuseItems; ++i) {
    const uint64_t r = cs + std::min<uint64_t>(i * kThreads + threadIdx.x, nwin - 1);
    klv[i] = key_len[r];
    vlv[i] = val_len[r];
  }
#pragma unroll
  for (int i = 0; i < kFuseItems; ++i) {
    const uint32_t j = i * kThreads + threadIdx.x;
    uint64_t sz = 0;
    if (j < nwin) {
      const uint64_t r = cs + j;
      const uint32_t kl = klv[i];
      sz = 6u + uint64_t(kl) + uint64_t(vlv[i]);
      if (j < kETile) {
        S.kl[j] = uint16_t(kl);
        if (kl == 0 && r < bad) bad = r;
        mn = sz < mn ? sz : mn;
      }
      wide |= sz > 0xffffffffull;
    }
    S.W[j + 1] = uint32_t(sz);
  }
  wide = __syncthreads_or(wide);
  uint64_t loc[kFuseItems], sum = 0;
#pragma unroll
  for (int i = 0; i < kFuseItems; ++i) {
    sum += S.W[1 + threadIdx.x * kFuseItems + i];
    loc[i] = sum;
  }
  uint64_t total;
  const uint64_t ex = wg_excl_scan(sum, S.sm, total);
#pragma unroll
  for (int i = 0; i < kFuseItems; ++i) S.W[1 + threadIdx.x * kFuseItems + i] = uint32_t(ex + loc[i]);
  if (threadIdx.x == 0) S.W[0] = 0;
  __syncthreads();
  const uint32_t rows = uint32_t(std::min<uint64_t>(n - cs, kETile));
  wide |= total >= 0xffffffffull;  // (so a saturated u32 target below exceeds every W)
  // next(a): first m > a - cs with W[m] >= W[a - cs] + T  (b = cs + m - 1)
  const uint32_t M = uint32_t(nwin) + 1;
  const bool complete = cs + nwin == n;
  const uint32_t a0 = threadIdx.x * kEItems;
  wmax = 0;
  far = false;
  uint32_t mb = 0;
  for (int i = 0; i < kEItems; ++i) {
    const uint32_t ar = a0 + i;
    if (ar >= rows) break;
    const uint32_t w0 = S.W[ar];
    const uint32_t target = T >= uint64_t(0xffffffffu - w0) ? 0xffffffffu : w0 + uint32_t(T);
    if (i == 0) {
      uint32_t L = ar + 1, H = M;
      while (L < H) {
        const uint32_t m = (L + H) >> 1;
        if (S.W[m] >= target)
          H = m;
        else
          L = m + 1;
      }
      mb = L;
    } else {
      mb = std::max(mb, ar + 1);
      while (mb < M && S.W[mb] < target) ++mb;
    }
    uint32_t d;
    if (mb < M)
      d = mb - ar;
    else if (complete)
      d = uint32_t(n - cs) - ar;
    else {
      far = true;
      d = 1;
    }
    S.nx[ar] = uint16_t(d);
    wmax = d > wmax ? d : wmax;
  }
  far |= wide;
  __syncthreads();
  return rows;
}

// E1 + E3 + E4: the level-0 chain table of each tile -- for every entry offset
// j < kCutS, where a chain entering at row j leaves the tile (its offset into
// the next one, <= kFuseLook) and how many blocks it starts on the way.
__global__ __launch_bounds__(kThreads) void okv_enc_cut_kernel(
    const uint16_t* __restrict__ key_len, const uint32_t* __restrict__ val_len, uint64_t n,
    uint64_t T, uint16_t* __restrict__ jts, uint16_t* __restrict__ jbs,
    uint64_t* __restrict__ tile_raw, EncTotals* __restrict__ tot) {
  __shared__ CutSmem S;
  const uint64_t cs = uint64_t(blockIdx.x) * kETile;
  uint64_t mn, bad, wmax;
  bool far;
  const uint32_t rows = cut_stage(key_len, val_len, n, T, cs, S, mn, bad, wmax, far);
  const uint32_t w_rows = S.W[rows];  // (before the entry tables overwrite W)
  __syncthreads();
  // entries 1..256, one lane each, one LDS read per block (tables jumping two
  // or four blocks per read cost more to build than the walks saved:
  // profiles/r5/session/enc_cut_dpp_jumps_ab.log); entry 0 enters the chain
  // of entry nx[0].
  // A chain enters this tile at most nx[0] rows in (the block it was in when
  // it crossed the tile start ends within the first nx[0] rows: bytes of rows
  // [cs, cs + j - 1) < T), so only those entries are walked; the others are
  // never reached and get an in-range placeholder.
  const uint32_t L0 = rows ? S.nx[0] : 1u;
  const uint32_t lim = rows ? min(L0, kCutS - 1) : 0u;
  // A tile whose blocks all have one row count L (fixed-size rows, C4) needs
  // no walks: the chain from j starts ceil((rows - j) / L) blocks here.
  bool eq = true;
  {
    const uint32_t a0 = threadIdx.x * kEItems;
    const uint32_t* n32 = reinterpret_cast<const uint32_t*>(S.nx + a0);
#pragma unroll
    for (int i = 0; i < kEItems / 2; ++i) {
      const uint32_t v = n32[i];
      if (a0 + 2 * i < rows) eq &= (v & 0xffffu) == L0;
      if (a0 + 2 * i + 1 < rows) eq &= (v >> 16) == L0;
    }
  }
  const bool uni = __syncthreads_and(eq);
  {
    const uint32_t j = threadIdx.x + 1;
    uint32_t pos = j > lim ? rows : j, cnt = 0;
    if (uni) {
      if (pos < rows) {
        cnt = (rows - pos + L0 - 1) / L0;
        pos += cnt * L0;
      }
    } else {
      while (pos < rows) {
        pos += S.nx[pos];
        ++cnt;
      }
    }
    S.c.ex[j] = j > lim ? 0u : pos - rows;
    S.c.nb[j] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t pos = 0, cnt = 0;
    if (rows) {
      pos = S.nx[0];
      cnt = 1;
      if (pos < rows && pos < kCutS) {
        cnt += S.c.nb[pos];
        pos = rows + S.c.ex[pos];
      } else {
        while (pos < rows) {
          pos += S.nx[pos];
          ++cnt;
        }
      }
    }
    S.c.ex[0] = pos - rows;
    S.c.nb[0] = cnt;
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < kCutS; j += kThreads) {
    jts[uint64_t(blockIdx.x) * kCutS + j] = uint16_t(S.c.ex[j]);
    jbs[uint64_t(blockIdx.x) * kCutS + j] = uint16_t(S.c.nb[j]);
  }
  mn = wave_min64(mn);
  bad = wave_min64(bad);
  wmax = wave_max64(wmax);
  const bool anyfar = __any(far);
  if ((threadIdx.x & 63) == 0) {
    if (mn < __atomic_load_n(&tot->min_size, __ATOMIC_RELAXED))
      atomicMin(&tot->min_size, (unsigned long long)mn);
    if (bad != kNone) atomicMin(&tot->bad_row, (unsigned long long)bad);
    if (wmax > __atomic_load_n(&tot->wmax, __ATOMIC_RELAXED))
      atomicMax(&tot->wmax, (unsigned long long)wmax);
    if (anyfar) atomicOr(&tot->far, 1ull);
  }
  // (the tiles' record bytes are summed by okv_enc_scan_kernel: one atomic add
  // per workgroup on one word cost 1.7 ms of C4's 2.1 ms cut launch)
  if (threadIdx.x == 0) tile_raw[blockIdx.x] = w_rows;
}

// The pointer doubling's level-0 table over chunks of kCutTiles tiles (W
// entries per chunk): the chunk's tiles' tables composed.  (One table per
// tile made every doubling level 4x larger: 0.69 GB of C4's side traffic.)
constexpr uint32_t kCutTiles = 4;
__global__ __launch_bounds__(kThreads) void okv_enc_compose_kernel(
    const uint16_t* __restrict__ jts, const uint16_t* __restrict__ jbs, uint64_t ntiles,
    uint64_t nch, uint32_t W, uint32_t* __restrict__ jt, uint32_t* __restrict__ jb) {
  const uint32_t gid = blockIdx.x * kThreads + threadIdx.x;  // (< nch * W < 2^32)
  const uint32_t c = gid / W, j = gid - c * W;
  if (c >= nch) return;
  uint32_t e = uint32_t(j), cnt = 0;
  const uint64_t t1 = std::min<uint64_t>(ntiles, (c + 1) * kCutTiles);
  for (uint64_t t = c * kCutTiles; t < t1; ++t) {  // (exit offsets are <= kFuseLook < kCutS)
    cnt += jbs[t * kCutS + e];
    e = jts[t * kCutS + e];
  }
  jt[gid] = e;
  jb[gid] = cnt;
}

// Each tile's entry row and the blocks before it, from its chunk's (E6) and
// the tables of the chunk's tiles before it.
__global__ __launch_bounds__(kThreads) void okv_enc_tile_entry_kernel(
    const uint16_t* __restrict__ jts, const uint16_t* __restrict__ jbs,
    const uint32_t* __restrict__ entry, const uint64_t* __restrict__ kbase, uint64_t ntiles,
    uint32_t* __restrict__ tentry, uint64_t* __restrict__ tkbase) {
  const uint64_t t = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (t >= ntiles) return;
  const uint64_t c = t / kCutTiles;
  uint32_t e = entry[c];
  uint64_t kb = kbase[c];
  for (uint64_t s = c * kCutTiles; s < t; ++s) {
    kb += jbs[s * kCutS + e];
    e = jts[s * kCutS + e];
  }
  tentry[t] = e;
  tkbase[t] = kb;
}

// E7 per tile: the chain from the tile's entry row (E6) in LDS; each block
// started here gets its first row, OriginalSize and FirstKey length.
__global__ __launch_bounds__(kThreads) void okv_enc_emit_tile_kernel(
    const uint16_t* __restrict__ key_len, const uint32_t* __restrict__ val_len, uint64_t n,
    uint64_t T, const uint32_t* __restrict__ entry, const uint64_t* __restrict__ kbase,
    uint64_t* __restrict__ first, uint64_t* __restrict__ orig, uint16_t* __restrict__ fkl,
    uint64_t nb, uint64_t ntiles, EncTotals* __restrict__ tot) {
  __shared__ CutSmem S;
  __shared__ uint16_t starts[kETile];
  __shared__ uint32_t s_m;
  const uint64_t c = blockIdx.x, cs = c * kETile;
  uint64_t mn, bad, wmax;
  bool far;
  const uint32_t rows = cut_stage(key_len, val_len, n, T, cs, S, mn, bad, wmax, far);
  // Wave 0 walks the chain from the tile's entry row, speculating on runs of
  // equal block lengths: with L = next(pos) - pos, lane j reads next() at
  // pos + j L; the lanes before the first whose block length differs (or that
  // is past the tile) are confirmed block starts -- up to 64 per round of two
  // LDS reads, one per round where every block differs.  (A four-block jump
  // table and a parallel expansion measured slower: 504 vs 370 us per C4
  // launch; so did a 64-row ballot search per block.)
  if (threadIdx.x < 64) {
    const uint32_t lane = threadIdx.x;
    uint32_t pos = entry[c], m = 0;
    while (pos < rows) {
      const uint32_t L = S.nx[pos];
      const uint32_t q = pos + lane * L;
      const bool in = q < rows;
      const uint32_t lq = S.nx[in ? q : 0u];
      const uint64_t brk = __ballot(!in || lq != L);
      const uint32_t k = brk ? uint32_t(__builtin_ctzll(brk)) : 64u;  // >= 1: lane 0 is pos
      if (lane < k) starts[m + lane] = uint16_t(q);
      m += k;
      pos += k * L;
    }
    if (lane == 0) s_m = m;
  }
  __syncthreads();
  const uint32_t m = s_m;
  const uint64_t k0 = kbase[c];
  if (k0 + m > nb) {
    if (threadIdx.x == 0) tot->fault = 1;
    return;
  }
  for (uint32_t i = threadIdx.x; i < m; i += kThreads) {
    const uint32_t a = starts[i];
    first[k0 + i] = cs + a;
    orig[k0 + i] = S.W[a + S.nx[a]] - S.W[a];
    fkl[k0 + i] = S.kl[a];
  }
  if (c == ntiles - 1 && threadIdx.x == 0) {
    if (k0 + m != nb) tot->fault = 1;
    first[nb] = n;
  }
}

// ---------------------------------------------------------------------------
// E8: per block OriginalSize (:160-163), BlockSize (Q2: len + DBS - len % DBS,
// :171-182), CompressedSize (LZ4 flag: the raw length, :165-167), meta index
// entry size (2 + len(FirstKey) + 40, block_stat.go:27-42) and tile scans.
// ---------------------------------------------------------------------------
struct StatParams {
  const uint64_t* orig;   // [nb] OriginalSize (the emit kernels)
  const uint16_t* fkl;    // [nb] FirstKey length
  uint64_t nb, D;
  uint32_t dshift;  // log2(D) when D is a power of two, else 64
  int lz4;
  Desc* desc;
  uint64_t* bsl;
  uint64_t* esl;
  uint64_t* btile_tot;
  uint64_t* etile_tot;
  EncTotals* tot;
};

__global__ __launch_bounds__(kThreads) void okv_enc_stat_kernel(StatParams P) {
  __shared__ uint64_t sm[kThreads / 64 + 1];
  const uint64_t base = uint64_t(blockIdx.x) * kETile + uint64_t(threadIdx.x) * kEItems;
  uint64_t lb[kEItems], le[kEItems];
  uint64_t sb = 0, se = 0, bmax = 0;
  uint64_t rawv[kEItems];  // loads first (clamped), so they are in flight together
  uint32_t fklv[kEItems];
#pragma unroll
  for (int i = 0; i < kEItems; ++i) {
    const uint64_t k = std::min<uint64_t>(base + i, P.nb - 1);
    rawv[i] = P.orig[k];
    fklv[i] = P.fkl[k];
  }
#pragma unroll
  for (int i = 0; i < kEItems; ++i) {
    const uint64_t k = base + i;
    if (k < P.nb) {
      const uint64_t raw = rawv[i];
      // (Q2: len + DBS - len % DBS; a power-of-two DBS -- the usual case -- by
      // shifts, else 32-bit division when both fit: a 64-bit division per
      // block was most of this kernel's instructions)
      const uint64_t bs = P.dshift < 64         ? ((raw >> P.dshift) + 1) << P.dshift
                          : (raw | P.D) >> 32   ? (raw / P.D + 1) * P.D
                                                : uint64_t(uint32_t(raw) / uint32_t(P.D) + 1) * P.D;
      const uint64_t es = 42u + fklv[i];
      Desc d;
      d.offset = 0;
      d.block_size = bs;
      d.original_size = raw;
      d.compressed_size = P.lz4 ? raw : 0;
      P.desc[k] = d;
      sb += bs;
      se += es;
      bmax = bs > bmax ? bs : bmax;
      if (k == P.nb - 1) P.tot->last_raw = raw;
    }
    lb[i] = sb;
    le[i] = se;
  }
  uint64_t tb, te;
  const uint64_t xb = wg_excl_scan(sb, sm, tb);
  const uint64_t xe = wg_excl_scan(se, sm, te);
#pragma unroll
  for (int i = 0; i < kEItems; ++i) {
    if (base + i < P.nb) {
      P.bsl[base + i] = xb + lb[i];
      P.esl[base + i] = xe + le[i];
    }
  }
  if (threadIdx.x == 0) {
    P.btile_tot[blockIdx.x] = tb;
    P.etile_tot[blockIdx.x] = te;
  }
  bmax = wave_max64(bmax);
  if ((threadIdx.x & 63) == 0 && bmax > __atomic_load_n(&P.tot->bmax, __ATOMIC_RELAXED))
    atomicMax(&P.tot->bmax, (unsigned long long)bmax);
}

// E9: Offset = running sum of BlockSize (:197-203); meta entry offsets.
__global__ __launch_bounds__(kThreads) void okv_enc_offset_kernel(
    Desc* __restrict__ desc, const uint64_t* __restrict__ bsl, const uint64_t* __restrict__ esl,
    const uint64_t* __restrict__ btile_pre, const uint64_t* __restrict__ etile_pre, uint64_t nb,
    const uint16_t* __restrict__ key_len, uint64_t n, const uint64_t* __restrict__ first,
    uint64_t* __restrict__ moff, EncTotals* __restrict__ tot, uint64_t bloom_extra) {
  const uint64_t k = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  // meta head: u16+FirstKey, u16+lastKey, bloom byte [+ u64 length + filter
  // bytes: bloom_extra], compression byte, index-type byte, u64 entry count
  // (:288-325)
  const uint64_t head = 2u + key_len[0] + 2u + key_len[n - 1] + 3u + 8u + bloom_extra;
  if (k == 0) tot->head = head;
  if (k >= nb) return;
  const uint64_t t = k / kETile;
  desc[k].offset = btile_pre[t] + bsl[k] - desc[k].block_size;
  // esl: E8's tile-inclusive prefix of entry sizes, so the exclusive one is
  // the previous block's (no second read of the block's first key length)
  moff[k] = head + etile_pre[t] + (k % kETile ? esl[k - 1] : 0u);
}

__device__ __forceinline__ void put_le(uint8_t* p, uint64_t v, int nbytes) {
  for (int i = 0; i < nbytes; ++i) p[i] = uint8_t(v >> (8 * i));
}
__device__ __forceinline__ void put_bytes(uint8_t* p, const uint8_t* s, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) p[i] = s[i];
}

#ifdef OKV_ABLATE  // the single-pass plan kernel (ablation build only, OKV_ENC_ONEPASS=1)
#include "okv_encode_ablate.inc"
#endif

// ---------------------------------------------------------------------------
// E10: pack.  One workgroup per block; lane l of a pass owns destination
// chunk q (16 bytes at Offset + 16q) and assembles it from the records that
// overlap it: header bytes synthesised from (klen, vlen), key and value bytes
// gathered from the arenas with two aligned 16-byte loads + funnel.  Chunks
// past OriginalSize are the zero padding.  Every chunk is stored whole, once.
// ---------------------------------------------------------------------------
struct PackParams {
  const uint8_t* key_arena;
  const uint64_t* key_off;
  const uint16_t* key_len;
  const uint8_t* val_arena;
  const uint64_t* val_off;
  const uint32_t* val_len;
  const uint64_t* pl;
  const uint64_t* tp;
  const uint64_t* first;
  const Desc* desc;
  uint8_t* seg;
  uint64_t* hash;  // BlockStat.Hash, written by kernels that hash in LDS
  uint8_t* meta;   // non-null: okv_enc_pack_lds_kernel also writes the blocks' meta
                   // index entries (BlockStat.toBytes, block_stat.go:27-42) here
  const uint64_t* moff;  // [nb] entry offsets within the meta block
  uint8_t* fk = nullptr;  // non-null: the LDS kernel keeps each block's first kFkStride bytes
};

struct __align__(16) PackSmem {
  uint64_t rel[kPackRows + 1];  // record start within the block
  uint64_t ko[kPackRows];
  uint64_t vo[kPackRows];
  uint32_t kl[kPackRows];
  uint32_t vl[kPackRows];
};

// Bytes [b, 16) of acc replaced by those of v (b clamped to [0, 16]).  Records
// are assembled segment by segment in increasing position, so each segment
// only has to overwrite from its own start: later segments overwrite its
// tail.  Four med3 + 64-bit shift + bfi per chunk.
__device__ __forceinline__ uint32_t suffix_mask(int32_t c) {
  c = min(max(c, 0), 4);
  return uint32_t(0xffffffffULL << (8 * c));
}
__device__ __forceinline__ uint4 replace_from(const uint4& acc, const uint4& v, int32_t b) {
  uint32_t m;
  uint4 r;
  m = suffix_mask(b);
  r.x = bsel(m, v.x, acc.x);
  m = suffix_mask(b - 4);
  r.y = bsel(m, v.y, acc.y);
  m = suffix_mask(b - 8);
  r.z = bsel(m, v.z, acc.z);
  m = suffix_mask(b - 12);
  r.w = bsel(m, v.w, acc.w);
  return r;
}

// 16 bytes whose byte j (for j in [s, e) intersected with [0, 16)) is
// src[j - s].  Only the 16-byte lines holding those bytes are loaded.
__device__ __forceinline__ uint4 seg_window(const uint8_t* src, int64_t s, int64_t e) {
  const int64_t lo = s > 0 ? s : 0;
  const int64_t hi = e < 16 ? e : 16;
  // (pointer arithmetic, not integer casts: the loads keep the arena's global
  // address space -- global_load, not flat_load, which also counts against
  // lgkmcnt and so holds up every LDS wait behind it)
  const uint8_t* v = src - s;  // window byte 0
  const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(v) & 15);
  const uint8_t* a = v - sh;
  const uint8_t* safe = v + lo - (reinterpret_cast<uintptr_t>(v + lo) & 15);
  const bool n0 = int64_t(16 - sh) > lo;
  const bool n1 = sh != 0 && hi > int64_t(16 - sh);
  const uint4 x = *reinterpret_cast<const uint4*>(n0 ? a : safe);
  const uint4 y = *reinterpret_cast<const uint4*>(n1 ? a + 16 : safe);
  return funnel32(x, y, sh);
}

// The 6 header bytes [u16 klen][u32 vlen] placed at window offset d (-5..15).
__device__ __forceinline__ uint4 header_window(uint32_t kl, uint32_t vl, int64_t d) {
  const uint4 H = make_uint4(kl | (vl << 16), vl >> 16, 0, 0);
  const uint4 Z = make_uint4(0, 0, 0, 0);
  return d > 0 ? funnel32(Z, H, uint32_t(16 - d)) : funnel32(H, Z, uint32_t(-d));
}

struct RecInfo {
  uint64_t rs;  // record start (block- or region-relative, same frame as pos)
  uint64_t ko, vo;
  uint32_t kl, vl;
};

// Destination chunk [pos, pos + 16): records i0, i0 + 1, ... (rec(i) gives
// them, valid while i < nrec) in increasing position; bytes no record covers
// are padding (zero).  i0 = the last record starting at or before pos.
template <class Rec>
__device__ __forceinline__ uint4 assemble_chunk(const PackParams& P, uint64_t pos, uint64_t i0,
                                                uint64_t nrec, Rec rec) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  int64_t last_end = 0;
  for (uint64_t i = i0; i < nrec; ++i) {
    const RecInfo r = rec(i);
    if (r.rs >= pos + 16) break;
    const int64_t hs = int64_t(r.rs) - int64_t(pos);
    const int64_t ks = hs + 6, vs = ks + int64_t(r.kl), ve = vs + int64_t(r.vl);
    if (ve <= 0) continue;  // record ends before this chunk (padding chunk)
    if (ks > 0) acc = replace_from(acc, header_window(r.kl, r.vl, hs), int32_t(hs > 0 ? hs : 0));
    if (vs > 0 && ks < 16)
      acc = replace_from(acc, seg_window(P.key_arena + r.ko, ks, vs), int32_t(ks > 0 ? ks : 0));
    if (r.vl && vs < 16)
      acc = replace_from(acc, seg_window(P.val_arena + r.vo, vs, ve), int32_t(vs > 0 ? vs : 0));
    last_end = ve;
  }
  if (last_end < 16) acc = replace_from(acc, make_uint4(0, 0, 0, 0), int32_t(last_end));
  return acc;
}

// E10, general blocks (more than kPackRows rows or larger than a region): one
// workgroup per block, rows staged kPackRows at a time; a chunk that runs into
// the next batch reads those records from HBM.
__global__ __launch_bounds__(kThreads) void okv_enc_pack_kernel(PackParams P) {
  __shared__ PackSmem sm;
  const uint64_t k = blockIdx.x;
  const Desc d = P.desc[k];
  const uint64_t r0 = P.first[k], r1 = P.first[k + 1];
  const uint64_t base = Pg(P.pl, P.tp, int64_t(r0) - 1);
  const uint64_t S = d.block_size;
  uint8_t* dst = P.seg + d.offset;
  for (uint64_t b0 = r0;; b0 += kPackRows) {
    const uint64_t b1 = std::min<uint64_t>(r1, b0 + kPackRows);
    const uint32_t nbat = uint32_t(b1 - b0);
    for (uint32_t i = threadIdx.x; i <= nbat; i += kThreads) {
      const uint64_t g = b0 + i;
      sm.rel[i] = Pg(P.pl, P.tp, int64_t(g) - 1) - base;
      if (i < nbat) {
        sm.ko[i] = P.key_off[g];
        sm.kl[i] = P.key_len[g];
        sm.vo[i] = P.val_off[g];
        sm.vl[i] = P.val_len[g];
      }
    }
    __syncthreads();
    const bool last = b1 == r1;
    const uint64_t q0 = (sm.rel[0] + 15) >> 4;
    const uint64_t q1 = last ? (S >> 4) : ((sm.rel[nbat] + 15) >> 4);
    auto rec = [&](uint64_t i) {
      RecInfo r;
      if (i < nbat) {
        r.rs = sm.rel[i];
        r.ko = sm.ko[i];
        r.vo = sm.vo[i];
        r.kl = sm.kl[i];
        r.vl = sm.vl[i];
      } else {  // the chunk runs into the next batch
        const uint64_t g = b0 + i;
        r.rs = Pg(P.pl, P.tp, int64_t(g) - 1) - base;
        r.ko = P.key_off[g];
        r.vo = P.val_off[g];
        r.kl = P.key_len[g];
        r.vl = P.val_len[g];
      }
      return r;
    };
    for (uint64_t q = q0 + threadIdx.x; q < q1; q += kThreads) {
      const uint64_t pos = q << 4;
      uint32_t lo = 0, hi = nbat;  // rel[lo] <= pos < rel[hi] (or pos in the padding)
      while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if (sm.rel[m] <= pos)
          lo = m;
        else
          hi = m;
      }
      *reinterpret_cast<uint4*>(dst + pos) = assemble_chunk(P, pos, lo, r1 - b0, rec);
    }
    if (last) break;
    __syncthreads();
  }
}

// E10, small blocks: one workgroup packs a region of G consecutive blocks
// (at most kPackRows records and kMaxChunks chunks).  Blocks start on 16-byte
// boundaries, so no chunk mixes two blocks.  A chunk -> record table built in
// LDS replaces the per-chunk search.
constexpr int kMaxRegion = 64;
constexpr uint32_t kMaxChunks = 4096;

struct __align__(16) RegionSmem {
  uint64_t out[kPackRows + 1];  // record start relative to the region; [nrow] = region end
  uint64_t ko[kPackRows];
  uint64_t vo[kPackRows];
  uint32_t kl[kPackRows];
  uint32_t vl[kPackRows];
  uint16_t qrow[kMaxChunks];    // last record starting at or before chunk q
  uint64_t bfirst[kMaxRegion + 1];
  uint64_t brel[kMaxRegion];    // block offset - region offset
  uint64_t bbase[kMaxRegion];   // P(first row - 1)
};

template <int V>  // diagnostic ablation (OKV_ENC_VARIANT): 0 product, 1 tables only,
                 // 2 tables + zero stores
__global__ __launch_bounds__(kThreads) void okv_enc_pack_region_kernel(PackParams P, uint64_t nb,
                                                                       uint32_t G) {
  __shared__ RegionSmem sm;
  const uint64_t k0 = uint64_t(blockIdx.x) * G;
  const uint32_t g = uint32_t(std::min<uint64_t>(G, nb - k0));
  const uint64_t O0 = P.desc[k0].offset;
  const Desc dl = P.desc[k0 + g - 1];
  const uint64_t nq = (dl.offset + dl.block_size - O0) >> 4;
  if (threadIdx.x <= g) {
    const uint32_t t = threadIdx.x;
    const uint64_t f = P.first[k0 + t];
    sm.bfirst[t] = f;
    if (t < g) {
      sm.brel[t] = P.desc[k0 + t].offset - O0;
      sm.bbase[t] = Pg(P.pl, P.tp, int64_t(f) - 1);
    }
  }
  __syncthreads();
  const uint64_t R0 = sm.bfirst[0];
  const uint32_t nrow = uint32_t(sm.bfirst[g] - R0);
  for (uint32_t i = threadIdx.x; i < nrow; i += kThreads) {
    const uint64_t r = R0 + i;
    uint32_t lo = 0, hi = g;  // block of row r: bfirst[lo] <= r < bfirst[hi]
    while (hi - lo > 1) {
      const uint32_t m = (lo + hi) >> 1;
      if (sm.bfirst[m] <= r)
        lo = m;
      else
        hi = m;
    }
    sm.out[i] = sm.brel[lo] + Pg(P.pl, P.tp, int64_t(r) - 1) - sm.bbase[lo];
    sm.ko[i] = P.key_off[r];
    sm.kl[i] = P.key_len[r];
    sm.vo[i] = P.val_off[r];
    sm.vl[i] = P.val_len[r];
  }
  if (threadIdx.x == 0) sm.out[nrow] = nq << 4;
  __syncthreads();
  // chunk q belongs to the record whose span [out[i], out[i+1]) holds byte 16q
  for (uint32_t i = threadIdx.x; i < nrow; i += kThreads) {
    const uint32_t qa = uint32_t((sm.out[i] + 15) >> 4), qb = uint32_t((sm.out[i + 1] + 15) >> 4);
    for (uint32_t q = qa; q < qb; ++q) sm.qrow[q] = uint16_t(i);
  }
  __syncthreads();
  auto rec = [&](uint64_t i) {
    RecInfo r;
    r.rs = sm.out[i];
    r.ko = sm.ko[i];
    r.vo = sm.vo[i];
    r.kl = sm.kl[i];
    r.vl = sm.vl[i];
    return r;
  };
  uint8_t* dst = P.seg + O0;
  if (V == 1) return;
  for (uint32_t q = threadIdx.x; q < nq; q += kThreads) {
    const uint64_t pos = uint64_t(q) << 4;
    if (V == 2)
      *reinterpret_cast<uint4*>(dst + pos) = make_uint4(sm.qrow[q], 0, 0, 0);
    else
      *reinterpret_cast<uint4*>(dst + pos) = assemble_chunk(P, pos, sm.qrow[q], nrow, rec);
  }
}

// E10, records smaller than a region: record-major assembly in LDS.  The
// region's G blocks (<= kImage bytes) are built in an LDS image: zeroed (the
// padding), then each lane ORs its records' header / key / value bytes in
// (16-byte source windows realigned to the destination, all loads of a field
// issued together), then the image is stored with aligned 16-byte stores.
// 16 KiB: 8 workgroups per CU, so one's XXH64 tail overlaps the others' copies
// (C4 pack + hash: 32 KiB 5.2 ms, 16 KiB 4.3 ms)
constexpr uint32_t kImage = 16384;
constexpr uint32_t kMetaImage = 32768;

// OR the first nbytes (<= 16; higher bytes of w must be zero) of w into the
// LDS byte image at byte address d.
__device__ __forceinline__ void lds_or16(uint32_t* img, uint32_t d, const uint4& w) {
  const uint32_t a = d & 3, k = d >> 2;
  const uint32_t sh = 8 * a;
  // w shifted left by a bytes across five dwords
  const uint32_t d0 = sh ? (w.x << sh) : w.x;
  const uint32_t d1 = sh ? __builtin_amdgcn_alignbyte(w.y, w.x, 4 - a) : w.y;
  const uint32_t d2 = sh ? __builtin_amdgcn_alignbyte(w.z, w.y, 4 - a) : w.z;
  const uint32_t d3 = sh ? __builtin_amdgcn_alignbyte(w.w, w.z, 4 - a) : w.w;
  const uint32_t d4 = sh ? (w.w >> (32 - sh)) : 0u;
  atomicOr(img + k, d0);
  atomicOr(img + k + 1, d1);
  atomicOr(img + k + 2, d2);
  atomicOr(img + k + 3, d3);
  if (d4) atomicOr(img + k + 4, d4);
}

// Up to 4 windows (len <= 64) of a field from 5 prefetched source lines.
struct Lines5 {
  uint4 l[5];
  uint32_t s;
  uint32_t nwin;
};
__device__ __forceinline__ Lines5 load_lines5(const uint8_t* src, uint32_t len) {
  Lines5 L;
  L.s = uint32_t(reinterpret_cast<uintptr_t>(src) & 15);
  const uint4* line = reinterpret_cast<const uint4*>(src - L.s);  // (global_load: seg_window)
  L.nwin = (len + 15) >> 4;
  const uint32_t nline = (L.s + len + 15) >> 4;
#pragma unroll
  for (int t = 0; t < 5; ++t)
    L.l[t] = uint32_t(t) < nline ? line[t] : make_uint4(0, 0, 0, 0);
  return L;
}
__device__ __forceinline__ void lds_put5(uint32_t* img, uint32_t d, const Lines5& L,
                                         uint32_t len) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (uint32_t(t) >= L.nwin) break;
    uint4 w = funnel32(L.l[t], L.l[t + 1], L.s);
    const int32_t rem = int32_t(len) - 16 * t;
    if (rem < 16) w = replace_from(w, make_uint4(0, 0, 0, 0), rem);
    lds_or16(img, d + 16 * t, w);
  }
}

// Copy len source bytes (len > 0) to image byte address d, 4 windows per
// round with the round's 5 source lines loaded first.
__device__ __forceinline__ void lds_copy_field(uint32_t* img, uint32_t d, const uint8_t* src,
                                               uint64_t len) {
  for (uint64_t j0 = 0; j0 < len; j0 += 64) {
    const uint32_t part = uint32_t(std::min<uint64_t>(64, len - j0));
    const Lines5 L = load_lines5(src + j0, part);
    lds_put5(img, d + uint32_t(j0), L, part);
  }
}

template <uint32_t IMG, int V = 0, bool kMeta = false, uint32_t NT = kThreads>  // V: diagnostic ablation (OKV_ENC_VARIANT 4: no hash,
                                   // 5: headers only, 6: loads without LDS writes;
                                   // 7: row positions by a workgroup scan, no pl reads (the product);
                                   // 8: 7 with registers capped for 8 waves)
                                   // kMeta (ablation, OKV_ENC_META_FUSED=1): the meta index
                                   // entries written here too (measured slower: 5.16-5.30
                                   // vs 4.31-4.39 ms pack, + 0.23 ms meta kernel saved)
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(V == 8 ? 8 : 1)))
void okv_enc_pack_lds_kernel(PackParams P, uint64_t nb, uint32_t G) {
  // V == 7, the product form (70 registers, 7 waves per SIMD); V == 8
  // (ablation) is the same code capped at 64 registers for 8 waves: it spills
  // (9 registers) and measured 4.88 vs 3.85 ms (profiles/r3/r3g/ablate_enc.log)
  // V == 9 (ablation): 7 with the block hashes computed by wave 0 from the
  // raw image while waves 1-3 store it (no second barrier, no precompute)
  constexpr bool kOverlap = V == 9;
  constexpr int VL = (V == 8 || V == 9) ? 7 : V;
  __shared__ uint4 img4[IMG / 16];
  __shared__ uint64_t bfirst[kMaxRegion + 1], brel[kMaxRegion], bbase[kMaxRegion];
  __shared__ uint32_t slim[kMaxRegion], blen[kMaxRegion];  // end of whole stripes, BlockSize
  __shared__ uint64_t borig[kMaxRegion], bcsz[kMaxRegion], bmoff[kMaxRegion];
  __shared__ uint32_t bfkl[kMaxRegion];  // key length of each block's first row (its FirstKey)
  uint32_t* img = reinterpret_cast<uint32_t*>(img4);
  const uint64_t k0 = uint64_t(blockIdx.x) * G;
  const uint32_t g = uint32_t(std::min<uint64_t>(G, nb - k0));
  // one HBM trip for everything that needs only the region's index: its
  // blocks' first rows and descriptors (clamped addresses, issued together;
  // round 4 waited for the region's extent before loading first[])
  const uint64_t frow = P.first[k0 + std::min<uint32_t>(threadIdx.x, g)];
  Desc dt{};
  if (threadIdx.x < 64) dt = P.desc[k0 + std::min<uint32_t>(threadIdx.x, g - 1)];
  const uint64_t O0 = P.desc[k0].offset;
  const Desc dl = P.desc[k0 + g - 1];
  const uint32_t nq = uint32_t((dl.offset + dl.block_size - O0) >> 4);
  if (threadIdx.x <= g) bfirst[threadIdx.x] = frow;
  for (uint32_t q = threadIdx.x; q < nq; q += NT) img4[q] = make_uint4(0, 0, 0, 0);
  if (threadIdx.x < 64) {  // g <= kMaxRegion = 64: wave 0
    const uint32_t t = threadIdx.x;
    uint64_t orig = 0;
    if (t < g) {  // (with first[], and the meta entry offset)
      brel[t] = dt.offset - O0;
      blen[t] = uint32_t(dt.block_size);
      slim[t] = uint32_t(dt.offset - O0 + (dt.block_size & ~uint64_t(31)));
      orig = dt.original_size;
      if constexpr (kMeta) {
        borig[t] = orig;
        bcsz[t] = dt.compressed_size;
        bmoff[t] = P.moff[k0 + t];
      }
    }
    // each block's start in the region's row stream: the OriginalSizes before it
    const uint64_t incl = wave_incl_scan(orig, int(t));
    if (t < g) bbase[t] = incl - orig;
  }
  __shared__ uint32_t s_wt[2][NT / 64];  // VL == 7: per-wave record-size totals
  __syncthreads();
  const uint64_t R0 = bfirst[0], R1 = bfirst[g];
  const uint64_t abs0 = VL == 7 ? 0 : Pg(P.pl, P.tp, int64_t(R0) - 1);
  uint32_t carry = 0;  // VL == 7: image bytes of the rows before this pass
  for (uint64_t base = R0; base < R1; base += NT) {  // uniform trip count (VL == 7 barriers)
    const uint64_t r = base + threadIdx.x;
    const bool live = r < R1;
    uint32_t kl = 0, vl = 0;
    uint64_t ko = 0, vo = 0;
    if (live) {
      kl = P.key_len[r];
      vl = P.val_len[r];
      ko = P.key_off[r];
      vo = P.val_off[r];
    }
    uint32_t srel = 0;  // VL == 7: region-relative start of record r's row stream
    if constexpr (VL == 7) {
      // exclusive scan of the record sizes in row order (< IMG bytes: u32)
      const uint32_t sz = live ? 6 + kl + vl : 0u;
      const uint32_t inc = wave_scan_dpp(sz);
      const uint32_t wave = threadIdx.x >> 6, par = uint32_t((base - R0) / NT) & 1;
      if ((threadIdx.x & 63) == 63) s_wt[par][wave] = inc;
      __syncthreads();
      uint32_t before = carry, tot = 0;
#pragma unroll
      for (uint32_t w = 0; w < NT / 64; ++w) {
        const uint32_t t = s_wt[par][w];
        before += w < wave ? t : 0u;
        tot += t;
      }
      srel = before + inc - sz;
      carry += tot;
    }
    if (!live) continue;
    uint32_t lo = 0, hi = g;  // block of row r
    while (hi - lo > 1) {
      const uint32_t m = (lo + hi) >> 1;
      if (bfirst[m] <= r)
        lo = m;
      else
        hi = m;
    }
    if (kMeta && r == bfirst[lo]) bfkl[lo] = kl;
    // (the other arms: the row's absolute row-stream position from the row
    // prefix, less the block's -- the region's first row's absolute position
    // abs0 plus the block's region-relative base)
    const uint32_t d = VL == 7 ? uint32_t(brel[lo] + srel - (bbase[lo] - bbase[0]))
                              : uint32_t(brel[lo] + Pg(P.pl, P.tp, int64_t(r) - 1) -
                                         (abs0 + bbase[lo]));
    if (VL == 5) {
      lds_or16(img, d, make_uint4(kl | (vl << 16), vl >> 16, 0, 0));
    } else if (VL == 6 && kl <= 64 && vl <= 64) {
      const Lines5 K = load_lines5(P.key_arena + ko, kl);
      const Lines5 Vl = load_lines5(P.val_arena + vo, vl);
      uint32_t x = 0;
#pragma unroll
      for (int t = 0; t < 5; ++t) x ^= K.l[t].x ^ K.l[t].w ^ Vl.l[t].y ^ Vl.l[t].z;
      lds_or16(img, d, make_uint4(kl | (vl << 16), vl >> 16, x == 0x9e3779b9u ? 1u : 0u, 0));
    } else if (kl <= 64 && vl <= 64) {  // all source lines of the record in flight at once
      const Lines5 K = load_lines5(P.key_arena + ko, kl);
      const Lines5 Vl = load_lines5(P.val_arena + vo, vl);
      lds_or16(img, d, make_uint4(kl | (vl << 16), vl >> 16, 0, 0));
      lds_put5(img, d + 6, K, kl);
      if (vl) lds_put5(img, d + 6 + kl, Vl, vl);
    } else {
      lds_or16(img, d, make_uint4(kl | (vl << 16), vl >> 16, 0, 0));
      lds_copy_field(img, d + 6, P.key_arena + ko, kl);
      if (vl) lds_copy_field(img, d + 6 + kl, P.val_arena + vo, vl);
    }
  }
  __syncthreads();
  uint4* dst = reinterpret_cast<uint4*>(P.seg + O0);
  if constexpr (kOverlap) {
    if (threadIdx.x >= 64) {
      for (uint32_t q = threadIdx.x - 64; q < nq; q += NT - 64) dst[q] = img4[q];
      return;
    }
  } else {
  // Store the image; each 16 bytes lying in whole 32-byte stripes of its block
  // are then replaced in place (same lane, so no barrier between) by their two
  // XXH64 round inputs x * PRIME64_2, computed by all 256 lanes: the four
  // hashing lanes per block are left with add, rotate, multiply per round.
  // (non-temporal stores: the segment is written once and read by no kernel
  // of this encode -- pack 4.53-4.55 -> 4.44-4.47 ms, profiles/r5/session/
  // enc_pack_nt_ab.log; non-temporal arena loads as well: 4.82-4.84 ms)
  for (uint32_t q = threadIdx.x; q < nq; q += NT) {
    const uint4 v = img4[q];
    store_nt16(&dst[q], v);
    if (VL == 4) continue;
    const uint32_t p = q << 4;
    uint32_t lo = 0, hi = g;  // block holding byte p
    while (hi - lo > 1) {
      const uint32_t m = (lo + hi) >> 1;
      if (uint32_t(brel[m]) <= p)
        lo = m;
      else
        hi = m;
    }
    // the block's first kFkStride bytes (its first record's header and key),
    // as stored, for the meta kernel -- which otherwise reads the block's first
    // line from the segment, one scattered line per block (blocks start
    // 16-byte aligned in the image: whole chunks; BlockSize >= 48 here)
    if (P.fk && p < uint32_t(brel[lo]) + kFkStride && p + 16 <= uint32_t(brel[lo]) + blen[lo])
      *reinterpret_cast<uint4*>(P.fk + (k0 + lo) * kFkStride + (p - uint32_t(brel[lo]))) = v;
    if constexpr (kMeta) {  // FirstKey bytes of the block's meta entry (block_stat.go:31-33)
      const uint32_t ks = uint32_t(brel[lo]) + 6, ke = ks + bfkl[lo];
      const uint32_t a0 = max(p, ks), a1 = min(p + 16, ke);
      uint8_t* m = P.meta + bmoff[lo] + 2 - ks;
      for (uint32_t x = a0; x < a1; ++x) m[x] = uint8_t(dword_at(v, x - p));
    }
    if (p + 16 <= slim[lo]) {
      const uint64_t a = ((uint64_t(v.y) << 32) | v.x) * XP2;
      const uint64_t c = ((uint64_t(v.w) << 32) | v.z) * XP2;
      img4[q] = make_uint4(uint32_t(a), uint32_t(a >> 32), uint32_t(c), uint32_t(c >> 32));
    }
  }
  if (VL == 4) return;
  // only LDS has to be ordered here (a __syncthreads would also wait for the
  // image's global stores)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // BlockStat.Hash = XXH64 of the padded block (segment_writer.go:185), from
  // the image: four lanes per block own XXH64's four accumulators.
  if (threadIdx.x < 4 * g) {
    const uint32_t b = threadIdx.x >> 2, q = threadIdx.x & 3;
    const uint32_t boff = uint32_t(brel[b]);
    const uint64_t len = blen[b];
    const uint64_t* w64 = reinterpret_cast<const uint64_t*>(img4) + (boff >> 3);
    uint64_t acc = (q == 0) ? XP1 + XP2 : (q == 1) ? XP2 : (q == 2) ? 0 : 0 - XP1;
    const uint32_t nstripe = uint32_t(len / 32);
    uint32_t st = 0;
    for (; st + 8 <= nstripe; st += 8) {  // 8 LDS reads ahead of the round chain
      uint64_t x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = w64[4 * (st + u) + q];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = kOverlap ? xround(acc, x[u]) : xround_pre(acc, x[u]);
    }
    for (; st < nstripe; ++st)
      acc = kOverlap ? xround(acc, w64[4 * st + q]) : xround_pre(acc, w64[4 * st + q]);
    const int lane = threadIdx.x & 63;
    const uint64_t a1 = __shfl(acc, (lane & ~3) + 1, 64);
    const uint64_t a2 = __shfl(acc, (lane & ~3) + 2, 64);
    const uint64_t a3 = __shfl(acc, (lane & ~3) + 3, 64);
    if (q == 0) {
      uint64_t h;
      if (len >= 32) {
        h = rotl64(acc, 1) + rotl64(a1, 7) + rotl64(a2, 12) + rotl64(a3, 18);
        h = (h ^ xround(0, acc)) * XP1 + XP4;
        h = (h ^ xround(0, a1)) * XP1 + XP4;
        h = (h ^ xround(0, a2)) * XP1 + XP4;
        h = (h ^ xround(0, a3)) * XP1 + XP4;
      } else {
        h = XP5;
      }
      h += len;
      const uint8_t* bytes = reinterpret_cast<const uint8_t*>(img4) + boff;
      uint32_t t = nstripe * 32;
      for (; t + 8 <= len; t += 8) {
        h ^= xround(0, w64[t / 8]);
        h = rotl64(h, 27) * XP1 + XP4;
      }
      if (t + 4 <= len) {
        const uint32_t v = uint32_t(bytes[t]) | (uint32_t(bytes[t + 1]) << 8) |
                           (uint32_t(bytes[t + 2]) << 16) | (uint32_t(bytes[t + 3]) << 24);
        h ^= uint64_t(v) * XP1;
        h = rotl64(h, 23) * XP2 + XP3;
        t += 4;
      }
      for (; t < len; ++t) {
        h ^= uint64_t(bytes[t]) * XP5;
        h = rotl64(h, 11) * XP1;
      }
      h ^= h >> 33;
      h *= XP2;
      h ^= h >> 29;
      h *= XP3;
      h ^= h >> 32;
      P.hash[k0 + b] = h;
      if constexpr (kMeta) {  // the rest of the entry: u16 len(FirstKey), then 5 x u64 (:27-42)
        uint8_t* m = P.meta + bmoff[b];
        const uint32_t kl = bfkl[b];
        put_le(m, kl, 2);
        m += 2 + kl;
        put_le(m, O0 + boff, 8);
        put_le(m + 8, len, 8);
        put_le(m + 16, borig[b], 8);
        put_le(m + 24, bcsz[b], 8);
        put_le(m + 32, h, 8);
      }
    }
  }
}

// E10 (general DataBlockSize, not a multiple of 16): one byte per lane.
__global__ __launch_bounds__(kThreads) void okv_enc_pack_bytes_kernel(PackParams P, uint64_t nb,
                                                                      uint64_t data_bytes) {
  for (uint64_t x = uint64_t(blockIdx.x) * kThreads + threadIdx.x; x < data_bytes;
       x += uint64_t(gridDim.x) * kThreads) {
    uint64_t lo = 0, hi = nb;  // block: desc[lo].offset <= x
    while (hi - lo > 1) {
      const uint64_t m = (lo + hi) >> 1;
      if (P.desc[m].offset <= x)
        lo = m;
      else
        hi = m;
    }
    const Desc d = P.desc[lo];
    const uint64_t p = x - d.offset;
    uint8_t byte = 0;
    if (p < d.original_size) {
      const uint64_t r0 = P.first[lo], r1 = P.first[lo + 1];
      const uint64_t base = Pg(P.pl, P.tp, int64_t(r0) - 1);
      uint64_t a = r0, b = r1;  // row: P(a-1) - base <= p
      while (b - a > 1) {
        const uint64_t m = (a + b) >> 1;
        if (Pg(P.pl, P.tp, int64_t(m) - 1) - base <= p)
          a = m;
        else
          b = m;
      }
      const uint64_t o = p - (Pg(P.pl, P.tp, int64_t(a) - 1) - base);
      const uint32_t kl = P.key_len[a], vl = P.val_len[a];
      if (o < 2)
        byte = uint8_t(kl >> (8 * o));
      else if (o < 6)
        byte = uint8_t(vl >> (8 * (o - 2)));
      else if (o < 6 + uint64_t(kl))
        byte = P.key_arena[P.key_off[a] + (o - 6)];
      else
        byte = P.val_arena[P.val_off[a] + (o - 6 - kl)];
    }
    P.seg[x] = byte;
  }
}

// ---------------------------------------------------------------------------
// E12: meta block = head + one entry per block (BlockStat.toBytes,
// block_stat.go:27-42), written at seg + data_bytes.
// ---------------------------------------------------------------------------

struct MetaParams {
  const uint8_t* key_arena;
  const uint64_t* key_off;
  const uint16_t* key_len;
  uint64_t n;
  const uint64_t* first;
  const Desc* desc;
  const uint64_t* hash;
  const uint64_t* moff;
  uint64_t nb;      // entries written by this launch
  uint64_t count;   // block index entries (the head's u64 count, :320)
  int comp_byte;
  uint8_t* meta;
  uint64_t bloom_len;  // ~0: no bloom filter; else its WriteTo length
  // the segment the pack kernel wrote (uncompressed blocks): each block's
  // FirstKey is read from its first record there, one line per block, instead
  // of through the row arrays (key_len, key_off and the key: three scattered
  // lines); null: through the row arrays
  const uint8_t* seg = nullptr;
  // non-null: each block's FirstKey length and (when <= kFkCap) bytes, kept by
  // the planner and the LDS pack kernel -- two coalesced reads per block
  const uint8_t* fk = nullptr;
  const uint16_t* fkl = nullptr;
};

__global__ __launch_bounds__(kThreads) void okv_enc_meta_kernel(MetaParams P) {
  const uint64_t k = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (k == 0) {  // generateMetaBlock head (:288-325)
    uint8_t* p = P.meta;
    const uint32_t k0 = P.key_len[0], kz = P.key_len[P.n - 1];
    put_le(p, k0, 2);
    put_bytes(p + 2, P.key_arena + P.key_off[0], k0);
    p += 2 + k0;
    put_le(p, kz, 2);
    put_bytes(p + 2, P.key_arena + P.key_off[P.n - 1], kz);
    p += 2 + kz;
    if (P.bloom_len != ~uint64_t(0)) {  // :295-300 (the filter bytes: a host copy)
      p[0] = 1;
      put_le(p + 1, P.bloom_len, 8);
      p += 9 + P.bloom_len;
    } else {
      p[0] = 0;  // :301-303
      p += 1;
    }
    p[0] = uint8_t(P.comp_byte);
    p[1] = 0;  // not a partitioned block index
    put_le(p + 2, P.count, 8);
  }
  if (k >= P.nb) return;
  uint8_t* p = P.meta + P.moff[k];
  const uint64_t r = P.first[k];
  const uint32_t kl = P.key_len[r];
  put_le(p, kl, 2);
  put_bytes(p + 2, P.key_arena + P.key_off[r], kl);
  p += 2 + kl;
  const Desc d = P.desc[k];
  put_le(p, d.offset, 8);
  put_le(p + 8, d.block_size, 8);
  put_le(p + 16, d.original_size, 8);
  put_le(p + 24, d.compressed_size, 8);
  put_le(p + 32, P.hash[k], 8);
}

// Block k's FirstKey (block_stat.go:31-33): the key of its first record.
__device__ __forceinline__ void first_key(const MetaParams& P, uint64_t k, const Desc& d,
                                          uint32_t& kl, const uint8_t*& key) {
  if (P.fk && P.fkl[k] <= kFkCap && d.block_size >= kFkStride) {
    kl = P.fkl[k];
    key = P.fk + k * kFkStride + 6;
  } else if (P.seg) {  // [u16 LE kl][u32 LE vl][key] at the block's start
    const uint8_t* rec = P.seg + d.offset;
    kl = uint32_t(rec[0]) | (uint32_t(rec[1]) << 8);
    key = rec + 6;
  } else {
    const uint64_t r = P.first[k];
    kl = P.key_len[r];
    key = P.key_arena + P.key_off[r];
  }
}

// E12 via LDS: one workgroup builds the entries of kThreads consecutive blocks
// (one contiguous byte range of the meta block, <= kMetaImage bytes) in an LDS
// image and stores it with aligned 16-byte stores; the range's unaligned head
// and tail bytes (shared with neighbouring workgroups) are stored bytewise.
__global__ __launch_bounds__(kThreads) void okv_enc_meta_lds_kernel(MetaParams P,
                                                                    uint64_t meta_bytes) {
  __shared__ uint4 img4[kMetaImage / 16 + 2];
  __shared__ int big;
  uint32_t* img = reinterpret_cast<uint32_t*>(img4);
  const uint64_t k0 = uint64_t(blockIdx.x) * kThreads;
  const uint64_t k1 = std::min<uint64_t>(P.nb, k0 + kThreads);
  const uint64_t lo = P.moff[k0];
  const uint64_t hi = k1 < P.nb ? P.moff[k1] : meta_bytes;
  const uint64_t a0 = lo & ~uint64_t(15);  // image byte 0 = meta byte a0
  const uint32_t nq = uint32_t((hi - a0 + 15) >> 4);
  if (threadIdx.x == 0) big = (hi - a0 + 15) > kMetaImage;
  __syncthreads();
  const uint64_t k = k0 + threadIdx.x;
  if (big) {  // long first keys: byte stores
    if (k < k1) {
      uint8_t* p = P.meta + P.moff[k];
      const Desc d = P.desc[k];
      uint32_t kl;
      const uint8_t* key;
      first_key(P, k, d, kl, key);
      put_le(p, kl, 2);
      put_bytes(p + 2, key, kl);
      p += 2 + kl;
      put_le(p, d.offset, 8);
      put_le(p + 8, d.block_size, 8);
      put_le(p + 16, d.original_size, 8);
      put_le(p + 24, d.compressed_size, 8);
      put_le(p + 32, P.hash[k], 8);
    }
    return;
  }
  for (uint32_t q = threadIdx.x; q < nq; q += kThreads) img4[q] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  if (k < k1) {
    const uint32_t d = uint32_t(P.moff[k] - a0);
    const Desc ds = P.desc[k];
    const uint64_t h = P.hash[k];
    uint32_t kl;
    const uint8_t* key;
    first_key(P, k, ds, kl, key);
    lds_or16(img, d, make_uint4(kl & 0xffffu, 0, 0, 0));  // only 2 bytes are non-zero
    if (kl) lds_copy_field(img, d + 2, key, kl);
    const uint32_t e = d + 2 + kl;
    lds_or16(img, e, make_uint4(uint32_t(ds.offset), uint32_t(ds.offset >> 32),
                                uint32_t(ds.block_size), uint32_t(ds.block_size >> 32)));
    lds_or16(img, e + 16, make_uint4(uint32_t(ds.original_size), uint32_t(ds.original_size >> 32),
                                     uint32_t(ds.compressed_size),
                                     uint32_t(ds.compressed_size >> 32)));
    lds_or16(img, e + 32, make_uint4(uint32_t(h), uint32_t(h >> 32), 0, 0));
  }
  __syncthreads();
  const uint8_t* ib = reinterpret_cast<const uint8_t*>(img4);
  for (uint32_t q = threadIdx.x; q < nq; q += kThreads) {
    const uint64_t c0 = a0 + 16 * uint64_t(q);
    if (c0 >= lo && c0 + 16 <= hi) {
      *reinterpret_cast<uint4*>(P.meta + c0) = img4[q];
    } else {  // shared with a neighbouring range
      for (uint32_t b = 0; b < 16; ++b)
        if (c0 + b >= lo && c0 + b < hi) P.meta[c0 + b] = ib[16 * q + b];
    }
  }
}

// ---------------------------------------------------------------------------
// Deterministic fixed-shape rows (oracle/pyoracle.py rows_fixed).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix_at(uint64_t seed, uint64_t w) {
  uint64_t z = seed + (w + 1) * 0x9E3779B97F4A7C15ULL;  // state after draw w
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kThreads) void okv_synth_fixed_kernel(
    uint64_t seed, uint64_t first_row, uint64_t n, uint32_t kl, uint32_t vl,
    uint8_t* __restrict__ key_arena, uint64_t* __restrict__ key_off,
    uint16_t* __restrict__ key_len, uint8_t* __restrict__ val_arena,
    uint64_t* __restrict__ val_off, uint32_t* __restrict__ val_len) {
  const uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint64_t row = first_row + i;
  uint8_t* k = key_arena + i * kl;
  for (uint32_t b = 0; b < kl; ++b) {
    const uint32_t from_end = kl - 1 - b;
    k[b] = from_end < 8 ? uint8_t(row >> (8 * from_end)) : 0;
  }
  const uint32_t wpr = (vl + 7) / 8;
  uint8_t* v = val_arena + i * vl;
  for (uint32_t w = 0; w < wpr; ++w) {
    const uint64_t x = splitmix_at(seed, row * wpr + w);
    const uint32_t nbytes = std::min<uint32_t>(8, vl - 8 * w);
    if (nbytes == 8 && (reinterpret_cast<uintptr_t>(v + 8 * w) & 7) == 0)
      *reinterpret_cast<uint64_t*>(v + 8 * w) = x;
    else
      for (uint32_t b = 0; b < nbytes; ++b) v[8 * w + b] = uint8_t(x >> (8 * b));
  }
  key_off[i] = i * kl;
  key_len[i] = uint16_t(kl);
  val_off[i] = i * vl;
  val_len[i] = vl;
}

}  // namespace okv

// ===========================================================================
// Host orchestration
// ===========================================================================
namespace okv {
namespace {

struct DevRows {
  const uint8_t* ka;
  const uint64_t* ko;
  const uint16_t* kl;
  const uint8_t* va;
  const uint64_t* vo;
  const uint32_t* vl;
  uint64_t n;
};

int dev_realloc(okv_ctx* ctx, void** p, size_t bytes) {
  if (*p) {
    OKV_HIP(hipStreamSynchronize(ctx->stream));
    (void)hipFree(*p);
    *p = nullptr;
  }
  OKV_HIP(hipMalloc(p, std::max<size_t>(bytes, 256)));
  return OKV_OK;
}

int enc_scratch(okv_ctx* ctx, EncScratch** out) {
  if (!ctx->enc) {
    EncScratch* e = new EncScratch();
    ctx->enc = e;
    OKV_HIP(hipMalloc(&e->d_tot, sizeof(EncTotals)));
    OKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&e->h_tot), sizeof(EncTotals), 0));
  }
  *out = ctx->enc;
  return OKV_OK;
}

int ensure_tiles(okv_ctx* ctx, EncScratch* e, uint64_t n) {
  const uint64_t nt = (n + kETile - 1) / kETile + 1;
  int rc;
  if (nt > e->cap_tiles || !e->tile_tot) {
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->tile_tot), nt * 8))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->tile_pre), nt * 8))) return rc;
    e->cap_tiles = nt;
  }
  return OKV_OK;
}

int ensure_rows(okv_ctx* ctx, EncScratch* e, uint64_t n) {
  const uint64_t nt = (n + kETile - 1) / kETile + 1;
  int rc;
  if (n > e->cap_rows || !e->pl) {
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->pl), n * 8))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->nx), n * 4))) return rc;
    e->cap_rows = n;
  }
  if (nt > e->cap_tiles || !e->tile_tot) {
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->tile_tot), nt * 8))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->tile_pre), nt * 8))) return rc;
    e->cap_tiles = nt;
  }
  return OKV_OK;
}

int ensure_jump(okv_ctx* ctx, EncScratch* e, size_t entries, uint64_t nch) {
  int rc;
  if (entries > e->cap_jump || !e->jt) {
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->jt), entries * 4))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->jb), entries * 4))) return rc;
    e->cap_jump = entries;
  }
  if (nch > e->cap_chunks || !e->entry) {
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->entry), nch * 4))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->kbase), nch * 8))) return rc;
    e->cap_chunks = nch;
  }
  return OKV_OK;
}

int ensure_blocks_enc(okv_ctx* ctx, EncScratch* e, uint64_t nb) {
  const uint64_t nbt = (nb + kETile - 1) / kETile + 1;
  int rc;
  if (nb + 1 > e->cap_blocks || !e->first) {
    const size_t c = nb + 1;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->first), c * 8))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->desc), c * sizeof(Desc)))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->hash), c * 8))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->bsl), c * 8))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->esl), c * 8))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->moff), c * 8))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->orig), c * 8))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->fkl), c * 2))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->fk), c * kFkStride))) return rc;
    e->cap_blocks = c;
  }
  if (nbt > e->cap_btiles || !e->btile) {
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->btile), 4 * nbt * 8))) return rc;
    e->cap_btiles = nbt;
  }
  return OKV_OK;
}

int read_enc_totals(okv_ctx* ctx, EncScratch* e) {
  OKV_HIP(hipMemcpyAsync(e->h_tot, e->d_tot, sizeof(EncTotals), hipMemcpyDeviceToHost,
                         ctx->stream));
  OKV_HIP(hipStreamSynchronize(ctx->stream));
  return OKV_OK;
}

void enc_mark(okv_ctx* ctx, EncScratch* e, int k) {  // 5 events per profiled call
  if (!ctx->prof) return;
  while (e->ev.size() < e->ev_used + 5) {
    hipEvent_t v;
    if (hipEventCreate(&v) != hipSuccess) return;
    e->ev.push_back(v);
  }
  (void)hipEventRecord(e->ev[e->ev_used + k], ctx->stream);
  if (k == 4) e->ev_used += 5;
}

uint32_t ceil_div(uint64_t a, uint64_t b) { return uint32_t((a + b - 1) / b); }

struct Plan {
  uint64_t nb, data_bytes, meta_bytes, file_bytes, last_raw;
  uint64_t head;  // meta head bytes (keys, bloom, compression, count)
  uint64_t w;     // most rows any block start can take (max next(a) - a)
  uint64_t bmax;  // largest BlockSize
  uint64_t avg_rec;  // mean record size
};

// E1-E2 (record-size prefix pl / tile_pre) for the pack kernels that read it,
// after a single-pass plan (which writes no per-row array).
int enc_row_prefix(okv_ctx* ctx, EncScratch* e, const DevRows& R, uint64_t T) {
  if (e->have_pl) return OKV_OK;
  int rc;
  if ((rc = ensure_rows(ctx, e, R.n))) return rc;
  const uint32_t ntiles = ceil_div(R.n, kETile);
  hipLaunchKernelGGL(okv_enc_size_next_kernel, dim3(ntiles), dim3(kThreads), 0, ctx->stream,
                     R.kl, R.vl, R.n, T, e->pl, e->tile_tot, e->nx, e->d_tot);
  hipLaunchKernelGGL(okv_enc_scan_kernel, dim3(1), dim3(1024), 0, ctx->stream, e->tile_tot,
                     uint64_t(ntiles), e->tile_pre, nullptr);
  OKV_HIP(hipGetLastError());
  e->have_pl = true;
  return OKV_OK;
}

#ifdef OKV_ABLATE  // A/B arm OKV_ENC_ONEPASS=1 (the single-pass plan, measured slower)
#include "okv_encode_ablate_host.inc"
#endif

int ensure_cut(okv_ctx* ctx, EncScratch* e, uint64_t ntiles) {
  int rc;
  if (ntiles * kCutS > e->cap_cut || !e->jts) {
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->jts), ntiles * kCutS * 2))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->jbs), ntiles * kCutS * 2))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->tentry), ntiles * 4))) return rc;
    if ((rc = dev_realloc(ctx, reinterpret_cast<void**>(&e->tkbase), ntiles * 8))) return rc;
    e->cap_cut = ntiles * kCutS;
  }
  return OKV_OK;
}

// Block boundaries, BlockStat sizes/offsets and meta layout (E1-E9).
int enc_plan(okv_ctx* ctx, EncScratch* e, const DevRows& R, const okv_encode_opts& o, Plan* pl,
             uint64_t* bad_row) {
  const uint64_t n = R.n;
  const uint64_t T = o.threshold_bytes, D = o.block_size;
  const uint32_t ntiles = ceil_div(n, kETile);
  int rc;
  // the tile cut (E1 + E3 + E4 in LDS per tile, no per-row arrays)
  if ((rc = ensure_cut(ctx, e, ntiles)) || (rc = ensure_tiles(ctx, e, n))) return rc;
  e->have_pl = false;
  hipLaunchKernelGGL(okv_enc_init_kernel, dim3(1), dim3(1), 0, ctx->stream, e->d_tot);
  hipLaunchKernelGGL(okv_enc_cut_kernel, dim3(ntiles), dim3(kThreads), 0, ctx->stream, R.kl, R.vl,
                     n, T, e->jts, e->jbs, e->tile_tot, e->d_tot);
  hipLaunchKernelGGL(okv_enc_sum_kernel, dim3(1), dim3(1024), 0, ctx->stream, e->tile_tot,
                     uint64_t(ntiles), &e->d_tot->total_raw);
  OKV_HIP(hipGetLastError());
  if ((rc = read_enc_totals(ctx, e))) return rc;
  const bool tile_cut = !e->h_tot->far;
  if (!tile_cut) {
    // a block longer than the lookahead: the general kernels (E1-E2 over every
    // row, E3 over the global prefix)
    if ((rc = ensure_rows(ctx, e, n))) return rc;
    e->have_pl = true;
    hipLaunchKernelGGL(okv_enc_init_kernel, dim3(1), dim3(1), 0, ctx->stream, e->d_tot);
    hipLaunchKernelGGL(okv_enc_size_next_kernel, dim3(ntiles), dim3(kThreads), 0, ctx->stream,
                       R.kl, R.vl, n, T, e->pl, e->tile_tot, e->nx, e->d_tot);
    hipLaunchKernelGGL(okv_enc_scan_kernel, dim3(1), dim3(1024), 0, ctx->stream, e->tile_tot,
                       uint64_t(ntiles), e->tile_pre, &e->d_tot->total_raw);
    hipLaunchKernelGGL(okv_enc_init_wmax_kernel, dim3(1), dim3(1), 0, ctx->stream, e->d_tot);
    hipLaunchKernelGGL(okv_enc_next_kernel, dim3(ntiles), dim3(kThreads), 0, ctx->stream, e->pl,
                       e->tile_pre, n, T, e->nx, e->d_tot);
    OKV_HIP(hipGetLastError());
    if ((rc = read_enc_totals(ctx, e))) return rc;
  }
  if (e->h_tot->bad_row != kNone) {
    *bad_row = e->h_tot->bad_row;
    return set_err(ctx, OKV_W_INVALID_KEY, "key cannot be empty (ErrInvalidKey)");
  }
  // chunking for the chain: C >= W rows per chunk (the tile cut: its tiles,
  // entered at offsets <= kFuseLook, so its tables are at most kCutS wide)
  const uint64_t wmax = std::max<uint64_t>(1, e->h_tot->wmax);
  const uint64_t W = tile_cut ? std::min<uint64_t>(wmax, kCutS) : wmax;
  uint64_t C = tile_cut ? uint64_t(kETile) * kCutTiles : 4096;
  while (C < W) C <<= 1;
  const uint64_t nch = (n + C - 1) / C;
  uint32_t levels = 0;
  while ((uint64_t(1) << levels) < nch) ++levels;  // 2^levels >= nch
  const uint64_t lv = nch * W;
  if (lv >= (uint64_t(1) << 32))  // (the chain-table kernels index with 32 bits)
    return set_err(ctx, OKV_E_ARG, "encode: too many rows for one call (chain table >= 2^32)");
  if ((rc = ensure_jump(ctx, e, lv * std::max<uint32_t>(levels, 1), nch))) return rc;
  if (tile_cut)
    hipLaunchKernelGGL(okv_enc_compose_kernel, dim3(ceil_div(lv, kThreads)), dim3(kThreads), 0,
                       ctx->stream, e->jts, e->jbs, uint64_t(ntiles), nch, uint32_t(W), e->jt,
                       e->jb);
  else
    hipLaunchKernelGGL(okv_enc_jump0_kernel, dim3(ceil_div(lv, kThreads)), dim3(kThreads), 0,
                       ctx->stream, e->nx, n, C, uint32_t(W), nch, e->jt, e->jb);
  for (uint32_t k = 1; k < levels; ++k)
    hipLaunchKernelGGL(okv_enc_jump_kernel, dim3(ceil_div(lv, kThreads)), dim3(kThreads), 0,
                       ctx->stream, e->jt + (k - 1) * lv, e->jb + (k - 1) * lv, e->jt + k * lv,
                       e->jb + k * lv, uint32_t(W), nch, uint64_t(1) << (k - 1), e->d_tot);
  hipLaunchKernelGGL(okv_enc_resolve_kernel, dim3(ceil_div(nch, kThreads)), dim3(kThreads), 0,
                     ctx->stream, e->jt, e->jb, levels, uint32_t(W), nch, e->entry, e->kbase,
                     e->d_tot);
  OKV_HIP(hipGetLastError());
  if ((rc = read_enc_totals(ctx, e))) return rc;
  const uint64_t nb = e->h_tot->nb;
  if (e->h_tot->fault || nb == 0 || nb > n || nb >= (uint64_t(1) << 32))
    return set_err(ctx, OKV_E_HIP, "encode: inconsistent block count");
  if ((rc = ensure_blocks_enc(ctx, e, nb))) return rc;
  const uint32_t nbt = ceil_div(nb, kETile);
  uint64_t* btot = e->btile;
  uint64_t* bpre = e->btile + e->cap_btiles;
  uint64_t* etot = e->btile + 2 * e->cap_btiles;
  uint64_t* epre = e->btile + 3 * e->cap_btiles;
  if (tile_cut) {
    hipLaunchKernelGGL(okv_enc_tile_entry_kernel, dim3(ceil_div(ntiles, kThreads)), dim3(kThreads),
                       0, ctx->stream, e->jts, e->jbs, e->entry, e->kbase, uint64_t(ntiles),
                       e->tentry, e->tkbase);
    hipLaunchKernelGGL(okv_enc_emit_tile_kernel, dim3(ntiles), dim3(kThreads), 0, ctx->stream,
                       R.kl, R.vl, n, T, e->tentry, e->tkbase, e->first, e->orig, e->fkl, nb,
                       uint64_t(ntiles), e->d_tot);
  }
  else
    hipLaunchKernelGGL(okv_enc_emit_kernel, dim3(ceil_div(nch, kThreads)), dim3(kThreads), 0,
                       ctx->stream, e->nx, n, C, nch, e->entry, e->kbase, e->first, nb, e->pl,
                       e->tile_pre, R.kl, e->orig, e->fkl, e->d_tot);
  StatParams sp;
  sp.orig = e->orig;
  sp.fkl = e->fkl;
  sp.nb = nb;
  sp.D = D;
  sp.dshift = 64;
  if (D && (D & (D - 1)) == 0)
    for (sp.dshift = 0; (uint64_t(1) << sp.dshift) != D; ++sp.dshift) {
    }
  sp.lz4 = o.compression == OKV_COMP_LZ4;
  sp.desc = e->desc;
  sp.bsl = e->bsl;
  sp.esl = e->esl;
  sp.btile_tot = btot;
  sp.etile_tot = etot;
  sp.tot = e->d_tot;
  hipLaunchKernelGGL(okv_enc_stat_kernel, dim3(nbt), dim3(kThreads), 0, ctx->stream, sp);
  hipLaunchKernelGGL(okv_enc_scan_kernel, dim3(1), dim3(1024), 0, ctx->stream, btot,
                     uint64_t(nbt), bpre, &e->d_tot->data_bytes);
  hipLaunchKernelGGL(okv_enc_scan_kernel, dim3(1), dim3(1024), 0, ctx->stream, etot,
                     uint64_t(nbt), epre, &e->d_tot->meta_ent);
  hipLaunchKernelGGL(okv_enc_offset_kernel, dim3(ceil_div(nb, kThreads)), dim3(kThreads), 0,
                     ctx->stream, e->desc, e->bsl, e->esl, bpre, epre, nb, R.kl, n, e->first,
                     e->moff, e->d_tot, o.bloom ? 8 + o.bloom_len : 0);
  OKV_HIP(hipGetLastError());
  if ((rc = read_enc_totals(ctx, e))) return rc;
  if (e->h_tot->fault) return set_err(ctx, OKV_E_HIP, "encode: block chain inconsistent");
  pl->nb = nb;
  pl->data_bytes = e->h_tot->data_bytes;
  pl->head = e->h_tot->head;
  pl->meta_bytes = e->h_tot->head + e->h_tot->meta_ent;
  pl->file_bytes = pl->data_bytes + pl->meta_bytes + 25;
  pl->last_raw = e->h_tot->last_raw;
  pl->w = wmax;  // (the chain tables above are capped at kCutS; blocks are not)
  pl->bmax = e->h_tot->bmax;
  pl->avg_rec = e->h_tot->total_raw / n;
  return OKV_OK;
}

// Blocks per chunk-major region launch (okv_enc_pack_region_kernel).
uint64_t pack_region_blocks(const Plan& pl) {
  return std::min<uint64_t>({uint64_t(kMaxRegion), kPackRows / std::max<uint64_t>(pl.w, 1),
                             uint64_t(kMaxChunks) * 16 / std::max<uint64_t>(pl.bmax, 1)});
}

// The product's pack launch (E10-E11): record-major LDS assembly + block hashes
// for small records, chunk-major regions for large ones, a per-block kernel
// or a byte kernel when the segment is not 16-byte aligned.  *hashed: the
// launch also wrote the block hashes.
int enc_pack(okv_ctx* ctx, EncScratch* e, const DevRows& R, const okv_encode_opts& o,
             const Plan& pl, uint8_t* seg, const PackParams& pp, bool* hashed, bool* fk_done) {
  // record-major LDS assembly pays off for small records (most chunks would
  // mix fields); large records take the chunk-major kernels, which read the
  // row prefix (E1-E2; a single-pass plan does not write it)
  const bool aligned = o.block_size % 16 == 0 && (reinterpret_cast<uintptr_t>(seg) & 15) == 0;
  const uint64_t GL = std::min<uint64_t>(kMaxRegion, kImage / std::max<uint64_t>(pl.bmax, 1));
  const uint64_t G = pack_region_blocks(pl);
  int rc;
  if (aligned && GL >= 1 && pl.avg_rec <= 512) {
    // small records: record-major LDS assembly, the block hashes and FirstKeys
    hipLaunchKernelGGL((okv_enc_pack_lds_kernel<kImage, 7>), dim3(ceil_div(pl.nb, GL)),
                       dim3(kThreads), 0, ctx->stream, pp, pl.nb, uint32_t(GL));
    *hashed = true;
    *fk_done = pp.fk != nullptr;
    return OKV_OK;
  }
  // the other kernels read the row prefix: computed here (the tile cut writes
  // none), so the parameters take its buffers after the call
  if ((rc = enc_row_prefix(ctx, e, R, o.threshold_bytes))) return rc;
  PackParams q = pp;
  q.pl = e->pl;
  q.tp = e->tile_pre;
  // precondition of every kernel below: the row prefix exists (round 5 launched
  // them with a null prefix after the tile cut stopped writing it -- an illegal
  // address on the device)
  if (!e->have_pl || !q.pl || !q.tp || e->cap_rows < R.n)
    return set_err(ctx, OKV_E_ARG, "enc_pack: row prefix missing for the chunk-major kernels");
  if (aligned && G >= 1) {  // large records: chunk-major regions
    hipLaunchKernelGGL(okv_enc_pack_region_kernel<0>, dim3(ceil_div(pl.nb, G)), dim3(kThreads), 0,
                       ctx->stream, q, pl.nb, uint32_t(G));
  } else if (aligned) {
    hipLaunchKernelGGL(okv_enc_pack_kernel, dim3(uint32_t(pl.nb)), dim3(kThreads), 0,
                       ctx->stream, q);
  } else {
    const uint32_t g = std::min<uint64_t>(65536, (pl.data_bytes + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(okv_enc_pack_bytes_kernel, dim3(std::max<uint32_t>(g, 1)),
                       dim3(kThreads), 0, ctx->stream, q, pl.nb, pl.data_bytes);
  }
  return OKV_OK;
}

#ifdef OKV_ABLATE  // the measured pack variants (OKV_ENC_VARIANT / _IMAGE / _META_FUSED)
#include "okv_encode_ablate_pack.inc"
#endif

// Data blocks, block hashes and the meta block into seg (E10-E12).
int enc_write(okv_ctx* ctx, EncScratch* e, const DevRows& R, const okv_encode_opts& o,
              const Plan& pl, uint8_t* seg) {
  enc_mark(ctx, e, 1);
  PackParams pp;
  pp.key_arena = R.ka;
  pp.key_off = R.ko;
  pp.key_len = R.kl;
  pp.val_arena = R.va;
  pp.val_off = R.vo;
  pp.val_len = R.vl;
  pp.pl = e->pl;  // (null until the row prefix is computed: enc_pack / the ablation arms)
  pp.tp = e->tile_pre;
  pp.first = e->first;
  pp.desc = e->desc;
  pp.seg = seg;
  pp.hash = e->hash;
  pp.meta = nullptr;
  pp.moff = e->moff;
  pp.fk = e->fk;
  bool hashed = false, meta_done = false, fk_done = false;
  int rc;
#ifdef OKV_ABLATE
  bool handled = false;  // an ablation knob chose the pack launch
  if ((rc = enc_pack_ablate(ctx, e, R, o, pl, seg, pp, &hashed, &meta_done, &handled))) return rc;
  if (!handled)
#endif
    if ((rc = enc_pack(ctx, e, R, o, pl, seg, pp, &hashed, &fk_done))) return rc;
  enc_mark(ctx, e, 2);
  if (!hashed) launch_hash(ctx->stream, seg, pl.data_bytes, e->desc, uint32_t(pl.nb), e->hash);
  enc_mark(ctx, e, 3);
  MetaParams mp;
  mp.key_arena = R.ka;
  mp.key_off = R.ko;
  mp.key_len = R.kl;
  mp.n = R.n;
  mp.first = e->first;
  mp.desc = e->desc;
  mp.hash = e->hash;
  mp.moff = e->moff;
  mp.nb = pl.nb;
  mp.count = pl.nb;
  mp.comp_byte = o.compression == OKV_COMP_LZ4 ? 2 : 0;
  mp.meta = seg + pl.data_bytes;
  mp.bloom_len = o.bloom ? o.bloom_len : ~uint64_t(0);
  mp.seg = o.compression == OKV_COMP_NONE ? seg : nullptr;
  mp.fk = fk_done ? e->fk : nullptr;
  mp.fkl = e->fkl;
  if (o.bloom && o.bloom_len)  // BloomFilter.WriteTo bytes at head - 10 - len (after flag + u64)
    OKV_HIP(hipMemcpyAsync(mp.meta + pl.head - 10 - o.bloom_len, o.bloom, o.bloom_len,
                           hipMemcpyHostToDevice, ctx->stream));
  if (meta_done || (reinterpret_cast<uintptr_t>(mp.meta) & 15) == 0) {
    // head bytes by the first lane of a one-block launch (nb = 0); entries via
    // LDS unless the pack kernel wrote them
    MetaParams head = mp;
    head.nb = 0;
    hipLaunchKernelGGL(okv_enc_meta_kernel, dim3(1), dim3(64), 0, ctx->stream, head);
    if (!meta_done)
      hipLaunchKernelGGL(okv_enc_meta_lds_kernel, dim3(ceil_div(pl.nb, kThreads)),
                         dim3(kThreads), 0, ctx->stream, mp, pl.meta_bytes);
  } else {
    hipLaunchKernelGGL(okv_enc_meta_kernel, dim3(ceil_div(pl.nb, kThreads)), dim3(kThreads), 0,
                       ctx->stream, mp);
  }
  enc_mark(ctx, e, 4);
  OKV_HIP(hipGetLastError());
  return OKV_OK;
}

// The 25-byte trailer (segment_writer.go:226-276): meta offset, XXH64(meta),
// version 1, magic 69696969696969 (:21).
void trailer_bytes(uint64_t meta_off, uint64_t meta_hash, uint8_t t[25]) {
  const uint64_t magic = 69696969696969ULL;
  for (int i = 0; i < 8; ++i) {
    t[i] = uint8_t(meta_off >> (8 * i));
    t[8 + i] = uint8_t(meta_hash >> (8 * i));
    t[17 + i] = uint8_t(magic >> (8 * i));
  }
  t[16] = 1;
}

// XXH64 over a byte stream fed in 32-byte-multiple pieces (segment_writer.go:248
// hashes the meta block with xxhash.Sum64: canonical XXH64, seed 0).
struct Xxh64Stream {
  static constexpr uint64_t P1 = 11400714785074694791ULL, P2 = 14029467366897019727ULL,
                            P3 = 1609587929392839161ULL, P4 = 9650029242287828579ULL,
                            P5 = 2870177450012600261ULL;
  uint64_t v[4] = {P1 + P2, P2, 0, 0 - P1};
  uint64_t len = 0;
  static uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
  static uint64_t rd64(const uint8_t* p) {
    uint64_t x;
    memcpy(&x, p, 8);
    return x;
  }
  static uint64_t xr(uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; }
  void stripes(const uint8_t* p, uint64_t n) {  // n % 32 == 0
    uint64_t a = v[0], b = v[1], c = v[2], d = v[3];
    for (const uint8_t* end = p + n; p < end; p += 32) {
      a = xr(a, rd64(p));
      b = xr(b, rd64(p + 8));
      c = xr(c, rd64(p + 16));
      d = xr(d, rd64(p + 24));
    }
    v[0] = a, v[1] = b, v[2] = c, v[3] = d;
    len += n;
  }
  uint64_t finish(const uint8_t* p, uint64_t n) {  // the last n < 32 bytes
    const uint64_t total = len + n;
    uint64_t h;
    if (len) {
      h = rotl(v[0], 1) + rotl(v[1], 7) + rotl(v[2], 12) + rotl(v[3], 18);
      for (uint64_t x : v) h = (h ^ xr(0, x)) * P1 + P4;
    } else {
      h = P5;
    }
    h += total;
    const uint8_t* end = p + n;
    for (; p + 8 <= end; p += 8) h = rotl(h ^ xr(0, rd64(p)), 27) * P1 + P4;
    if (p + 4 <= end) {
      uint32_t w;
      memcpy(&w, p, 4);
      h = rotl(h ^ (uint64_t(w) * P1), 23) * P2 + P3;
      p += 4;
    }
    for (; p < end; ++p) h = rotl(h ^ (uint64_t(*p) * P5), 11) * P1;
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
  }
};

// Close (segment_writer.go:226-276) on a device segment: the meta block comes
// back in pinned 8 MiB pieces on the context stream, double-buffered so the
// next piece's D2H overlaps this piece's XXH64; then the 25-byte trailer.
int close_device(okv_ctx* ctx, EncScratch* e, okv_encode_out* out) {
  constexpr uint64_t kPiece = 8ull << 20;  // multiple of 32 (XXH64 stripes)
  uint8_t* meta = out->seg + out->data_bytes;
  for (int i = 0; i < 2; ++i) {
    if (!e->close_buf[i]) OKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&e->close_buf[i]),
                                                kPiece, 0));
    if (!e->close_ev[i]) OKV_HIP(hipEventCreateWithFlags(&e->close_ev[i],
                                                         hipEventDisableTiming));
  }
  const uint64_t mb = out->meta_bytes, np = (mb + kPiece - 1) / kPiece;
  auto issue = [&](uint64_t k) -> int {
    const uint64_t o = k * kPiece, n = std::min(kPiece, mb - o);
    OKV_HIP(hipMemcpyAsync(e->close_buf[k & 1], meta + o, n, hipMemcpyDeviceToHost,
                           ctx->stream));
    OKV_HIP(hipEventRecord(e->close_ev[k & 1], ctx->stream));
    return OKV_OK;
  };
  Xxh64Stream xs;
  int rc;
  if (np && (rc = issue(0))) return rc;
  for (uint64_t k = 0; k < np; ++k) {
    OKV_HIP(hipEventSynchronize(e->close_ev[k & 1]));
    if (k + 1 < np && (rc = issue(k + 1))) return rc;
    const uint64_t n = std::min(kPiece, mb - k * kPiece);
    const uint64_t whole = k + 1 < np ? n : n & ~uint64_t(31);
    xs.stripes(e->close_buf[k & 1], whole);
    if (k + 1 == np) out->meta_hash = xs.finish(e->close_buf[k & 1] + whole, n - whole);
  }
  if (!np) out->meta_hash = xs.finish(nullptr, 0);
  static thread_local uint8_t t[25];
  trailer_bytes(out->data_bytes, out->meta_hash, t);
  OKV_HIP(hipMemcpyAsync(meta + out->meta_bytes, t, 25, hipMemcpyHostToDevice, ctx->stream));
  OKV_HIP(hipStreamSynchronize(ctx->stream));
  out->file_bytes = out->data_bytes + out->meta_bytes + 25;
  return OKV_OK;
}

void close_host(okv_encode_out* out) {
  uint8_t* meta = out->seg + out->data_bytes;
  out->meta_hash = okv_xxh64(meta, out->meta_bytes, 0);
  trailer_bytes(out->data_bytes, out->meta_hash, meta + out->meta_bytes);
  out->file_bytes = out->data_bytes + out->meta_bytes + 25;
}

}  // namespace
}  // namespace okv

// ===========================================================================
// C-ABI (include/okv_sst.h)
// ===========================================================================
using namespace okv;

extern "C" {

int okv_encode_rows(okv_ctx* ctx, const okv_rows* rows, const okv_encode_opts* opts,
                    okv_encode_out* out, uint32_t flags) {
  if (!ctx || !rows || !opts || !out) return OKV_E_ARG;
  out->n_blocks = out->data_bytes = out->meta_bytes = out->file_bytes = 0;
  out->meta_hash = 0;
  out->bad_row = kNone;
  if (opts->compression == OKV_COMP_ZSTD)
    return set_err(ctx, OKV_W_UNSUPPORTED, "zstd encode not implemented");
  if (opts->compression != OKV_COMP_NONE && opts->compression != OKV_COMP_LZ4)
    return set_err(ctx, OKV_E_ARG, "compression");
  if (opts->block_size == 0) return set_err(ctx, OKV_E_ARG, "block_size == 0");
  const uint64_t n = rows->n_rows;
  if (n == 0)  // Close with no open block: Go panics (Q1) or ErrNoRowsWritten (:221)
    return opts->strict_go ? set_err(ctx, OKV_W_NIL_WRITER, "Close on nil blockWriter (Q1)")
                           : set_err(ctx, OKV_W_NO_ROWS, "ErrNoRowsWritten");
  if (n >= (uint64_t(1) << 32) - kETile) return set_err(ctx, OKV_E_ARG, "n_rows >= 2^32");
  if (!rows->key_off || !rows->key_len || !rows->val_off || !rows->val_len ||
      (!rows->key_arena && rows->key_arena_bytes) || (!rows->val_arena && rows->val_arena_bytes))
    return set_err(ctx, OKV_E_ARG, "rows");
  OKV_HIP(hipSetDevice(ctx->device));
  EncScratch* e;
  int rc = enc_scratch(ctx, &e);
  if (rc) return rc;
  const bool dev = flags & OKV_F_DEVICE_PTRS;
  DevRows R;
  R.n = n;
  if (dev) {
    R.ka = rows->key_arena;
    R.ko = rows->key_off;
    R.kl = rows->key_len;
    R.va = rows->val_arena;
    R.vo = rows->val_off;
    R.vl = rows->val_len;
  } else {  // stage the host rows in one device buffer
    const auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    const size_t oka = 0, ova = oka + al(rows->key_arena_bytes),
                 oko = ova + al(rows->val_arena_bytes), okl = oko + al(n * 8),
                 ovo = okl + al(n * 2), ovl = ovo + al(n * 8), end = ovl + al(n * 4);
    if ((rc = grow(ctx, reinterpret_cast<void**>(&e->d_in), &e->cap_in, end + 64))) return rc;
    uint8_t* b = e->d_in;
    const hipMemcpyKind h2d = hipMemcpyHostToDevice;
    if (rows->key_arena_bytes)
      OKV_HIP(hipMemcpyAsync(b + oka, rows->key_arena, rows->key_arena_bytes, h2d, ctx->stream));
    if (rows->val_arena_bytes)
      OKV_HIP(hipMemcpyAsync(b + ova, rows->val_arena, rows->val_arena_bytes, h2d, ctx->stream));
    OKV_HIP(hipMemcpyAsync(b + oko, rows->key_off, n * 8, h2d, ctx->stream));
    OKV_HIP(hipMemcpyAsync(b + okl, rows->key_len, n * 2, h2d, ctx->stream));
    OKV_HIP(hipMemcpyAsync(b + ovo, rows->val_off, n * 8, h2d, ctx->stream));
    OKV_HIP(hipMemcpyAsync(b + ovl, rows->val_len, n * 4, h2d, ctx->stream));
    R.ka = b + oka;
    R.va = b + ova;
    R.ko = reinterpret_cast<const uint64_t*>(b + oko);
    R.kl = reinterpret_cast<const uint16_t*>(b + okl);
    R.vo = reinterpret_cast<const uint64_t*>(b + ovo);
    R.vl = reinterpret_cast<const uint32_t*>(b + ovl);
  }
  Plan pl;
  uint64_t bad = kNone;
  // the cut, sizes and offsets: E1-E9 (pointer doubling over chunks)
  bool general = true;
#ifdef OKV_ABLATE
  // A/B (OKV_ENC_ONEPASS=1): the single-pass plan kernel, falling back to E1-E9
  if (okv::knob("OKV_ENC_ONEPASS") && atoi(okv::knob("OKV_ENC_ONEPASS")))
    rc = enc_plan_fast(ctx, e, R, *opts, &pl, &bad, &general);
  else
#endif
    rc = OKV_OK, enc_mark(ctx, e, 0);
  if (!rc && general) rc = enc_plan(ctx, e, R, *opts, &pl, &bad);
  ctx->last_path = general ? 0u : OKV_PATH_ENC_ONEPASS;
  if (rc == OKV_W_INVALID_KEY) out->bad_row = bad;
  if (rc) return rc;
  out->n_blocks = pl.nb;
  out->data_bytes = pl.data_bytes;
  out->meta_bytes = pl.meta_bytes;
  out->file_bytes = pl.file_bytes;
  if (opts->strict_go && pl.last_raw >= opts->threshold_bytes)
    return set_err(ctx, OKV_W_NIL_WRITER, "Close on nil blockWriter (Q1): last row closed a block");
  const bool want_idx = out->blk_first_row || out->blk_desc || out->blk_hash;
  if (out->seg_cap < pl.file_bytes || (want_idx && out->blk_cap < pl.nb) || !out->seg)
    return set_err(ctx, OKV_E_CAPACITY, "encode output capacity too small (sizes set)");
  uint8_t* seg = out->seg;
  if (!dev) {
    if ((rc = grow(ctx, reinterpret_cast<void**>(&e->d_outseg), &e->cap_outseg,
                   pl.file_bytes + 64)))
      return rc;
    seg = e->d_outseg;
  }
  if ((rc = enc_write(ctx, e, R, *opts, pl, seg))) return rc;
  const hipMemcpyKind k = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  if (out->blk_first_row)
    OKV_HIP(hipMemcpyAsync(out->blk_first_row, e->first, (pl.nb + 1) * 8, k, ctx->stream));
  if (out->blk_desc)
    OKV_HIP(hipMemcpyAsync(out->blk_desc, e->desc, pl.nb * sizeof(Desc), k, ctx->stream));
  if (out->blk_hash)
    OKV_HIP(hipMemcpyAsync(out->blk_hash, e->hash, pl.nb * 8, k, ctx->stream));
  if (!dev) {
    OKV_HIP(hipMemcpyAsync(out->seg, seg, pl.data_bytes + pl.meta_bytes, k, ctx->stream));
    OKV_HIP(hipStreamSynchronize(ctx->stream));
    if (!(flags & OKV_F_NO_CLOSE)) close_host(out);
    return OKV_OK;
  }
  if (!(flags & OKV_F_NO_CLOSE)) return close_device(ctx, e, out);
  OKV_HIP(hipStreamSynchronize(ctx->stream));
  return OKV_OK;
}

int okv_encode_close(okv_ctx* ctx, okv_encode_out* out, uint32_t flags) {
  if (!ctx || !out || !out->seg || !out->meta_bytes) return OKV_E_ARG;
  if (out->seg_cap < out->data_bytes + out->meta_bytes + 25)
    return set_err(ctx, OKV_E_CAPACITY, "seg_cap");
  if (!(flags & OKV_F_DEVICE_PTRS)) {
    close_host(out);
    return OKV_OK;
  }
  OKV_HIP(hipSetDevice(ctx->device));
  EncScratch* e;
  int rc = enc_scratch(ctx, &e);
  if (rc) return rc;
  return close_device(ctx, e, out);
}

int okv_encode_profile_read(okv_ctx* ctx, double* ms, uint64_t* calls) {
  if (!ctx) return OKV_E_ARG;
  OKV_HIP(hipStreamSynchronize(ctx->stream));
  EncScratch* e = ctx->enc;
  if (e) {
    for (size_t i = 0; i + 5 <= e->ev_used; i += 5) {
      for (int k = 0; k < 4; ++k) {
        float t = 0.f;
        OKV_HIP(hipEventElapsedTime(&t, e->ev[i + k], e->ev[i + k + 1]));
        e->ms[k] += t;
      }
      e->calls++;
    }
    e->ev_used = 0;
  }
  for (int k = 0; k < 4; ++k) ms[k] = e ? e->ms[k] : 0.0;
  if (calls) *calls = e ? e->calls : 0;
  return OKV_OK;
}

int okv_encode_profile_reset(okv_ctx* ctx) {
  if (!ctx) return OKV_E_ARG;
  OKV_HIP(hipStreamSynchronize(ctx->stream));
  if (EncScratch* e = ctx->enc) {
    e->ev_used = 0;
    e->calls = 0;
    for (double& m : e->ms) m = 0;
  }
  return OKV_OK;
}

int okv_synth_rows_fixed(okv_ctx* ctx, uint64_t seed, uint64_t first_row, uint64_t n,
                         uint32_t key_len, uint32_t val_len, uint8_t* key_arena,
                         uint64_t* key_off, uint16_t* key_len_out, uint8_t* val_arena,
                         uint64_t* val_off, uint32_t* val_len_out) {
  if (!ctx || key_len > 65535 || !key_off || !key_len_out || !val_off || !val_len_out)
    return OKV_E_ARG;
  if (!n) return OKV_OK;
  OKV_HIP(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(okv_synth_fixed_kernel, dim3(ceil_div(n, kThreads)), dim3(kThreads), 0,
                     ctx->stream, seed, first_row, n, key_len, val_len, key_arena, key_off,
                     key_len_out, val_arena, val_off, val_len_out);
  OKV_HIP(hipGetLastError());
  OKV_HIP(hipStreamSynchronize(ctx->stream));
  return OKV_OK;
}

}  // extern "C"
