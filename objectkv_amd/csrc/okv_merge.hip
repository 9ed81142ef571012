// okv_merge.hip -- device k-way merge of decoded segments: the loop of
// snapshot_reader.Reader.GetRange (/root/reference/snapshot_reader/
// snapshot_reader.go:214-372) and the same newest-wins merge as a compaction
// feed (the reference compactor is a stub, sst/compactor.go:3-6).
//
// Inputs are K streams, each a sorted row range of one decoded segment (the
// okv_decode_out SoA), in the snapshot's priority order (:235-254): among equal
// keys the lowest stream index owns the key (findMaxIndexes keeps the first
// index, :404-424).  The merge is computed, not iterated:
//   1. prefix: per row the first 16 key bytes (big-endian words) and the key's
//      address;
//   2. rank: a row's place in the merged multiset is its index in its stream
//      plus, per other stream, a binary-searched count of smaller keys (<= for
//      streams before it, < after it); it owns its key iff no earlier stream
//      holds the key;
//   3. scatter to merged order; 4. scan of owner flags -> unique keys;
//   5. per unique key (in iteration direction) the Go loop's outcome: skipped
//      tombstone, tombstone rolled onto io.EOF (error), range break, emit,
//      emit followed by the stale-cursor break or error (a stream that ran out
//      leaves its cursor on its last key, :351-365);
//   6. scan of emits, first terminating event (limit included), compaction.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "okv_ctx.hpp"
#include "okv_kernels.hpp"
#include "okv_sst.h"

namespace okv {

namespace mrg {

struct Src {  // == okv_merge_src
  const uint8_t* ka;
  const uint64_t* ko;
  const uint16_t* kl;
  const uint8_t* va;
  const uint64_t* vo;
  const uint32_t* vl;
  uint64_t lo, hi;
  int32_t level;
  int32_t pad;
};
static_assert(sizeof(Src) == sizeof(okv_merge_src), "okv_merge_src layout");

constexpr uint32_t kMaxSrc = 64;

// Go loop outcome per unique key
enum : uint8_t {
  kSkip = 0,       // L0 tombstone owner: rolled forward (:316-333)
  kErr = 1,        // ... and a stream ran out on it: Next() returns io.EOF -> error
  kBreak = 2,      // outside the range: break before it (:340-347)
  kEmit = 3,       // appended (:350-354)
  kEmitBreak = 4,  // appended; a stream ran out on it: the stale cursor ends the loop (:336-338)
  kEmitErr = 5,    // appended; the stale cursor's owner is an L0 tombstone: io.EOF error
};

// The first 16 key bytes as two big-endian words, zero padded: with the length
// as the tie-break, comparing these orders keys as bytes.Compare does, so keys
// of <= 16 bytes never touch the arenas.
struct Key16 {
  uint64_t a, b;
};

struct Scratch {
  uint64_t cap_rows = 0;
  uint64_t* kaddr = nullptr;  // [N] key address
  Key16* pfx = nullptr;       // [N] big-endian first 16 key bytes (zero padded)
  uint32_t* klen = nullptr;   // [N]
  uint64_t* pos = nullptr;    // [N] merged position
  uint8_t* own = nullptr;     // [N] owns its key
  uint64_t* mg = nullptr;     // [N] merged order -> global row
  uint32_t* mown = nullptr;   // [N + 1] owner flag in merged order, then its exclusive scan
  uint64_t* uniq = nullptr;   // [N] unique key -> owning global row
  uint8_t* ev = nullptr;      // [N] outcome per unique key, direction order
  uint32_t* escan = nullptr;  // [N + 1] emit flags, then their exclusive scan
  uint32_t cap_blk = 0;
  uint32_t* bsum = nullptr;   // scan block sums
  uint64_t* split = nullptr;  // [ceil(N / 256)][K][2] rank-kernel search windows
  size_t cap_split = 0;
  Src* d_src = nullptr;
  uint64_t* d_base = nullptr;  // [K + 1] stream offsets in the global row numbering
  uint8_t* d_bound = nullptr;
  size_t cap_bound = 0;
  uint64_t* d_misc = nullptr;  // [0] first termination, [1] its code, [2..] per-stream end key index
  uint64_t* h_misc = nullptr;  // pinned
};

__device__ __forceinline__ uint32_t find_src(const uint64_t* __restrict__ base, uint32_t k,
                                             uint64_t g) {
  uint32_t lo = 0, hi = k;  // largest i with base[i] <= g
  while (hi - lo > 1) {
    const uint32_t m = (lo + hi) >> 1;
    if (base[m] <= g)
      lo = m;
    else
      hi = m;
  }
  return lo;
}

// Key bytes [off, off + 8) as a big-endian word, bytes past len read as 0;
// the eight loads are independent (one memory round trip).
__device__ __forceinline__ uint64_t be_word(const uint8_t* k, uint32_t len, uint32_t off) {
  uint64_t p = 0;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) p = (p << 8) | (off + i < len ? uint64_t(k[off + i]) : 0ull);
  return p;
}

// The first 16 bytes from the aligned line(s) holding them (the second only
// when the key runs into it: a line holding a valid byte never crosses the
// allocation), bytes past len zeroed, then byte-swapped to big-endian words.
__device__ __forceinline__ Key16 be_prefix(const uint8_t* k, uint32_t len) {
  if (len == 0) return Key16{0, 0};
  const uintptr_t a = reinterpret_cast<uintptr_t>(k);
  const uint4* line = reinterpret_cast<const uint4*>(a & ~uintptr_t(15));
  const uint32_t sh = uint32_t(a & 15), n = len < 16 ? len : 16;
  const uint4 x = line[0];
  const uint4 y = sh + n > 16 ? line[1] : make_uint4(0, 0, 0, 0);
  uint4 v = funnel32(x, y, sh);
  v.x &= byte_mask(0, int32_t(n), 0);
  v.y &= byte_mask(0, int32_t(n), 1);
  v.z &= byte_mask(0, int32_t(n), 2);
  v.w &= byte_mask(0, int32_t(n), 3);
  return Key16{__builtin_bswap64(uint64_t(v.x) | (uint64_t(v.y) << 32)),
               __builtin_bswap64(uint64_t(v.z) | (uint64_t(v.w) << 32))};
}

// bytes.Compare of two keys given their prefixes, lengths and addresses.
__device__ __forceinline__ int key_cmp(const Key16& pa, uint32_t la, const uint8_t* ka,
                                       const Key16& pb, uint32_t lb, const uint8_t* kb) {
  if (pa.a != pb.a) return pa.a < pb.a ? -1 : 1;
  if (pa.b != pb.b) return pa.b < pb.b ? -1 : 1;
  const uint32_t m = la < lb ? la : lb;
  for (uint32_t i = 16; i < m; i += 8) {
    const uint64_t x = be_word(ka, la, i), y = be_word(kb, lb, i);
    if (x != y) return x < y ? -1 : 1;
  }
  return la < lb ? -1 : (la > lb ? 1 : 0);
}

}  // namespace mrg

// 1. per-row key prefix and address
__global__ __launch_bounds__(256) void okv_merge_pfx_kernel(const mrg::Src* __restrict__ src,
                                                            const uint64_t* __restrict__ base,
                                                            uint32_t k, uint64_t n,
                                                            uint64_t* __restrict__ kaddr,
                                                            mrg::Key16* __restrict__ pfx,
                                                            uint32_t* __restrict__ klen) {
  const uint64_t g = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const uint32_t i = mrg::find_src(base, k, g);
  const mrg::Src s = src[i];
  const uint64_t r = s.lo + (g - base[i]);
  const uint8_t* kp = s.ka + s.ko[r];
  const uint32_t l = s.kl[r];
  kaddr[g] = reinterpret_cast<uint64_t>(kp);
  klen[g] = l;
  pfx[g] = mrg::be_prefix(kp, l);
}

namespace mrg {
// First global row in [lo, hi) whose key is > key (le) or >= key (!le): the
// count of stream rows <= / < key, offset by the stream base.
__device__ __forceinline__ uint64_t rank_in(const Key16* __restrict__ pfx,
                                            const uint32_t* __restrict__ klen,
                                            const uint64_t* __restrict__ kaddr, uint64_t lo,
                                            uint64_t hi, const Key16& p0, uint32_t l0,
                                            const uint8_t* k0, bool le) {
  while (lo < hi) {
    const uint64_t m = (lo + hi) >> 1;
    const int c = key_cmp(pfx[m], klen[m], reinterpret_cast<const uint8_t*>(kaddr[m]), p0, l0, k0);
    if (c < 0 || (c == 0 && le))
      lo = m + 1;
    else
      hi = m;
  }
  return lo;
}
}  // namespace mrg

// 2. merged position and ownership of every row.  A row's rank in stream j
// is monotone along its own stream, so when a workgroup's rows all come from
// one stream the ranks of its first and last row bound every lane's search
// window in stream j.  Those windows (prefix, length, address per row) are
// staged in LDS when they fit, so the lanes' searches run at LDS latency;
// otherwise the searches read the windows from HBM / L2.
constexpr uint32_t kRankWin = 1024;  // staged window rows per workgroup (28 KiB)

// 2a. the windows: for every rank workgroup (256 rows) the ranks of its first
// and last row in every other stream, one full-range search per lane (the
// searches are independent, so they overlap instead of holding a workgroup).
__global__ __launch_bounds__(256) void okv_merge_split_kernel(
    const uint64_t* __restrict__ base, uint32_t k, uint64_t n, const uint64_t* __restrict__ kaddr,
    const mrg::Key16* __restrict__ pfx, const uint32_t* __restrict__ klen,
    uint64_t* __restrict__ split) {
  const uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t nwg = (n + 255) / 256;
  if (t >= nwg * 2 * k) return;
  const uint64_t wg = t / (2 * k);
  const uint32_t q = uint32_t(t % (2 * k)), j = q >> 1;
  const uint64_t g0 = wg * 256, g1 = (g0 + 256 < n ? g0 + 256 : n) - 1;
  const uint64_t ge = (q & 1) ? g1 : g0;
  const uint32_t i = mrg::find_src(base, k, ge);
  split[t] = j == i ? 0
                    : mrg::rank_in(pfx, klen, kaddr, base[j], base[j + 1], pfx[ge], klen[ge],
                                   reinterpret_cast<const uint8_t*>(kaddr[ge]), j < i);
}

__global__ __launch_bounds__(256) void okv_merge_rank_kernel(
    const uint64_t* __restrict__ base, uint32_t k, uint64_t n, const uint64_t* __restrict__ kaddr,
    const mrg::Key16* __restrict__ pfx, const uint32_t* __restrict__ klen,
    const uint64_t* __restrict__ split, int stage, uint64_t* __restrict__ pos,
    uint8_t* __restrict__ own) {
  __shared__ uint64_t s_lo[mrg::kMaxSrc], s_hi[mrg::kMaxSrc];
  __shared__ uint32_t w_at[mrg::kMaxSrc + 1];
  __shared__ mrg::Key16 w_pfx[kRankWin];
  __shared__ uint64_t w_addr[kRankWin];
  __shared__ uint32_t w_len[kRankWin];
  const uint64_t g0 = uint64_t(blockIdx.x) * blockDim.x;
  const uint64_t g1 = (g0 + blockDim.x < n ? g0 + blockDim.x : n) - 1;
  const uint32_t i0 = mrg::find_src(base, k, g0), i1 = mrg::find_src(base, k, g1);
  const bool one = i0 == i1;
  if (one) {
    for (uint32_t t = threadIdx.x; t < 2 * k; t += blockDim.x) {
      const uint64_t r = split[uint64_t(blockIdx.x) * 2 * k + t];
      if (t & 1)
        s_hi[t >> 1] = r;
      else
        s_lo[t >> 1] = r;
    }
  }
  __syncthreads();
  bool staged = false;
  if (one && stage) {
    if (threadIdx.x == 0) {
      uint64_t tot = 0;
      for (uint32_t j = 0; j < k; ++j) {
        w_at[j] = uint32_t(tot < kRankWin ? tot : kRankWin);
        tot += s_hi[j] - s_lo[j];
      }
      w_at[k] = uint32_t(tot <= kRankWin ? tot : kRankWin + 1);  // > kRankWin: not staged
    }
    __syncthreads();
    staged = w_at[k] <= kRankWin;
    if (staged) {
      for (uint32_t j = 0; j < k; ++j) {
        const uint64_t lo = s_lo[j];
        const uint32_t w = uint32_t(s_hi[j] - lo), o = w_at[j];
        for (uint32_t t = threadIdx.x; t < w; t += blockDim.x) {
          w_pfx[o + t] = pfx[lo + t];
          w_len[o + t] = klen[lo + t];
          w_addr[o + t] = kaddr[lo + t];
        }
      }
    }
    __syncthreads();
  }
  const uint64_t g = g0 + threadIdx.x;
  if (g >= n) return;
  const uint32_t i = one ? i0 : mrg::find_src(base, k, g);
  const mrg::Key16 p0 = pfx[g];
  const uint32_t l0 = klen[g];
  const uint8_t* k0 = reinterpret_cast<const uint8_t*>(kaddr[g]);
  uint64_t rank = g - base[i];
  uint8_t owner = 1;
  for (uint32_t j = 0; j < k; ++j) {
    if (j == i) continue;
    const bool le = j < i;  // earlier streams own ties: count keys <= key
    uint64_t r;
    if (staged) {
      const uint32_t o = w_at[j];
      uint32_t lo = 0, hi = uint32_t(s_hi[j] - s_lo[j]);
      while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        const int c = mrg::key_cmp(w_pfx[o + m], w_len[o + m],
                                   reinterpret_cast<const uint8_t*>(w_addr[o + m]), p0, l0, k0);
        if (c < 0 || (c == 0 && le))
          lo = m + 1;
        else
          hi = m;
      }
      r = s_lo[j] + lo;
      // an earlier stream holding the key owns it: its row r - 1 equals the key
      if (le && r > base[j]) {
        const bool in = lo > 0;
        const int c = in ? mrg::key_cmp(w_pfx[o + lo - 1], w_len[o + lo - 1],
                                        reinterpret_cast<const uint8_t*>(w_addr[o + lo - 1]), p0,
                                        l0, k0)
                         : mrg::key_cmp(pfx[r - 1], klen[r - 1],
                                        reinterpret_cast<const uint8_t*>(kaddr[r - 1]), p0, l0, k0);
        if (c == 0) owner = 0;
      }
    } else {
      const uint64_t lo = one ? s_lo[j] : base[j], hi = one ? s_hi[j] : base[j + 1];
      r = mrg::rank_in(pfx, klen, kaddr, lo, hi, p0, l0, k0, le);
      if (le && r > base[j] &&
          mrg::key_cmp(pfx[r - 1], klen[r - 1], reinterpret_cast<const uint8_t*>(kaddr[r - 1]),
                       p0, l0, k0) == 0)
        owner = 0;
    }
    rank += r - base[j];
  }
  pos[g] = rank;
  own[g] = owner;
}

// 3. scatter into merged order
__global__ __launch_bounds__(256) void okv_merge_scatter_kernel(uint64_t n,
                                                                const uint64_t* __restrict__ pos,
                                                                const uint8_t* __restrict__ own,
                                                                uint64_t* __restrict__ mg,
                                                                uint32_t* __restrict__ mown) {
  const uint64_t g = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const uint64_t p = pos[g];
  mg[p] = g;
  mown[p] = own[g];
}

// Exclusive scan of u32 flags in place (three launches: block scans of 4096,
// one workgroup over the block sums, add).
__global__ __launch_bounds__(1024) void okv_mscan_block_kernel(uint32_t* __restrict__ x, uint64_t n,
                                                               uint32_t* __restrict__ bsum) {
  __shared__ uint32_t ws[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t b0 = uint64_t(blockIdx.x) * 4096 + uint64_t(threadIdx.x) * 4;
  uint32_t v[4], t = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    v[u] = b0 + u < n ? x[b0 + u] : 0;
    t += v[u];
  }
  const uint32_t inc = wave_incl_scan32(t, lane);
  if (lane == 63) ws[wave] = inc;
  __syncthreads();
  uint32_t before = 0, tot = 0;
  for (int w = 0; w < 16; ++w) {
    before += w < wave ? ws[w] : 0;
    tot += ws[w];
  }
  uint32_t run = before + inc - t;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    if (b0 + u < n) x[b0 + u] = run;
    run += v[u];
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}
__global__ __launch_bounds__(1024) void okv_mscan_sums_kernel(uint32_t* __restrict__ bsum,
                                                              uint32_t nb,
                                                              uint32_t* __restrict__ total) {
  __shared__ uint32_t ws[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {
    const uint32_t i = b0 + threadIdx.x;
    const uint32_t v = i < nb ? bsum[i] : 0;
    const uint32_t inc = wave_incl_scan32(v, lane);
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint32_t before = 0, tot = 0;
    for (int w = 0; w < 16; ++w) {
      before += w < wave ? ws[w] : 0;
      tot += ws[w];
    }
    if (i < nb) bsum[i] = carry + before + inc - v;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}
__global__ __launch_bounds__(1024) void okv_mscan_add_kernel(uint32_t* __restrict__ x, uint64_t n,
                                                             const uint32_t* __restrict__ bsum) {
  const uint64_t b0 = uint64_t(blockIdx.x) * 4096 + uint64_t(threadIdx.x) * 4;
  const uint32_t add = bsum[blockIdx.x];
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (b0 + u < n) x[b0 + u] += add;
}

// 4. unique keys: owners in merged order; mown holds the exclusive scan and the
// flag is re-derived from the scan step (flag = scan[p + 1] - scan[p]).
__global__ __launch_bounds__(256) void okv_merge_uniq_kernel(uint64_t n,
                                                             const uint32_t* __restrict__ mscan,
                                                             const uint64_t* __restrict__ mg,
                                                             uint64_t* __restrict__ uniq) {
  const uint64_t p = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (p >= n) return;
  if (mscan[p + 1] != mscan[p]) uniq[mscan[p]] = mg[p];
}

// Per stream: the unique-key index of its last row in iteration direction.
__global__ void okv_merge_ends_kernel(const uint64_t* __restrict__ base, uint32_t k, int dir,
                                      const uint64_t* __restrict__ pos,
                                      const uint32_t* __restrict__ mscan,
                                      uint64_t* __restrict__ ends) {
  const uint32_t j = threadIdx.x;
  if (j >= k) return;
  if (base[j + 1] == base[j]) {
    ends[j] = ~0ull;
    return;
  }
  const uint64_t g = dir == OKV_DIR_DESC ? base[j] : base[j + 1] - 1;
  const uint64_t p = pos[g];
  // the key's owner is the first row of its run in merged order
  ends[j] = uint64_t(mscan[p + 1]) - 1;
}

// 5. the Go loop's outcome per unique key, in direction order
__global__ __launch_bounds__(256) void okv_merge_event_kernel(
    const mrg::Src* __restrict__ src, const uint64_t* __restrict__ base, uint32_t k, uint64_t nu,
    int dir, int mode, int drop_tomb, const uint64_t* __restrict__ uniq,
    const uint64_t* __restrict__ kaddr, const mrg::Key16* __restrict__ pfx,
    const uint32_t* __restrict__ klen, const uint8_t* __restrict__ bound, uint32_t bound_len,
    const uint64_t* __restrict__ ends, uint8_t* __restrict__ ev, uint32_t* __restrict__ emit) {
  const uint64_t d = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (d >= nu) return;
  const uint64_t u = dir == OKV_DIR_DESC ? nu - 1 - d : d;
  const uint64_t g = uniq[u];
  const uint32_t i = mrg::find_src(base, k, g);
  const mrg::Src s = src[i];
  const uint64_t r = s.lo + (g - base[i]);
  const bool tomb = s.level == 0 && s.vl[r] == 0;
  uint8_t e;
  if (mode == OKV_MERGE_ALL) {
    e = (tomb && drop_tomb) ? mrg::kSkip : mrg::kEmit;
  } else {
    // streams that run out on this key; the lowest index is the stale owner
    bool end_here = false;
    uint32_t jmin = k;
    for (uint32_t j = 0; j < k; ++j)
      if (ends[j] == u) {
        end_here = true;
        jmin = j < jmin ? j : jmin;
      }
    if (tomb) {
      e = end_here ? mrg::kErr : mrg::kSkip;
    } else {
      const uint8_t* kp = reinterpret_cast<const uint8_t*>(kaddr[g]);
      const mrg::Key16 bp = mrg::be_prefix(bound, bound_len);
      const int c = mrg::key_cmp(pfx[g], klen[g], kp, bp, bound_len, bound);
      const bool out = dir == OKV_DIR_DESC ? c <= 0 : c >= 0;
      if (out) {
        e = mrg::kBreak;
      } else if (!end_here) {
        e = mrg::kEmit;
      } else {
        // the stale cursor of stream jmin sits on this key: its row is the
        // stream's last in direction
        const mrg::Src t = src[jmin];
        const uint64_t rj = dir == OKV_DIR_DESC ? t.lo : t.hi - 1;
        e = (t.level == 0 && t.vl[rj] == 0) ? mrg::kEmitErr : mrg::kEmitBreak;
      }
    }
  }
  ev[d] = e;
  emit[d] = e >= mrg::kEmit ? 1u : 0u;
}

// 6a. first terminating position (GetRange mode): misc[0] = atomicMin of
// (position << 3 | code) where code 1 = stop after (OK), 2 = stop after with
// error, 5 = error before, 6 = break before; limit stops after the limit-th
// emit.  A stop after key d and an event before key d + 1 share a position;
// the stop comes first in the Go loop, so its codes are the smaller.
__global__ __launch_bounds__(256) void okv_merge_term_kernel(uint64_t nu,
                                                             const uint8_t* __restrict__ ev,
                                                             const uint32_t* __restrict__ escan,
                                                             uint64_t limit,
                                                             unsigned long long* __restrict__ misc) {
  const uint64_t d = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (d >= nu) return;
  const uint8_t e = ev[d];
  unsigned long long key = ~0ull;
  if (e == mrg::kErr) {
    key = (unsigned long long)(d) << 3 | 5;
  } else if (e == mrg::kBreak) {
    key = (unsigned long long)(d) << 3 | 6;
  } else if (e >= mrg::kEmit) {
    const uint64_t cnt = uint64_t(escan[d]) + 1;  // emits through d
    if (cnt == limit || e == mrg::kEmitBreak)
      key = (unsigned long long)(d + 1) << 3 | 1;
    else if (e == mrg::kEmitErr)
      key = (unsigned long long)(d + 1) << 3 | 2;
  }
  if (key != ~0ull) atomicMin(misc, key);
}

// 6b. output rows: emits before the termination, in direction order
__global__ __launch_bounds__(256) void okv_merge_out_kernel(
    const mrg::Src* __restrict__ src, const uint64_t* __restrict__ base, uint32_t k, uint64_t nu,
    int dir, const uint64_t* __restrict__ uniq, const uint8_t* __restrict__ ev,
    const uint32_t* __restrict__ escan, uint64_t stop, uint64_t row_cap, uint32_t* __restrict__ osrc,
    uint64_t* __restrict__ orow, uint64_t* __restrict__ okoff, uint16_t* __restrict__ oklen,
    uint64_t* __restrict__ ovoff, uint32_t* __restrict__ ovlen, const uint8_t* kbase,
    const uint8_t* vbase) {
  const uint64_t d = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (d >= nu || d >= stop || ev[d] < mrg::kEmit) return;
  const uint64_t o = escan[d];
  if (o >= row_cap) return;
  const uint64_t u = dir == OKV_DIR_DESC ? nu - 1 - d : d;
  const uint64_t g = uniq[u];
  const uint32_t i = mrg::find_src(base, k, g);
  const mrg::Src s = src[i];
  const uint64_t r = s.lo + (g - base[i]);
  if (osrc) osrc[o] = i;
  if (orow) orow[o] = r;
  if (okoff) okoff[o] = uint64_t(s.ka - kbase) + s.ko[r];
  if (oklen) oklen[o] = s.kl[r];
  if (ovoff) ovoff[o] = uint64_t(s.va - vbase) + s.vo[r];
  if (ovlen) ovlen[o] = s.vl[r];
}

namespace {

int scan_u32(okv_ctx* ctx, mrg::Scratch* m, uint32_t* x, uint64_t n, uint32_t* total) {
  const uint32_t nb = uint32_t((n + 4095) / 4096);
  if (nb > m->cap_blk) {
    OKV_HIP(hipStreamSynchronize(ctx->stream));
    (void)hipFree(m->bsum);
    OKV_HIP(hipMalloc(&m->bsum, (size_t(nb) + 1) * 4));
    m->cap_blk = nb;
  }
  if (nb) {
    hipLaunchKernelGGL(okv_mscan_block_kernel, dim3(nb), dim3(1024), 0, ctx->stream, x, n,
                       m->bsum);
    hipLaunchKernelGGL(okv_mscan_sums_kernel, dim3(1), dim3(1024), 0, ctx->stream, m->bsum, nb,
                       total);
    hipLaunchKernelGGL(okv_mscan_add_kernel, dim3(nb), dim3(1024), 0, ctx->stream, x, n, m->bsum);
  } else {
    OKV_HIP(hipMemsetAsync(total, 0, 4, ctx->stream));
  }
  return OKV_OK;
}

int ensure(okv_ctx* ctx, mrg::Scratch* m, uint64_t n) {
  if (!m->d_src) {
    OKV_HIP(hipMalloc(&m->d_src, sizeof(mrg::Src) * mrg::kMaxSrc));
    OKV_HIP(hipMalloc(&m->d_base, 8 * (mrg::kMaxSrc + 1)));
    OKV_HIP(hipMalloc(&m->d_misc, 8 * (mrg::kMaxSrc + 8)));
    OKV_HIP(hipHostMalloc(&m->h_misc, 8 * (mrg::kMaxSrc + 8)));
  }
  if (n <= m->cap_rows && m->kaddr) return OKV_OK;
  OKV_HIP(hipStreamSynchronize(ctx->stream));
  void** ps[] = {reinterpret_cast<void**>(&m->kaddr), reinterpret_cast<void**>(&m->pfx),
                 reinterpret_cast<void**>(&m->klen),  reinterpret_cast<void**>(&m->pos),
                 reinterpret_cast<void**>(&m->own),   reinterpret_cast<void**>(&m->mg),
                 reinterpret_cast<void**>(&m->mown),  reinterpret_cast<void**>(&m->uniq),
                 reinterpret_cast<void**>(&m->ev),    reinterpret_cast<void**>(&m->escan)};
  const size_t sz[] = {8, sizeof(mrg::Key16), 4, 8, 1, 8, 4, 8, 1, 4};
  const uint64_t c = std::max<uint64_t>(n + n / 8, 4096);
  for (int q = 0; q < 10; ++q) {
    (void)hipFree(*ps[q]);
    *ps[q] = nullptr;
    OKV_HIP(hipMalloc(ps[q], sz[q] * (c + 16)));
  }
  m->cap_rows = c;
  return OKV_OK;
}

}  // namespace

void merge_release(okv_ctx* ctx) {
  mrg::Scratch* m = ctx->merge;
  if (!m) return;
  for (void* p : {static_cast<void*>(m->kaddr), static_cast<void*>(m->pfx),
                  static_cast<void*>(m->klen), static_cast<void*>(m->pos),
                  static_cast<void*>(m->own), static_cast<void*>(m->mg),
                  static_cast<void*>(m->mown), static_cast<void*>(m->uniq),
                  static_cast<void*>(m->ev), static_cast<void*>(m->escan),
                  static_cast<void*>(m->bsum), static_cast<void*>(m->split),
                  static_cast<void*>(m->d_src),
                  static_cast<void*>(m->d_base), static_cast<void*>(m->d_bound),
                  static_cast<void*>(m->d_misc)})
    (void)hipFree(p);
  if (m->h_misc) (void)hipHostFree(m->h_misc);
  delete m;
  ctx->merge = nullptr;
}

}  // namespace okv

using namespace okv;

extern "C" {

int okv_merge_rows(okv_ctx* ctx, const okv_merge_src* srcs, uint32_t nsrc,
                   const okv_merge_opts* opts, okv_merge_out* out, uint32_t flags) {
  if (!ctx || !opts || !out || (!srcs && nsrc) || nsrc > mrg::kMaxSrc) return OKV_E_ARG;
  if (!(flags & OKV_F_DEVICE_PTRS)) return OKV_E_ARG;  // sources are decoded device SoA
  if (opts->direction != OKV_DIR_ASC && opts->direction != OKV_DIR_DESC) return OKV_E_ARG;
  if (opts->mode != OKV_MERGE_GETRANGE && opts->mode != OKV_MERGE_ALL) return OKV_E_ARG;
  if (opts->mode == OKV_MERGE_GETRANGE && (opts->limit == 0 || (!opts->bound && opts->bound_len)))
    return OKV_E_ARG;
  OKV_HIP(hipSetDevice(ctx->device));
  if (!ctx->merge) ctx->merge = new mrg::Scratch();
  mrg::Scratch* m = ctx->merge;
  std::vector<uint64_t> base(nsrc + 1, 0);
  for (uint32_t i = 0; i < nsrc; ++i) {
    if (srcs[i].row_hi < srcs[i].row_lo) return OKV_E_ARG;
    base[i + 1] = base[i] + (srcs[i].row_hi - srcs[i].row_lo);
  }
  const uint64_t n = base[nsrc];
  if (n >= (1ull << 32) - 2) return OKV_E_ARG;  // u32 scans
  int rc;
  if ((rc = ensure(ctx, m, n))) return rc;
  hipStream_t s = ctx->stream;
  if (nsrc) {
    OKV_HIP(hipMemcpyAsync(m->d_src, srcs, sizeof(mrg::Src) * nsrc, hipMemcpyHostToDevice, s));
    OKV_HIP(hipMemcpyAsync(m->d_base, base.data(), 8 * (nsrc + 1), hipMemcpyHostToDevice, s));
  }
  const uint32_t blen = opts->mode == OKV_MERGE_GETRANGE ? uint32_t(opts->bound_len) : 0;
  if (opts->bound_len > 0xffff) return OKV_E_ARG;  // keys are at most 65535 bytes
  if ((rc = grow(ctx, reinterpret_cast<void**>(&m->d_bound), &m->cap_bound, blen + 16))) return rc;
  if (blen) OKV_HIP(hipMemcpyAsync(m->d_bound, opts->bound, blen, hipMemcpyHostToDevice, s));
  const dim3 b256(256);
  const dim3 gn(uint32_t((n + 255) / 256));
  out->n_rows = 0;
  out->n_unique = 0;
  out->status = 0;
  if (n == 0) return OKV_OK;
  hipLaunchKernelGGL(okv_merge_pfx_kernel, gn, b256, 0, s, m->d_src, m->d_base, nsrc, n, m->kaddr,
                     m->pfx, m->klen);
  if ((rc = grow(ctx, reinterpret_cast<void**>(&m->split), &m->cap_split,
                 8 * 2 * nsrc * ((n + 255) / 256))))
    return rc;
  {
    const uint64_t ns = 2 * nsrc * ((n + 255) / 256);
    hipLaunchKernelGGL(okv_merge_split_kernel, dim3(uint32_t((ns + 255) / 256)), b256, 0, s,
                       m->d_base, nsrc, n, m->kaddr, m->pfx, m->klen, m->split);
  }
  static const int stage = [] {
    const char* e = okv::knob("OKV_MERGE_STAGE");  // A/B knob: 0 = windows searched in HBM / L2
    return e ? atoi(e) : 1;
  }();
  hipLaunchKernelGGL(okv_merge_rank_kernel, gn, b256, 0, s, m->d_base, nsrc, n, m->kaddr, m->pfx,
                     m->klen, m->split, stage, m->pos, m->own);
  hipLaunchKernelGGL(okv_merge_scatter_kernel, gn, b256, 0, s, n, m->pos, m->own, m->mg, m->mown);
  OKV_HIP(hipMemsetAsync(m->mown + n, 0, 4, s));
  uint32_t* d_tot = reinterpret_cast<uint32_t*>(m->d_misc + 2 + mrg::kMaxSrc);
  if ((rc = scan_u32(ctx, m, m->mown, n + 1, d_tot))) return rc;  // mown[n] = 0 pad -> total
  hipLaunchKernelGGL(okv_merge_uniq_kernel, gn, b256, 0, s, n, m->mown, m->mg, m->uniq);
  hipLaunchKernelGGL(okv_merge_ends_kernel, dim3(1), dim3(64), 0, s, m->d_base, nsrc,
                     opts->direction, m->pos, m->mown, m->d_misc + 2);
  OKV_HIP(hipMemcpyAsync(m->h_misc, d_tot, 4, hipMemcpyDeviceToHost, s));
  OKV_HIP(hipStreamSynchronize(s));
  const uint64_t nu = *reinterpret_cast<uint32_t*>(m->h_misc);
  out->n_unique = nu;
  const dim3 gu(uint32_t((nu + 255) / 256));
  hipLaunchKernelGGL(okv_merge_event_kernel, gu, b256, 0, s, m->d_src, m->d_base, nsrc, nu,
                     opts->direction, opts->mode, opts->drop_tombstones, m->uniq, m->kaddr,
                     m->pfx, m->klen, m->d_bound, blen, m->d_misc + 2, m->ev, m->escan);
  OKV_HIP(hipMemsetAsync(m->escan + nu, 0, 4, s));
  uint32_t* d_etot = d_tot + 1;
  if ((rc = scan_u32(ctx, m, m->escan, nu + 1, d_etot))) return rc;
  uint64_t stop = nu;
  int32_t status = 0;
  if (opts->mode == OKV_MERGE_GETRANGE) {
    OKV_HIP(hipMemsetAsync(m->d_misc, 0xff, 8, s));
    hipLaunchKernelGGL(okv_merge_term_kernel, gu, b256, 0, s, nu, m->ev, m->escan, opts->limit,
                       reinterpret_cast<unsigned long long*>(m->d_misc));
    OKV_HIP(hipMemcpyAsync(m->h_misc, m->d_misc, 8, hipMemcpyDeviceToHost, s));
    OKV_HIP(hipStreamSynchronize(s));
    const uint64_t t = m->h_misc[0];
    if (t != ~0ull) {
      stop = t >> 3;
      const uint32_t code = uint32_t(t & 7);
      if (code == 2 || code == 5) status = OKV_M_EOF;
    }
  }
  // rows emitted before stop = escan[stop]
  OKV_HIP(hipMemcpyAsync(m->h_misc, m->escan + stop, 4, hipMemcpyDeviceToHost, s));
  OKV_HIP(hipStreamSynchronize(s));
  const uint64_t nrows = *reinterpret_cast<uint32_t*>(m->h_misc);
  out->n_rows = nrows;
  out->status = status;
  if (status) return OKV_OK;  // Go returns (nil, err): no rows
  if (nrows > out->row_cap) return OKV_E_CAPACITY;
  if (nrows)
    hipLaunchKernelGGL(okv_merge_out_kernel, gu, b256, 0, s, m->d_src, m->d_base, nsrc, nu,
                       opts->direction, m->uniq, m->ev, m->escan, stop, out->row_cap, out->src,
                       out->row, out->key_off, out->key_len, out->val_off, out->val_len,
                       out->key_base, out->val_base);
  OKV_HIP(hipGetLastError());
  if (!(flags & OKV_F_ASYNC)) OKV_HIP(hipStreamSynchronize(s));
  return OKV_OK;
}

}  // extern "C"
