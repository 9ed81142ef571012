// okv_ctx.hpp -- the per-GPU context shared by the decode (okv_decode.hip)
// and encode (okv_encode.hip) translation units.  Internal header.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

#include "okv_kernels.hpp"
#include "okv_sst.h"

namespace okv {
struct EncScratch;  // okv_encode.hip
void enc_release(okv_ctx* ctx);
namespace mrg {
struct Scratch;  // okv_merge.hip
}
void merge_release(okv_ctx* ctx);
// okv_decode.hip: enqueue XXH64 of each block's BlockSize bytes (device pointers).
void launch_hash(hipStream_t stream, const uint8_t* seg, uint64_t seg_bytes, const Desc* descs,
                 uint32_t nblk, uint64_t* out);
// okv_zstd.hip: zstd block decompression into per-block scratch regions.
void launch_zstd_cap(hipStream_t s, const Desc* descs, uint32_t nblk, uint64_t* cap_off);
// total: in, the first regions' total (cap_off[nblk]); out, the scratch bytes
// in use after the frames that outgrew their regions were decoded again
int zstd_run(okv_ctx* ctx, const uint8_t* seg, uint64_t seg_bytes, const Desc* descs,
             uint32_t nblk, uint64_t* total);
void launch_zstd_desc(hipStream_t s, const Desc* descs, uint32_t nblk, const uint64_t* cap_off,
                      const uint64_t* dec_len, Desc* out);
constexpr uint32_t kZstdLitBytes = 1u << 17;  // per-wave literal scratch (Block_Maximum_Size)
}  // namespace okv

struct okv_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;
  // pass-1/2 scratch
  okv::BlockCount* d_cnt = nullptr;
  okv::Prefix* d_lp = nullptr;
  okv::Prefix* d_tile_tot = nullptr;
  okv::Prefix* d_tile_pre = nullptr;
  uint32_t* d_rec = nullptr;       // nblk x kRCap record positions (pass 1, rec_index)
  uint32_t* d_big = nullptr;       // big-block list [nblk]
  uint32_t* d_ctr = nullptr;       // [0] count-kernel arrivals, [1..2] big-block counter slots
  uint32_t big_slot = 0;           // slot the next launch counts big blocks in
  size_t cap_blocks = 0;
  // single-pass small-block decode (okv_decode_fused_kernel)
  bool fused = true;               // OKV_DECODE_FUSED=0: passes 1-3 as separate launches
  uint32_t fused_max = 0;          // largest fused batch: resident-capacity bound (okv_open)
  bool zstd_one_pass = false;      // OKV_OPEN_ZSTD_ONE_PASS: every zstd block by the general kernel
  bool point = true;               // host-mode point path (okv_point_kernel); OKV_OPEN_NO_POINT: off
  uint32_t* f_flag = nullptr;      // [nblk] look-back flags, tagged with f_epoch
  okv::Prefix* f_agg = nullptr;
  okv::Prefix* f_incl = nullptr;
  unsigned long long* f_ctr = nullptr;  // block-index counter, f_base at the next call
  unsigned long long f_base = 0;
  uint32_t f_epoch = 0;
  // grouped single-pass small-block decode (ablation build, OKV_DECODE_GROUP=1)
  bool group = false;
  uint32_t* g_flag = nullptr;      // [groups] look-back flags, tagged with g_epoch
  okv::Prefix* g_agg = nullptr;
  okv::Prefix* g_incl = nullptr;
  size_t g_cap = 0;
  uint32_t g_epoch = 0;
  uint32_t last_path = 0;          // OKV_PATH_* of the last decode (okv_last_path)
  // okv_decode_chain: this context's pass 3 waits for chain's last pass 3
  okv_ctx* chain = nullptr;
  std::vector<okv_ctx*> chained_by;  // contexts whose chain is this one (unchained at close)
  hipEvent_t p3_done = nullptr;    // recorded after every pass 3 once created
  bool p3_rec = false;             // p3_done has been recorded
  size_t f_cap = 0;
  okv::Totals* d_tot = nullptr;
  okv::Totals* h_tot = nullptr;  // pinned
  // the longest block walk of the last okv_decode_plan, for that batch's tile
  // pass (tile_geo); keyed by the batch's device inputs
  unsigned long long* d_span = nullptr;
  unsigned long long* h_span = nullptr;  // pinned
  okv::SpanHint span_hint;
  // ablation build (OKV_DECODE_PIECES=1): large-block decodes in two pieces,
  // the second piece's header walk on stream2 under the first's tile pass
  bool pieces = false;
  bool stream_lb = false;
  uint64_t small_piece = 0;   // ablation build (OKV_SMALL_PIECE_MB): small-block decodes in pieces
  void* d_ptot = nullptr;     // two Totals: the running prefix between pieces  // ablation build (OKV_DECODE_STREAM=1): okv_decode_stream_kernel
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_piece[2] = {nullptr, nullptr};
  okv::Totals* d_tot2 = nullptr;   // totals of the first piece
  // host-mode staging buffers (device side)
  uint8_t* d_seg = nullptr;
  size_t cap_seg = 0;
  okv::Desc* d_desc = nullptr;
  size_t cap_desc = 0;
  void* d_out = nullptr;
  size_t cap_out = 0;
  uint64_t* d_hash = nullptr;
  size_t cap_hash = 0;
  // host-mode point reads (okv_point_kernel): one pinned slab holding the
  // staged blocks, their descriptors and every output
  uint8_t* h_slab = nullptr;
  uint32_t point_seq = 0;          // point-kernel call number (its slab completion word)
  size_t cap_slab = 0;
  // per-pass event timing (okv_profile)
  uint32_t gather_grid = 0;  // 0: default grid; else workgroups (OKV_GATHER_GRID)
  uint32_t gather_threads = 0;  // 0: by average block size; else 64 or 256 (OKV_GATHER_THREADS)
  bool gather_staged = true;    // 256-thread pass 3 stages value spans in LDS (OKV_GATHER_STAGED=0: off)
  uint32_t value_sweep = 8;     // large blocks: 8 = okv_tile_kernel (source tiles); 0 = the
                                // per-block staged pass 3; 1/2/4 = okv_rows_kernel +
                                // okv_value_sweep_kernel with 1/2/4 tiles per workgroup,
                                // unaligned loads; 5/6/7 = 4/2/3 tiles, aligned loads and lane
                                // shuffles (OKV_VALUE_SWEEP)
  uint32_t tile_kib = 16;       // okv_tile_kernel tile bytes / 1024 (OKV_TILE)
  bool tile_xcd = true;         // consecutive tiles on one XCD
  uint32_t tile_threads = 256;  // okv_tile_kernel workgroup width
  uint32_t tile_diag = 0;       // diagnostic arms (1: no chunk pass, 2: no DMA)
  void* d_hdr = nullptr;        // [nblk x kRCap] pass-1 record key lengths (u16)
  size_t cap_hdr = 0;
  void* d_vsrc = nullptr;       // [row] value sources (sweep hand-off)
  size_t cap_vsrc = 0;
  void* d_vtile = nullptr;      // [value-arena tile] owning rows
  size_t cap_vtile = 0;
  bool prof = false;
  std::vector<hipEvent_t> ev;  // 5 per timed call
  size_t ev_used = 0;
  double prof_ms[4] = {0, 0, 0, 0};  // count, scan, gather, zstd stage
  uint64_t prof_calls = 0;
  okv::EncScratch* enc = nullptr;  // encode scratch (okv_encode.hip)
  okv::mrg::Scratch* merge = nullptr;  // merge scratch (okv_merge.hip)
  // zstd decompression scratch (okv_zstd.hip)
  uint64_t* z_cap_off = nullptr;  // [nblk + 1] decompressed-region offsets
  uint64_t* z_dec_len = nullptr;  // [nblk]
  int32_t* z_status = nullptr;    // [nblk]
  okv::Desc* z_desc = nullptr;    // [nblk] descriptors of the decompressed blocks
  size_t z_cap_blocks = 0;
  uint8_t* z_dec = nullptr;       // decompressed blocks
  size_t z_cap_dec = 0;
  uint8_t* z_lit = nullptr;       // per-wave literal scratch (general kernel)
  size_t z_cap_lit = 0;
  uint8_t* z_blit = nullptr;      // per-block literal scratch (prologue -> executor)
  size_t z_cap_blit = 0;
  uint32_t* z_tabs = nullptr;     // per-block FSE tables (prologue -> sequence stage)
  size_t z_cap_tabs = 0;         // (+ kHufSlot u16 per block: Huffman tables, prologue -> stream stage)
  hipEvent_t z_ev = nullptr;      // the sequence count's copy (zstd_run)
  void* z_zb = nullptr;           // per-block zst::ZBlk
  size_t z_cap_zb = 0;
  uint64_t* z_seq_off = nullptr;  // [nblk + 1] sequence offsets
  size_t z_cap_seq_off = 0;
  uint64_t* z_seqs = nullptr;     // packed sequences
  size_t z_cap_seqs = 0;
  uint32_t* z_list = nullptr;     // [nblk] blocks decoded again (+ the count after them)
  size_t z_cap_list = 0;
  uint64_t* z_need = nullptr;     // [n] measured outputs, [n + 1] their regions
  size_t z_cap_need = 0;
  uint32_t z_retried = 0;         // blocks the last zstd decode decoded again
};

namespace okv {

// A/B and diagnostic knobs: read from the environment in the ablation build
// only (-DOKV_ABLATE, libokv_sst_ablate.so); the product library never reads
// the environment, so its kernels do not change with a process's settings.
inline const char* knob(const char* name) {
#ifdef OKV_ABLATE
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

inline int set_err(okv_ctx* c, int code, const char* what, hipError_t e = hipSuccess) {
  if (c) {
    c->err = what;
    if (e != hipSuccess) {
      c->err += ": ";
      c->err += hipGetErrorString(e);
    }
  }
  return code;
}

#define OKV_HIP(call)                                             \
  do {                                                            \
    hipError_t e_ = (call);                                       \
    if (e_ != hipSuccess) return set_err(ctx, OKV_E_HIP, #call, e_); \
  } while (0)

inline int grow(okv_ctx* ctx, void** p, size_t* cap, size_t need) {
  if (need <= *cap && *p) return OKV_OK;
  if (*p) {
    OKV_HIP(hipStreamSynchronize(ctx->stream));
    OKV_HIP(hipFree(*p));
    *p = nullptr;
  }
  size_t c = std::max<size_t>(need, 4096);
  c = (c + 4095) & ~size_t(4095);
  OKV_HIP(hipMalloc(p, c));
  *cap = c;
  return OKV_OK;
}

}  // namespace okv
