/*
 * okv_sst.h -- C-ABI of the MI355X-native SST block decode path
 * (libokv_sst.so, objectkv_amd/csrc/).
 *
 * This is the drop-in boundary for ObjectKV's Go `sst` package
 * (danthegoodman1/ObjectKV @ 2025-03-21).  The reference has no FFI: its seam
 * is the Go method
 *     func (s *SegmentReader) ReadBlockWithStat(stat BlockStat) ([]KVPair, error)
 *     (sst/segment_reader.go:295-355)
 * called by RowIter.Next/Seek (sst/segment_row_iter.go:83, :143, :165),
 * GetRow (segment_reader.go:392) and GetRange (:458).  A cgo shim
 *  replaces that method's body -- and a batched
 * `ReadBlocks([]BlockStat)` used by RowIter and the compaction feed -- with
 * okv_decode_blocks() below.  Metadata parsing (FetchAndLoadMetadata,
 * BytesToMetadata, segment_reader.go:91-238) stays in the host caller; it
 * yields the okv_block_desc array.
 *
 * Plain pointers and sizes only.  All inputs and outputs are owned by the
 * caller; the library owns only its context (device, stream, scratch) and
 * retains no pointer after a call returns.  Contexts are not thread safe
 * (like the Go types, segment_writer.go:57): use one okv_ctx per (device,
 * goroutine/thread).
 */
#ifndef OKV_SST_H
#define OKV_SST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OKV_ABI_VERSION 1

/* ---- return codes (int) -------------------------------------------------- */
#define OKV_OK 0
#define OKV_E_ARG (-1)      /* bad argument (NULL, misaligned device pointer, ...) */
#define OKV_E_HIP (-2)      /* HIP runtime failure; okv_last_error() has the text */
#define OKV_E_CAPACITY (-3) /* outputs too small: totals in okv_decode_out are set */
#define OKV_E_NOMEM (-4)
#define OKV_E_NODEV (-5)    /* no GPU / bad device id */

/* ---- per-block status (okv_decode_out.blk_status) ---------------------- */
/* Mirrors what ReadBlockWithStat does for that block (segment_reader.go). */
#define OKV_BLK_OK 0
#define OKV_BLK_EOF 1         /* Seek/Read error: offset >= segment length (:303-313) -> Go error */
#define OKV_BLK_SHORT 2       /* short read, ErrUnexpectedBytesRead (:314-316) -> Go error */
#define OKV_BLK_PANIC 3       /* record overruns the block buffer: mustReadBytes panics (:338-352, :506-512) */
#define OKV_BLK_UNSUPPORTED 4 /* zstd block: not decoded on device yet (:320-330) */
#define OKV_BLK_CAPACITY 5    /* output capacity exceeded (library-specific; never a Go outcome) */

/* ---- compression byte of the meta block (segment_reader.go:166-172) ----- */
#define OKV_COMP_NONE 0
#define OKV_COMP_ZSTD 1
#define OKV_COMP_LZ4 2 /* reference quirk Q7: decodes as an empty buffer */

/* ---- flags ---------------------------------------------------------------- */
#define OKV_F_DEVICE_PTRS 1u /* seg, descs and every output pointer are device pointers */
#define OKV_F_INDEX_ONLY 2u  /* key_off/val_off are byte offsets into seg; no arenas written */
#define OKV_F_ASYNC 4u       /* with DEVICE_PTRS: enqueue on the ctx stream and return;
                                totals are NOT filled (call okv_decode_totals after okv_sync) */

/* One data-block index entry: BlockStat (sst/block_stat.go:9-24) without
 * FirstKey and Hash, which the decode does not need. */
typedef struct okv_block_desc {
  uint64_t offset;          /* BlockStat.Offset         */
  uint64_t block_size;      /* BlockStat.BlockSize      */
  uint64_t original_size;   /* BlockStat.OriginalSize   */
  uint64_t compressed_size; /* BlockStat.CompressedSize */
} okv_block_desc;

/*
 * Output of a batched decode, structure-of-arrays (DESIGN.md "Output layout").
 * Global row g of block b is row (g - row_start[b]) of ReadBlockWithStat(b),
 * in block order (callers reverse per block for DirectionDescending,
 * segment_row_iter.go:89-92).  Per row:
 *   key bytes   = key_arena[key_off[g] .. +key_len[g]]   (full decode)
 *               = seg[key_off[g] .. +key_len[g]]         (OKV_F_INDEX_ONLY)
 *   value bytes = val_arena[val_off[g] .. +val_len[g]]   (likewise)
 *   a length of 0 is Go's nil slice (Q4: readBytes returns nil, :490-493).
 * In full-decode mode each block's keys (values) are packed contiguously at
 * key_base[b] (val_base[b]); each block region is zero-padded to a multiple
 * of 16 bytes, so key_base/val_base are 16-byte aligned.
 * A block whose status is not OKV_BLK_OK contributes no rows and no bytes.
 */
typedef struct okv_decode_out {
  uint64_t *row_start; /* [nblk+1] exclusive scan of rows per block  */
  uint64_t *key_base;  /* [nblk]   (full decode; may be NULL)          */
  uint64_t *val_base;  /* [nblk]   (full decode; may be NULL)          */
  int32_t *blk_status; /* [nblk]   OKV_BLK_*                           */
  uint64_t *key_off;   /* [row_cap] */
  uint16_t *key_len;   /* [row_cap] */
  uint64_t *val_off;   /* [row_cap] */
  uint32_t *val_len;   /* [row_cap] */
  uint8_t *key_arena;  /* [key_cap] (full decode) */
  uint8_t *val_arena;  /* [val_cap] (full decode) */
  uint64_t row_cap, key_cap, val_cap;
  /* filled on return (synchronous calls): */
  uint64_t n_rows;        /* total rows */
  uint64_t key_bytes;     /* arena extent used (sum of 16-byte padded block regions) */
  uint64_t val_bytes;     /* likewise for values */
  uint64_t n_bad_blocks;  /* blocks whose status != OKV_BLK_OK */
} okv_decode_out;

typedef struct okv_ctx okv_ctx;

/* Context bound to one GPU (HIP device ordinal).  Creates its own stream
 * unless okv_open_on_stream is used (stream = a hipStream_t, opaque here). */
okv_ctx *okv_open(int device);
okv_ctx *okv_open_on_stream(int device, void *stream);
void okv_close(okv_ctx *ctx);
const char *okv_last_error(const okv_ctx *ctx);
void *okv_stream(const okv_ctx *ctx);
int okv_sync(okv_ctx *ctx);
int okv_abi_version(void);

/*
 * Size query (pass 1 + scan only): totals needed by okv_decode_blocks for
 * these blocks.  Same inputs and flags as okv_decode_blocks (ASYNC ignored).
 */
int okv_decode_plan(okv_ctx *ctx, const uint8_t *seg, uint64_t seg_bytes,
                    const okv_block_desc *descs, uint32_t nblk, int compression,
                    uint32_t flags, uint64_t *n_rows, uint64_t *key_bytes,
                    uint64_t *val_bytes);

/*
 * Batched ReadBlockWithStat over `nblk` blocks of one segment.
 *   seg/seg_bytes : the segment file bytes (what the io.ReadSeeker holds).
 *                   Device pointers must be 16-byte aligned; the kernels issue
 *                   only aligned loads that contain at least one byte of
 *                   [seg, seg+seg_bytes).
 *   compression   : the meta block's compression byte (OKV_COMP_*).
 * Returns OKV_OK, OKV_E_CAPACITY (totals set; nothing else is valid), or a
 * negative error.  Per-block outcomes are in out->blk_status.
 */
int okv_decode_blocks(okv_ctx *ctx, const uint8_t *seg, uint64_t seg_bytes,
                      const okv_block_desc *descs, uint32_t nblk, int compression,
                      okv_decode_out *out, uint32_t flags);

/* After an OKV_F_ASYNC decode and okv_sync(): copy the device totals into out. */
int okv_decode_totals(okv_ctx *ctx, okv_decode_out *out);

/* XXH64 (cespare/xxhash/v2 v2.2.0 semantics, seed 0 in the reference) of a
 * host buffer. */
uint64_t okv_xxh64(const void *data, size_t len, uint64_t seed);

/* Device XXH64 of each block's BlockSize bytes at its Offset -- the value the
 * writer stored in BlockStat.Hash (segment_writer.go:185).  hashes[nblk]. */
int okv_hash_blocks(okv_ctx *ctx, const uint8_t *seg, uint64_t seg_bytes,
                    const okv_block_desc *descs, uint32_t nblk, uint64_t *hashes,
                    uint32_t flags);

/* Per-kernel timing with HIP events recorded on the context stream around
 * each launch of okv_decode_blocks (pass 1 count, pass 2 scan, pass 3
 * copy/index).  okv_profile(ctx, 1) enables and resets; okv_profile_read
 * synchronises the stream and returns the summed milliseconds per pass
 * (ms[3]) and the number of decode calls timed. */
int okv_profile(okv_ctx *ctx, int enable);
int okv_profile_read(okv_ctx *ctx, double *ms, uint64_t *calls);

/* Device / pinned-host memory helpers for callers without another allocator. */
void *okv_device_alloc(okv_ctx *ctx, size_t bytes);
void okv_device_free(okv_ctx *ctx, void *p);
void *okv_host_alloc(size_t bytes); /* pinned (hipHostMalloc) */
void okv_host_free(void *p);
int okv_memcpy(okv_ctx *ctx, void *dst, const void *src, size_t bytes, int kind /*0 H2D, 1 D2H, 2 D2D*/);

#ifdef __cplusplus
}
#endif
#endif /* OKV_SST_H */
