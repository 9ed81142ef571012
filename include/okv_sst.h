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

#define OKV_ABI_VERSION 6 /* 2: okv_encode_opts.bloom / bloom_len, and okv_profile_read writes
                             4 doubles (ms[4]: the zstd stage slot was added);
                             3: okv_open_ex / okv_open_opts
                             4: okv_decode_chain
                             5: OKV_OPEN_NO_POINT / OKV_PATH_POINT (host-mode point path)
                             6: okv_point_get (GetRow's block step, one row back) */

/* ---- return codes (int) -------------------------------------------------- */
#define OKV_OK 0
#define OKV_E_ARG (-1)      /* bad argument (NULL, misaligned device pointer, ...) */
#define OKV_E_HIP (-2)      /* HIP runtime failure; okv_last_error() has the text */
#define OKV_E_CAPACITY (-3) /* outputs too small: totals in okv_decode_out are set */
#define OKV_E_NOMEM (-4)
#define OKV_E_NODEV (-5)    /* no GPU / bad device id */

/* Go SegmentWriter sentinels returned by the encode (values shared with
 * okv_host.h and the test oracle; segment_writer.go:69-74) */
#define OKV_W_KEY_TOO_LARGE (-101)   /* ErrKeyTooLarge */
#define OKV_W_VALUE_TOO_LARGE (-102) /* ErrValueTooLarge */
#define OKV_W_CLOSED (-103)          /* ErrWriterClosed */
#define OKV_W_INVALID_KEY (-104)     /* ErrInvalidKey: empty key (WriteRow :89-91) */
#define OKV_W_NIL_WRITER (-105)      /* Go panics in Close when no block is open (:212, Q1) */
#define OKV_W_UNSUPPORTED (-106)     /* zstd level > 0: encoder not implemented */
#define OKV_W_NO_ROWS (-107)         /* ErrNoRowsWritten (:221-223) */

/* ---- per-block status (okv_decode_out.blk_status) ---------------------- */
/* Mirrors what ReadBlockWithStat does for that block (segment_reader.go). */
#define OKV_BLK_OK 0
#define OKV_BLK_EOF 1         /* Seek/Read error: offset >= segment length (:303-313) -> Go error */
#define OKV_BLK_SHORT 2       /* short read, ErrUnexpectedBytesRead (:314-316) -> Go error */
#define OKV_BLK_PANIC 3       /* record overruns the block buffer: mustReadBytes panics (:338-352, :506-512) */
#define OKV_BLK_UNSUPPORTED 4 /* zstd block under OKV_F_INDEX_ONLY (no spans into seg exist) */
#define OKV_BLK_CAPACITY 5    /* the caller's output capacity (row_cap / key_cap / val_cap) is
                                 exceeded (library-specific; never with okv_decode_plan sizes) */
#define OKV_BLK_ZSTD_ERROR 6  /* zstd.NewReader / io.Copy error (:321-330) -> Go error */

/* ---- compression byte of the meta block (segment_reader.go:166-172) ----- */
#define OKV_COMP_NONE 0
#define OKV_COMP_ZSTD 1 /* decoded on the device (okv_zstd.hip); not with OKV_F_INDEX_ONLY */
#define OKV_COMP_LZ4 2 /* reference quirk Q7: decodes as an empty buffer */

/* ---- flags ---------------------------------------------------------------- */
#define OKV_F_DEVICE_PTRS 1u /* seg, descs and every output pointer are device pointers */
#define OKV_F_INDEX_ONLY 2u  /* key_off/val_off are byte offsets into seg; no arenas written */
#define OKV_F_ASYNC 4u       /* with DEVICE_PTRS: enqueue on the ctx stream and return;
                                totals are NOT filled (call okv_decode_totals after okv_sync) */
#define OKV_F_NO_CLOSE 8u    /* encode: stop after blocks + block index + meta block; the
                                meta XXH64 and the 25-byte trailer are left to okv_encode_close */

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

/* Context options (okv_open_ex).  The library reads no environment variables:
 * every choice a caller can make is here. */
#define OKV_OPEN_NO_FUSED 1u      /* batches of <= 512 small blocks: three launches (count, scan,
                                     gather) instead of the single-pass kernel, whose workgroups
                                     wait for each other -- for devices whose compute slots other
                                     work may hold; the outputs are identical */
#define OKV_OPEN_ZSTD_ONE_PASS 2u /* zstd blocks: the one-wave-per-block decoder for every block
                                     (one launch, no host synchronisation between stages: lower
                                     latency for a few blocks); outputs identical */
#define OKV_OPEN_NO_POINT 4u      /* host-mode calls never take the point path (okv_point_kernel:
                                     <= 16 small uncompressed blocks in one launch over pinned
                                     memory): every batch is staged to device memory and decoded
                                     by the device-resident kernels; outputs identical */
typedef struct okv_open_opts {
  uint32_t size;  /* sizeof(okv_open_opts) */
  uint32_t flags; /* OKV_OPEN_* */
} okv_open_opts;
/* stream may be NULL (the context creates its own); opts may be NULL (defaults). */
okv_ctx *okv_open_ex(int device, void *stream, const okv_open_opts *opts);
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

/*
 * Consecutive-segment pipelining (a reader decoding segment after segment: a
 * compaction feed, a scan over a level).  After okv_decode_chain(ctx, after),
 * every decode on ctx starts its pass 3 (the bandwidth-bound kernels) only
 * once the pass 3 last enqueued on `after` has finished.  Two contexts chained
 * to each other, decoding alternate segments on their own streams, run each
 * decode's header walk (pass 1, latency-bound) under the other's pass 3,
 * while their pass-3 kernels never run concurrently.  after = NULL unchains.
 * Both contexts must be on the same device and be driven from one host thread;
 * okv_close of either unchains the pair.  The caller's current device is kept.
 */
int okv_decode_chain(okv_ctx *ctx, okv_ctx *after);

/*
 * GetRow's block step (segment_reader.go:387-404) on one block, host memory:
 * ReadBlockWithStat of the block -- every record walked with Go's checks --
 * then the first row whose key equals `key` (bytes.Equal, :398), in one
 * point-path launch (okv_point_kernel: the block and the key in, that one
 * row out; no row arrays come back).
 *   out->status : the block's OKV_BLK_* outcome (rows exist only when OK);
 *   out->found  : 1 (key / val point at the row's bytes, valid until the next
 *                 call on ctx), 0 (no such row), or -1 (the block is not a
 *                 point-path block -- zstd, BlockSize > 64 KiB, a key longer
 *                 than 8 KiB, or more than 1 024 rows: use okv_decode_blocks).
 * Returns OKV_OK or a negative error.  (ABI 6.)
 */
typedef struct okv_point_row {
  int32_t status;
  int32_t found;
  const uint8_t *key;
  uint64_t key_len;
  const uint8_t *val;
  uint64_t val_len;
} okv_point_row;

int okv_point_get(okv_ctx *ctx, const uint8_t *seg, uint64_t seg_bytes,
                  const okv_block_desc *desc, int compression, const uint8_t *key,
                  uint64_t key_len, okv_point_row *out);

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

/* ======================================================================== *
 * Encode: SegmentWriter.WriteRow x n -> Close (segment_writer.go:80-328)
 * ======================================================================== */

/* Rows to encode, structure of arrays (the okv_decode_out layout, so a decode
 * feeds an encode directly -- the compaction shape).  Row i is
 *   key   = key_arena[key_off[i] .. +key_len[i]]
 *   value = val_arena[val_off[i] .. +val_len[i]]
 * in the order WriteRow would be called ("expected that rows are written in
 * order", segment_writer.go:78; the writer does not check it and neither do
 * we).  key_arena_bytes / val_arena_bytes are the arena extents (host mode
 * stages that many bytes; device mode uses them only for validation). */
typedef struct okv_rows {
  const uint8_t *key_arena;
  const uint64_t *key_off;
  const uint16_t *key_len;
  const uint8_t *val_arena;
  const uint64_t *val_off;
  const uint32_t *val_len;
  uint64_t n_rows;
  uint64_t key_arena_bytes, val_arena_bytes;
} okv_rows;

/* SegmentWriterOptions (segment_writer_option.go:5-16).  The bloom filter is
 * an opaque pass-through: the caller runs BloomFilter.Add per row
 * (segment_writer.go:133-136) and hands over BloomFilter.WriteTo's bytes; the
 * meta block then carries [1][u64 LE length][bytes] (:295-300), else [0]. */
typedef struct okv_encode_opts {
  uint64_t threshold_bytes; /* DataBlockThresholdBytes (default 3584) */
  uint64_t block_size;      /* DataBlockSize (default 4096) */
  int compression;          /* OKV_COMP_NONE, or OKV_COMP_LZ4: Go writes raw bytes with
                               CompressedSize = OriginalSize and meta byte 2 (Q7);
                               OKV_COMP_ZSTD -> OKV_W_UNSUPPORTED */
  int strict_go;            /* 1: a Close with no open block panics in Go (Q1) ->
                               OKV_W_NIL_WRITER; 0: write the footer normally */
  const uint8_t *bloom;     /* host bytes of BloomFilter.WriteTo, or NULL (BloomFilter nil) */
  uint64_t bloom_len;
} okv_encode_opts;

/* Output: the segment file, written as the Go writer writes it:
 *   seg[0 .. data_bytes)                      data blocks (BlockStat order)
 *   seg[data_bytes .. +meta_bytes)            meta block (generateMetaBlock :284-328)
 *   seg[data_bytes + meta_bytes .. +25)       trailer: u64 meta offset, u64 XXH64(meta),
 *                                             u8 version 1, u64 magic (:226-276)
 * plus the block index as arrays.  Any of blk_first_row / blk_desc / blk_hash
 * may be NULL.  FirstKey of block b = key of row blk_first_row[b]. */
typedef struct okv_encode_out {
  uint8_t *seg;
  uint64_t seg_cap;
  uint64_t *blk_first_row;  /* [blk_cap + 1]; entry n_blocks = n_rows */
  okv_block_desc *blk_desc; /* [blk_cap] Offset, BlockSize, OriginalSize, CompressedSize */
  uint64_t *blk_hash;       /* [blk_cap] BlockStat.Hash */
  uint64_t blk_cap;
  /* filled on return (also with OKV_E_CAPACITY): */
  uint64_t n_blocks;
  uint64_t data_bytes;  /* sum of BlockSize == meta block offset */
  uint64_t meta_bytes;
  uint64_t file_bytes;  /* data + meta + 25: Close()'s first return value */
  uint64_t meta_hash;   /* 0 with OKV_F_NO_CLOSE until okv_encode_close */
  uint64_t bad_row;     /* OKV_W_INVALID_KEY: the first row with an empty key */
} okv_encode_out;

/*
 * Encode rows into one segment on the GPU.  flags: OKV_F_DEVICE_PTRS (rows and
 * every output pointer are device pointers; seg must be 16-byte aligned),
 * OKV_F_NO_CLOSE.  Returns OKV_OK; OKV_E_CAPACITY (sizes in out set, nothing
 * written: call again with seg_cap >= file_bytes and blk_cap >= n_blocks --
 * a call with zero capacities is the size query); OKV_W_INVALID_KEY (bad_row
 * set); OKV_W_NIL_WRITER (strict_go and the last row closed a block, or no
 * rows); OKV_W_NO_ROWS (no rows, strict_go == 0); OKV_W_UNSUPPORTED; or an
 * OKV_E_* error.
 */
int okv_encode_rows(okv_ctx *ctx, const okv_rows *rows, const okv_encode_opts *opts,
                    okv_encode_out *out, uint32_t flags);

/* Close after OKV_F_NO_CLOSE: XXH64 of the meta block on the host (one
 * sequential hash, segment_writer.go:248) and the trailer written into seg.
 * flags: OKV_F_DEVICE_PTRS as given to okv_encode_rows. */
int okv_encode_close(okv_ctx *ctx, okv_encode_out *out, uint32_t flags);

/* Per-phase encode timing (HIP events on the ctx stream, enabled by
 * okv_profile(ctx, 1)): ms[4] = cut (E1-E9), pack, block hash, meta block,
 * summed over the profiled okv_encode_rows calls. */
int okv_encode_profile_read(okv_ctx *ctx, double *ms, uint64_t *calls);
int okv_encode_profile_reset(okv_ctx *ctx);

/* Deterministic C1/C2/C4 rows on the device: key = row index big-endian in
 * key_len bytes, value = val_len bytes of splitmix64(seed) 8-byte LE words,
 * drawn in row order (oracle/pyoracle.py rows_fixed).  Rows first_row ..
 * first_row + n - 1, packed: key_off[i] = i * key_len, val_off[i] = i * val_len
 * (relative to this call's arenas).  All pointers are device pointers. */
int okv_synth_rows_fixed(okv_ctx *ctx, uint64_t seed, uint64_t first_row, uint64_t n,
                         uint32_t key_len, uint32_t val_len, uint8_t *key_arena,
                         uint64_t *key_off, uint16_t *key_len_out, uint8_t *val_arena,
                         uint64_t *val_off, uint32_t *val_len_out);

/* ======================================================================== *
 * Merge: snapshot_reader.Reader.GetRange's k-way merge
 * (/root/reference/snapshot_reader/snapshot_reader.go:214-372) on the device,
 * and the same newest-wins merge as a compaction feed.
 * ======================================================================== */
#define OKV_MERGE_GETRANGE 0 /* the Go loop exactly: range bound, limit, tombstones, and the
                                stale cursor of a stream that ran out (:336-365) */
#define OKV_MERGE_ALL 1      /* every key's owning row (compaction); L0 tombstones dropped
                                iff drop_tombstones */
#define OKV_DIR_ASC 0        /* sst.DirectionAscending  (segment_row_iter.go:22-25) */
#define OKV_DIR_DESC 1       /* sst.DirectionDescending */
#define OKV_M_EOF 1          /* okv_merge_out.status: GetRange returns an error because a
                                RowIter.Next hit io.EOF rolling a tombstone forward (:316-331) */

/* One merge input: rows [row_lo, row_hi) of a decoded segment (the okv_decode_out
 * layout, device pointers), sorted ascending by key as the Go writer writes them.
 * For GetRange this is the stream RowIter(direction).Seek(startRange) yields
 * (ascending: rows >= start; descending: rows <= end, consumed from row_hi - 1).
 * Inputs are given in the snapshot's priority order (:235-254); among equal keys
 * the lowest index owns the key (findMaxIndexes, :404-424). */
typedef struct okv_merge_src {
  const uint8_t *key_arena;
  const uint64_t *key_off;
  const uint16_t *key_len;
  const uint8_t *val_arena;
  const uint64_t *val_off;
  const uint32_t *val_len; /* 0 = Go nil: an L0 row with a nil value is a tombstone */
  uint64_t row_lo, row_hi;
  int32_t level; /* SegmentRecord.Level */
  int32_t pad;
} okv_merge_src;

typedef struct okv_merge_opts {
  int mode;            /* OKV_MERGE_* */
  int direction;       /* OKV_DIR_* */
  int drop_tombstones; /* OKV_MERGE_ALL only */
  int pad;
  uint64_t limit;      /* OKV_MERGE_GETRANGE: > 0 (Go panics on 0: the caller's check) */
  const uint8_t *bound; /* host bytes: end (ascending) or start (descending), :340-347 */
  uint64_t bound_len;
} okv_merge_opts;

/* Output rows in iteration order: which input and row, and optionally an
 * index-only SoA whose offsets are relative to key_base / val_base (callers pass
 * the lowest input arena address), so the result feeds okv_encode_rows directly.
 * Any array pointer may be NULL. */
typedef struct okv_merge_out {
  uint32_t *src;
  uint64_t *row;
  uint64_t *key_off;
  uint16_t *key_len;
  uint64_t *val_off;
  uint32_t *val_len;
  const uint8_t *key_base;
  const uint8_t *val_base;
  uint64_t row_cap;
  /* filled on return: */
  uint64_t n_rows;   /* rows returned (set also with OKV_E_CAPACITY) */
  uint64_t n_unique; /* distinct keys across the inputs */
  int32_t status;    /* 0, or OKV_M_EOF (no rows are written) */
  int32_t pad;
} okv_merge_out;

/* flags: OKV_F_DEVICE_PTRS (required), OKV_F_ASYNC. At most 64 inputs. */
int okv_merge_rows(okv_ctx *ctx, const okv_merge_src *srcs, uint32_t nsrc,
                   const okv_merge_opts *opts, okv_merge_out *out, uint32_t flags);

/* Per-kernel timing with HIP events recorded on the context stream around
 * each stage of okv_decode_blocks.  okv_profile(ctx, 1) enables and resets;
 * okv_profile_read synchronises the stream and returns the summed
 * milliseconds per stage, ms[4] = {pass 1 count, pass 2 scan, pass 3 gather
 * (+ big-block copy / index), zstd decompression (0 for uncompressed)}, and
 * the number of decode calls timed.  ms must hold 4 doubles (ABI 2 and later;
 * ABI 1 wrote 3). */
int okv_profile(okv_ctx *ctx, int enable);
int okv_profile_read(okv_ctx *ctx, double *ms, uint64_t *calls);

/* The pass-3 kernels the context's last okv_decode_blocks call launched (a
 * bitmask of OKV_PATH_*), for tests and benchmarks that must show which
 * shipping kernel ran.  Set before the call returns, async or not. */
#define OKV_PATH_FUSED 1u  /* okv_decode_fused_kernel: passes 1-3 in one launch */
#define OKV_PATH_SMALL 2u  /* okv_gather_small_kernel: one wave per small block */
#define OKV_PATH_TILE 4u   /* okv_tile_kernel: large blocks, source tiles */
#define OKV_PATH_SWEEP 8u  /* okv_rows_kernel + okv_value_sweep_kernel */
#define OKV_PATH_STAGED 16u /* okv_gather_staged_kernel as the pass */
#define OKV_PATH_GATHER 32u /* okv_gather_kernel (unstaged) */
#define OKV_PATH_BIG 64u    /* okv_copy_kernel / okv_index_kernel for big blocks (always
                               launched after a non-fused pass; exits when none) */
#define OKV_PATH_ZSTD 128u  /* the zstd stage ran first */
#define OKV_PATH_STREAM 1024u   /* okv_decode_stream_kernel (ablation builds only,
                                     OKV_DECODE_STREAM=1): passes 1-3 in one launch for any batch
                                     of small blocks, prefix by decoupled look-back */
#define OKV_PATH_ENC_ONEPASS 512u /* okv_encode_rows used the single-pass plan kernel: ablation
                                     builds only (OKV_ENC_ONEPASS=1); the product runs E1-E9 */
#define OKV_PATH_ZSTD_REGROW 256u /* zstd frames outgrew their first output region and were
                                     measured and decoded again (io.Copy inflates them all) */
#define OKV_PATH_GROUP 4096u /* okv_group_kernel (ablation builds only, OKV_DECODE_GROUP=1):
                                  a large batch of small blocks in one pass, 16 blocks per
                                  workgroup, the prefix by decoupled look-back; measured
                                  slower than passes 1-3 */
#define OKV_PATH_POINT 2048u /* okv_point_kernel: a host-mode call of a few small uncompressed
                                blocks (GetRow, GetRange) in one launch over pinned memory */
uint32_t okv_last_path(const okv_ctx *ctx);

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
