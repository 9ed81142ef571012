/*
 * okv_host.h -- host-side C++ mirror of the Go sst API, exported as C for
 * non-Go callers (the Python harness, C/C++ services).  A Go caller keeps its
 * own sst.SegmentWriter/SegmentReader and binds only okv_sst.h.
 *
 *   okv_writer_*      sst.SegmentWriter   (sst/segment_writer.go:35-328)
 *   okv_meta_*        sst.SegmentReader.FetchAndLoadMetadata / BytesToMetadata
 *                     (sst/segment_reader.go:91-238)
 *   okv_reader_*      sst.SegmentReader + RowIter over the GPU batched decode
 *                     (segment_reader.go:264-475, segment_row_iter.go:32-212)
 *   okv_synth_*       deterministic synthetic segments
 *
 * Error codes mirror the Go sentinels; see the OKV_W_* / OKV_M_* values.
 */
#ifndef OKV_HOST_H
#define OKV_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "okv_sst.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Go error sentinels (values shared with the test oracle) */
/* OKV_W_* (SegmentWriter sentinels) are defined in okv_sst.h */
#define OKV_M_MAGIC (-201)           /* ErrInvalidMagicNumber      segment_reader.go:84 */
#define OKV_M_VERSION (-202)         /* ErrUnknownSegmentVersion   :81 */
#define OKV_M_HASH (-203)            /* ErrMismatchedMetaBlockHash :82 */
#define OKV_M_INVALID (-204)         /* ErrInvalidMetaBlock        :83 */
#define OKV_M_PANIC (-205)           /* mustReadBytes panic while parsing */
#define OKV_M_IO (-206)              /* Seek/Read error */
#define OKV_M_MAKESLICE (-207)       /* make([]byte, negative) panic :124 */
#define OKV_M_BLOOM (-208)           /* BloomFilter.ReadFrom error: parseBloomFilterBlock :160-163 */
#define OKV_R_NO_ROWS (-301)         /* ErrNoRows          :357 */
#define OKV_R_EOF (-302)             /* io.EOF from RowIter.Next */
#define OKV_R_CLOSED (-303)          /* ErrClosed          segment_row_iter.go:27 */
#define OKV_R_ALREADY_CLOSED (-304)  /* ErrAlreadyClosed   segment_reader.go:478 */
#define OKV_R_BLOCK_EOF (-305)       /* ReadBlockWithStat: reader.Read error (:310-313) */
#define OKV_R_BLOCK_SHORT (-306)     /* ReadBlockWithStat: ErrUnexpectedBytesRead (:314-316) */
#define OKV_R_PANIC (-307)           /* a Go panic: mustReadBytes (:506-512) or rows[0] of an
                                        empty block (segment_row_iter.go:95, :147) */
#define OKV_R_UNSUPPORTED (-308)     /* a block the device decode does not support */
#define OKV_R_GPU (-309)             /* the GPU decode itself failed (okv_last_error) */
#define OKV_R_ZSTD (-310)            /* zstd decoder error: ReadBlockWithStat's io.Copy error
                                        (segment_reader.go:326-330) */

/* ---- SegmentWriter ------------------------------------------------------- */
typedef struct okv_writer okv_writer;
/* SegmentWriterOptions (segment_writer_option.go:5-16). */
okv_writer *okv_writer_new(uint64_t threshold_bytes, uint64_t block_size, int zstd_level, int lz4);
/* options.BloomFilter != nil (segment_writer_option.go:20): the meta block
 * carries [1][u64 LE len][bytes] (segment_writer.go:295-300).  bytes =
 * BloomFilter.WriteTo, computed by the caller (BloomFilter.Add per row,
 * :133-136); an opaque pass-through here.  Call any time before Close. */
void okv_writer_set_bloom(okv_writer *w, const uint8_t *bytes, uint64_t len);
int okv_writer_write_row(okv_writer *w, const uint8_t *key, size_t klen, const uint8_t *val,
                         size_t vlen);
/* Close (segment_writer.go:211-282).  strict_go != 0 reproduces the Go panic
 * when no row is pending (Q1) as OKV_W_NIL_WRITER; strict_go == 0 emits the
 * footer normally (documented divergence). */
int okv_writer_close(okv_writer *w, int strict_go, uint64_t *file_len, uint64_t *meta_len);
const uint8_t *okv_writer_data(const okv_writer *w, uint64_t *len);
const uint8_t *okv_writer_meta(const okv_writer *w, uint64_t *len);
uint64_t okv_writer_num_blocks(const okv_writer *w);
/* index entry i: descriptor + hash + first key (pointer valid until free) */
int okv_writer_block(const okv_writer *w, uint64_t i, okv_block_desc *desc, uint64_t *hash,
                     const uint8_t **first_key, uint64_t *first_key_len);
void okv_writer_free(okv_writer *w);

/* ---- metadata ------------------------------------------------------------ */
typedef struct okv_meta okv_meta;
/* FetchAndLoadMetadata over buf (what the reader holds) with the file length
 * given to NewSegmentReader (file_bytes). */
int okv_meta_fetch(const uint8_t *buf, uint64_t buf_len, int64_t file_bytes, okv_meta **out);
int okv_meta_parse(const uint8_t *meta, uint64_t meta_len, okv_meta **out); /* BytesToMetadata */
uint64_t okv_meta_num_blocks(const okv_meta *m);       /* entries in file order */
int okv_meta_compression(const okv_meta *m);
const okv_block_desc *okv_meta_descs(const okv_meta *m); /* file order */
const uint8_t *okv_meta_first_key(const okv_meta *m, uint64_t *len);
const uint8_t *okv_meta_last_key(const okv_meta *m, uint64_t *len);
int okv_meta_block(const okv_meta *m, uint64_t i, okv_block_desc *desc, uint64_t *hash,
                   const uint8_t **first_key, uint64_t *first_key_len);
void okv_meta_free(okv_meta *m);
/* The meta block's bloom filter (parseBloomFilterBlock :183-201) and its Test
 * (probeBloomFilter :245-258; bits-and-blooms v2.0.3 + murmur3 v1.1.0 +
 * bitset v1.1.11 restated on the host, filter bytes parity-unpinned).
 * okv_meta_bloom_test: 1 maybe present (also with no filter), 0 absent,
 * OKV_R_PANIC for a filter with m == 0 (Go's integer division panic). */
int okv_meta_has_bloom(const okv_meta *m);
int okv_meta_bloom_test(const okv_meta *m, const uint8_t *key, size_t klen);

/* ---- SegmentReader / RowIter over the GPU decode -------------------------- */
/* A row as Go's KVPair (segment_reader.go:285-288): NULL pointer = nil slice.
 * Rows returned by okv_reader_read_block / _get_row / _get_range stay valid
 * until the next such call on the reader (or okv_reader_free); the rows an
 * iterator returns stay valid while it serves the same block. */
typedef struct okv_row {
  const uint8_t *key;
  uint64_t key_len;
  const uint8_t *val;
  uint64_t val_len;
} okv_row;

typedef struct okv_reader okv_reader;
typedef struct okv_iter okv_iter;

/* NewSegmentReader (segment_reader.go:65-72) over `len` bytes (what the
 * io.ReadSeeker holds; copied) with the file length `file_bytes`.  Block reads
 * are GPU calls on `ctx` bounded as the cgo shim's ReadBlocks:
 * GetRow / ReadBlockWithStat decode one block, GetRange the blocks its btree
 * walks select, RowIter the block and the next 255 in its direction (the
 * iteration window, which later reads are served from); each call stages
 * only its blocks' span of the bytes. */
okv_reader *okv_reader_open(okv_ctx *ctx, const uint8_t *data, uint64_t len, int64_t file_bytes);
int okv_reader_fetch_metadata(okv_reader *r);                                  /* :91-141 */
int okv_reader_load_metadata(okv_reader *r, const uint8_t *meta, uint64_t len); /* :147 + :75 */
int okv_reader_num_blocks(okv_reader *r, uint64_t *n); /* btree entries (unique first keys) */
/* ReadBlockWithStat on the i-th btree entry in ascending FirstKey order (:295-355).
 * *rows points to n rows (valid until free). */
int okv_reader_read_block(okv_reader *r, uint64_t i, const okv_row **rows, uint64_t *n);
int okv_reader_get_row(okv_reader *r, const uint8_t *key, size_t klen, okv_row *out); /* :362 */
/* GetRange [start, end) (:410-475); an empty start is UnboundStart, end == {0xff} UnboundEnd.
 * Go ranges a map over the candidate blocks; this returns them in ascending FirstKey order. */
int okv_reader_get_range(okv_reader *r, const uint8_t *start, size_t slen, const uint8_t *end,
                         size_t elen, const okv_row **rows, uint64_t *n);
int okv_reader_close(okv_reader *r); /* :481-487 (OKV_R_ALREADY_CLOSED the second time) */
void okv_reader_free(okv_reader *r);
/* I/O of the reader's block reads so far: GPU decode calls, blocks decoded,
 * bytes staged (the storage bytes the calls read). */
typedef struct okv_reader_io {
  uint64_t calls, blocks, bytes_staged;
} okv_reader_io;
int okv_reader_io_stats(const okv_reader *r, okv_reader_io *io);

/* RowIter (segment_row_iter.go:11-212); direction 0 ascending, 1 descending. */
okv_iter *okv_reader_row_iter(okv_reader *r, int direction);
int okv_iter_next(okv_iter *it, okv_row *out);                     /* OKV_R_EOF at the end */
int okv_iter_seek(okv_iter *it, const uint8_t *key, size_t klen); /* empty = UnboundStart */
void okv_iter_free(okv_iter *it);

/* ---- synthetic segments (bench / tests) ---------------------------------- */
#define OKV_SYNTH_FIXED 0 /* C1/C2: 16 B big-endian index key, 64 B splitmix64(seed) value */
#define OKV_SYNTH_ZIPF 1  /* C3: key 8..256 B (P ~ (L-7)^-1.1), value 0..4096 B */
/* Writes rows until `nrows` are written (nrows > 0) or until `nblocks` blocks
 * are flushed with one more row open; returns a closed writer. */
okv_writer *okv_synth_segment(int kind, uint64_t seed, uint64_t nrows, uint64_t nblocks,
                              uint64_t threshold, uint64_t block_size);

#ifdef __cplusplus
}
#endif
#endif
