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
#define OKV_W_KEY_TOO_LARGE (-101)   /* ErrKeyTooLarge   segment_writer.go:71 */
#define OKV_W_VALUE_TOO_LARGE (-102) /* ErrValueTooLarge :72 */
#define OKV_W_CLOSED (-103)          /* ErrWriterClosed  :69 */
#define OKV_W_INVALID_KEY (-104)     /* ErrInvalidKey    :74 */
#define OKV_W_NIL_WRITER (-105)      /* Go panics in Close (:212) -- see okv_writer_close */
#define OKV_W_UNSUPPORTED (-106)     /* zstd level > 0: encoder not implemented */
#define OKV_W_NO_ROWS (-107)         /* ErrNoRowsWritten :73 (reachable only with strict_go == 0) */
#define OKV_M_MAGIC (-201)           /* ErrInvalidMagicNumber      segment_reader.go:84 */
#define OKV_M_VERSION (-202)         /* ErrUnknownSegmentVersion   :81 */
#define OKV_M_HASH (-203)            /* ErrMismatchedMetaBlockHash :82 */
#define OKV_M_INVALID (-204)         /* ErrInvalidMetaBlock        :83 */
#define OKV_M_PANIC (-205)           /* mustReadBytes panic while parsing */
#define OKV_M_IO (-206)              /* Seek/Read error */
#define OKV_M_MAKESLICE (-207)       /* make([]byte, negative) panic :124 */
#define OKV_R_NO_ROWS (-301)         /* ErrNoRows          :357 */
#define OKV_R_EOF (-302)             /* io.EOF from RowIter.Next */
#define OKV_R_CLOSED (-303)          /* ErrClosed          segment_row_iter.go:27 */
#define OKV_R_ALREADY_CLOSED (-304)  /* ErrAlreadyClosed   segment_reader.go:478 */
#define OKV_R_BLOCK (-305)           /* block decode error / panic (see okv_reader_last_block_status) */

/* ---- SegmentWriter ------------------------------------------------------- */
typedef struct okv_writer okv_writer;
/* SegmentWriterOptions (segment_writer_option.go:5-16).  BloomFilter is not
 * supported (bloom bytes are parity-unpinned). */
okv_writer *okv_writer_new(uint64_t threshold_bytes, uint64_t block_size, int zstd_level, int lz4);
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
