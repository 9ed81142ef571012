/*
 * okv_oracle.h -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Plain-C CPU restatement of ObjectKV's Go `sst/` segment path
 * (/root/reference @ 2025-03-21).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this.  The product path
 * (objectkv_amd/, libokv_sst.so) never links or calls it.
 *
 * Parity pinning: the Go toolchain is absent in this image and on the GPU
 * box, so the reference cannot be built or run.  This restatement is pinned
 * by (1) every known answer asserted in the reference's own tests
 * (sst/segment_reader_test.go, segment_row_iter_test.go,
 * segment_writer_test.go), (2) the XXH64 specification
 * (cespare/xxhash/v2 v2.2.0 = canonical XXH64, seed 0), cross-checked
 * against the Python `xxhash` 3.8.1 package, and (3) an independent Python
 * restatement (oracle/pyoracle.py) that must agree byte for byte.
 */
#ifndef OKV_ORACLE_H
#define OKV_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (values shared with include/okv_sst.h) --------------- */
/* writer (segment_writer.go:68-75) */
#define OREF_OK 0
#define OREF_ERR_KEY_TOO_LARGE (-101)   /* ErrKeyTooLarge    :71 */
#define OREF_ERR_VALUE_TOO_LARGE (-102) /* ErrValueTooLarge  :72 */
#define OREF_ERR_WRITER_CLOSED (-103)   /* ErrWriterClosed   :69 */
#define OREF_ERR_INVALID_KEY (-104)     /* ErrInvalidKey     :74 */
#define OREF_PANIC_NIL_WRITER (-105)    /* Close() :212 defer on nil blockWriter (Q1) */
#define OREF_ERR_UNSUPPORTED (-106)     /* zstd encoder not restated (parity unpinned) */
/* metadata (segment_reader.go:79-85) */
#define OREF_ERR_MAGIC (-201)        /* ErrInvalidMagicNumber */
#define OREF_ERR_VERSION (-202)      /* ErrUnknownSegmentVersion */
#define OREF_ERR_META_HASH (-203)    /* ErrMismatchedMetaBlockHash */
#define OREF_ERR_META_INVALID (-204) /* ErrInvalidMetaBlock (0 entries) */
#define OREF_PANIC_META (-205)       /* mustReadBytes panic while parsing meta */
#define OREF_ERR_IO (-206)           /* Seek/Read error (EOF, negative position) */
#define OREF_PANIC_MAKESLICE (-207)  /* make([]byte, negative) :124 */

/* per-block decode status (segment_reader.go:295-355) */
#define OREF_BLK_OK 0
#define OREF_BLK_EOF 1         /* reader.Read / Seek error (:303-313) */
#define OREF_BLK_SHORT 2       /* ErrUnexpectedBytesRead error (:314-316) */
#define OREF_BLK_PANIC 3       /* mustReadBytes panic in the record loop (:338-352, :506-512) */
#define OREF_BLK_UNSUPPORTED 4 /* index-only spans of a zstd block; libzstd missing */
#define OREF_BLK_ZSTD 6        /* zstd.NewReader / io.Copy error (:321-330) */

/* Go runtime maxAlloc on 64-bit linux (1 << heapAddrBits, heapAddrBits = 48):
 * make([]byte, n) panics for n above it (runtime/malloc.go, runtime/slice.go) */
#define OREF_GO_MAX_ALLOC (1ull << 48)

#define OREF_COMP_NONE 0
#define OREF_COMP_ZSTD 1
#define OREF_COMP_LZ4 2

/* ---- XXH64 ------------------------------------------------------------- */
uint64_t oref_xxh64(const void *data, size_t len, uint64_t seed);

/* ---- SegmentWriter (segment_writer.go:35-328, block_stat.go:27-42) ----- */
typedef struct oref_writer oref_writer;
oref_writer *oref_writer_new(uint64_t threshold_bytes, uint64_t block_size, int zstd_level,
                             int lz4);
int oref_writer_write_row(oref_writer *w, const uint8_t *key, size_t klen, const uint8_t *val,
                          size_t vlen);
/* On success: *file and *file_len hold the whole segment, *meta and *meta_len the
 * meta block (both owned by the writer until oref_writer_free). */
int oref_writer_close(oref_writer *w, const uint8_t **file, uint64_t *file_len,
                      const uint8_t **meta, uint64_t *meta_len);
/* bytes written to the external writer so far (blocks + footer) */
const uint8_t *oref_writer_bytes(const oref_writer *w, uint64_t *len);
uint64_t oref_writer_num_blocks(const oref_writer *w);
/* options.BloomFilter != nil: the meta block carries [1][u64 len][bytes]
 * (segment_writer.go:295-300); bytes = BloomFilter.WriteTo, opaque here. */
void oref_writer_set_bloom(oref_writer *w, const uint8_t *bytes, uint64_t len);
void oref_writer_free(oref_writer *w);

/* ---- block index entry ------------------------------------------------- */
typedef struct {
  uint64_t offset, block_size, original_size, compressed_size;
} oref_block_desc;

/* ---- Metadata (segment_reader.go:91-238) ------------------------------- */
typedef struct {
  const uint8_t *first_key;
  uint64_t first_key_len;
  const uint8_t *last_key;
  uint64_t last_key_len;
  int has_bloom;
  uint64_t bloom_off, bloom_len; /* opaque bytes inside the meta block */
  int compression;               /* 0 none / 1 zstd / 2 lz4 (:166-172) */
  uint64_t n_entries;            /* entries in FILE order */
  const uint8_t **entry_key;     /* pointers into the meta bytes */
  uint64_t *entry_key_len;
  uint64_t *entry_offset, *entry_block_size, *entry_original_size, *entry_compressed_size,
      *entry_hash;
} oref_meta;

/* BytesToMetadata over meta bytes; returns OREF_OK or an error code. */
int oref_parse_meta(const uint8_t *meta, uint64_t meta_len, oref_meta *out);
/* FetchAndLoadMetadata: buf is what the io.ReadSeeker holds, file_bytes is
 * the length passed to NewSegmentReader (they differ in the corruption
 * tests, segment_reader_test.go:727-830).  On success *meta_off and *meta_len
 * locate the meta bytes inside buf. */
int oref_fetch_meta(const uint8_t *buf, uint64_t buf_len, int64_t file_bytes, oref_meta *out,
                    uint64_t *meta_off, uint64_t *meta_len);
void oref_meta_free(oref_meta *m);

/* ---- ReadBlockWithStat (segment_reader.go:295-355) --------------------- */
/* Go-semantics decode of one block: allocates a block copy and one heap copy
 * per key and value (mustReadBytes, :489-512); empty -> NULL (Q4). */
typedef struct {
  uint8_t *key;
  uint64_t key_len;
  uint8_t *val;
  uint64_t val_len;
} oref_kv;
typedef struct {
  oref_kv *rows;
  uint64_t n, cap;
} oref_rows;
int oref_read_block(const uint8_t *seg, uint64_t seg_len, const oref_block_desc *d,
                    int compression, oref_rows *out);
void oref_rows_free(oref_rows *r);

/* CPU baseline: decode blocks [b0, b1) with Go allocation semantics on
 * `threads` threads; returns rows decoded (sum) and writes total key+value
 * bytes to *payload.  Used only by bench.py's cpu_baseline leg. */
uint64_t oref_decode_range_go(const uint8_t *seg, uint64_t seg_len, const oref_block_desc *d,
                              uint64_t nblk, int compression, int threads, uint64_t *payload);
/* CPU encode baseline: `threads` key-range shards, each its own segment, with
 * Go's per-row rowBuf allocation; returns 0 or the first writer error. */
int oref_encode_go(const uint8_t *key_arena, const uint64_t *key_off, const uint16_t *key_len,
                   const uint8_t *val_arena, const uint64_t *val_off, const uint32_t *val_len,
                   uint64_t n, uint64_t threshold, uint64_t block_size, int lz4, int threads,
                   uint64_t *file_bytes);

/* One segment from SoA rows on one thread (full-size encode parity): every
 * row written, the writer returned for ONE oref_writer_close, then
 * oref_writer_free; *rc = 0 or the first writer error. */
oref_writer *oref_encode_soa(const uint8_t *key_arena, const uint64_t *key_off,
                             const uint16_t *key_len, const uint8_t *val_arena,
                             const uint64_t *val_off, const uint32_t *val_len, uint64_t n,
                             uint64_t threshold, uint64_t block_size, int *rc);

/* CPU baselines of bench.py configs (Go semantics; `threads` independent
 * copies of the job run concurrently):
 * C1 -- WriteRow x n + Close + a full ascending read with ReadBlockWithStat's
 * per-row copies; returns rows read (all threads), *file_bytes summed. */
uint64_t oref_roundtrip_go(const uint8_t *key_arena, const uint64_t *key_off,
                           const uint16_t *key_len, const uint8_t *val_arena,
                           const uint64_t *val_off, const uint32_t *val_len, uint64_t n,
                           uint64_t threshold, uint64_t block_size, int threads,
                           uint64_t *file_bytes);
/* CM -- decode every block of k segments (newest first), merge ascending with
 * the newest segment owning a key, write the merge with the Go writer;
 * returns the merged rows of one compaction (0 on error). */
uint64_t oref_compact_go(int k, const uint8_t *const *segs, const uint64_t *seg_lens,
                         const oref_block_desc *const *descs, const uint64_t *nblks,
                         uint64_t threshold, uint64_t block_size, int threads,
                         uint64_t *out_bytes);

/* ---- SoA restatement of the product's output layout -------------------- */
/* Pass 1: per-block (status, rows, key bytes, value bytes). */
void oref_block_counts(const uint8_t *seg, uint64_t seg_len, const oref_block_desc *d,
                       uint64_t nblk, int compression, int32_t *status, uint64_t *rows,
                       uint64_t *kbytes, uint64_t *vbytes);
/* Full layout (DESIGN.md "Output layout"): index_only=1 -> offsets into seg,
 * no arenas.  Arrays must be sized from oref_block_counts. */
void oref_decode_soa(const uint8_t *seg, uint64_t seg_len, const oref_block_desc *d,
                     uint64_t nblk, int compression, int index_only, uint64_t *row_start,
                     uint64_t *key_base, uint64_t *val_base, uint64_t *key_off,
                     uint16_t *key_len, uint64_t *val_off, uint32_t *val_len,
                     uint8_t *key_arena, uint8_t *val_arena, int32_t *status);

#ifdef __cplusplus
}
#endif
#endif
