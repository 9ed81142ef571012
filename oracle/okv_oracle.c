/*
 * okv_oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of ObjectKV's Go
 * sst/ segment path.  See okv_oracle.h for the pinning statement.  Every
 * function cites the reference file:line it restates (/root/reference/...).
 * Never linked into the product (libokv_sst.so); loaded only by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 */
#include "okv_oracle.h"

#include <dlfcn.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================= */
/* XXH64 -- github.com/cespare/xxhash/v2 v2.2.0 (go.mod:7) implements the    */
/* canonical XXH64 with seed 0; call sites segment_writer.go:185, :248 and  */
/* segment_reader.go:130.  Restated from the public XXH64 specification.    */
/* ======================================================================= */
#define P1 11400714785074694791ULL
#define P2 14029467366897019727ULL
#define P3 1609587929392839161ULL
#define P4 9650029242287828579ULL
#define P5 2870177450012600261ULL

static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t rd64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}
static inline uint32_t rd32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint16_t rd16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline uint64_t xround(uint64_t acc, uint64_t in) {
  acc += in * P2;
  acc = rotl64(acc, 31);
  return acc * P1;
}
static inline uint64_t xmerge(uint64_t acc, uint64_t v) {
  acc ^= xround(0, v);
  return acc * P1 + P4;
}

uint64_t oref_xxh64(const void *data, size_t len, uint64_t seed) {
  const uint8_t *p = (const uint8_t *)data, *end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uint8_t *lim = end - 32;
    do {
      v1 = xround(v1, rd64(p));
      v2 = xround(v2, rd64(p + 8));
      v3 = xround(v3, rd64(p + 16));
      v4 = xround(v4, rd64(p + 24));
      p += 32;
    } while (p <= lim);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xmerge(h, v1);
    h = xmerge(h, v2);
    h = xmerge(h, v3);
    h = xmerge(h, v4);
  } else {
    h = seed + P5;
  }
  h += (uint64_t)len;
  while (p + 8 <= end) {
    h ^= xround(0, rd64(p));
    h = rotl64(h, 27) * P1 + P4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= (uint64_t)rd32(p) * P1;
    h = rotl64(h, 23) * P2 + P3;
    p += 4;
  }
  while (p < end) {
    h ^= (uint64_t)(*p) * P5;
    h = rotl64(h, 11) * P1;
    p++;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

/* ======================================================================= */
/* growable byte buffer (stands in for bytes.Buffer)                        */
/* ======================================================================= */
typedef struct {
  uint8_t *p;
  uint64_t n, cap;
} obuf;
static void ob_reserve(obuf *b, uint64_t extra) {
  if (b->n + extra <= b->cap) return;
  uint64_t c = b->cap ? b->cap : 256;
  while (c < b->n + extra) c *= 2;
  b->p = (uint8_t *)realloc(b->p, c);
  b->cap = c;
}
static void ob_put(obuf *b, const void *src, uint64_t n) {
  ob_reserve(b, n);
  if (n) memcpy(b->p + b->n, src, n);
  b->n += n;
}
static void ob_zero(obuf *b, uint64_t n) {
  ob_reserve(b, n);
  memset(b->p + b->n, 0, n);
  b->n += n;
}
static void ob_u8(obuf *b, uint8_t v) { ob_put(b, &v, 1); }
static void ob_u16(obuf *b, uint16_t v) {
  uint8_t t[2] = {(uint8_t)v, (uint8_t)(v >> 8)};
  ob_put(b, t, 2);
}
static void ob_u32(obuf *b, uint32_t v) {
  uint8_t t[4];
  for (int i = 0; i < 4; i++) t[i] = (uint8_t)(v >> (8 * i));
  ob_put(b, t, 4);
}
static void ob_u64(obuf *b, uint64_t v) {
  uint8_t t[8];
  for (int i = 0; i < 8; i++) t[i] = (uint8_t)(v >> (8 * i));
  ob_put(b, t, 8);
}

/* ======================================================================= */
/* SegmentWriter                                                            */
/* ======================================================================= */
typedef struct {
  obuf first_key;
  uint64_t offset, block_size, original_size, compressed_size, hash;
} oref_stat; /* BlockStat block_stat.go:9-24 */

struct oref_writer {
  uint64_t threshold, dbs; /* SegmentWriterOptions segment_writer_option.go:5-16 */
  int zstd_level, lz4;
  int writer_open;          /* s.blockWriter != nil */
  obuf block;               /* s.blockBuffer */
  uint64_t raw;             /* s.currentRawBlockSize */
  obuf cur_first_key;       /* s.currentBlockStartKey (copied; Q8 aliasing not modelled) */
  obuf last_key;            /* s.lastKey */
  obuf file;                /* the external io.Writer */
  uint64_t offset;          /* s.currentByteOffset */
  oref_stat *idx;           /* s.blockIndex */
  uint64_t nidx, capidx;
  int closed;
  obuf meta;
  int has_bloom; /* options.BloomFilter != nil (segment_writer_option.go:20) */
  obuf bloom;    /* its WriteTo bytes, supplied by the caller (opaque here) */
};

oref_writer *oref_writer_new(uint64_t threshold_bytes, uint64_t block_size, int zstd_level,
                             int lz4) { /* NewSegmentWriter segment_writer.go:58-66 */
  oref_writer *w = (oref_writer *)calloc(1, sizeof(*w));
  w->threshold = threshold_bytes;
  w->dbs = block_size;
  w->zstd_level = zstd_level;
  w->lz4 = lz4;
  return w;
}

/* flushCurrentDataBlock segment_writer.go:148-204 */
static int flush_block(oref_writer *w) {
  int use_zstd = w->zstd_level > 0, use_lz4 = !use_zstd && w->lz4;
  if (w->capidx == w->nidx) {
    w->capidx = w->capidx ? 2 * w->capidx : 64;
    w->idx = (oref_stat *)realloc(w->idx, w->capidx * sizeof(oref_stat));
  }
  oref_stat *st = &w->idx[w->nidx++];
  memset(st, 0, sizeof(*st));
  st->offset = w->offset;                                   /* :161 */
  st->original_size = w->raw;                               /* :162 */
  ob_put(&st->first_key, w->cur_first_key.p, w->cur_first_key.n); /* :163 */
  if (use_zstd || use_lz4) st->compressed_size = w->block.n; /* :165-167 */
  uint64_t rem = w->dbs - w->block.n % w->dbs;              /* :169, always >= 1 (Q2) */
  if (rem > 0) ob_zero(&w->block, rem);                     /* :171 */
  st->block_size = w->block.n;                              /* :180 */
  st->hash = oref_xxh64(w->block.p, w->block.n, 0);         /* :185 */
  ob_put(&w->file, w->block.p, w->block.n);                 /* :191 */
  w->offset += w->block.n;                                  /* :202 */
  w->block.n = 0;
  w->writer_open = 0;                                       /* :200 */
  return OREF_OK;
}

/* WriteRow segment_writer.go:80-146 */
int oref_writer_write_row(oref_writer *w, const uint8_t *key, size_t klen, const uint8_t *val,
                          size_t vlen) {
  if (klen > 65535) return OREF_ERR_KEY_TOO_LARGE;                 /* :81 */
  if ((uint64_t)vlen > 0xFFFFFFFFULL) return OREF_ERR_VALUE_TOO_LARGE; /* :84 */
  if (w->closed) return OREF_ERR_WRITER_CLOSED;                    /* :87 */
  if (klen == 0) return OREF_ERR_INVALID_KEY;                      /* :90 */
  if (w->zstd_level > 0) return OREF_ERR_UNSUPPORTED;              /* :105-111 not restated */
  if (!w->writer_open) {                                           /* :95-115 */
    w->cur_first_key.n = 0;
    ob_put(&w->cur_first_key, key, klen);
    w->raw = 0;
    w->block.n = 0;
    w->writer_open = 1;
  }
  w->last_key.n = 0; /* :118 */
  ob_put(&w->last_key, key, klen);
  ob_u16(&w->block, (uint16_t)klen); /* :121-127 */
  ob_u32(&w->block, (uint32_t)vlen);
  ob_put(&w->block, key, klen);
  ob_put(&w->block, val, vlen);
  w->raw += 6 + klen + vlen; /* :131 */
  if (w->block.n >= w->threshold) return flush_block(w); /* :138-143 */
  return OREF_OK;
}

/* BlockStat.toBytes block_stat.go:27-42 */
static void stat_to_bytes(obuf *m, const oref_stat *s) {
  ob_u16(m, (uint16_t)s->first_key.n);
  ob_put(m, s->first_key.p, s->first_key.n);
  ob_u64(m, s->offset);
  ob_u64(m, s->block_size);
  ob_u64(m, s->original_size);
  ob_u64(m, s->compressed_size);
  ob_u64(m, s->hash);
}

/* Close segment_writer.go:211-282, generateMetaBlock :284-328 */
int oref_writer_close(oref_writer *w, const uint8_t **file, uint64_t *file_len,
                      const uint8_t **meta, uint64_t *meta_len) {
  if (!w->writer_open) return OREF_PANIC_NIL_WRITER; /* :212 defer on nil interface (Q1) */
  int rc = flush_block(w);                           /* :214-219 */
  if (rc) return rc;
  /* :221 ErrNoRowsWritten is unreachable (Q1) */
  uint64_t meta_start = w->offset; /* :226 */
  obuf *m = &w->meta;
  m->n = 0;
  const oref_stat *f = &w->idx[0];
  ob_u16(m, (uint16_t)f->first_key.n); /* :288-292 */
  ob_put(m, f->first_key.p, f->first_key.n);
  ob_u16(m, (uint16_t)w->last_key.n);
  ob_put(m, w->last_key.p, w->last_key.n);
  if (w->has_bloom) { /* :295-300: flag 1, u64 length, BloomFilter.WriteTo bytes */
    ob_u8(m, 1);
    ob_u64(m, w->bloom.n);
    ob_put(m, w->bloom.p, w->bloom.n);
  } else {
    ob_u8(m, 0); /* :301-303 */
  }
  int use_zstd = w->zstd_level > 0, use_lz4 = !use_zstd && w->lz4;
  ob_u8(m, use_zstd ? 1 : (use_lz4 ? 2 : 0)); /* :306-314 */
  ob_u8(m, 0);                                /* :317 simple index */
  ob_u64(m, w->nidx);                         /* :320 */
  for (uint64_t i = 0; i < w->nidx; i++) stat_to_bytes(m, &w->idx[i]); /* :323-325 */
  ob_put(&w->file, m->p, m->n);                  /* :228 */
  w->offset += m->n;
  ob_u64(&w->file, meta_start);                  /* :238 */
  ob_u64(&w->file, oref_xxh64(m->p, m->n, 0));   /* :248-249 */
  ob_u8(&w->file, 1);                            /* :259 version */
  ob_u64(&w->file, 69696969696969ULL);           /* :269 MagicNumber :21 */
  w->offset += 25;
  w->closed = 1; /* :279 */
  if (file) *file = w->file.p;
  if (file_len) *file_len = w->offset;
  if (meta) *meta = m->p;
  if (meta_len) *meta_len = m->n;
  return OREF_OK;
}

const uint8_t *oref_writer_bytes(const oref_writer *w, uint64_t *len) {
  if (len) *len = w->file.n;
  return w->file.p;
}
uint64_t oref_writer_num_blocks(const oref_writer *w) { return w->nidx; }

/* BloomFilter != nil: the writer serialises these bytes into the meta block
 * (the caller runs BloomFilter.Add per row, segment_writer.go:133-136, and
 * hands over WriteTo's bytes before Close; the filter is opaque here). */
void oref_writer_set_bloom(oref_writer *w, const uint8_t *bytes, uint64_t len) {
  w->has_bloom = 1;
  w->bloom.n = 0;
  ob_put(&w->bloom, bytes, len);
}

void oref_writer_free(oref_writer *w) {
  if (!w) return;
  free(w->bloom.p);
  for (uint64_t i = 0; i < w->nidx; i++) free(w->idx[i].first_key.p);
  free(w->idx);
  free(w->block.p);
  free(w->cur_first_key.p);
  free(w->last_key.p);
  free(w->file.p);
  free(w->meta.p);
  free(w);
}

/* ======================================================================= */
/* Metadata                                                                 */
/* ======================================================================= */
/* bytes.Reader + mustReadBytes (segment_reader.go:489-512): a read of n>0
 * bytes panics unless n bytes remain; n == 0 returns nil without reading. */
typedef struct {
  const uint8_t *p;
  uint64_t n, i;
} rd_t;
static int must_read(rd_t *r, uint64_t n, const uint8_t **out) {
  if (n == 0) {
    *out = NULL;
    return 0;
  }
  if (r->i >= r->n || r->n - r->i < n) return -1;
  *out = r->p + r->i;
  r->i += n;
  return 0;
}

/* BytesToMetadata segment_reader.go:147-181, parseBloomFilterBlock :183-201,
 * parseBlockIndex :206-238 */
int oref_parse_meta(const uint8_t *meta, uint64_t meta_len, oref_meta *o) {
  memset(o, 0, sizeof(*o));
  rd_t r = {meta, meta_len, 0};
  const uint8_t *t;
  if (must_read(&r, 2, &t)) return OREF_PANIC_META; /* :152 */
  o->first_key_len = rd16(t);
  if (must_read(&r, o->first_key_len, &o->first_key)) return OREF_PANIC_META; /* :153 */
  if (must_read(&r, 2, &t)) return OREF_PANIC_META;                           /* :154 */
  o->last_key_len = rd16(t);
  if (must_read(&r, o->last_key_len, &o->last_key)) return OREF_PANIC_META; /* :155 */
  if (must_read(&r, 1, &t)) return OREF_PANIC_META;                         /* :184 */
  o->has_bloom = t[0] == 1;
  if (o->has_bloom) {
    if (must_read(&r, 8, &t)) return OREF_PANIC_META; /* :191 */
    o->bloom_len = rd64(t);
    o->bloom_off = r.i;
    if (must_read(&r, o->bloom_len, &t)) return OREF_PANIC_META; /* :192 */
    /* bloom.ReadFrom (bits-and-blooms v2.0.3) is not restated: opaque bytes */
  }
  if (must_read(&r, 1, &t)) return OREF_PANIC_META; /* :166 */
  o->compression = (t[0] == 1) ? 1 : (t[0] == 2 ? 2 : 0);
  if (must_read(&r, 1, &t)) return OREF_PANIC_META; /* :209 index type, skipped */
  if (must_read(&r, 8, &t)) return OREF_PANIC_META; /* :212 */
  uint64_t n = rd64(t);
  if (n == 0) return OREF_ERR_META_INVALID; /* :213-215 */
  /* every entry needs >= 42 bytes; a count beyond that would panic while parsing */
  if (n > (meta_len - r.i) / 42) return OREF_PANIC_META;
  o->entry_key = (const uint8_t **)calloc(n, sizeof(void *));
  o->entry_key_len = (uint64_t *)calloc(n, 8);
  o->entry_offset = (uint64_t *)calloc(n, 8);
  o->entry_block_size = (uint64_t *)calloc(n, 8);
  o->entry_original_size = (uint64_t *)calloc(n, 8);
  o->entry_compressed_size = (uint64_t *)calloc(n, 8);
  o->entry_hash = (uint64_t *)calloc(n, 8);
  for (uint64_t i = 0; i < n; i++) { /* :221-235 */
    if (must_read(&r, 2, &t)) goto panic;
    o->entry_key_len[i] = rd16(t);
    if (must_read(&r, o->entry_key_len[i], &o->entry_key[i])) goto panic;
    uint64_t *dst[5] = {o->entry_offset, o->entry_block_size, o->entry_original_size,
                        o->entry_compressed_size, o->entry_hash};
    for (int k = 0; k < 5; k++) {
      if (must_read(&r, 8, &t)) goto panic;
      dst[k][i] = rd64(t);
    }
  }
  o->n_entries = n;
  return OREF_OK;
panic:
  oref_meta_free(o);
  return OREF_PANIC_META;
}

void oref_meta_free(oref_meta *m) {
  free(m->entry_key);
  free(m->entry_key_len);
  free(m->entry_offset);
  free(m->entry_block_size);
  free(m->entry_original_size);
  free(m->entry_compressed_size);
  free(m->entry_hash);
  memset(m, 0, sizeof(*m));
}

/* FetchAndLoadMetadata segment_reader.go:91-141 */
int oref_fetch_meta(const uint8_t *buf, uint64_t buf_len, int64_t file_bytes, oref_meta *out,
                    uint64_t *meta_off, uint64_t *meta_len) {
  memset(out, 0, sizeof(*out));
  if (buf_len < 25) return OREF_ERR_IO; /* Seek(-25, End) -> negative position :93 */
  const uint8_t *tail = buf + buf_len - 25; /* :99-100 */
  if (rd64(tail + 17) != 69696969696969ULL) return OREF_ERR_MAGIC; /* :105-108 */
  if (tail[16] != 1) return OREF_ERR_VERSION;                       /* :110-113 */
  uint64_t moff = rd64(tail), mhash = rd64(tail + 8);                /* :115-116 */
  if ((int64_t)moff < 0) return OREF_ERR_IO;                         /* :119 Seek */
  int64_t mlen = file_bytes - (int64_t)moff - 25;                    /* :124 */
  if (mlen < 0) return OREF_PANIC_MAKESLICE;
  /* :125 bytes.Reader.Read: EOF when positioned at/after the end (even for a
   * zero-length read); otherwise copies what is available without checking n. */
  if (moff >= buf_len) return OREF_ERR_IO;
  uint64_t avail = buf_len - moff;
  uint8_t *mb = (uint8_t *)calloc((size_t)mlen + 1, 1);
  memcpy(mb, buf + moff, (size_t)((uint64_t)mlen < avail ? (uint64_t)mlen : avail));
  int rc;
  if (oref_xxh64(mb, (size_t)mlen, 0) != mhash || (uint64_t)mlen > avail) { /* :130-132 */
    /* (a short meta read that still matched its hash would need a 64-bit
     * collision; treated as a mismatch) */
    rc = OREF_ERR_META_HASH;
  } else {
    rc = oref_parse_meta(buf + moff, (uint64_t)mlen, out); /* :134 (bytes identical to mb) */
  }
  free(mb);
  if (rc == OREF_OK) {
    if (meta_off) *meta_off = moff;
    if (meta_len) *meta_len = (uint64_t)mlen;
  }
  return rc;
}

/* ======================================================================= */
/* ReadBlockWithStat (segment_reader.go:295-355)                            */
/* ======================================================================= */
/* zstd: zstd.NewReader(bytes.NewReader(rawBlockBytes[:CompressedSize])) and
 * io.Copy (:320-330), klauspost/compress v1.17.9 = standard RFC 8878 decoding
 * of every frame in the slice.  Checker: the system libzstd (dlopen, no
 * headers needed), the RFC's reference implementation. */
typedef size_t (*zstd_dec_fn)(void *, size_t, const void *, size_t);
typedef unsigned (*zstd_iserr_fn)(size_t);
typedef int (*zstd_code_fn)(size_t);
typedef void *(*zstd_mkd_fn)(void);
typedef size_t (*zstd_freed_fn)(void *);
typedef size_t (*zstd_begin_fn)(void *);
typedef size_t (*zstd_fh_fn)(void *, const void *, size_t);
typedef size_t (*zstd_next_fn)(void *);
typedef int (*zstd_nit_fn)(void *);
typedef size_t (*zstd_cont_fn)(void *, void *, size_t, const void *, size_t);
/* ZSTD_frameHeader (zstd.h 1.4.x) */
typedef struct {
  unsigned long long frameContentSize, windowSize;
  unsigned blockSizeMax;
  int frameType;
  unsigned headerSize, dictID, checksumFlag;
} zstd_fh_t;
static zstd_dec_fn z_dec;
static zstd_iserr_fn z_iserr;
static zstd_code_fn z_code;
static zstd_mkd_fn z_mkd;
static zstd_freed_fn z_freed;
static zstd_begin_fn z_begin;
static zstd_fh_fn z_fh;
static zstd_next_fn z_next;
static zstd_nit_fn z_nit;
static zstd_cont_fn z_cont;
static pthread_once_t z_once = PTHREAD_ONCE_INIT;
static void zstd_load(void) {
  void *h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) return;
  z_dec = (zstd_dec_fn)dlsym(h, "ZSTD_decompress");
  z_iserr = (zstd_iserr_fn)dlsym(h, "ZSTD_isError");
  z_code = (zstd_code_fn)dlsym(h, "ZSTD_getErrorCode");
  z_mkd = (zstd_mkd_fn)dlsym(h, "ZSTD_createDCtx");
  z_freed = (zstd_freed_fn)dlsym(h, "ZSTD_freeDCtx");
  z_begin = (zstd_begin_fn)dlsym(h, "ZSTD_decompressBegin");
  z_fh = (zstd_fh_fn)dlsym(h, "ZSTD_getFrameHeader");
  z_next = (zstd_next_fn)dlsym(h, "ZSTD_nextSrcSizeToDecompress");
  z_nit = (zstd_nit_fn)dlsym(h, "ZSTD_nextInputType");
  z_cont = (zstd_cont_fn)dlsym(h, "ZSTD_decompressContinue");
}
/* RFC 8878 3.1.1.2.3-4: a block decompresses to at most Block_Maximum_Size =
 * min(Window_Size, 128 KiB) (ZSTD_frameHeader.blockSizeMax).  libzstd 1.4.8's
 * one-shot decoder does not enforce it (a 200 KiB RLE block decodes); the
 * device decoder does, as the RFC and newer libzstd do.  Replays the frames
 * block by block (ZSTD_decompressContinue) into out (out_len bytes, the
 * one-shot result's length); 0 if any block exceeds its limit or the
 * block-wise API rejects the input (e.g. legacy v0.5-v0.7 frames, which the
 * 1.4.8 one-shot path still accepts and RFC 8878 does not define). */
static int zstd_blocks_within_max(const uint8_t *src, uint64_t n, uint8_t *out, uint64_t out_len) {
  void *d = z_mkd();
  if (!d) return 0;
  uint64_t at = 0, pos = 0;
  int ok = 1;
  while (ok && at < n) {
    zstd_fh_t fh;
    size_t r = z_fh(&fh, src + at, (size_t)(n - at));
    if (z_iserr(r) || r != 0 || z_iserr(z_begin(d))) {
      ok = 0;
      break;
    }
    for (;;) {
      size_t need = z_next(d);
      if (need == 0) break;
      if (need > n - at) {
        ok = 0;
        break;
      }
      int kind = z_nit(d); /* ZSTDnit_block = 2, ZSTDnit_lastBlock = 3 */
      size_t m = z_cont(d, out + pos, (size_t)(out_len + 64 - pos), src + at, need);
      if (z_iserr(m) || ((kind == 2 || kind == 3) && fh.frameType == 0 && m > fh.blockSizeMax)) {
        ok = 0;
        break;
      }
      at += need;
      pos += m;
    }
  }
  z_freed(d);
  return ok && pos == out_len;
}
/* Every frame of src[0, n), the whole output whatever OriginalSize says (Go's
 * io.Copy inflates the frames before its record walk); hint sizes the first
 * buffer only. */
static int zstd_block(const uint8_t *src, uint64_t n, uint64_t hint, uint8_t **out,
                      uint64_t *out_len) {
  pthread_once(&z_once, zstd_load);
  if (!z_dec || !z_iserr || !z_code || !z_mkd || !z_freed || !z_begin || !z_fh || !z_next ||
      !z_nit || !z_cont)
    return OREF_BLK_UNSUPPORTED;
  uint64_t cap = (hint < (1ull << 24) ? hint : (1ull << 24)) + 65536;
  for (;;) {
    uint8_t *buf = (uint8_t *)malloc(cap + 64);
    size_t r = z_dec(buf, cap, n ? src : (const uint8_t *)"", n);
    if (!z_iserr(r)) {
      if (!zstd_blocks_within_max(n ? src : (const uint8_t *)"", n, buf, r)) {
        free(buf);
        return OREF_BLK_ZSTD;
      }
      *out = buf;
      *out_len = r;
      return OREF_BLK_OK;
    }
    free(buf);
    if (z_code(r) != 70 /* dstSize_tooSmall */ || cap > (1ull << 31)) return OREF_BLK_ZSTD;
    cap *= 2;
  }
}

/* Shared bounds logic: the raw buffer is seg[off, off+block_size) (:309-316),
 * for LZ4 an empty buffer (:331-333), for zstd the decompressed frames (then
 * *owned is set and the caller frees it).  Returns the block status. */
static int block_buffer(const uint8_t *seg, uint64_t seg_len, const oref_block_desc *d,
                        int compression, const uint8_t **buf, uint64_t *buf_len,
                        uint8_t **owned) {
  *owned = NULL;
  if ((int64_t)d->offset < 0) return OREF_BLK_EOF; /* Seek error :303-306 */
  /* make([]byte, stat.BlockSize) (:309): the uint64 converts to int; a length
   * that is negative as int or above the runtime's maxAlloc panics
   * ("makeslice: len out of range", runtime/slice.go makeslice; maxAlloc =
   * 1 << heapAddrBits = 2^48 on linux/amd64 and linux/arm64, runtime/malloc.go) */
  if (d->block_size > OREF_GO_MAX_ALLOC) return OREF_BLK_PANIC;
  if (d->offset >= seg_len) return OREF_BLK_EOF;   /* bytes.Reader.Read io.EOF :310-313 */
  uint64_t avail = seg_len - d->offset;
  if (avail < d->block_size) return OREF_BLK_SHORT; /* :314-316 */
  if (compression == OREF_COMP_ZSTD) {
    if (d->compressed_size > d->block_size) return OREF_BLK_PANIC; /* slice bounds :321 */
    uint8_t *o = NULL;
    uint64_t n = 0;
    int st = zstd_block(seg + d->offset, d->compressed_size, d->original_size, &o, &n);
    if (st) return st;
    *owned = o;
    *buf = o;
    *buf_len = n;
    return OREF_BLK_OK;
  }
  *buf = seg + d->offset;
  *buf_len = (compression == OREF_COMP_LZ4) ? 0 : d->block_size; /* :331-335 (Q7) */
  return OREF_BLK_OK;
}

/* The record loop :338-352: `for consumed < OriginalSize`, each mustReadBytes
 * needing its full length (zero-length reads are free and yield nil, Q4). */
typedef void (*row_cb)(void *ctx, uint64_t rec, uint64_t klen, uint64_t vlen);
static int walk_records(const uint8_t *buf, uint64_t len, uint64_t orig, row_cb cb, void *ctx) {
  uint64_t p = 0;
  /* `totalReadBytes < int(stat.OriginalSize)` (:340): int(OriginalSize) is
   * negative from 2^63 on, so the loop runs no iteration (nil rows, no error) */
  if ((int64_t)orig < 0) orig = 0;
  while (p < orig) {
    if (len - p < 2) return OREF_BLK_PANIC; /* p <= len always holds here */
    uint64_t kl = rd16(buf + p);
    if (len - p < 6) return OREF_BLK_PANIC;
    uint64_t vl = rd32(buf + p + 2);
    if (kl && len - p - 6 < kl) return OREF_BLK_PANIC;
    if (vl && len - p - 6 - kl < vl) return OREF_BLK_PANIC;
    if (cb) cb(ctx, p, kl, vl);
    p += 6 + kl + vl;
  }
  return OREF_BLK_OK;
}

/* ---- Go's allocation fast path for the CPU baselines ---------------------
 * Go serves each make([]byte, n) from the P's mcache span of its size class:
 * no lock and no contention between Ps.  glibc malloc contends past ~16
 * threads on the GPU box's host, which a Go program would not,
 * so the baseline jobs (oref_*_go) allocate from a per-thread bump arena
 * (16-byte granules, like the small size classes) whose frees are no-ops; a
 * decode or encode job resets it between blocks / rows once 4 MiB are in use
 * (the GC's own work is not counted).  Outside those jobs (the oracle proper)
 * the functions below are plain malloc / realloc / free. */
typedef struct arena_chunk {
  struct arena_chunk *next;
  size_t cap, used;
  uint8_t *data;
} arena_chunk;
static __thread arena_chunk *t_arena;
static __thread int t_arena_on;
static __thread size_t t_arena_since;  /* bytes handed out since the last reset */
/* chunks of finished jobs, kept faulted-in for the next job (threads are
 * created per call; touching fresh pages would make every pass pay page faults) */
static arena_chunk *g_pool;
static size_t g_pool_n;  /* chunks pooled (capped: kPoolMax; the rest are freed) */
static pthread_mutex_t g_pool_mu = PTHREAD_MUTEX_INITIALIZER;
static const size_t kArenaChunk = (size_t)16 << 20;
static const size_t kPoolMax = 64; /* 1 GiB of faulted-in chunks kept across jobs */

static void arena_begin(void) {
  t_arena_on = 1;
  t_arena_since = 0;
}
static void arena_release(arena_chunk *c) { /* to the pool (standard-size chunks) or freed */
  if (c->cap != kArenaChunk) {
    free(c->data);
    free(c);
    return;
  }
  pthread_mutex_lock(&g_pool_mu);
  if (g_pool_n < kPoolMax) {
    c->next = g_pool;
    g_pool = c;
    g_pool_n++;
    c = NULL;
  }
  pthread_mutex_unlock(&g_pool_mu);
  if (c) {
    free(c->data);
    free(c);
  }
}
/* Free every pooled chunk (the CPU baselines call it after a sweep, so the
 * process does not keep the sweep's peak arena memory). */
void oref_arena_trim(void) {
  pthread_mutex_lock(&g_pool_mu);
  arena_chunk *c = g_pool;
  g_pool = NULL;
  g_pool_n = 0;
  pthread_mutex_unlock(&g_pool_mu);
  while (c) {
    arena_chunk *n = c->next;
    free(c->data);
    free(c);
    c = n;
  }
}
static void arena_reset(void) {
  if (!t_arena) return;
  arena_chunk *keep = t_arena, *c = keep->next;
  while (c) {
    arena_chunk *n = c->next;
    arena_release(c);
    c = n;
  }
  keep->next = NULL;
  keep->used = 0;
  t_arena_since = 0;
}
static void arena_end(void) {
  arena_reset();
  if (t_arena) arena_release(t_arena);
  t_arena = NULL;
  t_arena_on = 0;
}
static void *go_alloc(size_t n) {
  if (!t_arena_on) return malloc(n ? n : 1);
  n = n ? (n + 15) & ~(size_t)15 : 16;
  if (!t_arena || t_arena->used + n > t_arena->cap) {
    arena_chunk *c = NULL;
    if (n <= kArenaChunk) {
      pthread_mutex_lock(&g_pool_mu);
      if ((c = g_pool)) {
        g_pool = c->next;
        g_pool_n--;
      }
      pthread_mutex_unlock(&g_pool_mu);
    }
    if (!c) {
      c = (arena_chunk *)malloc(sizeof(*c));
      c->cap = n > kArenaChunk ? n : kArenaChunk;
      c->data = (uint8_t *)malloc(c->cap);
    }
    c->used = 0;
    c->next = t_arena;
    t_arena = c;
  }
  void *p = t_arena->data + t_arena->used;
  t_arena->used += n;
  t_arena_since += n;
  return p;
}
static void go_free(void *p) {
  if (!t_arena_on) free(p);
}
static void *go_realloc(void *p, size_t old, size_t n) {
  if (!t_arena_on) return realloc(p, n);
  void *q = go_alloc(n); /* append growth: a new backing array, the old one is garbage */
  if (p && old) memcpy(q, p, old < n ? old : n);
  return q;
}
static void arena_maybe_reset(void) {
  if (t_arena_on && t_arena_since > ((size_t)4 << 20)) arena_reset();
}

typedef struct {
  const uint8_t *buf;
  oref_rows *out;
} go_ctx;
static void go_row(void *c, uint64_t rec, uint64_t kl, uint64_t vl) {
  go_ctx *g = (go_ctx *)c;
  oref_rows *o = g->out;
  if (o->n == o->cap) { /* append growth :351 */
    const size_t old = o->cap * sizeof(oref_kv);
    o->cap = o->cap ? 2 * o->cap : 4;
    o->rows = (oref_kv *)go_realloc(o->rows, old, o->cap * sizeof(oref_kv));
  }
  oref_kv *kv = &o->rows[o->n++];
  kv->key_len = kl;
  kv->val_len = vl;
  kv->key = kl ? (uint8_t *)go_alloc(kl) : NULL; /* readBytes :490-494 */
  if (kl) memcpy(kv->key, g->buf + rec + 6, kl);
  kv->val = vl ? (uint8_t *)go_alloc(vl) : NULL;
  if (vl) memcpy(kv->val, g->buf + rec + 6 + kl, vl);
}

int oref_read_block(const uint8_t *seg, uint64_t seg_len, const oref_block_desc *d,
                    int compression, oref_rows *out) {
  memset(out, 0, sizeof(*out));
  const uint8_t *buf = NULL;
  uint64_t len = 0;
  uint8_t *owned = NULL;
  int st = block_buffer(seg, seg_len, d, compression, &buf, &len, &owned);
  if (st) return st;
  /* rawBlockBytes := make([]byte, BlockSize); Read (:309-310) -- a copy */
  uint8_t *copy = (uint8_t *)go_alloc(len ? len : 1);
  if (len) memcpy(copy, buf, len);
  free(owned);
  go_ctx g = {copy, out};
  st = walk_records(copy, len, d->original_size, go_row, &g);
  go_free(copy);
  if (st) oref_rows_free(out);
  return st;
}

void oref_rows_free(oref_rows *r) {
  for (uint64_t i = 0; i < r->n; i++) {
    go_free(r->rows[i].key);
    go_free(r->rows[i].val);
  }
  go_free(r->rows);
  memset(r, 0, sizeof(*r));
}

/* ---- CPU baseline (Go allocation semantics, N threads) ----------------- */
typedef struct {
  const uint8_t *seg;
  uint64_t seg_len;
  const oref_block_desc *d;
  uint64_t b0, b1;
  int comp;
  uint64_t rows, payload;
} job_t;
static void *job_run(void *a) {
  job_t *j = (job_t *)a;
  arena_begin();
  for (uint64_t b = j->b0; b < j->b1; b++) {
    oref_rows r;
    if (oref_read_block(j->seg, j->seg_len, &j->d[b], j->comp, &r) == OREF_BLK_OK) {
      j->rows += r.n;
      for (uint64_t i = 0; i < r.n; i++) j->payload += r.rows[i].key_len + r.rows[i].val_len;
      oref_rows_free(&r);
    }
    arena_maybe_reset();
  }
  arena_end();
  return NULL;
}
uint64_t oref_decode_range_go(const uint8_t *seg, uint64_t seg_len, const oref_block_desc *d,
                              uint64_t nblk, int compression, int threads, uint64_t *payload) {
  if (threads < 1) threads = 1;
  job_t *jobs = (job_t *)calloc((size_t)threads, sizeof(job_t));
  pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; t++) {
    jobs[t] = (job_t){seg, seg_len, d, nblk * t / threads, nblk * (t + 1) / threads, compression,
                      0, 0};
    if (threads > 1)
      pthread_create(&th[t], NULL, job_run, &jobs[t]);
    else
      job_run(&jobs[t]);
  }
  uint64_t rows = 0, pay = 0;
  for (int t = 0; t < threads; t++) {
    if (threads > 1) pthread_join(th[t], NULL);
    rows += jobs[t].rows;
    pay += jobs[t].payload;
  }
  free(jobs);
  free(th);
  if (payload) *payload = pay;
  return rows;
}

/* CPU baseline for the encode: SegmentWriter.WriteRow x n + Close with Go's
 * per-row allocation (rowBuf := make([]byte, 6+len(key)+len(val)) and two
 * copies, segment_writer.go:121-125).  `threads` writers encode contiguous
 * row ranges as separate segments (key-range shards). */
typedef struct {
  const uint8_t *ka, *va;
  const uint64_t *ko, *vo;
  const uint16_t *kl;
  const uint32_t *vl;
  uint64_t lo, hi, T, D;
  int lz4;
  uint64_t bytes;
  int rc;
} enc_job;

static void *enc_run(void *arg) {
  enc_job *j = (enc_job *)arg;
  oref_writer *w = oref_writer_new(j->T, j->D, 0, j->lz4);
  j->rc = 0;
  arena_begin();
  for (uint64_t i = j->lo; i < j->hi && !j->rc; i++) {
    const size_t k = j->kl[i], v = j->vl[i];
    uint8_t *row = (uint8_t *)go_alloc(6 + k + v); /* :121 make */
    memcpy(row + 6, j->ka + j->ko[i], k);          /* :124 */
    memcpy(row + 6 + k, j->va + j->vo[i], v);      /* :125 */
    j->rc = oref_writer_write_row(w, row + 6, k, row + 6 + k, v);
    go_free(row);
    arena_maybe_reset();
  }
  arena_end();
  uint64_t flen = 0;
  /* Close panics in Go when the last WriteRow flushed (Q1); the rows are
     written either way, and the throughput baseline counts them */
  if (!j->rc) {
    j->rc = oref_writer_close(w, NULL, &flen, NULL, NULL);
    if (j->rc == OREF_PANIC_NIL_WRITER) j->rc = 0;
  }
  j->bytes = flen;
  oref_writer_free(w);
  return NULL;
}

int oref_encode_go(const uint8_t *key_arena, const uint64_t *key_off, const uint16_t *key_len,
                   const uint8_t *val_arena, const uint64_t *val_off, const uint32_t *val_len,
                   uint64_t n, uint64_t threshold, uint64_t block_size, int lz4, int threads,
                   uint64_t *file_bytes) {
  if (threads < 1) threads = 1;
  enc_job *jobs = (enc_job *)calloc((size_t)threads, sizeof(enc_job));
  pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; t++) {
    jobs[t] = (enc_job){key_arena, val_arena, key_off, val_off, key_len, val_len,
                        n * t / threads, n * (t + 1) / threads, threshold, block_size, lz4, 0, 0};
    if (threads > 1)
      pthread_create(&th[t], NULL, enc_run, &jobs[t]);
    else
      enc_run(&jobs[t]);
  }
  int rc = 0;
  uint64_t bytes = 0;
  for (int t = 0; t < threads; t++) {
    if (threads > 1) pthread_join(th[t], NULL);
    if (jobs[t].rc) rc = jobs[t].rc;
    bytes += jobs[t].bytes;
  }
  free(jobs);
  free(th);
  if (file_bytes) *file_bytes = bytes;
  return rc;
}

/* One segment from SoA rows, single-threaded: WriteRow for every row
 * (segment_writer.go:80-146); the caller then calls oref_writer_close once
 * (:211-328).  The oracle side of the full-size encode parity test; *rc = 0
 * or the first writer error. */
oref_writer *oref_encode_soa(const uint8_t *key_arena, const uint64_t *key_off,
                             const uint16_t *key_len, const uint8_t *val_arena,
                             const uint64_t *val_off, const uint32_t *val_len, uint64_t n,
                             uint64_t threshold, uint64_t block_size, int *rc) {
  oref_writer *w = oref_writer_new(threshold, block_size, 0, 0);
  *rc = 0;
  for (uint64_t i = 0; i < n && !*rc; i++)
    *rc = oref_writer_write_row(w, key_arena + key_off[i], key_len[i], val_arena + val_off[i],
                                val_len[i]);
  return w;
}

/* ======================================================================= */
/* CPU baselines for bench.py configs C1 and CM (Go semantics)               */
/* ======================================================================= */
/* C1: one segment round trip -- WriteRow x n with Go's per-row rowBuf
 * (segment_writer.go:121), Close, then a full ascending read block by block
 * (RowIter.Next -> ReadBlockWithStat, segment_row_iter.go:63-95) with its
 * per-row copies.  `threads` independent round trips run concurrently. */
typedef struct {
  const uint8_t *ka, *va;
  const uint64_t *ko, *vo;
  const uint16_t *kl;
  const uint32_t *vl;
  uint64_t n, T, D;
  uint64_t rows, bytes;
  int rc;
} rt_job;

static void *rt_run(void *arg) {
  rt_job *j = (rt_job *)arg;
  enc_job e = {j->ka, j->va, j->ko, j->vo, j->kl, j->vl, 0, j->n, j->T, j->D, 0, 0, 0};
  oref_writer *w = oref_writer_new(j->T, j->D, 0, 0);
  j->rc = 0;
  arena_begin();
  for (uint64_t i = 0; i < j->n && !j->rc; i++) {
    const size_t k = e.kl[i], v = e.vl[i];
    uint8_t *row = (uint8_t *)go_alloc(6 + k + v);
    memcpy(row + 6, e.ka + e.ko[i], k);
    memcpy(row + 6 + k, e.va + e.vo[i], v);
    j->rc = oref_writer_write_row(w, row + 6, k, row + 6 + k, v);
    go_free(row);
    arena_maybe_reset();
  }
  const uint8_t *file = NULL;
  uint64_t flen = 0;
  if (!j->rc) j->rc = oref_writer_close(w, &file, &flen, NULL, NULL);
  j->rows = 0;
  j->bytes = flen;
  for (uint64_t b = 0; b < w->nidx && !j->rc; b++) {
    const oref_stat *st = &w->idx[b];
    oref_block_desc d = {st->offset, st->block_size, st->original_size, st->compressed_size};
    oref_rows r = {0, 0, 0};
    if (oref_read_block(file, flen, &d, 0, &r) == OREF_BLK_OK) j->rows += r.n;
    oref_rows_free(&r);
    arena_maybe_reset();
  }
  arena_end();
  oref_writer_free(w);
  return NULL;
}

uint64_t oref_roundtrip_go(const uint8_t *key_arena, const uint64_t *key_off,
                           const uint16_t *key_len, const uint8_t *val_arena,
                           const uint64_t *val_off, const uint32_t *val_len, uint64_t n,
                           uint64_t threshold, uint64_t block_size, int threads,
                           uint64_t *file_bytes) {
  if (threads < 1) threads = 1;
  rt_job *jobs = (rt_job *)calloc((size_t)threads, sizeof(rt_job));
  pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; t++) {
    jobs[t] = (rt_job){key_arena, val_arena, key_off, val_off, key_len, val_len, n, threshold,
                       block_size, 0, 0, 0};
    if (threads > 1)
      pthread_create(&th[t], NULL, rt_run, &jobs[t]);
    else
      rt_run(&jobs[t]);
  }
  uint64_t rows = 0, bytes = 0;
  for (int t = 0; t < threads; t++) {
    if (threads > 1) pthread_join(th[t], NULL);
    rows += jobs[t].rc ? 0 : jobs[t].rows;
    bytes += jobs[t].bytes;
  }
  free(jobs);
  free(th);
  if (file_bytes) *file_bytes = bytes;
  return rows;
}

/* CM: one compaction step -- every block of K input segments decoded with
 * ReadBlockWithStat's semantics (per-row copies), a k-way merge ascending in
 * which the first (newest) segment holding a key owns it (the L0 rule of
 * snapshot_reader.GetRange, snapshot_reader.go:294-331), and the merged rows
 * written with the Go writer (WriteRow + Close).  `threads` independent
 * compactions of the same inputs run concurrently.  Returns the merged rows
 * of one compaction (0 on error); *in_bytes = sum of input BlockSize. */
typedef struct {
  int k;
  const uint8_t *const *segs;
  const uint64_t *lens;
  const oref_block_desc *const *descs;
  const uint64_t *nblks;
  uint64_t T, D;
  uint64_t rows_out, bytes_out;
  int rc;
} cm_job;

static int kv_less(const oref_kv *a, const oref_kv *b) {
  const uint64_t n = a->key_len < b->key_len ? a->key_len : b->key_len;
  const int c = n ? memcmp(a->key, b->key, n) : 0;
  return c < 0 || (c == 0 && a->key_len < b->key_len);
}
static int kv_equal(const oref_kv *a, const oref_kv *b) {
  return a->key_len == b->key_len && (!a->key_len || !memcmp(a->key, b->key, a->key_len));
}

static void *cm_run(void *arg) {
  cm_job *j = (cm_job *)arg;
  oref_rows *all = (oref_rows *)calloc((size_t)j->k, sizeof(oref_rows));
  j->rc = 0;
  arena_begin();  /* (no reset: the decoded rows live until the merge has written them) */
  for (int s = 0; s < j->k && !j->rc; s++) { /* decode: ReadBlockWithStat per block */
    for (uint64_t b = 0; b < j->nblks[s] && !j->rc; b++) {
      oref_rows r = {0, 0, 0};
      if (oref_read_block(j->segs[s], j->lens[s], &j->descs[s][b], 0, &r) != OREF_BLK_OK) {
        j->rc = -1;
      } else {
        for (uint64_t i = 0; i < r.n; i++) { /* append (the RowIter's rows) */
          if (all[s].n == all[s].cap) {
            const size_t old = all[s].cap * sizeof(oref_kv);
            all[s].cap = all[s].cap ? 2 * all[s].cap : 1024;
            all[s].rows = (oref_kv *)go_realloc(all[s].rows, old, all[s].cap * sizeof(oref_kv));
          }
          all[s].rows[all[s].n++] = r.rows[i];
        }
        go_free(r.rows); /* the row copies now belong to all[s] */
      }
    }
  }
  oref_writer *w = oref_writer_new(j->T, j->D, 0, 0);
  uint64_t *pos = (uint64_t *)calloc((size_t)j->k, sizeof(uint64_t));
  j->rows_out = 0;
  while (!j->rc) { /* k-way merge: smallest key; ties -> lowest (newest) segment */
    int best = -1;
    for (int s = 0; s < j->k; s++)
      if (pos[s] < all[s].n && (best < 0 || kv_less(&all[s].rows[pos[s]], &all[best].rows[pos[best]])))
        best = s;
    if (best < 0) break;
    const oref_kv *kv = &all[best].rows[pos[best]];
    for (int s = 0; s < j->k; s++) /* shadowed versions of the same key */
      if (s != best && pos[s] < all[s].n && kv_equal(&all[s].rows[pos[s]], kv)) pos[s]++;
    j->rc = oref_writer_write_row(w, kv->key, kv->key_len, kv->val, kv->val_len);
    pos[best]++;
    j->rows_out++;
  }
  uint64_t flen = 0;
  /* Close panics in Go when the last WriteRow flushed (Q1); the rows are
     written either way, and the throughput baseline counts them */
  if (!j->rc) {
    j->rc = oref_writer_close(w, NULL, &flen, NULL, NULL);
    if (j->rc == OREF_PANIC_NIL_WRITER) j->rc = 0;
  }
  j->bytes_out = flen;
  oref_writer_free(w);
  for (int s = 0; s < j->k; s++) oref_rows_free(&all[s]);
  arena_end();
  free(all);
  free(pos);
  return NULL;
}

uint64_t oref_compact_go(int k, const uint8_t *const *segs, const uint64_t *seg_lens,
                         const oref_block_desc *const *descs, const uint64_t *nblks,
                         uint64_t threshold, uint64_t block_size, int threads,
                         uint64_t *out_bytes) {
  if (threads < 1) threads = 1;
  cm_job *jobs = (cm_job *)calloc((size_t)threads, sizeof(cm_job));
  pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; t++) {
    jobs[t] = (cm_job){k, segs, seg_lens, descs, nblks, threshold, block_size, 0, 0, 0};
    if (threads > 1)
      pthread_create(&th[t], NULL, cm_run, &jobs[t]);
    else
      cm_run(&jobs[t]);
  }
  uint64_t rows = 0, bytes = 0;
  int rc = 0;
  for (int t = 0; t < threads; t++) {
    if (threads > 1) pthread_join(th[t], NULL);
    if (jobs[t].rc) rc = jobs[t].rc;
    rows = jobs[t].rows_out;
    bytes += jobs[t].bytes_out;
  }
  free(jobs);
  free(th);
  if (out_bytes) *out_bytes = bytes;
  return rc ? 0 : rows;
}

/* ======================================================================= */
/* SoA restatement of the product output layout                 */
/* ======================================================================= */
typedef struct {
  uint64_t rows, kb, vb;
} cnt_ctx;
static void cnt_row(void *c, uint64_t rec, uint64_t kl, uint64_t vl) {
  (void)rec;
  cnt_ctx *k = (cnt_ctx *)c;
  k->rows++;
  k->kb += kl;
  k->vb += vl;
}

void oref_block_counts(const uint8_t *seg, uint64_t seg_len, const oref_block_desc *d,
                       uint64_t nblk, int compression, int32_t *status, uint64_t *rows,
                       uint64_t *kbytes, uint64_t *vbytes) {
  for (uint64_t b = 0; b < nblk; b++) {
    const uint8_t *buf = NULL;
    uint64_t len = 0;
    cnt_ctx c = {0, 0, 0};
    uint8_t *owned = NULL;
    int st = block_buffer(seg, seg_len, &d[b], compression, &buf, &len, &owned);
    if (!st) st = walk_records(buf, len, d[b].original_size, cnt_row, &c);
    free(owned);
    if (st) c = (cnt_ctx){0, 0, 0}; /* a failed block contributes no rows */
    status[b] = st;
    rows[b] = c.rows;
    kbytes[b] = c.kb;
    vbytes[b] = c.vb;
  }
}

typedef struct {
  const uint8_t *buf;
  uint64_t blk_off;
  int index_only;
  uint64_t g, kpos, vpos; /* next global row, next arena byte */
  uint64_t *key_off, *val_off;
  uint16_t *key_len;
  uint32_t *val_len;
  uint8_t *ka, *va;
} soa_ctx;
static void soa_row(void *c, uint64_t rec, uint64_t kl, uint64_t vl) {
  soa_ctx *s = (soa_ctx *)c;
  uint64_t g = s->g++;
  s->key_len[g] = (uint16_t)kl;
  s->val_len[g] = (uint32_t)vl;
  if (s->index_only) {
    s->key_off[g] = s->blk_off + rec + 6;
    s->val_off[g] = s->blk_off + rec + 6 + kl;
  } else {
    s->key_off[g] = s->kpos;
    s->val_off[g] = s->vpos;
    if (kl) memcpy(s->ka + s->kpos, s->buf + rec + 6, kl);
    if (vl) memcpy(s->va + s->vpos, s->buf + rec + 6 + kl, vl);
    s->kpos += kl;
    s->vpos += vl;
  }
}

static inline uint64_t round16(uint64_t x) { return (x + 15) & ~(uint64_t)15; }

void oref_decode_soa(const uint8_t *seg, uint64_t seg_len, const oref_block_desc *d,
                     uint64_t nblk, int compression, int index_only, uint64_t *row_start,
                     uint64_t *key_base, uint64_t *val_base, uint64_t *key_off,
                     uint16_t *key_len, uint64_t *val_off, uint32_t *val_len,
                     uint8_t *key_arena, uint8_t *val_arena, int32_t *status) {
  uint64_t g = 0, kb = 0, vb = 0;
  for (uint64_t b = 0; b < nblk; b++) {
    row_start[b] = g;
    if (!index_only) {
      key_base[b] = kb;
      val_base[b] = vb;
    }
    const uint8_t *buf = NULL;
    uint64_t len = 0;
    uint8_t *owned = NULL;
    int st = block_buffer(seg, seg_len, &d[b], compression, &buf, &len, &owned);
    if (!st && index_only && compression == OREF_COMP_ZSTD)
      st = OREF_BLK_UNSUPPORTED; /* spans into seg do not exist for zstd blocks */
    if (!st) st = walk_records(buf, len, d[b].original_size, NULL, NULL); /* validate first */
    status[b] = st;
    if (st) {
      free(owned);
      continue;
    }
    soa_ctx s = {buf, d[b].offset, index_only, g, kb, vb, key_off, val_off, key_len, val_len,
                 key_arena, val_arena};
    walk_records(buf, len, d[b].original_size, soa_row, &s);
    free(owned);
    g = s.g;
    if (!index_only) {
      /* each block's arena region is padded with zeros to a 16-byte multiple */
      uint64_t kend = round16(s.kpos), vend = round16(s.vpos);
      if (kend > s.kpos) memset(key_arena + s.kpos, 0, kend - s.kpos);
      if (vend > s.vpos) memset(val_arena + s.vpos, 0, vend - s.vpos);
      kb = kend;
      vb = vend;
    }
  }
  row_start[nblk] = g;
}
