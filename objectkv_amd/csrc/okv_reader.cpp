// okv_reader.cpp -- host C++ mirror of sst.SegmentReader / RowIter / GetRow /
// GetRange (/root/reference/sst/segment_reader.go:65-487,
// segment_row_iter.go:11-212) whose block reads come from the batched GPU
// decode (okv_decode_blocks).  The Go control flow is restated statement by
// statement, quirks included (they are cited inline); only ReadBlockWithStat's
// record loop moved to the device.  No CPU decode fallback exists: without a
// GPU context block reads fail with OKV_R_GPU.
//
// Block reads are bounded exactly as the cgo shim's (INTEGRATION.md
// ReadBlocks): a GPU call decodes
//   * GetRow / ReadBlockWithStat (:362-404, :295): the one block it reads;
//   * GetRange (:410-475): the block set its btree walks select (:421-458);
//   * RowIter.Next / Seek (segment_row_iter.go:83, :143, :165): the block and
//     the next kIterWindow - 1 in the iteration direction, kept as the
//     iteration window (later reads of those blocks are served from it);
// and stages only the bytes [min Offset, max Offset + BlockSize) of the batch
// (clamped to the storage), with the offsets rebased onto that span so Go's
// outcomes are kept: a block at or past the end reads as io.EOF, one running
// past it is short, a negative Offset is a Seek error, an oversized BlockSize
// the makeslice panic (segment_reader.go:303-316).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "okv_host.h"
#include "okv_sst.h"

namespace {

typedef std::vector<uint8_t> Bytes;

// A Go []byte: nil and empty are distinct values (statLastKey == nil tests,
// segment_row_iter.go:47) but compare equal (bytes.Equal / bytes.Compare).
struct GoBytes {
  bool nil = true;
  Bytes b;
  static GoBytes of(const uint8_t* p, uint64_t n) {  // mustReadBytes: n == 0 -> nil
    GoBytes g;
    if (n) {
      g.nil = false;
      g.b.assign(p, p + n);
    }
    return g;
  }
};

int bcmp(const uint8_t* a, size_t al, const uint8_t* b, size_t bl) {  // bytes.Compare
  const size_t n = al < bl ? al : bl;
  const int c = n ? std::memcmp(a, b, n) : 0;
  if (c) return c < 0 ? -1 : 1;
  return al < bl ? -1 : (al > bl ? 1 : 0);
}
int bcmp(const Bytes& a, const Bytes& b) { return bcmp(a.data(), a.size(), b.data(), b.size()); }

struct Entry {  // BlockStat (block_stat.go:9-24) as stored in the btree
  Bytes first_key;
  okv_block_desc d;
  uint64_t hash;
  uint64_t file_index;  // position in the meta block (the decode batch)
};

}  // namespace

namespace {

// iterWindow: blocks per GPU call while iterating.
constexpr size_t kIterWindow = 256;

// One GPU decode of a batch of blocks (okv_decode_blocks), with the rows of
// each batch entry built lazily.  Shared: the iteration window, an iterator's
// current block and the last GetRow / GetRange results may all hold it.
template <class T>
using Arr = std::unique_ptr<T[]>;  // uninitialised: the decode writes what is read
template <class T>
Arr<T> arr(uint64_t n) {
  return Arr<T>(new T[n ? n : 1]);
}
struct Batch {
  std::vector<uint32_t> entries;  // file_entries index of each batch entry
  std::vector<int32_t> status;
  std::vector<uint64_t> row_start;
  Arr<uint64_t> key_off, val_off;
  Arr<uint16_t> key_len;
  Arr<uint32_t> val_len;
  Arr<uint8_t> key_arena, val_arena;
  std::vector<std::vector<okv_row>> rows;
  std::vector<bool> built;
};
typedef std::shared_ptr<Batch> BatchP;

}  // namespace

struct okv_reader {
  okv_ctx* ctx = nullptr;
  std::vector<uint8_t> data;  // what the io.ReadSeeker reads (the storage)
  int64_t file_bytes = 0;
  bool closed = false;
  // metadata (SegmentMetadata, segment_reader.go:43-55)
  bool have_meta = false;
  int compression = 0;
  GoBytes first_key, last_key;
  std::unique_ptr<okv_meta, void (*)(okv_meta*)> meta{nullptr, okv_meta_free};  // (its bloom filter)
  std::vector<Entry> file_entries;  // meta block order
  std::vector<Entry> tree;          // google/btree.BTreeG ordered by FirstKey (ReplaceOrInsert)
  // the iteration window: its batch and each file entry's slot in it (-1: absent)
  BatchP window;
  std::vector<int32_t> window_slot;
  BatchP last_read;    // the last ReadBlockWithStat batch outside the window (GetRow)
  BatchP range_batch;  // the last GetRange batch
  std::vector<okv_row> range_out;
  std::vector<uint8_t> point_key, point_val;  // GetRow's row from okv_point_get
  okv_reader_io io{};  // GPU calls, blocks decoded, bytes staged
};

struct okv_iter {
  okv_reader* s;
  int direction;
  GoBytes stat_last_key;               // statLastKey
  bool rows_nil = true;                // blockRows == nil
  std::vector<okv_row> rows;           // blockRows
  BatchP rows_batch;                   // keeps blockRows' bytes alive
  int64_t idx = 0;                     // blockRowIdx
};

namespace {

// ---- btree helpers (google/btree v1.1.2 semantics over a sorted vector) ----
size_t lower(const okv_reader* r, const uint8_t* k, size_t kl) {  // first item >= k
  size_t lo = 0, hi = r->tree.size();
  while (lo < hi) {
    const size_t m = (lo + hi) / 2;
    if (bcmp(r->tree[m].first_key.data(), r->tree[m].first_key.size(), k, kl) < 0)
      lo = m + 1;
    else
      hi = m;
  }
  return lo;
}
size_t upper(const okv_reader* r, const uint8_t* k, size_t kl) {  // first item > k
  size_t lo = 0, hi = r->tree.size();
  while (lo < hi) {
    const size_t m = (lo + hi) / 2;
    if (bcmp(r->tree[m].first_key.data(), r->tree[m].first_key.size(), k, kl) <= 0)
      lo = m + 1;
    else
      hi = m;
  }
  return lo;
}

int load_meta(okv_reader* r, okv_meta* m) {
  r->compression = okv_meta_compression(m);
  uint64_t n = 0;
  const uint8_t* p = okv_meta_first_key(m, &n);
  r->first_key = GoBytes::of(p, n);
  p = okv_meta_last_key(m, &n);
  r->last_key = GoBytes::of(p, n);
  const uint64_t nb = okv_meta_num_blocks(m);
  r->file_entries.clear();
  r->tree.clear();
  for (uint64_t i = 0; i < nb; ++i) {
    Entry e;
    const uint8_t* fk;
    uint64_t fl;
    okv_meta_block(m, i, &e.d, &e.hash, &fk, &fl);
    e.first_key.assign(fk, fk + fl);
    e.file_index = i;
    r->file_entries.push_back(e);
    // ReplaceOrInsert (segment_reader.go:234): an equal FirstKey replaces (Q9)
    const size_t pos = lower(r, e.first_key.data(), e.first_key.size());
    if (pos < r->tree.size() && bcmp(r->tree[pos].first_key, e.first_key) == 0)
      r->tree[pos] = e;
    else
      r->tree.insert(r->tree.begin() + pos, e);
  }
  r->meta.reset(m);  // kept for GetRow's bloom probe
  r->have_meta = true;
  r->window.reset();
  r->window_slot.assign(r->file_entries.size(), -1);
  r->last_read.reset();
  r->range_batch.reset();
  return OKV_OK;
}

int ensure_meta(okv_reader* r) {  // "Fetches the metadata if not already loaded"
  if (r->have_meta) return OKV_OK;
  return okv_reader_fetch_metadata(r);
}

// ReadBlocks: one GPU decode of the given file entries,
// staging only their span of the storage.
// The bytes a batch of these file entries stages: the span of the blocks with
// a non-negative Offset inside the storage (the others fail before any read:
// Seek error, or io.EOF at / past the end), and the descriptors rebased onto
// it (offsets >= the storage end stay >= the span end -- io.EOF --, a
// BlockSize past the end stays short; negative ones keep their sign).
void stage_span(const okv_reader* r, const std::vector<uint32_t>& entries,
                std::vector<okv_block_desc>* descs, const uint8_t** seg, uint64_t* n) {
  const uint64_t nbytes = r->data.size();
  uint64_t lo = UINT64_MAX, hi = 0;
  for (uint32_t e : entries) {
    const okv_block_desc& d = r->file_entries[e].d;
    if (int64_t(d.offset) < 0 || d.offset >= nbytes) continue;
    lo = std::min(lo, d.offset);
    hi = std::max(hi, d.offset + std::min(d.block_size, nbytes - d.offset));
  }
  if (lo > hi) lo = hi = 0;
  descs->resize(entries.size());
  for (size_t i = 0; i < entries.size(); ++i) {
    (*descs)[i] = r->file_entries[entries[i]].d;
    if (int64_t((*descs)[i].offset) >= 0) (*descs)[i].offset -= lo;
  }
  *seg = hi > lo ? r->data.data() + lo : nullptr;
  *n = hi - lo;
}

int decode_batch(okv_reader* r, const std::vector<uint32_t>& entries, BatchP* out) {
  if (!r->ctx) return OKV_R_GPU;
  const uint32_t nb = uint32_t(entries.size());
  std::vector<okv_block_desc> descs;
  const uint8_t* seg;
  uint64_t n;
  stage_span(r, entries, &descs, &seg, &n);
  uint64_t rows = 0, kb = 0, vb = 0;
  int rc;
  // a small batch (GetRow's one block) sizes its outputs from bounds (one GPU
  // walk); a large one (an iteration window, GetRange) from the plan, so it
  // allocates what it fills; zstd (decompressed sizes) always plans
  if (r->compression == OKV_COMP_ZSTD || n > (uint64_t(1) << 20)) {
    rc = okv_decode_plan(r->ctx, seg, n, descs.data(), nb, r->compression, 0, &rows, &kb, &vb);
    if (rc) return OKV_R_GPU;
  } else {
    // bounds from the descriptors: a block's records lie in its BlockSize
    // bytes inside the span (>= 6 bytes each), each region pads to 16 bytes;
    // the decode then sizes its device outputs the same way (one walk)
    for (const okv_block_desc& d : descs) {
      uint64_t span = 0;
      if (r->compression != OKV_COMP_LZ4 && int64_t(d.offset) >= 0 && d.offset < n)
        span = std::min<uint64_t>(d.block_size, n - d.offset);
      rows += span / 6;
      kb += span + 16;
    }
    vb = kb;
  }
  BatchP B = std::make_shared<Batch>();
  B->entries = entries;
  B->row_start.assign(nb + 1, 0);
  B->status.assign(nb, 0);
  B->key_off = arr<uint64_t>(rows + 1);
  B->val_off = arr<uint64_t>(rows + 1);
  B->key_len = arr<uint16_t>(rows + 1);
  B->val_len = arr<uint32_t>(rows + 1);
  B->key_arena = arr<uint8_t>(kb + 16);
  B->val_arena = arr<uint8_t>(vb + 16);
  std::vector<uint64_t> kbase(nb + 1), vbase(nb + 1);
  okv_decode_out o;
  std::memset(&o, 0, sizeof(o));
  o.row_start = B->row_start.data();
  o.key_base = kbase.data();
  o.val_base = vbase.data();
  o.blk_status = B->status.data();
  o.key_off = B->key_off.get();
  o.key_len = B->key_len.get();
  o.val_off = B->val_off.get();
  o.val_len = B->val_len.get();
  o.key_arena = B->key_arena.get();
  o.val_arena = B->val_arena.get();
  o.row_cap = rows;
  o.key_cap = kb;
  o.val_cap = vb;
  rc = okv_decode_blocks(r->ctx, seg, n, descs.data(), nb, r->compression, &o, 0);
  if (rc) return OKV_R_GPU;
  B->rows.assign(nb, {});
  B->built.assign(nb, false);
  r->io.calls++;
  r->io.blocks += nb;
  r->io.bytes_staged += n;
  *out = B;
  return OKV_OK;
}

// A block's ReadBlockWithStat outcome (segment_reader.go:295-355) as the
// reader's error: the Go error / panic, or OKV_OK.
int block_rc(int32_t st) {
  switch (st) {
    case OKV_BLK_OK: return OKV_OK;
    case OKV_BLK_EOF: return OKV_R_BLOCK_EOF;
    case OKV_BLK_SHORT: return OKV_R_BLOCK_SHORT;
    case OKV_BLK_PANIC: return OKV_R_PANIC;
    case OKV_BLK_UNSUPPORTED: return OKV_R_UNSUPPORTED;
    case OKV_BLK_ZSTD_ERROR: return OKV_R_ZSTD;
    default: return OKV_R_GPU;  // (capacity: the plan sized every output)
  }
}

// ReadBlockWithStat's outcome for batch entry `slot`: its rows, or the Go
// error / panic.
int batch_rows(Batch& B, uint32_t slot, const std::vector<okv_row>** rows) {
  if (const int rc = block_rc(B.status[slot])) return rc;
  if (!B.built[slot]) {
    std::vector<okv_row>& out = B.rows[slot];
    for (uint64_t g = B.row_start[slot]; g < B.row_start[slot + 1]; ++g) {
      okv_row row;
      row.key_len = B.key_len[g];
      row.val_len = B.val_len[g];
      row.key = row.key_len ? B.key_arena.get() + B.key_off[g] : nullptr;  // nil (Q4)
      row.val = row.val_len ? B.val_arena.get() + B.val_off[g] : nullptr;
      out.push_back(row);
    }
    B.built[slot] = true;
  }
  *rows = &B.rows[slot];
  return OKV_OK;
}

// ReadBlockWithStat(stat) for the btree entry at tree position t: served from
// the iteration window when it holds the block, else a one-block GPU call
// (GetRow stages BlockSize bytes, not the segment).  *keep owns the rows.
int read_block(okv_reader* r, size_t t, const std::vector<okv_row>** rows, BatchP* keep) {
  int rc = ensure_meta(r);
  if (rc) return rc;
  const uint32_t e = uint32_t(r->tree[t].file_index);
  if (r->window && r->window_slot[e] >= 0) {
    // the rows must outlive a later window replacement (okv_host.h: valid
    // until the next read_block / get_row / get_range call)
    r->last_read = r->window;
    *keep = r->window;
    return batch_rows(*r->window, uint32_t(r->window_slot[e]), rows);
  }
  BatchP B;
  if ((rc = decode_batch(r, {e}, &B))) return rc;
  r->last_read = B;
  *keep = B;
  return batch_rows(*B, 0, rows);
}

// RowIter's block read (segment_row_iter.go:83, :143, :165): on a window miss
// it decodes this block and the next kIterWindow - 1 btree entries in the
// iteration direction in one batch, which becomes the window.
int read_block_iter(okv_reader* r, size_t t, int direction, const std::vector<okv_row>** rows,
                    BatchP* keep) {
  int rc = ensure_meta(r);
  if (rc) return rc;
  const uint32_t e = uint32_t(r->tree[t].file_index);
  if (r->window && r->window_slot[e] >= 0) {
    *keep = r->window;
    return batch_rows(*r->window, uint32_t(r->window_slot[e]), rows);
  }
  std::vector<uint32_t> batch{e};  // the block itself first
  if (direction == 1) {
    for (size_t i = t; i-- > 0 && batch.size() < kIterWindow;)
      batch.push_back(uint32_t(r->tree[i].file_index));
  } else {
    for (size_t i = t + 1; i < r->tree.size() && batch.size() < kIterWindow; ++i)
      batch.push_back(uint32_t(r->tree[i].file_index));
  }
  BatchP B;
  if ((rc = decode_batch(r, batch, &B))) {
    // a failure of the whole window call (e.g. an allocation for a later,
    // highly inflating block) is not this block's outcome: read it alone, as
    // Go's Next would, and keep the current window
    if (batch.size() == 1 || (rc = decode_batch(r, {e}, &B))) return rc;
    *keep = B;
    return batch_rows(*B, 0, rows);
  }
  if (r->window)
    for (uint32_t x : r->window->entries) r->window_slot[x] = -1;
  r->window = B;
  for (uint32_t i = 0; i < uint32_t(batch.size()); ++i) r->window_slot[batch[i]] = int32_t(i);
  *keep = B;
  return batch_rows(*B, 0, rows);
}

}  // namespace

extern "C" {

okv_reader* okv_reader_open(okv_ctx* ctx, const uint8_t* data, uint64_t len, int64_t file_bytes) {
  okv_reader* r = new okv_reader();
  r->ctx = ctx;
  if (len) r->data.assign(data, data + len);
  r->file_bytes = file_bytes;
  return r;
}

int okv_reader_fetch_metadata(okv_reader* r) {  // FetchAndLoadMetadata :91-141
  okv_meta* m = nullptr;
  const int rc = okv_meta_fetch(r->data.empty() ? nullptr : r->data.data(), r->data.size(),
                                r->file_bytes, &m);
  if (rc) return rc;
  return load_meta(r, m);
}

int okv_reader_load_metadata(okv_reader* r, const uint8_t* meta, uint64_t len) {
  okv_meta* m = nullptr;  // BytesToMetadata :147 + LoadCachedMetadata :75
  const int rc = okv_meta_parse(meta, len, &m);
  if (rc) return rc;
  return load_meta(r, m);
}

int okv_reader_num_blocks(okv_reader* r, uint64_t* n) {
  const int rc = ensure_meta(r);
  if (rc) return rc;
  *n = r->tree.size();
  return OKV_OK;
}

int okv_reader_read_block(okv_reader* r, uint64_t i, const okv_row** rows, uint64_t* n) {
  int rc = ensure_meta(r);
  if (rc) return rc;
  if (i >= r->tree.size()) return OKV_E_ARG;
  const std::vector<okv_row>* v = nullptr;
  BatchP keep;
  if ((rc = read_block(r, size_t(i), &v, &keep))) return rc;
  *rows = v->empty() ? nullptr : v->data();
  *n = v->size();
  return OKV_OK;
}

int okv_reader_get_row(okv_reader* r, const uint8_t* key, size_t klen, okv_row* out) {
  int rc = ensure_meta(r);  // GetRow :362-404
  if (rc) return rc;
  // bloom probe (:371-378, probeBloomFilter :245-258) on the host: a key the
  // filter rejects costs no block read and no GPU call
  if (okv_meta_has_bloom(r->meta.get())) {
    const int t = okv_meta_bloom_test(r->meta.get(), key, klen);
    if (t < 0) return t;                 // Go's panic (a filter with m == 0)
    if (t == 0) return OKV_R_NO_ROWS;    // "did not find row in bloom filter"
  }
  const size_t up = upper(r, key, klen);  // DescendLessOrEqual first item (:381-385)
  if (up == 0) return OKV_R_NO_ROWS;
  const uint32_t e = uint32_t(r->tree[up - 1].file_index);
  if (r->ctx && !(r->window && r->window_slot[e] >= 0) && r->compression != OKV_COMP_ZSTD) {
    // ReadBlockWithStat + the row loop (:387-403) in one point-path launch:
    // only the matching row comes back (found == -1: not a point-path block)
    std::vector<okv_block_desc> d;
    const uint8_t* seg;
    uint64_t n;
    stage_span(r, {e}, &d, &seg, &n);
    okv_point_row pr;
    if (okv_point_get(r->ctx, seg, n, d.data(), r->compression, key, klen, &pr)) return OKV_R_GPU;
    if (okv_last_path(r->ctx) == OKV_PATH_POINT) {  // a launch, whatever it found
      r->io.calls++;
      r->io.blocks++;
      r->io.bytes_staged += n;
    }
    if (pr.found != -1) {
      if (const int brc = block_rc(pr.status)) return brc;
      if (pr.found == 0) return OKV_R_NO_ROWS;  // "did not find row in block"
      // (valid until the next read call, okv_host.h)
      r->point_key.assign(pr.key, pr.key + pr.key_len);
      r->point_val.assign(pr.val, pr.val + pr.val_len);
      out->key_len = pr.key_len;
      out->val_len = pr.val_len;
      out->key = pr.key_len ? r->point_key.data() : nullptr;  // nil (Q4)
      out->val = pr.val_len ? r->point_val.data() : nullptr;
      return OKV_OK;
    }
  }
  const std::vector<okv_row>* rows = nullptr;
  BatchP keep;
  if ((rc = read_block(r, up - 1, &rows, &keep))) return rc;
  for (const okv_row& row : *rows)
    if (bcmp(row.key, row.key_len, key, klen) == 0) {  // bytes.Equal (:398)
      *out = row;
      return OKV_OK;
    }
  return OKV_R_NO_ROWS;
}

int okv_reader_get_range(okv_reader* r, const uint8_t* start, size_t slen, const uint8_t* end,
                         size_t elen, const okv_row** rows_out, uint64_t* n) {
  int rc = ensure_meta(r);  // GetRange :410-475
  if (rc) return rc;
  const bool unbound_start = slen == 0;                     // bytes.Equal(start, nil) :418
  const bool unbound_end = elen == 1 && end[0] == 0xff;     // :419
  const size_t N = r->tree.size();
  std::vector<bool> pick(N, false);  // the stats map (:422), deduplicated by first key
  if (unbound_start) {
    for (size_t i = 0; i < lower(r, end, elen); ++i) pick[i] = true;  // AscendLessThan (:427)
  } else {
    for (size_t i = upper(r, start, slen); i-- > 0;) {  // DescendLessOrEqual(start) (:432-435)
      pick[i] = true;
      if (!(bcmp(start, slen, r->tree[i].first_key.data(), r->tree[i].first_key.size()) <= 0))
        break;
    }
  }
  const size_t up = upper(r, end, elen);  // DescendLessOrEqual(end), first item only (:440-443)
  if (up > 0) pick[up - 1] = true;
  for (size_t i = lower(r, end, elen); i < N; ++i) {  // AscendGreaterOrEqual(end) (:446-453)
    if (!unbound_end && bcmp(end, elen, r->tree[i].first_key.data(),
                             r->tree[i].first_key.size()) <= 0)
      break;
    pick[i] = true;
  }
  // the candidate blocks in one batch (Go ranges over a map, in random order;
  // ascending FirstKey order here, :457), served from the window when it holds
  // every one of them
  std::vector<uint32_t> list;
  for (size_t i = 0; i < N; ++i)
    if (pick[i]) list.push_back(uint32_t(r->tree[i].file_index));
  BatchP B;
  bool from_window = r->window != nullptr;
  for (uint32_t e : list) from_window = from_window && r->window_slot[e] >= 0;
  if (from_window) {
    B = r->window;
  } else if (!list.empty() && (rc = decode_batch(r, list, &B))) {
    return rc;
  }
  r->range_batch = B;
  r->range_out.clear();
  for (uint32_t k = 0; k < uint32_t(list.size()); ++k) {
    const uint32_t slot = from_window ? uint32_t(r->window_slot[list[k]]) : k;
    const std::vector<okv_row>* rows = nullptr;
    if ((rc = batch_rows(*B, slot, &rows))) return rc;
    for (const okv_row& row : *rows) {  // :462-471
      if (bcmp(start, slen, row.key, row.key_len) <= 0) {
        if (!unbound_end && bcmp(row.key, row.key_len, end, elen) >= 0) break;
        r->range_out.push_back(row);
      }
    }
  }
  *rows_out = r->range_out.empty() ? nullptr : r->range_out.data();
  *n = r->range_out.size();
  return OKV_OK;
}

int okv_reader_close(okv_reader* r) {  // Close :481-487
  if (r->closed) return OKV_R_ALREADY_CLOSED;
  r->closed = true;
  return OKV_OK;
}

void okv_reader_free(okv_reader* r) { delete r; }

int okv_reader_io_stats(const okv_reader* r, okv_reader_io* io) {
  if (!r || !io) return OKV_E_ARG;
  *io = r->io;
  return OKV_OK;
}

okv_iter* okv_reader_row_iter(okv_reader* r, int direction) {  // RowIter :264-283
  if (ensure_meta(r)) return nullptr;
  okv_iter* it = new okv_iter();
  it->s = r;
  it->direction = direction;
  return it;
}

void okv_iter_free(okv_iter* it) { delete it; }

int okv_iter_next(okv_iter* it, okv_row* out) {  // RowIter.Next segment_row_iter.go:32-96
  okv_reader* s = it->s;
  if (s->closed) return OKV_R_CLOSED;  // :33-35
  if (!it->rows_nil && it->idx < int64_t(it->rows.size()) && it->idx >= 0) {  // :37-42
    *out = it->rows[size_t(it->idx)];
    it->idx++;
    return OKV_OK;
  }
  size_t stat = SIZE_MAX;
  if (it->direction == 1) {  // DirectionDescending (:45-61)
    if (it->stat_last_key.nil && it->idx > -1) it->stat_last_key = s->last_key;
    const Bytes& k = it->stat_last_key.b;
    for (size_t i = upper(s, k.data(), k.size()); i-- > 0;) {
      if (bcmp(k, s->tree[i].first_key) == 0) continue;  // same key: keep going
      it->stat_last_key = GoBytes::of(s->tree[i].first_key.data(), s->tree[i].first_key.size());
      stat = i;
      break;
    }
  } else {  // ascending (:62-75)
    const Bytes& k = it->stat_last_key.b;
    for (size_t i = lower(s, k.data(), k.size()); i < s->tree.size(); ++i) {
      if (bcmp(k, s->tree[i].first_key) == 0) continue;
      it->stat_last_key = GoBytes::of(s->tree[i].first_key.data(), s->tree[i].first_key.size());
      stat = i;
      break;
    }
  }
  if (stat == SIZE_MAX) return OKV_R_EOF;  // :78-81
  const std::vector<okv_row>* rows = nullptr;
  BatchP keep;
  const int rc = read_block_iter(s, stat, it->direction, &rows, &keep);  // :83-86
  if (rc) return rc;
  it->rows = *rows;
  it->rows_batch = keep;
  it->rows_nil = rows->empty();  // a block with no rows decodes to a nil slice
  if (it->direction == 1) std::reverse(it->rows.begin(), it->rows.end());  // :89-92
  it->idx = 1;                                                            // :94
  if (it->rows.empty()) return OKV_R_PANIC;  // rows[0] of an empty block (:95)
  *out = it->rows[0];
  return OKV_OK;
}

int okv_iter_seek(okv_iter* it, const uint8_t* key, size_t klen) {  // Seek :102-207
  okv_reader* s = it->s;
  const bool unbound_start = klen == 0;                  // :105
  const bool unbound_end = klen == 1 && key[0] == 0xff;  // :106
  size_t stat = SIZE_MAX;
  if (s->tree.empty()) return OKV_R_PANIC;
  if (unbound_start) {
    stat = 0;  // Min (:108-109)
  } else if (unbound_end) {
    stat = s->tree.size() - 1;  // Max (:110-112)
  } else {
    for (size_t i = upper(s, key, klen); i-- > 0;) {  // DescendLessOrEqual (:114-117)
      stat = i;
      if (!(bcmp(key, klen, s->tree[i].first_key.data(), s->tree[i].first_key.size()) <= 0))
        break;
    }
  }
  std::vector<okv_row> rows;  // `rows` (:121), nil until assigned
  it->idx = 0;                // :123
  if (stat == SIZE_MAX) {     // :124-156
    if (it->direction == 0) {
      const Entry& first = s->tree.front();
      if (bcmp(key, klen, first.first_key.data(), first.first_key.size()) < 0) {
        stat = 0;
      } else {
        stat = s->tree.size() - 1;
        it->idx = int64_t(rows.size()) - 1;  // len(nil) - 1 == -1 (:137)
      }
    } else {
      const size_t last = s->tree.size() - 1;
      const std::vector<okv_row>* lr = nullptr;
      BatchP keep;
      const int rc = read_block_iter(s, last, it->direction, &lr, &keep);  // :143-146
      if (rc) return rc;
      if (lr->empty()) return OKV_R_PANIC;  // rows[len(rows)-1] (:147)
      const okv_row& lastrow = lr->back();
      if (bcmp(key, klen, lastrow.key, lastrow.key_len) > 0) {
        stat = last;
      } else {
        stat = 0;
        it->idx = int64_t(lr->size()) - 1;  // (:154)
      }
    }
  }
  const Entry& se = s->tree[stat];
  it->stat_last_key = GoBytes::of(se.first_key.data(), se.first_key.size());  // :162
  const std::vector<okv_row>* br = nullptr;
  BatchP keep;
  const int rrc = read_block_iter(s, stat, it->direction, &br, &keep);  // :165-168 -- the error is discarded
  if (rrc == OKV_R_PANIC) return rrc;
  it->rows_nil = rrc != OKV_OK || br->empty();
  it->rows = (rrc == OKV_OK) ? *br : std::vector<okv_row>();
  it->rows_batch = rrc == OKV_OK ? keep : BatchP();
  if (it->direction == 1) std::reverse(it->rows.begin(), it->rows.end());  // :170-172
  if ((it->direction == 0 && unbound_end) || (it->direction == 1 && unbound_start)) {
    it->idx = int64_t(it->rows.size());  // :174-175
  } else {
    for (;;) {  // :178-196
      okv_row row;
      const int rc = okv_iter_next(it, &row);
      if (rc == OKV_R_EOF) return OKV_OK;
      if (rc) return rc;
      if (it->direction == 1 && bcmp(row.key, row.key_len, key, klen) <= 0) break;
      if (it->direction == 0 && bcmp(row.key, row.key_len, key, klen) >= 0) break;
    }
    it->idx--;  // :198
  }
  if (unbound_start && it->direction == 1) it->idx = -1;  // :201-204
  return OKV_OK;
}

}  // extern "C"
