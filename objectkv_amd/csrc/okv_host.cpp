// okv_host.cpp -- host-side C++ mirror of ObjectKV's Go sst API (writer,
// metadata) plus XXH64 and the deterministic synthetic workloads.
// Reference: /root/reference/sst/segment_writer.go, block_stat.go,
// segment_reader.go.  This is product code; the independent CPU oracle used
// to check it lives in oracle/ and is never linked here.
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "okv_host.h"
#include "okv_sst.h"

namespace {

// ---------------------------------------------------------------------------
// XXH64 (cespare/xxhash/v2 v2.2.0 computes canonical XXH64; the reference
// hashes with seed 0 at segment_writer.go:185, :248, segment_reader.go:130)
// ---------------------------------------------------------------------------
constexpr uint64_t P1 = 11400714785074694791ULL, P2 = 14029467366897019727ULL,
                   P3 = 1609587929392839161ULL, P4 = 9650029242287828579ULL,
                   P5 = 2870177450012600261ULL;
inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t rd64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;  // x86-64 / little-endian host
}
inline uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline uint16_t rd16(const uint8_t* p) { return uint16_t(p[0] | (p[1] << 8)); }
inline uint64_t xr(uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; }

uint64_t xxh64(const uint8_t* p, size_t len, uint64_t seed) {
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uint8_t* lim = end - 32;
    do {
      v1 = xr(v1, rd64(p));
      v2 = xr(v2, rd64(p + 8));
      v3 = xr(v3, rd64(p + 16));
      v4 = xr(v4, rd64(p + 24));
      p += 32;
    } while (p <= lim);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    for (uint64_t v : {v1, v2, v3, v4}) h = (h ^ xr(0, v)) * P1 + P4;
  } else {
    h = seed + P5;
  }
  h += uint64_t(len);
  for (; p + 8 <= end; p += 8) h = rotl(h ^ xr(0, rd64(p)), 27) * P1 + P4;
  if (p + 4 <= end) {
    h = rotl(h ^ (uint64_t(rd32(p)) * P1), 23) * P2 + P3;
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

inline void put16(std::vector<uint8_t>& b, uint16_t v) {
  b.push_back(uint8_t(v));
  b.push_back(uint8_t(v >> 8));
}
inline void put32(std::vector<uint8_t>& b, uint32_t v) {
  for (int i = 0; i < 4; ++i) b.push_back(uint8_t(v >> (8 * i)));
}
inline void put64(std::vector<uint8_t>& b, uint64_t v) {
  for (int i = 0; i < 8; ++i) b.push_back(uint8_t(v >> (8 * i)));
}
inline void putb(std::vector<uint8_t>& b, const uint8_t* p, size_t n) {
  if (n) b.insert(b.end(), p, p + n);
}

struct Stat {  // BlockStat block_stat.go:9-24
  std::vector<uint8_t> first_key;
  okv_block_desc d;
  uint64_t hash;
};

}  // namespace

// ---------------------------------------------------------------------------
// SegmentWriter (segment_writer.go:35-328)
// ---------------------------------------------------------------------------
struct okv_writer {
  uint64_t threshold, dbs;  // DataBlockThresholdBytes, DataBlockSize
  int zstd_level, lz4;
  bool open = false;        // s.blockWriter != nil
  std::vector<uint8_t> block;
  uint64_t raw = 0;         // currentRawBlockSize
  std::vector<uint8_t> cur_first, last_key;
  std::vector<uint8_t> file;  // the external writer's bytes
  uint64_t offset = 0;        // currentByteOffset
  std::vector<Stat> index;    // blockIndex
  std::vector<uint8_t> meta;
  bool closed = false;
  bool has_bloom = false;      // options.BloomFilter != nil
  std::vector<uint8_t> bloom;  // its WriteTo bytes (opaque pass-through)

  void flush() {  // flushCurrentDataBlock :148-204
    const bool use_zstd = zstd_level > 0, use_lz4 = !use_zstd && lz4;
    Stat st;
    st.first_key = cur_first;
    st.d.offset = offset;
    st.d.original_size = raw;
    st.d.compressed_size = (use_zstd || use_lz4) ? block.size() : 0;  // :165-167
    const uint64_t rem = dbs - block.size() % dbs;  // :169 -- always >= 1 (Q2)
    block.resize(block.size() + rem, 0);
    st.d.block_size = block.size();
    st.hash = xxh64(block.data(), block.size(), 0);  // :185
    putb(file, block.data(), block.size());         // :191
    offset += block.size();
    block.clear();
    open = false;  // :200
    index.push_back(std::move(st));
  }
};

extern "C" {

uint64_t okv_xxh64(const void* data, size_t len, uint64_t seed) {
  return xxh64(static_cast<const uint8_t*>(data), len, seed);
}

okv_writer* okv_writer_new(uint64_t threshold_bytes, uint64_t block_size, int zstd_level,
                           int lz4) {
  if (block_size == 0) return nullptr;
  okv_writer* w = new okv_writer();
  w->threshold = threshold_bytes;
  w->dbs = block_size;
  w->zstd_level = zstd_level;
  w->lz4 = lz4;
  return w;
}

int okv_writer_write_row(okv_writer* w, const uint8_t* key, size_t klen, const uint8_t* val,
                         size_t vlen) {  // WriteRow :80-146
  if (klen > 0xFFFF) return OKV_W_KEY_TOO_LARGE;
  if (uint64_t(vlen) > 0xFFFFFFFFull) return OKV_W_VALUE_TOO_LARGE;
  if (w->closed) return OKV_W_CLOSED;
  if (klen == 0) return OKV_W_INVALID_KEY;
  if (w->zstd_level > 0) return OKV_W_UNSUPPORTED;
  if (!w->open) {
    w->cur_first.assign(key, key + klen);
    w->raw = 0;
    w->block.clear();
    w->open = true;
  }
  w->last_key.assign(key, key + klen);
  put16(w->block, uint16_t(klen));
  put32(w->block, uint32_t(vlen));
  putb(w->block, key, klen);
  putb(w->block, val, vlen);
  w->raw += 6 + klen + vlen;
  if (w->block.size() >= w->threshold) w->flush();
  return OKV_OK;
}

int okv_writer_close(okv_writer* w, int strict_go, uint64_t* file_len, uint64_t* meta_len) {
  if (w->closed && !w->open) return strict_go ? OKV_W_NIL_WRITER : OKV_W_CLOSED;
  if (!w->open && strict_go) return OKV_W_NIL_WRITER;  // :212 (Q1)
  if (w->open) w->flush();                             // :214-219
  if (w->index.empty()) return OKV_W_NO_ROWS;          // ErrNoRowsWritten :221
  const uint64_t meta_start = w->offset;
  std::vector<uint8_t>& m = w->meta;  // generateMetaBlock :284-328
  m.clear();
  put16(m, uint16_t(w->index[0].first_key.size()));
  putb(m, w->index[0].first_key.data(), w->index[0].first_key.size());
  put16(m, uint16_t(w->last_key.size()));
  putb(m, w->last_key.data(), w->last_key.size());
  if (w->has_bloom) {  // :295-300
    m.push_back(1);
    put64(m, w->bloom.size());
    putb(m, w->bloom.data(), w->bloom.size());
  } else {
    m.push_back(0);  // :301-303
  }
  const bool use_zstd = w->zstd_level > 0, use_lz4 = !use_zstd && w->lz4;
  m.push_back(use_zstd ? 1 : (use_lz4 ? 2 : 0));
  m.push_back(0);  // simple block index
  put64(m, w->index.size());
  for (const Stat& s : w->index) {  // BlockStat.toBytes block_stat.go:27-42
    put16(m, uint16_t(s.first_key.size()));
    putb(m, s.first_key.data(), s.first_key.size());
    put64(m, s.d.offset);
    put64(m, s.d.block_size);
    put64(m, s.d.original_size);
    put64(m, s.d.compressed_size);
    put64(m, s.hash);
  }
  putb(w->file, m.data(), m.size());
  w->offset += m.size();
  put64(w->file, meta_start);            // :238
  put64(w->file, xxh64(m.data(), m.size(), 0));  // :248
  w->file.push_back(1);                  // :259 version
  put64(w->file, 69696969696969ULL);     // :269 MagicNumber
  w->offset += 25;
  w->closed = true;
  if (file_len) *file_len = w->offset;
  if (meta_len) *meta_len = m.size();
  return OKV_OK;
}

const uint8_t* okv_writer_data(const okv_writer* w, uint64_t* len) {
  if (len) *len = w->file.size();
  return w->file.data();
}
const uint8_t* okv_writer_meta(const okv_writer* w, uint64_t* len) {
  if (len) *len = w->meta.size();
  return w->meta.data();
}
uint64_t okv_writer_num_blocks(const okv_writer* w) { return w->index.size(); }
int okv_writer_block(const okv_writer* w, uint64_t i, okv_block_desc* desc, uint64_t* hash,
                     const uint8_t** first_key, uint64_t* first_key_len) {
  if (i >= w->index.size()) return OKV_E_ARG;
  const Stat& s = w->index[i];
  if (desc) *desc = s.d;
  if (hash) *hash = s.hash;
  if (first_key) *first_key = s.first_key.data();
  if (first_key_len) *first_key_len = s.first_key.size();
  return OKV_OK;
}
void okv_writer_set_bloom(okv_writer* w, const uint8_t* bytes, uint64_t len) {
  w->has_bloom = true;
  w->bloom.assign(bytes, bytes + len);
}
void okv_writer_free(okv_writer* w) { delete w; }

}  // extern "C"

// ---------------------------------------------------------------------------
// Metadata (segment_reader.go:91-238)
// ---------------------------------------------------------------------------
struct okv_meta {
  std::vector<uint8_t> bytes;  // owned copy of the meta block
  uint64_t fk_off = 0, fk_len = 0, lk_off = 0, lk_len = 0;
  bool has_bloom = false;
  uint64_t bloom_off = 0, bloom_len = 0;
  // the filter BloomFilter.ReadFrom decoded (parseBloomFilterBlock :197-198)
  uint64_t bloom_m = 0, bloom_k = 0, bloom_length = 0;
  std::vector<uint64_t> bloom_words;
  int compression = 0;
  std::vector<okv_block_desc> descs;  // file order
  std::vector<uint64_t> hashes, key_off, key_len;
};

namespace {
struct MetaReader {  // bytes.Reader + mustReadBytes (:489-512)
  const uint8_t* p;
  uint64_t n, i = 0;
  bool must(uint64_t k, uint64_t* at) {
    if (k == 0) {
      *at = i;
      return true;
    }
    if (i >= n || n - i < k) return false;
    *at = i;
    i += k;
    return true;
  }
};

// ---- the bloom filter (parseBloomFilterBlock :183-201, probeBloomFilter
// :245-258), restated from the published algorithms of the pinned versions
// (go.sum): github.com/bits-and-blooms/bloom v2.0.3, github.com/spaolacci/
// murmur3 v1.1.0, github.com/willf/bitset v1.1.11.  Filter bytes are
// PARITY-UNPINNED (no reference test asserts them; oracle/bloom_ref.py is the
// independent restatement the tests compare against).

// murmur3.Sum128 (MurmurHash3_x64_128, seed 0) -> (h1, h2)
void murmur3_128(const uint8_t* p, size_t n, uint64_t* o1, uint64_t* o2) {
  const uint64_t c1 = 0x87C37B91114253D5ULL, c2 = 0x4CF5AD432745937FULL;
  uint64_t h1 = 0, h2 = 0;
  const size_t nb = n / 16;
  for (size_t i = 0; i < nb; ++i) {
    uint64_t k1 = rd64(p + 16 * i), k2 = rd64(p + 16 * i + 8);
    k1 *= c1; k1 = rotl(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52DCE729;
    k2 *= c2; k2 = rotl(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495AB5;
  }
  const uint8_t* t = p + 16 * nb;
  const size_t tl = n & 15;
  uint64_t k1 = 0, k2 = 0;
  for (size_t i = tl; i > 8; --i) k2 = (k2 << 8) | t[i - 1];
  if (tl > 8) { k2 *= c2; k2 = rotl(k2, 33); k2 *= c1; h2 ^= k2; }
  for (size_t i = tl < 8 ? tl : 8; i > 0; --i) k1 = (k1 << 8) | t[i - 1];
  if (tl) { k1 *= c1; k1 = rotl(k1, 31); k1 *= c2; h1 ^= k1; }
  h1 ^= uint64_t(n);
  h2 ^= uint64_t(n);
  h1 += h2;
  h2 += h1;
  auto fmix = [](uint64_t k) {
    k ^= k >> 33; k *= 0xFF51AFD7ED558CCDULL; k ^= k >> 33; k *= 0xC4CEB9FE1A85EC53ULL;
    return k ^ (k >> 33);
  };
  h1 = fmix(h1);
  h2 = fmix(h2);
  h1 += h2;
  h2 += h1;
  *o1 = h1;
  *o2 = h2;
}

inline uint64_t rdbe64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
  return v;
}

// BloomFilter.ReadFrom (bloom v2.0.3): binary.Read(BigEndian) of m and k, then
// bitset.ReadFrom (v1.1.11): u64 length, New(length) -- wordsNeeded(length)
// words, or length 0 when that allocation panics (recovered: "type mismatch")
// -- and binary.Read of the words.  Any short read is an error (io.EOF /
// io.ErrUnexpectedEOF); trailing bytes are not read.
bool bloom_read_from(okv_meta* m) {
  const uint8_t* b = m->bytes.data() + m->bloom_off;
  const uint64_t n = m->bloom_len;
  if (n < 24) return false;  // m, k, length
  m->bloom_m = rdbe64(b);
  m->bloom_k = rdbe64(b + 8);
  m->bloom_length = rdbe64(b + 16);
  const uint64_t cap = ~uint64_t(0);
  const uint64_t words = m->bloom_length > cap - 64 + 1 ? cap >> 6 : (m->bloom_length + 63) >> 6;
  // words beyond the bytes present: binary.Read fails (or make panicked first,
  // which New recovers into a length mismatch: an error either way)
  if (words > (n - 24) / 8) return false;
  m->bloom_words.resize(size_t(words));
  for (uint64_t i = 0; i < words; ++i) m->bloom_words[size_t(i)] = rdbe64(b + 24 + 8 * i);
  return true;
}

int parse_meta(okv_meta* m) {  // BytesToMetadata :147-181
  MetaReader r{m->bytes.data(), m->bytes.size()};
  const uint8_t* b = m->bytes.data();
  uint64_t at;
  if (!r.must(2, &at)) return OKV_M_PANIC;
  m->fk_len = rd16(b + at);
  if (!r.must(m->fk_len, &m->fk_off)) return OKV_M_PANIC;
  if (!r.must(2, &at)) return OKV_M_PANIC;
  m->lk_len = rd16(b + at);
  if (!r.must(m->lk_len, &m->lk_off)) return OKV_M_PANIC;
  if (!r.must(1, &at)) return OKV_M_PANIC;  // parseBloomFilterBlock :183-201
  m->has_bloom = b[at] == 1;
  if (m->has_bloom) {
    if (!r.must(8, &at)) return OKV_M_PANIC;
    m->bloom_len = rd64(b + at);
    if (!r.must(m->bloom_len, &m->bloom_off)) return OKV_M_PANIC;
    if (!bloom_read_from(m)) return OKV_M_BLOOM;  // "error in parseBloomFilterBlock" (:160-163)
  }
  if (!r.must(1, &at)) return OKV_M_PANIC;  // :166-172
  m->compression = b[at] == 1 ? OKV_COMP_ZSTD : (b[at] == 2 ? OKV_COMP_LZ4 : OKV_COMP_NONE);
  if (!r.must(1, &at)) return OKV_M_PANIC;  // parseBlockIndex :209
  if (!r.must(8, &at)) return OKV_M_PANIC;
  const uint64_t n = rd64(b + at);
  if (n == 0) return OKV_M_INVALID;                // :213-215
  if (n > (r.n - r.i) / 42) return OKV_M_PANIC;     // cannot hold n entries
  m->descs.resize(n);
  m->hashes.resize(n);
  m->key_off.resize(n);
  m->key_len.resize(n);
  for (uint64_t e = 0; e < n; ++e) {  // :221-235
    if (!r.must(2, &at)) return OKV_M_PANIC;
    m->key_len[e] = rd16(b + at);
    if (!r.must(m->key_len[e], &m->key_off[e])) return OKV_M_PANIC;
    if (!r.must(40, &at)) return OKV_M_PANIC;
    m->descs[e] = {rd64(b + at), rd64(b + at + 8), rd64(b + at + 16), rd64(b + at + 24)};
    m->hashes[e] = rd64(b + at + 32);
  }
  return OKV_OK;
}
}  // namespace

extern "C" {

int okv_meta_parse(const uint8_t* meta, uint64_t meta_len, okv_meta** out) {
  okv_meta* m = new okv_meta();
  m->bytes.assign(meta, meta + meta_len);
  const int rc = parse_meta(m);
  if (rc) {
    delete m;
    return rc;
  }
  *out = m;
  return OKV_OK;
}

int okv_meta_fetch(const uint8_t* buf, uint64_t buf_len, int64_t file_bytes, okv_meta** out) {
  // FetchAndLoadMetadata :91-141
  if (buf_len < 25) return OKV_M_IO;
  const uint8_t* tail = buf + buf_len - 25;
  if (rd64(tail + 17) != 69696969696969ULL) return OKV_M_MAGIC;
  if (tail[16] != 1) return OKV_M_VERSION;
  const uint64_t moff = rd64(tail), mhash = rd64(tail + 8);
  if (int64_t(moff) < 0) return OKV_M_IO;
  const int64_t mlen = file_bytes - int64_t(moff) - 25;
  if (mlen < 0) return OKV_M_MAKESLICE;
  if (moff >= buf_len) return OKV_M_IO;
  std::vector<uint8_t> mb(size_t(mlen), 0);
  const uint64_t avail = buf_len - moff;
  std::memcpy(mb.data(), buf + moff, size_t(uint64_t(mlen) < avail ? uint64_t(mlen) : avail));
  if (xxh64(mb.data(), mb.size(), 0) != mhash) return OKV_M_HASH;
  okv_meta* m = new okv_meta();
  m->bytes = std::move(mb);
  const int rc = parse_meta(m);
  if (rc) {
    delete m;
    return rc;
  }
  *out = m;
  return OKV_OK;
}

uint64_t okv_meta_num_blocks(const okv_meta* m) { return m->descs.size(); }
int okv_meta_compression(const okv_meta* m) { return m->compression; }
const okv_block_desc* okv_meta_descs(const okv_meta* m) { return m->descs.data(); }
const uint8_t* okv_meta_first_key(const okv_meta* m, uint64_t* len) {
  if (len) *len = m->fk_len;
  return m->bytes.data() + m->fk_off;
}
const uint8_t* okv_meta_last_key(const okv_meta* m, uint64_t* len) {
  if (len) *len = m->lk_len;
  return m->bytes.data() + m->lk_off;
}
int okv_meta_block(const okv_meta* m, uint64_t i, okv_block_desc* desc, uint64_t* hash,
                   const uint8_t** first_key, uint64_t* first_key_len) {
  if (i >= m->descs.size()) return OKV_E_ARG;
  if (desc) *desc = m->descs[i];
  if (hash) *hash = m->hashes[i];
  if (first_key) *first_key = m->bytes.data() + m->key_off[i];
  if (first_key_len) *first_key_len = m->key_len[i];
  return OKV_OK;
}
void okv_meta_free(okv_meta* m) { delete m; }

int okv_meta_has_bloom(const okv_meta* m) { return m && m->has_bloom ? 1 : 0; }

// BloomFilter.Test (bloom v2.0.3): baseHashes = murmur3 Sum128 of key, then of
// key ++ [1] (the hasher keeps its state); bit i of k is
// (h[i % 2] + i * h[2 + ((i + i % 2) % 4) / 2]) % m, tested by bitset.Test (a
// position >= the bitset's length reads false).  m == 0 is Go's integer
// division panic.
int okv_meta_bloom_test(const okv_meta* m, const uint8_t* key, size_t klen) {
  if (!m || !m->has_bloom) return 1;  // probeBloomFilter: no filter, no probe
  if (m->bloom_k == 0) return 1;
  if (m->bloom_m == 0) return OKV_R_PANIC;
  uint64_t h[4];
  murmur3_128(key, klen, &h[0], &h[1]);
  std::vector<uint8_t> k1(key, key + klen);
  k1.push_back(1);
  murmur3_128(k1.data(), k1.size(), &h[2], &h[3]);
  for (uint64_t i = 0; i < m->bloom_k; ++i) {
    const uint64_t loc = (h[i % 2] + i * h[2 + ((i + (i % 2)) % 4) / 2]) % m->bloom_m;
    if (loc >= m->bloom_length) return 0;
    if (!((m->bloom_words[size_t(loc >> 6)] >> (loc & 63)) & 1)) return 0;
  }
  return 1;
}

// ---------------------------------------------------------------------------
// Synthetic segments (BASELINE.md / SURVEY.md §8d)
// ---------------------------------------------------------------------------
okv_writer* okv_synth_segment(int kind, uint64_t seed, uint64_t nrows, uint64_t nblocks,
                              uint64_t threshold, uint64_t block_size) {
  okv_writer* w = okv_writer_new(threshold, block_size, 0, 0);
  if (!w) return nullptr;
  if (nblocks) w->file.reserve(size_t((nblocks + 2) * block_size));
  uint64_t s = seed;
  auto next = [&s]() {  // splitmix64
    s += 0x9E3779B97F4A7C15ULL;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
  };
  auto fill = [&](uint8_t* dst, uint64_t n) {  // 8-byte LE words, truncated
    for (uint64_t i = 0; i < n; i += 8) {
      const uint64_t v = next();
      const uint64_t k = n - i < 8 ? n - i : 8;
      std::memcpy(dst + i, &v, size_t(k));
    }
  };
  std::vector<double> cdf;
  if (kind == OKV_SYNTH_ZIPF) {
    double cum = 0.0;
    for (int L = 8; L <= 256; ++L) {
      cum += std::pow(double(L - 7), -1.1);
      cdf.push_back(cum);
    }
  }
  std::vector<uint8_t> key(256), val(4097);
  for (uint64_t i = 0;; ++i) {
    if (nrows && i >= nrows) break;
    if (nblocks && w->index.size() >= nblocks && w->open) break;
    uint64_t kl, vl;
    if (kind == OKV_SYNTH_FIXED) {
      kl = 16;
      vl = 64;
      std::memset(key.data(), 0, 8);
      for (int b = 0; b < 8; ++b) key[8 + b] = uint8_t(i >> (56 - 8 * b));
      fill(val.data(), vl);
    } else {
      const double u = double(next() >> 11) * (1.0 / 9007199254740992.0);
      const double t = u * cdf.back();
      uint64_t c = 0;  // number of cdf entries <= t (bisect_right)
      {
        uint64_t lo = 0, hi = cdf.size();
        while (lo < hi) {
          const uint64_t mid = (lo + hi) / 2;
          if (cdf[mid] <= t) lo = mid + 1; else hi = mid;
        }
        c = lo;
      }
      kl = 8 + c;
      if (kl > 256) kl = 256;
      vl = next() % 4097;
      for (int b = 0; b < 8; ++b) key[b] = uint8_t(i >> (56 - 8 * b));
      fill(key.data() + 8, kl - 8);
      fill(val.data(), vl);
    }
    if (okv_writer_write_row(w, key.data(), kl, val.data(), vl) != OKV_OK) {
      okv_writer_free(w);
      return nullptr;
    }
  }
  if (okv_writer_close(w, 0, nullptr, nullptr) != OKV_OK) {
    okv_writer_free(w);
    return nullptr;
  }
  return w;
}

}  // extern "C"
