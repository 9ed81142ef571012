"""pyoracle -- TEST INFRASTRUCTURE ONLY: an independent pure-Python restatement
of ObjectKV's Go ``sst/`` segment path (reference snapshot 2025-03-21).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this module; the product (``objectkv_amd``) never does.

Parity pinning (DESIGN.md "Oracle"): the Go toolchain is absent here and on
the GPU box, so the reference cannot run.  This restatement is pinned by
every known answer asserted in the reference's own tests (SURVEY.md §8c,
checked in tests/test_oracle.py), by the XXH64 specification (cespare/xxhash
v2.2.0, cross-checked against the ``xxhash`` 3.8.1 package) and by agreement
with the separate C restatement in ``oracle/okv_oracle.c``.

Every function cites the reference ``file:line`` it restates.
"""
from __future__ import annotations

import bisect
import struct

MAGIC = 69696969696969  # sst/segment_writer.go:21
TRAILER = 25  # segment_reader.go:93, :124 (Q3: SEGMENT.md says 17)

# ---- error model -----------------------------------------------------------


class GoError(Exception):
    """A Go ``error`` return; ``kind`` names the sentinel."""

    def __init__(self, kind, msg=""):
        super().__init__(f"{kind}: {msg}" if msg else kind)
        self.kind = kind


class GoPanic(Exception):
    """A Go panic (mustReadBytes, nil deref, index out of range)."""


ErrKeyTooLarge = "ErrKeyTooLarge"  # segment_writer.go:71
ErrValueTooLarge = "ErrValueTooLarge"  # :72
ErrWriterClosed = "ErrWriterClosed"  # :69
ErrInvalidKey = "ErrInvalidKey"  # :74
ErrInvalidMagicNumber = "ErrInvalidMagicNumber"  # segment_reader.go:84
ErrUnknownSegmentVersion = "ErrUnknownSegmentVersion"  # :81
ErrMismatchedMetaBlockHash = "ErrMismatchedMetaBlockHash"  # :82
ErrInvalidMetaBlock = "ErrInvalidMetaBlock"  # :83
ErrUnexpectedBytesRead = "ErrUnexpectedBytesRead"  # :477
ErrAlreadyClosed = "ErrAlreadyClosed"  # :478
ErrNoRows = "ErrNoRows"  # :357
ErrBloomReadFrom = "ErrBloomReadFrom"  # BytesToMetadata: "error in parseBloomFilterBlock" (:160-163)
ErrClosed = "ErrClosed"  # segment_row_iter.go:27
EOF = "EOF"  # io.EOF
ErrIO = "ErrIO"  # any other Seek/Read error
FATAL = {ErrInvalidMagicNumber, ErrUnknownSegmentVersion, ErrMismatchedMetaBlockHash,
         ErrInvalidMetaBlock}  # all wrap FatalError :80

# per-block status codes shared with include/okv_sst.h
BLK_OK, BLK_EOF, BLK_SHORT, BLK_PANIC, BLK_UNSUPPORTED = 0, 1, 2, 3, 4
BLK_ZSTD_ERROR = 6  # zstd.NewReader / io.Copy error (segment_reader.go:321-330)
COMP_NONE, COMP_ZSTD, COMP_LZ4 = 0, 1, 2

# ---- XXH64 (cespare/xxhash v2.2.0; segment_writer.go:185, :248) --------------
_M = (1 << 64) - 1
_P1, _P2, _P3, _P4, _P5 = (11400714785074694791, 14029467366897019727,
                           1609587929392839161, 9650029242287828579,
                           2870177450012600261)


def _rotl(x, r):
    return ((x << r) | (x >> (64 - r))) & _M


def _round(acc, lane):
    return (_rotl((acc + lane * _P2) & _M, 31) * _P1) & _M


def xxh64_py(data: bytes, seed: int = 0) -> int:
    """Pure-Python XXH64 from the public spec (slow; cross-check only)."""
    n = len(data)
    i = 0
    if n >= 32:
        v = [(seed + _P1 + _P2) & _M, (seed + _P2) & _M, seed & _M, (seed - _P1) & _M]
        while i + 32 <= n:
            for k in range(4):
                v[k] = _round(v[k], int.from_bytes(data[i + 8 * k:i + 8 * k + 8], "little"))
            i += 32
        h = (_rotl(v[0], 1) + _rotl(v[1], 7) + _rotl(v[2], 12) + _rotl(v[3], 18)) & _M
        for k in range(4):
            h = ((h ^ _round(0, v[k])) * _P1 + _P4) & _M
    else:
        h = (seed + _P5) & _M
    h = (h + n) & _M
    while i + 8 <= n:
        h ^= _round(0, int.from_bytes(data[i:i + 8], "little"))
        h = (_rotl(h, 27) * _P1 + _P4) & _M
        i += 8
    if i + 4 <= n:
        h ^= (int.from_bytes(data[i:i + 4], "little") * _P1) & _M
        h = (_rotl(h, 23) * _P2 + _P3) & _M
        i += 4
    while i < n:
        h ^= (data[i] * _P5) & _M
        h = (_rotl(h, 11) * _P1) & _M
        i += 1
    h ^= h >> 33
    h = (h * _P2) & _M
    h ^= h >> 29
    h = (h * _P3) & _M
    h ^= h >> 32
    return h


try:  # the pinned third-party C implementation, when present (it is here)
    import xxhash as _xx

    def xxh64(data: bytes, seed: int = 0) -> int:
        return _xx.xxh64_intdigest(data, seed)
except ImportError:  # pragma: no cover
    xxh64 = xxh64_py

# ---- types -------------------------------------------------------------------


class BlockStat:
    """block_stat.go:9-24."""

    __slots__ = ("FirstKey", "Offset", "BlockSize", "OriginalSize", "CompressedSize", "Hash")

    def __init__(self, FirstKey=None, Offset=0, BlockSize=0, OriginalSize=0,
                 CompressedSize=0, Hash=0):
        self.FirstKey = FirstKey
        self.Offset = Offset
        self.BlockSize = BlockSize
        self.OriginalSize = OriginalSize
        self.CompressedSize = CompressedSize
        self.Hash = Hash

    def to_bytes(self) -> bytes:  # block_stat.go:27-42
        fk = self.FirstKey or b""
        return (struct.pack("<H", len(fk)) + fk +
                struct.pack("<QQQQQ", self.Offset, self.BlockSize, self.OriginalSize,
                            self.CompressedSize, self.Hash))

    def desc(self):
        return (self.Offset, self.BlockSize, self.OriginalSize, self.CompressedSize)

    def __repr__(self):
        return (f"BlockStat({self.FirstKey!r}, off={self.Offset}, size={self.BlockSize}, "
                f"orig={self.OriginalSize}, comp={self.CompressedSize}, hash={self.Hash})")


class KVPair:
    """segment_reader.go:285-288; ``None`` stands for a nil slice (Q4)."""

    __slots__ = ("Key", "Value")

    def __init__(self, Key=None, Value=None):
        self.Key = Key
        self.Value = Value

    def __repr__(self):
        return f"KVPair({self.Key!r}, {self.Value!r})"


def _b(x):  # Go treats a nil slice as empty in bytes.Equal / bytes.Compare
    return b"" if x is None else x


# ---- SegmentWriter (segment_writer.go) ---------------------------------------


class SegmentWriterOptions:
    """segment_writer_option.go:5-16; defaults :18-27.  BloomFilter: an object
    with add(key) and to_bytes() (oracle/bloom_ref.py restates bits-and-blooms
    v2.0.3; its bytes are parity-unpinned), or None."""

    def __init__(self, DataBlockThresholdBytes=3584, DataBlockSize=4096,
                 ZSTDCompressionLevel=0, LZ4Compression=False, BloomFilter=None):
        self.DataBlockThresholdBytes = DataBlockThresholdBytes
        self.DataBlockSize = DataBlockSize
        self.ZSTDCompressionLevel = ZSTDCompressionLevel
        self.LZ4Compression = LZ4Compression
        self.BloomFilter = BloomFilter


class SegmentWriter:
    """NewSegmentWriter segment_writer.go:58-66 over an in-memory sink."""

    def __init__(self, opts: SegmentWriterOptions):
        self.options = opts
        self.external = bytearray()  # the io.Writer (tests may append to it)
        self.block_open = False  # s.blockWriter != nil
        self.block = bytearray()
        self.raw = 0
        self.cur_first_key = None
        self.last_key = None
        self.offset = 0
        self.index: list[BlockStat] = []
        self.closed = False

    def WriteRow(self, key: bytes, val: bytes):  # :80-146
        if len(key) > 0xFFFF:
            raise GoError(ErrKeyTooLarge)
        if len(val) > 0xFFFFFFFF:
            raise GoError(ErrValueTooLarge)
        if self.closed:
            raise GoError(ErrWriterClosed)
        if len(key) == 0:
            raise GoError(ErrInvalidKey)
        if self.options.ZSTDCompressionLevel > 0:
            raise NotImplementedError("klauspost zstd encoder is parity-unpinned offline")
        if not self.block_open:  # :95-115
            self.cur_first_key = bytes(key)
            self.raw = 0
            self.block = bytearray()
            self.block_open = True
        self.last_key = bytes(key)  # :118
        self.block += struct.pack("<HI", len(key), len(val)) + key + val  # :121-127
        self.raw += 6 + len(key) + len(val)  # :131
        if self.options.BloomFilter is not None:  # :133-136
            self.options.BloomFilter.add(bytes(key))
        if len(self.block) >= self.options.DataBlockThresholdBytes:  # :138
            self._flush()

    def _flush(self):  # flushCurrentDataBlock :148-204
        o = self.options
        use_zstd = o.ZSTDCompressionLevel > 0
        use_lz4 = (not use_zstd) and o.LZ4Compression
        st = BlockStat(self.cur_first_key, self.offset, 0, self.raw)
        if use_zstd or use_lz4:
            st.CompressedSize = len(self.block)  # :165-167
        rem = o.DataBlockSize - len(self.block) % o.DataBlockSize  # :169 (Q2)
        if rem > 0:
            self.block += bytes(rem)
        st.BlockSize = len(self.block)  # :180
        st.Hash = xxh64(bytes(self.block))  # :185
        self.index.append(st)
        self.external += self.block  # :191
        self.block_open = False  # :200
        self.offset += len(self.block)  # :202

    def Close(self):  # :211-282
        if not self.block_open:
            raise GoPanic("defer s.blockWriter.Close() on nil interface (Q1)")  # :212
        self._flush()
        meta_start = self.offset
        meta = self._meta()
        self.external += meta
        self.offset += len(meta)
        self.external += struct.pack("<QQBQ", meta_start, xxh64(meta), 1, MAGIC)  # :238-276
        self.offset += TRAILER
        self.closed = True
        return self.offset, meta

    def _meta(self) -> bytes:  # generateMetaBlock :284-328
        o = self.options
        fk = self.index[0].FirstKey
        m = bytearray()
        m += struct.pack("<H", len(fk)) + fk
        m += struct.pack("<H", len(self.last_key)) + self.last_key
        if o.BloomFilter is not None:  # :295-300
            bb = o.BloomFilter.to_bytes()
            m += b"\x01" + struct.pack("<Q", len(bb)) + bb
        else:
            m += b"\x00"  # :301-303
        use_zstd = o.ZSTDCompressionLevel > 0
        use_lz4 = (not use_zstd) and o.LZ4Compression
        m += bytes([1 if use_zstd else (2 if use_lz4 else 0)])  # :306-314
        m += b"\x00"  # :317
        m += struct.pack("<Q", len(self.index))  # :320
        for st in self.index:
            m += st.to_bytes()
        return bytes(m)


# ---- reader side ---------------------------------------------------------------


class _Reader:
    """bytes.Reader as used through mustReadBytes (segment_reader.go:489-512)."""

    def __init__(self, data):
        self.data = data
        self.i = 0

    def must(self, n):
        if n == 0:
            return None  # readBytes :490-493
        if self.i >= len(self.data) or len(self.data) - self.i < n:
            raise GoPanic(ErrUnexpectedBytesRead)  # :506-512
        out = bytes(self.data[self.i:self.i + n])
        self.i += n
        return out


class BlockIndex:
    """google/btree v1.1.2 BTreeG[BlockStat] ordered by FirstKey with
    ReplaceOrInsert (segment_reader.go:217-234; Q9 equal first keys collapse)."""

    def __init__(self):
        self.keys: list[bytes] = []
        self.items: list[BlockStat] = []

    def replace_or_insert(self, st):
        k = _b(st.FirstKey)
        i = bisect.bisect_left(self.keys, k)
        if i < len(self.keys) and self.keys[i] == k:
            self.items[i] = st
        else:
            self.keys.insert(i, k)
            self.items.insert(i, st)

    def Len(self):
        return len(self.items)

    def Get(self, key):
        k = _b(key)
        i = bisect.bisect_left(self.keys, k)
        if i < len(self.keys) and self.keys[i] == k:
            return self.items[i], True
        return BlockStat(), False

    def Min(self):
        return (self.items[0], True) if self.items else (BlockStat(), False)

    def Max(self):
        return (self.items[-1], True) if self.items else (BlockStat(), False)

    def ascend(self):
        return list(self.items)

    def ascend_ge(self, pivot):
        return self.items[bisect.bisect_left(self.keys, _b(pivot)):]

    def ascend_lt(self, pivot):
        return self.items[:bisect.bisect_left(self.keys, _b(pivot))]

    def descend_le(self, pivot):
        return self.items[:bisect.bisect_right(self.keys, _b(pivot))][::-1]


class SegmentMetadata:
    """segment_reader.go:43-55."""

    def __init__(self):
        self.BloomFilter = None
        self.ZSTDCompression = False
        self.LZ4Compression = False
        self.FirstKey = None
        self.LastKey = None
        self.BlockIndex = BlockIndex()
        self.entries: list[BlockStat] = []  # file order (not in the Go struct)

    @property
    def compression(self):
        if self.ZSTDCompression:
            return COMP_ZSTD
        return COMP_LZ4 if self.LZ4Compression else COMP_NONE


def bytes_to_metadata(meta: bytes) -> SegmentMetadata:
    """BytesToMetadata segment_reader.go:147-181 (+ :183-201, :206-238)."""
    md = SegmentMetadata()
    r = _Reader(meta)
    n = struct.unpack("<H", r.must(2))[0]
    md.FirstKey = r.must(n)
    n = struct.unpack("<H", r.must(2))[0]
    md.LastKey = r.must(n)
    if r.must(1)[0] == 1:  # :184
        blen = struct.unpack("<Q", r.must(8))[0]
        md.BloomFilter = r.must(blen)  # WriteTo bytes; GetRow probes them (bloom_ref)
        from oracle.bloom_ref import BloomFilter
        try:  # bloomFilter.ReadFrom (:197-200)
            md._bloom = BloomFilter.from_bytes(md.BloomFilter)
        except ValueError as e:
            raise GoError(ErrBloomReadFrom, f"error in parseBloomFilterBlock: {e}")
    c = r.must(1)[0]
    md.ZSTDCompression = c == 1
    md.LZ4Compression = c == 2
    r.must(1)  # :209
    num = struct.unpack("<Q", r.must(8))[0]
    if num == 0:
        raise GoError(ErrInvalidMetaBlock, "had no data block entries")
    for _ in range(num):
        kl = struct.unpack("<H", r.must(2))[0]
        st = BlockStat(r.must(kl))
        (st.Offset, st.BlockSize, st.OriginalSize, st.CompressedSize,
         st.Hash) = struct.unpack("<QQQQQ", r.must(40))
        md.entries.append(st)
        md.BlockIndex.replace_or_insert(st)
    return md


# Go runtime maxAlloc on 64-bit linux: 1 << heapAddrBits (48) (runtime/malloc.go);
# make([]byte, n) panics above it (runtime/slice.go makeslice)
GO_MAX_ALLOC = 1 << 48


def read_block(seg: bytes, desc, compression: int):
    """ReadBlockWithStat segment_reader.go:295-355 on raw bytes.

    Returns (status, rows) with rows a list of KVPair (None for nil).
    ``desc`` = (offset, block_size, original_size[, compressed_size]).
    """
    off, bsize, orig = desc[0], desc[1], desc[2]
    if off >= (1 << 63):
        return BLK_EOF, None  # Seek(int64(Offset)) error: negative position (:303-306)
    if bsize > GO_MAX_ALLOC:
        # make([]byte, stat.BlockSize) (:309): negative as int, or above the
        # runtime's maxAlloc -> "makeslice: len out of range" panic
        return BLK_PANIC, None
    if off >= len(seg):
        return BLK_EOF, None  # bytes.Reader.Read io.EOF (:310-313)
    if len(seg) - off < bsize:
        return BLK_SHORT, None  # :314-316
    if compression == COMP_ZSTD:
        # zstd.NewReader(bytes.NewReader(rawBlockBytes[:stat.CompressedSize])) + io.Copy
        # (:320-330); the decoder is klauspost v1.17.9 (standard RFC 8878 frames),
        # checked here with libzstd (oracle/zstd_ref.py)
        csize = desc[3] if len(desc) > 3 else 0
        if csize > bsize:
            return BLK_PANIC, None  # slice bounds out of range
        from oracle import zstd_ref
        buf = zstd_ref.decompress(seg[off:off + csize], orig)
        if buf is None:
            return BLK_ZSTD_ERROR, None
    else:
        buf = b"" if compression == COMP_LZ4 else seg[off:off + bsize]  # :331-335 (Q7)
    rows = None
    p = 0
    n = len(buf)
    if orig >= (1 << 63):
        orig = 0  # `totalReadBytes < int(stat.OriginalSize)` (:340): negative bound, no iteration
    while p < orig:  # :340
        if n - p < 2:
            return BLK_PANIC, None
        kl = buf[p] | (buf[p + 1] << 8)
        if n - p < 6:
            return BLK_PANIC, None
        vl = int.from_bytes(buf[p + 2:p + 6], "little")
        if kl and n - p - 6 < kl:
            return BLK_PANIC, None
        if vl and n - p - 6 - kl < vl:
            return BLK_PANIC, None
        key = bytes(buf[p + 6:p + 6 + kl]) if kl else None
        val = bytes(buf[p + 6 + kl:p + 6 + kl + vl]) if vl else None
        if rows is None:
            rows = []
        rows.append(KVPair(key, val))
        p += 6 + kl + vl
    return BLK_OK, rows


class SegmentReader:
    """NewSegmentReader segment_reader.go:65-72 over bytes.Reader semantics."""

    def __init__(self, data: bytes, file_bytes: int):
        self.data = bytes(data)
        self.fileBytes = file_bytes
        self.metadata: SegmentMetadata | None = None
        self.closed = False

    def LoadCachedMetadata(self, md):  # :75-77
        self.metadata = md

    def BytesToMetadata(self, meta):  # :147
        return bytes_to_metadata(meta)

    def FetchAndLoadMetadata(self):  # :91-141
        d = self.data
        if len(d) < TRAILER:
            raise GoError(ErrIO, "seek negative position")
        tail = d[-TRAILER:]
        if struct.unpack("<Q", tail[17:25])[0] != MAGIC:
            raise GoError(ErrInvalidMagicNumber)
        if tail[16] != 1:
            raise GoError(ErrUnknownSegmentVersion)
        moff, mhash = struct.unpack("<QQ", tail[:16])
        mlen = self.fileBytes - moff - TRAILER
        if mlen < 0:
            raise GoPanic("makeslice: len out of range")
        if moff >= len(d):
            raise GoError(EOF)
        mb = bytes(d[moff:moff + mlen])
        mb = mb + bytes(mlen - len(mb))  # Read copies what is available (:125)
        if xxh64(mb) != mhash:
            raise GoError(ErrMismatchedMetaBlockHash)
        self.metadata = bytes_to_metadata(mb)
        return self.metadata

    def _md(self):
        if self.metadata is None:
            self.FetchAndLoadMetadata()
        return self.metadata

    def ReadBlockWithStat(self, st: BlockStat):  # :295-355
        md = self._md()
        status, rows = read_block(self.data, st.desc(), md.compression)
        if status == BLK_PANIC:
            raise GoPanic(ErrUnexpectedBytesRead)
        if status == BLK_SHORT:
            raise GoError(ErrUnexpectedBytesRead, "when reading raw block bytes")
        if status == BLK_EOF:
            raise GoError(EOF)
        if status == BLK_UNSUPPORTED:
            raise NotImplementedError("zstd")
        return rows

    def GetRow(self, key):  # :362-404
        md = self._md()
        if md.BloomFilter is not None:  # :371-378 (probeBloomFilter :245-258)
            try:
                maybe = md._bloom.test(_b(key))
            except ZeroDivisionError:  # a filter with m == 0: Go's runtime panic
                raise GoPanic("integer divide by zero")
            if not maybe:
                raise GoError(ErrNoRows, "did not find row in bloom filter")
        cand = md.BlockIndex.descend_le(key)
        if not cand:
            raise GoError(ErrNoRows, "did not find potential block")
        for pair in self.ReadBlockWithStat(cand[0]) or []:
            if _b(pair.Key) == _b(key):
                return pair
        raise GoError(ErrNoRows, "did not find row in block")

    def GetRange(self, start, end):  # :410-475
        md = self._md()
        bi = md.BlockIndex
        unbound_start = _b(start) == b""
        unbound_end = _b(end) == b"\xff"
        stats = {}
        if unbound_start:
            for it in bi.ascend_lt(end):
                stats[_b(it.FirstKey)] = it
        else:
            for it in bi.descend_le(start):
                stats[_b(it.FirstKey)] = it
                if not (_b(start) <= _b(it.FirstKey)):
                    break
        for it in bi.descend_le(end)[:1]:
            stats[_b(it.FirstKey)] = it
        for it in bi.ascend_ge(end):
            if not unbound_end and _b(end) <= _b(it.FirstKey):
                break
            stats[_b(it.FirstKey)] = it
        out = []
        # Go ranges over a map (random order); restated in ascending FirstKey order
        for k in sorted(stats):
            for row in self.ReadBlockWithStat(stats[k]) or []:
                if _b(start) <= _b(row.Key):
                    if not unbound_end and _b(row.Key) >= _b(end):
                        break
                    out.append(row)
        return out

    def RowIter(self, direction):  # :264-283
        self._md()
        return RowIter(self, direction)

    def Close(self):  # :481-487
        if self.closed:
            raise GoError(ErrAlreadyClosed)
        self.closed = True


DirectionAscending, DirectionDescending = 0, 1  # segment_row_iter.go:22-25
UnboundStart = None  # segment_reader.go:60
UnboundEnd = b"\xff"  # :62


class RowIter:
    """segment_row_iter.go:11-212, restated statement by statement."""

    def __init__(self, s: SegmentReader, direction: int):
        self.statLastKey = None
        self.blockRows = None
        self.blockRowIdx = 0
        self.s = s
        self.direction = direction

    def Next(self):  # :32-96
        if self.s.closed:
            raise GoError(ErrClosed)
        if self.blockRows is not None and 0 <= self.blockRowIdx < len(self.blockRows):
            pair = self.blockRows[self.blockRowIdx]
            self.blockRowIdx += 1
            return pair
        md = self.s.metadata
        stat = None
        if self.direction == DirectionDescending:
            if self.statLastKey is None and self.blockRowIdx > -1:
                self.statLastKey = md.LastKey
            for it in md.BlockIndex.descend_le(self.statLastKey):
                if _b(self.statLastKey) == _b(it.FirstKey):
                    continue
                self.statLastKey = it.FirstKey
                stat = it
                break
        else:
            for it in md.BlockIndex.ascend_ge(self.statLastKey):
                if _b(self.statLastKey) == _b(it.FirstKey):
                    continue
                self.statLastKey = it.FirstKey
                stat = it
                break
        if stat is None:
            raise GoError(EOF)
        rows = self.s.ReadBlockWithStat(stat)
        self.blockRows = rows
        if self.direction == DirectionDescending and rows is not None:
            rows.reverse()
        self.blockRowIdx = 1
        if not rows:
            raise GoPanic("index out of range [0] with length 0")
        return rows[0]

    def Seek(self, key):  # :102-207
        md = self.s.metadata
        bi = md.BlockIndex
        unbound_start = _b(key) == b""
        unbound_end = _b(key) == b"\xff"
        stat = None
        if unbound_start:
            stat = bi.Min()[0]
        elif unbound_end:
            stat = bi.Max()[0]
        else:
            for it in bi.descend_le(key):
                stat = it
                if not (_b(key) <= _b(it.FirstKey)):
                    break
        rows = None
        self.blockRowIdx = 0
        if stat is None:
            if self.direction == DirectionAscending:
                first = bi.Min()[0]
                if _b(key) < _b(first.FirstKey):
                    stat = first
                else:
                    stat = bi.Max()[0]
                    self.blockRowIdx = (len(rows) if rows else 0) - 1
            else:
                last = bi.Max()[0]
                rows = self.s.ReadBlockWithStat(last)
                if not rows:
                    raise GoPanic("index out of range [-1]")
                if _b(key) > _b(rows[-1].Key):
                    stat = last
                else:
                    stat = bi.Min()[0]
                    self.blockRowIdx = len(rows) - 1
        self.statLastKey = stat.FirstKey
        try:
            rows = self.s.ReadBlockWithStat(stat)
        except GoError:  # :165-168 discards the error
            rows = None
        self.blockRows = rows
        if self.direction == DirectionDescending and rows is not None:
            rows.reverse()
        if ((self.direction == DirectionAscending and unbound_end) or
                (self.direction == DirectionDescending and unbound_start)):
            self.blockRowIdx = len(rows) if rows else 0
        else:
            while True:
                try:
                    row = self.Next()
                except GoError as e:
                    if e.kind == EOF:
                        return
                    raise
                if self.direction == DirectionDescending and _b(row.Key) <= _b(key):
                    break
                if self.direction == DirectionAscending and _b(row.Key) >= _b(key):
                    break
            self.blockRowIdx -= 1
        if unbound_start and self.direction == DirectionDescending:
            self.blockRowIdx = -1

    def CloseReader(self):  # :210-212
        return self.s.Close()


# ---- product output layout (DESIGN.md "Output layout") ----------------------


def decode_soa(seg: bytes, descs, compression: int, index_only: bool = False):
    """SoA restatement of the batched decode, built on read_block().

    Returns a dict of Python lists / bytes that tests compare bit-for-bit with
    the HIP path: status, row_start[nblk+1], key_base, val_base, key_off,
    key_len, val_off, val_len, key_arena, val_arena.  Arena regions are
    padded with zeros to a 16-byte multiple per block.
    """
    out = {k: [] for k in ("status", "row_start", "key_base", "val_base", "key_off",
                           "key_len", "val_off", "val_len")}
    ka, va = bytearray(), bytearray()
    g = 0
    for d in descs:
        out["row_start"].append(g)
        out["key_base"].append(len(ka))
        out["val_base"].append(len(va))
        status, rows = read_block(seg, d, compression)
        if index_only and compression == COMP_ZSTD and status == BLK_OK:
            status, rows = BLK_UNSUPPORTED, None  # spans into seg do not exist for zstd
        out["status"].append(status)
        if status != BLK_OK:
            continue
        rec = 0
        for r in rows or []:
            kl, vl = len(_b(r.Key)), len(_b(r.Value))
            out["key_len"].append(kl)
            out["val_len"].append(vl)
            if index_only:
                out["key_off"].append(d[0] + rec + 6)
                out["val_off"].append(d[0] + rec + 6 + kl)
            else:
                out["key_off"].append(len(ka))
                out["val_off"].append(len(va))
                ka += _b(r.Key)
                va += _b(r.Value)
            rec += 6 + kl + vl
            g += 1
        ka += bytes(-len(ka) % 16)
        va += bytes(-len(va) % 16)
    out["row_start"].append(g)
    if index_only:
        out["key_base"] = out["val_base"] = None
    out["key_arena"] = bytes(ka)
    out["val_arena"] = bytes(va)
    return out


# ---- deterministic synthetic workloads (BASELINE.md / SURVEY.md §8d) --------


class SplitMix64:
    def __init__(self, seed):
        self.s = seed & _M

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & _M
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M
        return z ^ (z >> 31)

    def bytes(self, n):
        words = (n + 7) // 8
        return b"".join(self.next().to_bytes(8, "little") for _ in range(words))[:n]


def rows_fixed(n, seed=1, key_len=16, val_len=64):
    """C1/C2 rows: key = row index big-endian in key_len bytes; value =
    val_len bytes from splitmix64(seed) (8-byte little-endian words)."""
    rng = SplitMix64(seed)
    for i in range(n):
        yield i.to_bytes(key_len, "big"), rng.bytes(val_len)


def zipf_cdf(lo=8, hi=256, s=1.1):
    cum, c = 0.0, []
    for L in range(lo, hi + 1):
        cum += float(L - lo + 1) ** (-s)
        c.append(cum)
    return c


def rows_zipf(seed=3, lo=8, hi=256, vmax=4096):
    """C3 rows (unbounded generator): key length L in [lo,hi] with
    P(L) ~ (L-lo+1)^-1.1, key = 8-byte big-endian row index + (L-8) random
    bytes, value length uniform on [0, vmax]."""
    rng = SplitMix64(seed)
    cdf = zipf_cdf(lo, hi)
    total = cdf[-1]
    i = 0
    while True:
        u = (rng.next() >> 11) * (1.0 / (1 << 53))
        t = u * total
        L = lo + bisect.bisect_right(cdf, t)
        if L > hi:
            L = hi
        vlen = rng.next() % (vmax + 1)
        key = i.to_bytes(8, "big") + rng.bytes(L - 8)
        val = rng.bytes(vlen)
        yield key, val
        i += 1


def build_segment(rows_iter, nblocks_target=None, nrows=None, threshold=3584, block_size=4096,
                  lz4=False):
    """Write rows until `nrows` are written, or until `nblocks_target` blocks
    are flushed and one more row is open (so Close never hits Q1).  Returns
    (file_bytes, meta_bytes, writer)."""
    w = SegmentWriter(SegmentWriterOptions(threshold, block_size, LZ4Compression=lz4))
    written = 0
    for key, val in rows_iter:
        if nrows is not None and written >= nrows:
            break
        if nblocks_target is not None and len(w.index) >= nblocks_target and w.block_open:
            break
        w.WriteRow(key, val)
        written += 1
    if nblocks_target is not None and not w.block_open:
        raise RuntimeError("row source ended on a block boundary")
    flen, meta = w.Close()
    return bytes(w.external), meta, w
