"""The reference's own Go tests, restated once and run against two
implementations (tests/test_oracle.py: the CPU oracle; tests/test_reader_gpu.py:
the product SegmentReader/RowIter over the GPU decode).  Every assertion
cites the Go test line it restates (/root/reference/sst/*_test.go).

An implementation adapter provides:
  write(rows, **opts) -> (segment bytes, file length, meta bytes)
  reader(data, file_bytes) -> object with Go-named methods
  stats(reader, meta) -> [(FirstKey, Offset, BlockSize, OriginalSize, CompressedSize)]
                         in btree (FirstKey) order, via BytesToMetadata
  read_block(reader, i) -> ReadBlockWithStat of btree entry i (list of pairs, or None)
  GoError / GoPanic exception classes (.kind = Go sentinel name), EOF = "EOF"
  DirectionAscending, DirectionDescending, UnboundStart, UnboundEnd, FATAL
"""
from __future__ import annotations

import random

import pytest

R200 = [(b"key%03d" % i, b"value%03d" % i) for i in range(200)]


def _b(x):
    return b"" if x is None else x


def _kind(impl, fn, *a):
    with pytest.raises(impl.GoError) as e:
        fn(*a)
    return e.value.kind


def case_read_uncompressed(impl):
    """TestReadUncompressed, segment_reader_test.go:12-269."""
    seg, flen, meta = impl.write(R200)
    r = impl.reader(seg, flen)
    st = impl.stats(r, meta)
    fk, lk = impl.first_last(r, meta)
    assert fk == b"key000" and lk == b"key199"  # :61-66
    assert len(st) == 2  # :77
    assert st[0][:5] == (b"key000", 0, 4096, 3600, 0)  # :81-92
    assert st[1][:5] == (b"key180", 4096, 4096, 400, 0)  # :94-105
    rows = impl.read_block(r, 0)
    assert rows[0].Key == b"key000" and rows[0].Value == b"value000"  # :116-121
    rows2 = impl.read_block(r, 1)
    assert len(rows) + len(rows2) == 200  # :131
    assert rows2[0].Key == b"key180" and rows2[0].Value == b"value180"  # :135-140
    assert rows2[-1].Key == b"key199" and rows2[-1].Value == b"value199"  # :142-147
    assert r.GetRow(b"key000").Value == b"value000"  # :150-159
    assert _kind(impl, r.GetRow, b"fuhguiregui") == "ErrNoRows"  # :161-164
    assert r.GetRow(b"key101").Key == b"key101"  # :166-172
    assert r.GetRow(b"key101").Value == b"value101"  # :173-179
    row = r.GetRow(b"key199")
    assert row.Key == b"key199" and row.Value == b"value199"  # :181-190
    g = r.GetRange(b"key000", b"key180")  # :193-212
    assert len(g) == 180 and g[0].Key == b"key000" and g[0].Value == b"value000"
    assert g[-1].Key == b"key179" and g[-1].Value == b"value179"
    assert len(r.GetRange(b"", b"key180")) == 180  # :215-222
    g = r.GetRange(b"key180", b"\xff")  # :224-244
    assert len(g) == 20 and g[0].Key == b"key180" and g[0].Value == b"value180"
    assert g[-1].Key == b"key199" and g[-1].Value == b"value199"
    g = r.GetRange(b"key199", b"\xff")  # :246-259
    assert len(g) == 1 and g[0].Key == b"key199" and g[0].Value == b"value199"
    r.Close()  # :261-264
    assert _kind(impl, r.Close) == "ErrAlreadyClosed"  # :265-268


def case_read_blank_value(impl):
    """TestReadBlankRecordUncompressed, segment_reader_test.go:271-326."""
    seg, flen, meta = impl.write(R200 + [(b"key200", b"")])
    r = impl.reader(seg, flen)
    row = r.GetRow(b"key200")
    assert row.Key == b"key200" and _b(row.Value) == b""  # :316-325
    assert row.Value is None  # readBytes(0) returns nil (segment_reader.go:490-493, Q4)


def case_read_single_row(impl):
    """TestReadSingleRecordUncompressed, segment_reader_test.go:328-511."""
    seg, flen, meta = impl.write(R200[:1])
    r = impl.reader(seg, flen)
    st = impl.stats(r, meta)
    assert impl.first_last(r, meta) == (b"key000", b"key000")  # :373-378
    assert len(st) == 1 and st[0][:5] == (b"key000", 0, 4096, 20, 0)  # :388-403
    rows = impl.read_block(r, 0)
    assert rows[0].Key == b"key000" and rows[-1].Value == b"value000"  # :414-426
    assert r.GetRow(b"key000").Value == b"value000"  # :429-438
    assert _kind(impl, r.GetRow, b"fuhguiregui") == "ErrNoRows"  # :440-443
    assert len(r.GetRange(b"key000", b"key000")) == 0  # :457-464
    assert len(r.GetRange(b"", b"key000")) == 0  # :466-473
    g = r.GetRange(b"", b"\xff")  # :476-495
    assert len(g) == 1 and g[0].Key == b"key000" and g[0].Value == b"value000"
    g = r.GetRange(b"key000", b"\xff")  # :497-510
    assert len(g) == 1 and g[0].Key == b"key000"


def case_corrupt_file_end(impl):
    """TestReadCorruptFileEnd, segment_reader_test.go:727-776 (crypto/rand
    replaced by a seeded generator)."""
    seg, flen, meta = impl.write(R200)
    rnd = bytes(random.Random(1).getrandbits(8) for _ in range(10))
    r = impl.reader(seg + rnd, flen)
    kind = _kind(impl, r.FetchAndLoadMetadata)
    assert kind == "ErrInvalidMagicNumber" and kind in impl.FATAL  # :773


def case_corrupt_file_middle(impl):
    """TestReadCorruptFileMiddle, segment_reader_test.go:778-830: 10 bytes land
    in the sink before the first block, shifting every offset."""
    seg, flen, meta = impl.write(R200)
    rnd = bytes(random.Random(2).getrandbits(8) for _ in range(10))
    r = impl.reader(rnd + seg, flen)  # what the sink holds after the corruption
    kind = _kind(impl, r.FetchAndLoadMetadata)
    assert kind == "ErrMismatchedMetaBlockHash" and kind in impl.FATAL  # :827


def case_row_iter_next(impl):
    """TestRowIterNext, segment_row_iter_test.go:12-134."""
    seg, flen, meta = impl.write(R200)
    r = impl.reader(seg, flen)
    it = r.RowIter(impl.DirectionAscending)
    row = it.Next()
    assert row.Key == b"key000" and row.Value == b"value000"  # :53-62
    row = it.Next()
    assert row.Key == b"key001" and row.Value == b"value001"  # :64-73
    for _ in range(198):
        row = it.Next()
    assert row.Key == b"key199" and row.Value == b"value199"  # :75-87
    assert _kind(impl, it.Next) == impl.EOF  # :89-92
    it = r.RowIter(impl.DirectionDescending)  # :94-98
    row = it.Next()
    assert row.Key == b"key199" and row.Value == b"value199"  # :100-109
    row = it.Next()
    assert row.Key == b"key198" and row.Value == b"value198"  # :110-119
    for _ in range(197):
        row = it.Next()
    assert row.Key == b"key001" and row.Value == b"value001"  # :121-133


def case_row_iter_seek(impl):
    """TestRowIterSeek, segment_row_iter_test.go:136-378."""
    seg, flen, meta = impl.write(R200)
    r = impl.reader(seg, flen)
    it = r.RowIter(impl.DirectionAscending)
    it.Seek(b"key010")  # :177-192
    row = it.Next()
    assert row.Key == b"key010" and row.Value == b"value010"
    assert it.Next().Key == b"key011"  # :194-204
    it.Seek(impl.UnboundStart)  # :206-222
    assert it.Next().Key == b"key000"
    it.Seek(b"key200")  # :224-233
    assert _kind(impl, it.Next) == impl.EOF
    it.Seek(impl.UnboundEnd)  # :235-244
    assert _kind(impl, it.Next) == impl.EOF
    it = r.RowIter(impl.DirectionDescending)  # :246-250
    it.Seek(b"key010")  # :252-267
    assert it.Next().Key == b"key010"
    assert it.Next().Key == b"key009"  # :269-279
    it.Seek(impl.UnboundStart)  # :281-290
    assert _kind(impl, it.Next) == impl.EOF
    it.Seek(impl.UnboundEnd)  # :292-307
    row = it.Next()
    assert row.Key == b"key199" and row.Value == b"value199"
    it.Seek(b"key200")  # :309-325
    assert it.Next().Key == b"key199"
    it.Seek(b"key")  # :327-336
    assert _kind(impl, it.Next) == impl.EOF
    it.Seek(impl.UnboundEnd)  # :338-354
    assert it.Next().Key == b"key199"
    it.Seek(b"key000")  # :356-372
    row = it.Next()
    assert row.Key == b"key000" and row.Value == b"value000"
    assert _kind(impl, it.Next) == impl.EOF  # :374-377


def case_rollover(impl):
    """TestRollover, segment_row_iter_test.go:380-450, with the options the Go
    test uses: DefaultSegmentWriterOptions, whose BloomFilter is
    NewWithEstimates(100000, 1e-6) (segment_writer_option.go:20) -- the meta
    block carries the filter (segment_writer.go:295-300) and the reader must
    parse past it (segment_reader.go:183-201)."""
    rows = [(b"key%03d" % i, b"value%03d-I-SHOULD-NOT-SHOW" % i) for i in range(1, 200, 2)]
    seg, flen, meta = impl.write(rows + [(b"key900", b"value900")], BloomFilter="default")
    assert meta[2 + 6 + 2 + 6] == 1  # bloom flag after the first/last keys
    r = impl.reader(seg, flen)
    it = r.RowIter(impl.DirectionDescending)
    it.Seek(b"key006")  # :420-423
    got = [it.Next().Key for _ in range(3)]  # :425-443
    assert got == [b"key005", b"key003", b"key001"]
    assert _kind(impl, it.Next) == impl.EOF  # :445-449
    # GetRow behind the bloom probe (segment_reader.go:371-378), hit and miss
    assert r.GetRow(b"key005").Value == b"value005-I-SHOULD-NOT-SHOW"
    assert _kind(impl, r.GetRow, b"key004") == "ErrNoRows"


def case_rollover_no_bloom(impl):
    """TestRollover's rows written with BloomFilter = nil."""
    rows = [(b"key%03d" % i, b"value%03d-I-SHOULD-NOT-SHOW" % i) for i in range(1, 200, 2)]
    seg, flen, meta = impl.write(rows + [(b"key900", b"value900")])
    assert meta[2 + 6 + 2 + 6] == 0
    r = impl.reader(seg, flen)
    it = r.RowIter(impl.DirectionDescending)
    it.Seek(b"key006")
    assert [it.Next().Key for _ in range(3)] == [b"key005", b"key003", b"key001"]
    assert _kind(impl, it.Next) == impl.EOF


def case_larger_than_block(impl):
    """TestSegmentWriterLargerThanBlock, segment_writer_test.go:73-112, read back."""
    rows = [(b"a" * 511, b"b" * 10000)] + [(b"key%d" % i, b"value%d" % i) for i in range(200)]
    seg, flen, meta = impl.write(rows)
    r = impl.reader(seg, flen)
    st = impl.stats(r, meta)
    assert sorted(s[1:4] for s in st) == [(0, 12288, 10517), (12288, 4096, 3600),
                                          (16384, 4096, 180)]
    got = []
    it = r.RowIter(impl.DirectionAscending)
    while True:
        try:
            got.append(it.Next())
        except impl.GoError as e:
            assert e.kind == impl.EOF
            break
    assert len(got) == 201
    assert got[0].Key == b"a" * 511 and got[0].Value == b"b" * 10000


CASES = [case_read_uncompressed, case_read_blank_value, case_read_single_row,
         case_corrupt_file_end, case_corrupt_file_middle, case_row_iter_next,
         case_row_iter_seek, case_rollover, case_rollover_no_bloom, case_larger_than_block]
