"""The reference's Go tests (tests/reference_cases.py) against the product:
the C++ SegmentWriter mirror writes, and the C++ SegmentReader/RowIter
mirror reads through the batched GPU decode (okv_reader.cpp)."""
from __future__ import annotations

import pytest

import objectkv_amd as okv
from objectkv_amd import reader as R
from tests import reference_cases as RC

pytestmark = pytest.mark.gpu


class ProductImpl:
    GoError, GoPanic, EOF, FATAL = R.GoError, R.GoPanic, "EOF", R.FATAL
    DirectionAscending, DirectionDescending = R.DirectionAscending, R.DirectionDescending
    UnboundStart, UnboundEnd = R.UnboundStart, R.UnboundEnd
    decoder = None

    @staticmethod
    def write(rows, **kw):
        bloom = None
        if kw.get("BloomFilter") == "default":  # the caller's filter; bytes pass through
            from oracle.bloom_ref import default_filter
            bloom = default_filter()
        w = okv.SegmentWriter(kw.get("DataBlockThresholdBytes", 3584),
                              kw.get("DataBlockSize", 4096), bloom=bloom)
        for k, v in rows:
            w.WriteRow(k, v)
        flen, meta = w.Close()
        return w.data().tobytes(), flen, meta

    @classmethod
    def reader(cls, data, file_bytes):
        return R.SegmentReader(data, file_bytes, cls.decoder)

    @staticmethod
    def stats(r, meta):
        md = r.BytesToMetadata(meta)
        ent = sorted(zip(md.first_keys, md.descs.tolist()))
        return [(k, *d) for k, d in ent]

    @staticmethod
    def first_last(r, meta):
        md = r.BytesToMetadata(meta)
        return md.first_key, md.last_key

    @staticmethod
    def read_block(r, i):
        return r.ReadBlock(i)


@pytest.mark.parametrize("case", RC.CASES, ids=lambda c: c.__name__)
def test_reference_cases_product(case, decoder):
    ProductImpl.decoder = decoder
    case(ProductImpl)


def test_product_reader_matches_oracle_on_random_iteration(decoder):
    """Random Seek/Next sequences: product RowIter == oracle RowIter."""
    import random
    from oracle import pyoracle as P
    rng = random.Random(5)
    rows = [(b"k%05d" % i, bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 300))))
            for i in range(0, 3000, 3)]
    w = okv.SegmentWriter()
    pw = P.SegmentWriter(P.SegmentWriterOptions())
    for k, v in rows:
        w.WriteRow(k, v)
        pw.WriteRow(k, v)
    flen, meta = w.Close()
    pw.Close()
    data = w.data().tobytes()
    assert data == bytes(pw.external)
    for direction in (0, 1):
        pr = R.SegmentReader(data, flen, decoder)
        orr = P.SegmentReader(data, flen)
        it, oit = pr.RowIter(direction), orr.RowIter(direction)
        for step in range(300):
            if rng.random() < 0.15:
                key = rng.choice([b"", b"\xff", b"k", b"z", b"k%05d" % rng.randrange(3100)])
                it.Seek(key)
                oit.Seek(key or None)
                continue
            try:
                want = oit.Next()
            except P.GoError as e:
                with pytest.raises(R.GoError) as g:
                    it.Next()
                assert g.value.kind == e.kind
                continue
            got = it.Next()
            assert (got.Key, got.Value) == (want.Key, want.Value), step


# ---- bounded block reads (the cgo shim's ReadBlocks) --------

def _segment(nrows=6000, vmax=300, seed=9):
    import random
    rng = random.Random(seed)
    rows = [(b"k%06d" % i, bytes(rng.getrandbits(8) for _ in range(rng.randint(0, vmax))))
            for i in range(nrows)]
    w = okv.SegmentWriter()
    for k, v in rows:
        w.WriteRow(k, v)
    flen, meta = w.Close()
    return rows, w.data().tobytes(), flen, meta


def test_getrow_stages_one_block(decoder):
    """GetRow decodes exactly the block the btree floor picks
    (segment_reader.go:381-392): one GPU call staging that block's BlockSize."""
    from oracle import pyoracle as P
    rows, data, flen, meta = _segment()
    md = P.bytes_to_metadata(meta)
    pr = R.SegmentReader(data, flen, decoder)
    for k, v in (rows[0], rows[2999], rows[-1]):
        before = pr.io_stats()
        assert pr.GetRow(k).Value == (v or None)
        after = pr.io_stats()
        assert after["calls"] - before["calls"] == 1
        assert after["blocks"] - before["blocks"] == 1
        st = max((e for e in md.entries if e.FirstKey <= k), key=lambda e: e.FirstKey)
        assert after["bytes_staged"] - before["bytes_staged"] == st.BlockSize


def test_rowiter_window_batches(decoder):
    """RowIter decodes 256 blocks per GPU call in its direction and serves the
    rest of the window without a call; rows equal the oracle's."""
    from oracle import pyoracle as P
    rows, data, flen, meta = _segment(nrows=30000, vmax=120)
    nb = len(P.bytes_to_metadata(meta).entries)
    assert nb > 600
    for direction in (0, 1):
        pr = R.SegmentReader(data, flen, decoder)
        it = pr.RowIter(direction)
        got = []
        while True:
            try:
                p = it.Next()
            except R.GoError as e:
                assert e.kind == "EOF"
                break
            got.append((p.Key, p.Value or b""))
        want = rows if direction == 0 else rows[::-1]
        assert got == want
        io = pr.io_stats()
        assert io["calls"] == -(-nb // 256) and io["blocks"] == nb


def test_getrange_stages_selected_blocks(decoder):
    """GetRange decodes the block set its btree walks select (:421-458) in one
    call: the floor of start (and the block below it when start equals a first
    key) and the floor of end -- Go reads no block in between, so rows there
    are not returned, by the oracle either.  Rows equal the oracle's."""
    from oracle import pyoracle as P
    rows, data, flen, meta = _segment()
    md = P.bytes_to_metadata(meta)
    pr = R.SegmentReader(data, flen, decoder)
    orr = P.SegmentReader(data, flen)
    start, end = rows[1000][0], rows[1400][0]
    got = pr.GetRange(start, end)
    want = orr.GetRange(start, end)
    assert [(r.Key, r.Value) for r in got] == [(r.Key, r.Value) for r in want]
    io = pr.io_stats()
    keys = sorted(e.FirstKey for e in md.entries)
    lo = max(i for i, k in enumerate(keys) if k <= start)
    picked = {lo}
    if keys[lo] == start and lo:  # the descending walk goes on past an equal key (:434)
        lo -= 1
        picked.add(lo)
    hi = max(i for i, k in enumerate(keys) if k <= end)  # DescendLessOrEqual(end), one item (:440-443)
    picked.add(hi)
    assert hi - lo > 2  # the range spans blocks the walks do not pick
    assert io["calls"] == 1 and io["blocks"] == len(picked)
    by_key = {e.FirstKey: e for e in md.entries}
    span = by_key[keys[hi]].Offset + by_key[keys[hi]].BlockSize - by_key[keys[lo]].Offset
    assert io["bytes_staged"] == span


def _with_descs(data, meta, edit):
    """The segment with its meta block rewritten: edit(i, BlockStat) changes
    entries in place; the meta hash is recomputed so the metadata loads."""
    import struct
    from oracle import pyoracle as P
    md = P.bytes_to_metadata(meta)
    for i, st in enumerate(md.entries):
        edit(i, st)
    moff, = struct.unpack_from("<Q", data, len(data) - 25)
    head_len = 2 + struct.unpack_from("<H", meta, 0)[0]
    head_len += 2 + struct.unpack_from("<H", meta, head_len)[0]
    head = meta[:head_len] + bytes([0, 0, 0]) + struct.pack("<Q", len(md.entries))
    new_meta = head + b"".join(st.to_bytes() for st in md.entries)
    seg = data[:moff] + new_meta
    return seg + struct.pack("<QQBQ", moff, P.xxh64(new_meta), 1, P.MAGIC)


def test_go_int_conversions_through_reader(decoder):
    """Descriptors past Go's int() conversions (segment_reader.go:303-340):
    a negative Offset is a Seek error, a BlockSize above the runtime's maxAlloc
    (2^48) panics in make before any read, OriginalSize >= 2^63 walks no record
    (nil rows, no error).  Product reader == oracle ReadBlockWithStat."""
    from oracle import pyoracle as P
    rows, data, flen, meta = _segment(nrows=400)
    n = len(data)

    def edit(i, st):
        if i == 0:
            st.OriginalSize = 1 << 63
        elif i == 1:
            st.OriginalSize = (1 << 64) - 1
        elif i == 2:
            st.BlockSize = (1 << 48) + 1
        elif i == 3:
            st.BlockSize = 1 << 63
        elif i == 4:
            st.BlockSize = 1 << 48  # allocatable: short read
        elif i == 5:
            st.Offset, st.BlockSize = n + 10, 1 << 50  # make panics before io.EOF
        elif i == 6:
            st.Offset = (1 << 63) + 5  # Seek error before the make panic
            st.BlockSize = 1 << 60
        elif i == 7:
            st.Offset = n + 100  # io.EOF
    seg = _with_descs(data, meta, edit)
    md = P.bytes_to_metadata(seg[struct_off(seg):len(seg) - 25])
    pr = R.SegmentReader(seg, len(seg), decoder)
    tree = sorted(md.entries, key=lambda e: e.FirstKey)
    assert pr.NumBlocks() == len(tree)
    seen = set()
    for i, st in enumerate(tree):
        status, want = P.read_block(seg, st.desc(), P.COMP_NONE)
        seen.add(status)
        if status == P.BLK_OK:
            got = pr.ReadBlock(i)
            assert [(r.Key, r.Value) for r in (got or [])] == \
                [(r.Key, r.Value) for r in (want or [])], i
        elif status == P.BLK_PANIC:
            with pytest.raises(R.GoPanic):
                pr.ReadBlock(i)
        else:
            with pytest.raises(R.GoError) as e:
                pr.ReadBlock(i)
            assert e.value.kind == ("EOF" if status == P.BLK_EOF else "ErrUnexpectedBytesRead")
    assert seen >= {P.BLK_OK, P.BLK_PANIC, P.BLK_EOF, P.BLK_SHORT}
    # OriginalSize >= 2^63: no record walked, nil rows, no error
    assert P.read_block(seg, md.entries[0].desc(), P.COMP_NONE) == (P.BLK_OK, None)
    assert pr.ReadBlock([e.FirstKey for e in tree].index(md.entries[0].FirstKey)) is None


def struct_off(seg):
    import struct
    return struct.unpack_from("<Q", seg, len(seg) - 25)[0]


@pytest.mark.parametrize("nblk", [1, 4096, 65536])
def test_getrow_on_large_segment_stages_one_block(decoder, nblk):
    """GetRow on C3-shaped segments up to 65 536 x 64 KiB (4.3 GB, offsets past
    4 GiB): one block staged, the row equals the writer's."""
    from objectkv_amd import sst as S
    w = S.synth_segment(1, 3, nblocks=nblk, threshold=57344, block_size=65536)
    data = w.data()
    pr = R.SegmentReader(data, len(data), decoder)
    n = pr.NumBlocks()
    last = pr.ReadBlock(n - 1)
    io = pr.io_stats()
    assert io["calls"] == 1 and io["blocks"] == 1 and io["bytes_staged"] == 65536
    k = last[-1].Key
    assert pr.GetRow(k).Key == k
    assert pr.io_stats()["bytes_staged"] == 2 * 65536


def test_getrow_rows_outlive_window_replacement(decoder):
    """Rows GetRow serves from the iteration window stay valid until the next
    GetRow / ReadBlock / GetRange call (okv_host.h), even when a later RowIter
    replaces the window: iterate, free the iterator, GetRow (from the
    window), seek a new iterator far away (window miss), then read the row's
    bytes through the returned pointers (okv_reader.cpp
    read_block)."""
    import ctypes as C
    from objectkv_amd._lib import Row, lib
    rows, data, flen, meta = _segment(nrows=12000, vmax=300)
    pr = R.SegmentReader(data, flen, decoder)
    L = lib()
    it = L.okv_reader_row_iter(pr._h, 0)
    row = Row()
    assert L.okv_iter_next(it, C.byref(row)) == 0  # window = the first 256 blocks
    L.okv_iter_free(it)
    k, v = rows[700]
    kb = C.create_string_buffer(k, len(k))
    got = Row()
    before = pr.io_stats()["calls"]
    assert L.okv_reader_get_row(pr._h, kb, len(k), C.byref(got)) == 0
    assert pr.io_stats()["calls"] == before  # served from the window
    it2 = L.okv_reader_row_iter(pr._h, 0)
    far = rows[-5][0]
    assert L.okv_iter_seek(it2, C.create_string_buffer(far, len(far)), len(far)) == 0
    assert pr.io_stats()["calls"] > before  # the window moved
    junk = [bytes(4096) for _ in range(2000)]  # reuse freed memory if any was freed
    assert C.string_at(got.key, got.key_len) == k
    assert (C.string_at(got.val, got.val_len) if got.val_len else b"") == v
    L.okv_iter_free(it2)
    del junk
