"""Snapshot reader oracle (oracle/snapshot_oracle.py) pinned to the reference's
own known answers: snapshot_reader_test.go TestGetRow (:196-245),
TestGetRangeAscending (:276-375), TestGetRangeDescending (:377-476),
TestFindMaxIndexes (:478-529), and the quirks the restatement keeps."""
from __future__ import annotations

import pytest

from oracle import pyoracle as P
from oracle import snapshot_oracle as S
from tests import snapshot_cases as SC


def _reader():
    segs = SC.reference_segments()
    data = {sid: (d, n) for sid, _l, d, n, _m in segs}

    def factory(rec):
        d, n = data[rec.ID]
        return P.SegmentReader(d, n)

    r = S.Reader(factory)
    recs = []
    for sid, lvl, _d, _n, meta in segs:
        md = P.bytes_to_metadata(meta)
        recs.append(S.SegmentRecord(sid, lvl, md.FirstKey, md.LastKey))
    r.UpdateSegments(recs, None)
    return r, recs


def test_reference_get_row():  # :196-245
    r, recs = _reader()
    assert r.GetRow(b"key000") == b"value000"
    assert r.GetRow(b"key001") == b"value001"
    assert r.GetRow(b"key900") == b"value900"
    for k in (b"key999", b"key800"):
        with pytest.raises(P.GoError) as e:
            r.GetRow(k)
        assert e.value.kind == P.ErrNoRows
    r.UpdateSegments(None, [recs[3]])
    with pytest.raises(P.GoError) as e:
        r.GetRow(b"key900")
    assert e.value.kind == P.ErrNoRows


def _keys(rows):
    return [x.Key for x in rows]


@pytest.mark.parametrize("direction", [P.DirectionAscending, P.DirectionDescending])
def test_reference_get_range(direction):  # :276-476
    r, _ = _reader()
    asc = direction == P.DirectionAscending
    order = (lambda ks: ks == sorted(ks)) if asc else (lambda ks: ks == sorted(ks, reverse=True))
    rows = r.GetRange(b"key000", b"key006", 100, direction)
    assert len(rows) == 7 and order(_keys(rows))
    rows = r.GetRange(b"key000", b"key006", 2, direction)
    assert len(rows) == 2 and order(_keys(rows))
    rows = r.GetRange(b"key010", b"key106", 10, direction)
    assert len(rows) == 10 and order(_keys(rows))
    assert len(r.GetRange(b"key00", b"key0000", 2, direction)) == 1
    if asc:
        assert len(r.GetRange(b"key000", b"key0000", 2, direction)) == 1
        assert len(r.GetRange(b"key900", b"key901", 2, direction)) == 1
    else:
        assert len(r.GetRange(b"key00", b"key000", 2, direction)) == 1
        assert len(r.GetRange(b"key899", b"key901", 2, direction)) == 1
    assert len(r.GetRange(b"key901", b"key910", 100, direction) or []) == 0


def test_reference_get_range_values():
    """What the reference test's comments state: seg1's buried rows never show,
    "key0010" shows between key001 and key002, the L1 duplicates are hidden."""
    r, _ = _reader()
    rows = r.GetRange(b"key000", b"key006", 100, P.DirectionAscending)
    assert _keys(rows) == [b"key000", b"key001", b"key0010", b"key002", b"key003",
                           b"key004", b"key005"]
    assert all(b"NOT" not in x.Value for x in rows)


def test_reference_find_max_indexes():  # :478-529
    items = [P.KVPair(b"b"), P.KVPair(b"b"), P.KVPair(b"a"), P.KVPair(b"b")]
    assert S.find_max_indexes(items, lambda a, b: S._cmp(a.Key, b.Key)) == [0, 1, 3]
    assert S.find_max_indexes(items, lambda a, b: -S._cmp(a.Key, b.Key)) == [2]


def test_get_range_quirks():
    """Kept as the Go loop has them: an exhausted segment stalls the merge at
    its last key (the stale cursor equals lastKey); limit 0 panics; start >=
    end is ErrInvalidRange."""
    r, _ = _reader()
    # 1-0 / 1-1 end at key198, 2-1 at key199, 2-0 continues to key900
    rows = r.GetRange(b"key190", P.UnboundEnd, 100, P.DirectionAscending)
    assert _keys(rows)[-1] in (b"key198", b"key199") and b"key900" not in _keys(rows)
    with pytest.raises(P.GoPanic):
        r.GetRange(b"key000", b"key006", 0, P.DirectionAscending)
    with pytest.raises(P.GoError) as e:
        r.GetRange(b"key006", b"key000", 5, P.DirectionAscending)
    assert e.value.kind == S.ErrInvalidRange


def test_random_snapshot_oracle_consistency():
    """The restated loop agrees with a direct newest-wins merge wherever no
    stream runs out inside the range (the quirk-free region)."""
    segs, keys = SC.random_snapshot(3, nseg=4)
    data = {sid: (d, n) for sid, _l, d, n, _m in segs}
    r = S.Reader(lambda rec: P.SegmentReader(*data[rec.ID]))
    recs = [S.SegmentRecord(sid, lvl, P.bytes_to_metadata(m).FirstKey,
                            P.bytes_to_metadata(m).LastKey) for sid, lvl, _d, _n, m in segs]
    r.UpdateSegments(recs, None)
    for k in keys[::17]:
        try:
            v = r.GetRow(k)
        except P.GoError as e:
            assert e.kind == P.ErrNoRows
            continue
        assert v is None or isinstance(v, bytes)


def _quirk_reader():
    segs = SC.quirk_segments()
    data = {sid: (d, n) for sid, _l, d, n, _m in segs}
    r = S.Reader(lambda rec: P.SegmentReader(*data[rec.ID]))
    recs = [S.SegmentRecord(sid, lvl, P.bytes_to_metadata(m).FirstKey,
                            P.bytes_to_metadata(m).LastKey) for sid, lvl, _d, _n, m in segs]
    r.UpdateSegments(recs, None)
    return r, segs


def test_get_range_eof_quirks():
    r, _ = _quirk_reader()
    # a tombstone that ends its stream: Next() -> io.EOF is returned as an error
    with pytest.raises(P.GoError) as e:
        r.GetRange(b"k00", b"k99", 100, P.DirectionAscending)
    assert e.value.kind == P.EOF
    # the tombstone check (:302) precedes the range check (:330): a range that
    # ends at the tombstone's key still rolls it onto io.EOF
    with pytest.raises(P.GoError) as e:
        r.GetRange(b"k00", b"k20", 100, P.DirectionAscending)
    assert e.value.kind == P.EOF
    # the range ends at a live row before the tombstone: no error
    rows = r.GetRange(b"k00", b"k19", 100, P.DirectionAscending)
    assert [x.Key for x in rows][-1] == b"k18"
    # the stale cursor of "C" (L0 tombstone at k25) after k25 is emitted from "5"
    with pytest.raises(P.GoError) as e:
        r.GetRange(b"k21", b"k99", 100, P.DirectionAscending)
    assert e.value.kind == P.EOF


def test_descending_seek_on_block_first_key():
    """RowIter.Seek walks DescendLessOrEqual while FirstKey == key
    (segment_row_iter.go:113-116): a descending seek onto a block's first key
    starts in the previous block, so that row is not returned."""
    r, segs = _quirk_reader()
    md = P.bytes_to_metadata(segs[3][4])
    # only segment "0" (multi-block L1): with the L0 segments present the
    # segment search descending from `end` stops at "1" (:182-191)
    r.UpdateSegments(None, [S.SegmentRecord(sid, lvl, P.bytes_to_metadata(m).FirstKey,
                                            P.bytes_to_metadata(m).LastKey)
                            for sid, lvl, _d, _n, m in segs[:3]])
    # a block first key and a range (start, end] = (k31, fk] that holds fk
    fk = next(e.FirstKey for e in md.entries if e.FirstKey > b"k32")
    rows = r.GetRange(b"k31", fk, 100, P.DirectionDescending)
    keys = [x.Key for x in rows]
    assert fk not in keys and keys[0] < fk and keys[-1] > b"k31"
