"""CPU restatement of the reference's snapshot reader (test infrastructure).

Restates /root/reference/snapshot_reader/snapshot_reader.go and
snapshot_iter.go statement by statement on top of the sst restatement in
oracle/pyoracle.py (SegmentReader / RowIter).  Only tests/ and bench.py's
cpu_baseline leg use this module; the product path is
objectkv_amd/snapshot.py over the device merge (objectkv_amd/csrc/okv_merge.hip).

Pinned by the reference's own known answers (tests/test_snapshot.py re-asserts
snapshot_reader_test.go: TestGetRow :196-245, TestGetRangeAscending :276-375,
TestGetRangeDescending :377-476, TestFindMaxIndexes :478-529).  The Go
toolchain is absent, so nothing here is checked against Go output directly.
"""
from __future__ import annotations

import functools

from oracle import pyoracle as P

ErrInvalidRange = "ErrInvalidRange"          # snapshot_reader.go:203
ErrNoNextIndexFound = "ErrNoNextIndexFound"  # :374


def _b(x):
    return P._b(x)


def _cmp(a, b) -> int:  # bytes.Compare (nil == empty)
    a, b = _b(a), _b(b)
    return (a > b) - (a < b)


class SegmentRecord:
    """segment_record.go:5-12 (Metadata carries FirstKey / LastKey)."""

    def __init__(self, ID: str, Level: int, FirstKey, LastKey):
        self.ID, self.Level, self.FirstKey, self.LastKey = ID, Level, FirstKey, LastKey

    def __repr__(self):
        return f"SegmentRecord({self.ID!r}, L{self.Level})"


def block_range_less(a: SegmentRecord, b: SegmentRecord) -> bool:  # :29-61
    c = _cmp(a.FirstKey, b.FirstKey)
    if c != 0:
        return c < 0
    if len(_b(a.LastKey)) == 0:
        return False
    if len(_b(b.LastKey)) == 0:
        return True
    c = _cmp(a.LastKey, b.LastKey)
    if c != 0:
        return c < 0
    if a.ID == "":
        return False
    if b.ID == "":
        return True
    return a.ID < b.ID


class _Tree:
    """google/btree BTreeG with a less function: ReplaceOrInsert / Delete /
    DescendLessOrEqual (items equal under `less` replace each other)."""

    def __init__(self, less):
        self.less = less
        self.items: list = []

    def _eq(self, a, b):
        return not self.less(a, b) and not self.less(b, a)

    def replace_or_insert(self, it):
        for i, x in enumerate(self.items):
            if self._eq(x, it):
                self.items[i] = it
                return
        self.items.append(it)
        self.items.sort(key=functools.cmp_to_key(
            lambda a, b: -1 if self.less(a, b) else (1 if self.less(b, a) else 0)))

    def delete(self, it) -> bool:
        for i, x in enumerate(self.items):
            if self._eq(x, it):
                del self.items[i]
                return True
        return False

    def descend_le(self, pivot):
        """Items <= pivot (not less(pivot, item)), descending."""
        for x in reversed(self.items):
            if not self.less(pivot, x):
                yield x


def first_value(a, b, direction) -> int:  # :379-398
    r = _cmp(a, b)
    if r == 0:
        return 0
    if direction == P.DirectionDescending:
        return 1 if r > 0 else -1
    return 1 if r < 0 else -1


def find_max_indexes(arr, compare):  # :404-424
    if len(arr) == 0:
        return None
    mx = arr[0]
    idx = [0]
    for i in range(1, len(arr)):
        c = compare(arr[i], mx)
        if c > 0:
            mx = arr[i]
            idx = [i]
        elif c == 0:
            idx.append(i)
    return idx


class Reader:
    """snapshot_reader.go:16-27, 63-74 (NewReader)."""

    def __init__(self, factory):
        self.segmentIDTree = _Tree(lambda a, b: a.ID < b.ID)
        self.blockRangeTree = _Tree(block_range_less)
        self.readerFactory = factory

    def UpdateSegments(self, add, drop):  # :80-96
        for d in drop or []:
            if not self.segmentIDTree.delete(d):
                continue
            self.blockRangeTree.delete(d)
        for a in add or []:
            self.segmentIDTree.replace_or_insert(a)
            self.blockRangeTree.replace_or_insert(a)

    def getPossibleSegmentsForKey(self, key):  # :149-170
        out = []
        for rec in self.blockRangeTree.descend_le(SegmentRecord("", 0, key, None)):
            in_range = _cmp(key, rec.FirstKey) >= 0 and _cmp(key, rec.LastKey) <= 0
            if in_range:
                out.append(rec)
            if not in_range:
                break
        return out

    def getPossibleSegmentsForRange(self, start, end):  # :172-193
        out = []
        for rec in self.blockRangeTree.descend_le(SegmentRecord("", 0, end, None)):
            in_range = not (_cmp(start, rec.LastKey) > 0 or _cmp(end, rec.FirstKey) < 0)
            if in_range:
                out.append(rec)
            if not in_range:
                break
        return out

    def GetRow(self, key):  # :98-146
        segs = self.getPossibleSegmentsForKey(key)
        segs.sort(key=functools.cmp_to_key(_getrow_cmp))
        for seg in segs:
            reader = self.readerFactory(seg)
            try:
                row = reader.GetRow(key)
            except P.GoError as e:
                if e.kind == P.ErrNoRows:
                    continue
                raise
            if _b(row.Value) == b"" and seg.Level == 0:
                raise P.GoError(P.ErrNoRows)
            return row.Value
        raise P.GoError(P.ErrNoRows)

    def GetRange(self, start, end, limit, direction):  # :214-372
        if _cmp(start, end) >= 0:
            raise P.GoError(ErrInvalidRange)
        segs = self.getPossibleSegmentsForRange(start, end)
        if len(segs) == 0:
            return None
        segs.sort(key=functools.cmp_to_key(lambda a, b: _getrange_cmp(a, b, direction)))
        iters, cursors = [], []
        start_range = end if direction == P.DirectionDescending else start
        for seg in segs:  # :259-290 (errgroup per segment, waited in turn)
            reader = self.readerFactory(seg)
            it = reader.RowIter(direction)
            it.Seek(start_range)
            iters.append(it)
            cursors.append(it.Next())  # io.EOF here is a GetRange error
        if limit < 0:
            raise P.GoPanic("makeslice: len out of range")
        rows = []
        last_key = None
        while True:
            nxt = find_max_indexes(cursors, lambda a, b: first_value(a.Key, b.Key, direction))
            if not nxt:
                raise P.GoError(ErrNoNextIndexFound)
            if segs[nxt[0]].Level == 0 and cursors[nxt[0]].Value is None:
                for ind in nxt:  # :316-331: any EOF is an error
                    cursors[ind] = iters[ind].Next()
                continue
            row = cursors[nxt[0]]
            if _b(last_key) != b"" and _b(row.Key) == _b(last_key):
                break
            if direction == P.DirectionAscending and _cmp(row.Key, end) >= 0:
                break
            if direction == P.DirectionDescending and _cmp(row.Key, start) <= 0:
                break
            last_key = row.Key
            if len(rows) >= limit:  # rows[addedRowIndex] with addedRowIndex == limit
                raise P.GoPanic("index out of range")
            rows.append(row)
            if len(rows) >= limit:
                break
            for ind in nxt:  # :351-365: io.EOF leaves the cursor in place
                try:
                    cursors[ind] = iters[ind].Next()
                except P.GoError as e:
                    if e.kind != P.EOF:
                        raise
        return rows

    def RowIter(self, start, direction, bufferSize=100):  # :430-443
        return Iter(self, start, direction, bufferSize)


def _getrow_cmp(a, b):  # :103-110 (less -> cmp)
    def less(x, y):
        if x.Level != y.Level:
            return x.Level < y.Level
        return x.ID > y.ID
    return -1 if less(a, b) else (1 if less(b, a) else 0)


def _getrange_cmp(a, b, direction):  # :235-254
    def less(x, y):
        if x.Level != y.Level:
            return x.Level < y.Level
        if x.Level == 0 and y.Level == 0:
            return x.ID > y.ID
        if direction == P.DirectionAscending:
            return _cmp(x.FirstKey, y.FirstKey) < 0
        return _cmp(x.LastKey, y.LastKey) > 0
    return -1 if less(a, b) else (1 if less(b, a) else 0)


class Iter:
    """snapshot_iter.go:11-116."""

    def __init__(self, reader, start, direction, bufferSize):
        self.reader, self.lastKey, self.direction = reader, start, direction
        self.bufferSize = bufferSize
        self.rowBuffer: list = []
        self.done = False

    def Next(self):  # :37-47
        self._check_load()
        return self.rowBuffer.pop(0)

    def Peek(self):  # :51-61
        self._check_load()
        return self.rowBuffer[0]

    def _check_load(self):  # :65-108
        if self.rowBuffer:
            return
        if self.done:
            raise P.GoError(P.EOF)
        if self.direction == P.DirectionDescending:
            s, e = P.UnboundStart, self.lastKey
        else:
            s, e = self.lastKey, P.UnboundEnd
        rows = self.reader.GetRange(s, e, self.bufferSize, self.direction)
        if not rows:
            self.done = True
            raise P.GoError(P.EOF)
        self.rowBuffer = []
        for i, r in enumerate(rows):
            if i == 0 and _b(r.Key) == _b(self.lastKey):
                continue
            self.rowBuffer.append(r)
        if not self.rowBuffer:  # i.rowBuffer.Back() is nil: .Value panics
            raise P.GoPanic("nil pointer dereference")
        self.lastKey = self.rowBuffer[-1].Key


def next_possible_key(key, direction):  # utils.go:8-24
    nk = bytearray(512)
    kb = _b(key)
    nk[:len(kb)] = kb[:512]
    for i in range(511, -1, -1):
        if nk[i] == 0 and direction == P.DirectionAscending:
            nk[i] += 1
            break
        if nk[i] > 0 and direction == P.DirectionDescending:
            nk[i] -= 1
            break
    return bytes(nk)
