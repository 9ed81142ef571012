"""GPU parity of the snapshot reader (objectkv_amd/snapshot.py over the device
merge okv_merge_rows) against the oracle restatement of snapshot_reader.go
(oracle/snapshot_oracle.py): the reference's own test segments, randomized
overlapping L0/L1 snapshots with tombstones, Iter paging, and the device
compaction (decode -> merge -> encode)."""
from __future__ import annotations

import random

import numpy as np
import pytest

import objectkv_amd as okv
from objectkv_amd import snapshot as SN
from oracle import pyoracle as P
from oracle import snapshot_oracle as SO
from tests import snapshot_cases as SC

pytestmark = pytest.mark.gpu


def _pair(segs, decoder):
    data = {sid: (d, n) for sid, _l, d, n, _m in segs}
    orc = SO.Reader(lambda rec: P.SegmentReader(*data[rec.ID]))
    dev = SN.Reader(lambda rec: data[rec.ID], decoder)
    orecs, drecs = [], []
    for sid, lvl, _d, _n, meta in segs:
        md = P.bytes_to_metadata(meta)
        orecs.append(SO.SegmentRecord(sid, lvl, md.FirstKey, md.LastKey))
        drecs.append(SN.SegmentRecord(sid, lvl, md.FirstKey, md.LastKey))
    orc.UpdateSegments(orecs, None)
    dev.UpdateSegments(drecs, None)
    return orc, dev, orecs, drecs


def _outcome(fn):
    try:
        rows = fn()
    except (P.GoError, SN.SnapshotError) as e:
        return ("err", e.kind)
    except (P.GoPanic, SN.SnapshotPanic):
        return ("panic",)
    if rows is None:
        return ("nil",)
    return ("rows", [(r.Key, r.Value) for r in rows])


def _same_range(orc, dev, start, end, limit, direction):
    a = _outcome(lambda: orc.GetRange(start, end, limit, direction))
    b = _outcome(lambda: dev.GetRange(start, end, limit, direction))
    assert a == b, (start, end, limit, direction, a, b)
    return a


def test_reference_snapshot_on_device(decoder):
    """snapshot_reader_test.go's calls (:196-476), device vs oracle."""
    orc, dev, orecs, drecs = _pair(SC.reference_segments(), decoder)
    for k in (b"key000", b"key001", b"key900", b"key999", b"key800", b"key0010", b"key198"):
        assert _outcome(lambda: [P.KVPair(k, orc.GetRow(k))]) == \
            _outcome(lambda: [SN.KVPair(k, dev.GetRow(k))])
    calls = [(b"key000", b"key006", 100), (b"key000", b"key006", 2), (b"key010", b"key106", 10),
             (b"key00", b"key0000", 2), (b"key000", b"key0000", 2), (b"key900", b"key901", 2),
             (b"key901", b"key910", 100), (b"key00", b"key000", 2), (b"key899", b"key901", 2),
             (b"key190", P.UnboundEnd, 100), (P.UnboundStart, b"key050", 1000),
             (b"key006", b"key000", 5), (b"key000", b"key006", 0)]
    for d in (P.DirectionAscending, P.DirectionDescending):
        for s, e, lim in calls:
            _same_range(orc, dev, s, e, lim, d)
    rows = dev.GetRange(b"key000", b"key006", 100, P.DirectionAscending)
    assert [r.Key for r in rows] == [b"key000", b"key001", b"key0010", b"key002", b"key003",
                                     b"key004", b"key005"]
    orc.UpdateSegments(None, [orecs[3]])
    dev.UpdateSegments(None, [drecs[3]])
    assert _outcome(lambda: [P.KVPair(b"", orc.GetRow(b"key900"))]) == \
        _outcome(lambda: [SN.KVPair(b"", dev.GetRow(b"key900"))])


@pytest.mark.parametrize("seed", range(6))
def test_random_snapshot_get_range(decoder, seed):
    segs, keys = SC.random_snapshot(seed, nseg=3 + seed % 4)
    orc, dev, _, _ = _pair(segs, decoder)
    rng = random.Random(100 + seed)
    probes = keys + [k + b"\x00" for k in keys[::7]] + [b"", b"k", b"z", P.UnboundEnd]
    nonempty = 0
    for _ in range(60):
        a, b = rng.choice(probes), rng.choice(probes)
        if SO._cmp(a, b) > 0 and rng.random() < 0.85:
            a, b = b, a
        if rng.random() < 0.1:
            a = P.UnboundStart
        lim = rng.choice([1, 2, 3, 7, 50, 10_000])
        d = rng.choice([P.DirectionAscending, P.DirectionDescending])
        out = _same_range(orc, dev, a, b, lim, d)
        nonempty += out[0] == "rows" and len(out[1]) > 0
    for k in keys[::5]:
        assert _outcome(lambda: [P.KVPair(k, orc.GetRow(k))]) == \
            _outcome(lambda: [SN.KVPair(k, dev.GetRow(k))])
    assert nonempty > 5


def test_snapshot_iter_paging(decoder):
    """snapshot_iter.go: Next/Peek paging through GetRange, to io.EOF or the
    empty-page panic, device vs oracle."""
    for seed in (11, 12, 13):
        segs, keys = SC.random_snapshot(seed, nseg=3)
        orc, dev, _, _ = _pair(segs, decoder)
        for d, start in ((P.DirectionAscending, keys[3]), (P.DirectionDescending, keys[-4])):
            for buf in (3, 17):
                oi, di = orc.RowIter(start, d, buf), dev.RowIter(start, d, buf)
                for _ in range(400):
                    a = _outcome(lambda: [oi.Next()])
                    b = _outcome(lambda: [di.Next()])
                    assert a == b
                    if a[0] != "rows":
                        break


def _py_merge(segs, drop):
    """Newest-wins over whole segments in priority order (GetRange's owner
    rule, snapshot_reader.go:294-331) -> sorted rows."""
    seen = {}
    for sid, lvl, d, n, _m in segs:
        r = P.SegmentReader(d, n)
        md = r.FetchAndLoadMetadata()
        for st in md.entries:
            for kv in r.ReadBlockWithStat(st) or []:
                if kv.Key not in seen:
                    seen[kv.Key] = (lvl, kv.Value)
    out = []
    for k in sorted(seen):
        lvl, v = seen[k]
        if drop and lvl == 0 and v is None:
            continue
        out.append((k, v))
    return out


@pytest.mark.parametrize("drop", [True, False])
def test_device_compaction(decoder, drop):
    """compact(): decode -> merge -> encode on the GPU equals the restated
    writer over the newest-wins merge, byte for byte."""
    segs, _ = SC.random_snapshot(21, nseg=5, rows_per_seg=(200, 900), keyspace=1500)
    order = sorted(segs, key=lambda s: (s[1], [-ord(c) for c in s[0]]))  # level, ID desc
    enc = okv.Encoder(0)
    dsegs = [(SN.DeviceSegment(enc, d, n), lvl) for _sid, lvl, d, n, _m in order]
    got = SN.compact(dsegs, enc, drop_tombstones=drop)
    want_rows = _py_merge(order, drop)
    w = P.SegmentWriter(P.SegmentWriterOptions())
    for k, v in want_rows:
        w.WriteRow(k, v or b"")
    nbytes, _meta = w.Close()
    assert got.n_rows == len(want_rows)
    assert got.file_bytes == nbytes
    assert got.seg.tobytes() == bytes(w.external)
    enc.close()


def test_merge_abi_all_mode(decoder):
    """okv_merge_rows directly: random sub-ranges of several sorted streams,
    OKV_MERGE_ALL ascending and descending, against a Python merge."""
    import torch
    rng = random.Random(7)
    segs, _ = SC.random_snapshot(31, nseg=6, rows_per_seg=(50, 400))
    dsegs = [SN.DeviceSegment(decoder, d, n) for _sid, _l, d, n, _m in segs]
    levels = [lvl for _sid, lvl, _d, _n, _m in segs]
    for trial in range(8):
        srcs, want = [], {}
        for i, ds in enumerate(dsegs):
            lo = rng.randrange(0, ds.n // 2 + 1)
            hi = rng.randrange(lo, ds.n + 1)
            srcs.append((ds.t, lo, hi, levels[i]))
            for r in range(lo, hi):
                want.setdefault(ds.key(r), (i, r))
        drop = trial % 2 == 0
        keys = sorted(k for k, (i, r) in want.items()
                      if not (drop and levels[i] == 0 and dsegs[i].value(r) is None))
        for d in (okv._lib.DIR_ASC, okv._lib.DIR_DESC):
            cap = sum(hi - lo for _t, lo, hi, _l in srcs) + 1
            out = {"src": torch.empty(cap, dtype=torch.int32, device="cuda"),
                   "row": torch.empty(cap, dtype=torch.int64, device="cuda")}
            mo = decoder.merge_device(srcs, okv._lib.MERGE_ALL, d, 0, None, drop, out,
                                      row_cap=cap)
            n = int(mo.n_rows)
            got = list(zip(out["src"][:n].cpu().tolist(), out["row"][:n].cpu().tolist()))
            exp = [want[k] for k in (keys if d == okv._lib.DIR_ASC else keys[::-1])]
            assert got == exp
            assert mo.n_unique == len(want)


def test_quirk_snapshot_on_device(decoder):
    """Tombstone rolled onto io.EOF, stale L0-tombstone cursor, descending
    seeks onto block first keys: device vs oracle, every (start, end) pair."""
    segs = SC.quirk_segments()
    orc, dev, _, _ = _pair(segs, decoder)
    probes = [b"k%02d" % i for i in range(0, 62, 3)] + [b"k20", b"k25", b"k21"]
    md = P.bytes_to_metadata(segs[3][4])
    probes += [st.FirstKey for st in md.entries]
    kinds = set()
    for a in probes:
        for b in probes:
            for d in (P.DirectionAscending, P.DirectionDescending):
                for lim in (0, 2, 100):
                    kinds.add(_same_range(orc, dev, a, b, lim, d)[0:2][0])
    assert {"rows", "err", "panic"} <= kinds
