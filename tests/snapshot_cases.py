"""Segment sets for the snapshot-merge tests (shared by the CPU oracle tests
and the GPU parity tests).

reference_segments() rebuilds prepareTestReader
(/root/reference/snapshot_reader/snapshot_reader_test.go:19-194) with the
restated writer; random_snapshot() makes overlapping L0/L1 segment sets with
tombstones (empty values) for randomized parity.
"""
from __future__ import annotations

import random

from oracle import pyoracle as P


def _write(rows):
    w = P.SegmentWriter(P.SegmentWriterOptions())
    for k, v in rows:
        w.WriteRow(k, v)
    n, meta = w.Close()
    return bytes(w.external), n, meta


def reference_segments():
    """[(ID, Level, segment bytes, file length, meta bytes)] as :19-194 builds them."""
    rows1 = []
    for i in range(0, 200, 2):
        rows1.append((b"key%03d" % i, b"value%03d-ISHOULDNOTSHOW" % i))
        if i == 0:
            rows1.append((b"key0010", b"value0010"))
    rows11 = [(b"key%03d" % i, b"value%03d" % i) for i in range(0, 200, 2)]
    rows2 = [(b"key%03d" % i, b"value%03d" % i) for i in range(1, 200, 2)]
    rows3 = [(b"key%03d" % i, b"value%03d-I-SHOULD-NOT-SHOW" % i) for i in range(1, 200, 2)]
    rows3.append((b"key900", b"value900"))
    out = []
    for sid, lvl, rows in (("1-0", 0, rows1), ("1-1", 0, rows11), ("2-1", 0, rows2),
                           ("2-0", 1, rows3)):
        data, n, meta = _write(rows)
        out.append((sid, lvl, data, n, meta))
    return out


def random_snapshot(seed, nseg=5, keyspace=400, rows_per_seg=(20, 160), tomb_frac=0.15,
                    vmax=40):
    """Segments over a shared key space: each holds a sorted random subset of
    keys; L0 segments may hold tombstones (empty values)."""
    rng = random.Random(seed)
    keys = sorted({b"k%05d" % rng.randrange(keyspace * 3) + bytes(rng.randrange(3))
                   for _ in range(keyspace)})
    out = []
    for s in range(nseg):
        level = 0 if s < nseg - 2 else rng.choice((1, 2))
        n = min(len(keys), rng.randint(*rows_per_seg))
        lo = rng.randrange(0, max(1, len(keys) - n))
        pick = sorted(rng.sample(range(lo, min(len(keys), lo + 3 * n)), n))
        rows = []
        for i in pick:
            tomb = level == 0 and rng.random() < tomb_frac
            v = b"" if tomb else b"s%d-%s-" % (s, keys[i]) + bytes(rng.randrange(256)
                                                                  for _ in range(rng.randrange(vmax)))
            rows.append((keys[i], v))
        data, n_bytes, meta = _write(rows)
        out.append((f"{s + 1:04d}-{rng.randrange(100)}", level, data, n_bytes, meta))
    return out, keys


def quirk_segments():
    """Crafted snapshot for the Go loop's edge paths (snapshot_reader.go:294-365):
    "A" (newest L0) ends with a tombstone at k20 -> GetRange rolls it forward
    onto io.EOF; "C" (older L0) ends with a tombstone at k25 while the owner of
    k25 continues -> the stale cursor is an L0 tombstone -> io.EOF; "B" (L1)
    spans multiple 4 KiB blocks, so descending seeks land on block first keys."""
    a = [(b"k%02d" % i, b"a%02d" % i) for i in range(10, 20)] + [(b"k20", b"")]
    c = [(b"k%02d" % i, b"c%02d" % i) for i in range(22, 25)] + [(b"k25", b"")]
    d = [(b"k%02d" % i, b"d%02d" % i) for i in range(21, 31)]
    b = [(b"k%02d" % i, b"b%02d-" % i + bytes(700)) for i in range(0, 61)]  # 61: Q1
    out = []
    for sid, lvl, rows in (("9", 0, a), ("1", 0, c), ("5", 0, d), ("0", 1, b)):
        data, n, meta = _write(rows)
        out.append((sid, lvl, data, n, meta))
    return out
