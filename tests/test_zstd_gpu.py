"""GPU parity for zstd blocks (okv_zstd.hip): the device decompression +
record walk must equal the CPU oracle, whose zstd checker is libzstd
(oracle/zstd_ref.py; klauspost v1.17.9 is not available offline)."""
from __future__ import annotations

import numpy as np
import pytest

import objectkv_amd as okv
from objectkv_amd import reader as R
from oracle import coracle as CO
from oracle import pyoracle as P
from tests import zstd_cases as ZC

pytestmark = pytest.mark.gpu

SOA = ("row_start", "key_off", "key_len", "val_off", "val_len", "key_base", "val_base")


def _check(decoder, seg, descs, index_only=False):
    d = np.array(descs, np.uint64).reshape(-1, 4)
    got = decoder.decode(np.frombuffer(seg, np.uint8), d, P.COMP_ZSTD, index_only=index_only)
    ref = CO.decode_soa(seg, CO.descs_array(descs), P.COMP_ZSTD, index_only)
    assert np.array_equal(got.status, ref["status"])
    for k in SOA:
        if index_only and k in ("key_base", "val_base"):
            continue
        assert np.array_equal(getattr(got, k), ref[k]), k
    if not index_only:
        assert got.key_arena.tobytes() == ref["key_arena"].tobytes()
        assert got.val_arena.tobytes() == ref["val_arena"].tobytes()
    return got


@pytest.mark.parametrize("case", ZC.cases(), ids=lambda c: c[0])
def test_zstd_cases(decoder, case):
    name, seg, descs, _note = case
    got = _check(decoder, seg, descs)
    assert int(got.status.max()) == 0, name
    _check(decoder, seg, descs, index_only=True)  # every block OKV_BLK_UNSUPPORTED


@pytest.mark.parametrize("case", ZC.corrupt_cases(), ids=lambda c: c[0])
def test_zstd_corrupt(decoder, case):
    name, seg, descs = case
    _check(decoder, seg, descs)


def test_zstd_segment_through_product_reader(decoder):
    """RowIter / GetRow / GetRange over a zstd segment (C++ reader mirror)."""
    rows = ZC._rows(21, 2500)
    seg, flen, _meta = ZC.Z.zstd_segment(rows, 3584, 4096, level=7)
    pr = R.SegmentReader(seg, flen, decoder)
    orr = P.SegmentReader(seg, flen)
    it, oit = pr.RowIter(R.DirectionAscending), orr.RowIter(0)
    n = 0
    while True:
        try:
            a = it.Next()
        except R.GoError as e:
            assert e.kind == "EOF"
            break
        b = oit.Next()
        assert (a.Key, a.Value) == (b.Key, b.Value)
        n += 1
    assert n == len(rows)
    k, v = rows[1234]
    assert pr.GetRow(k).Value == (v or None)
    got = pr.GetRange(rows[100][0], rows[900][0])
    want = orr.GetRange(rows[100][0], rows[900][0])
    assert [(r.Key, r.Value) for r in got] == [(r.Key, r.Value) for r in want]
