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
