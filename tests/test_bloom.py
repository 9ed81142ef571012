"""GetRow's bloom probe on the host (segment_reader.go:245-258, :371-378;
parseBloomFilterBlock :183-201): the product's C++ restatement of
bits-and-blooms v2.0.3 ReadFrom / Test (okv_meta_bloom_test) against the
independent Python restatement (oracle/bloom_ref.py).  No GPU: metadata
parsing and the probe are host code.

Parity unpinned: no reference test asserts filter bytes or Test results
(the Go module is not vendored); what is pinned is that both restatements
agree key by key, that members always test positive (no false negatives),
and the reference's TestRollover with DefaultSegmentWriterOptions (bloom on)
passes through the product reader (tests/test_reader_gpu.py)."""
from __future__ import annotations

import ctypes as C
import struct

import numpy as np
import pytest

import objectkv_amd as okv
from objectkv_amd import _lib
from oracle import bloom_ref as B
from oracle import pyoracle as P


def _meta_handle(meta: bytes):
    h = C.c_void_p()
    buf = C.create_string_buffer(bytes(meta), len(meta))
    rc = _lib.lib().okv_meta_parse(buf, len(meta), C.byref(h))
    return rc, h


def _meta_with_bloom(bloom_bytes: bytes) -> bytes:
    """A minimal meta block (BytesToMetadata layout) carrying the given
    BloomFilter.WriteTo bytes and one block index entry."""
    m = struct.pack("<H", 1) + b"a" + struct.pack("<H", 1) + b"z"
    m += b"\x01" + struct.pack("<Q", len(bloom_bytes)) + bloom_bytes
    m += b"\x00" + b"\x00" + struct.pack("<Q", 1)
    m += struct.pack("<H", 1) + b"a" + struct.pack("<QQQQQ", 0, 4096, 100, 0, 0)
    return m


def _test(h, key: bytes) -> int:
    return _lib.lib().okv_meta_bloom_test(h, key, len(key))


def test_bloom_probe_matches_python_restatement():
    """The default filter (NewWithEstimates(100000, 1e-6)) with 5 000 members
    written by the product writer: every member tests positive, and 20 000
    keys (members, non-members, empty, long) test the same on both sides."""
    f = B.default_filter()
    rng = np.random.default_rng(9)
    members = [b"key%06d" % i for i in range(0, 10000, 2)]
    w = okv.SegmentWriter(3584, 4096, bloom=f)
    for k in members:
        w.WriteRow(k, b"v")
    _, meta = w.Close()
    rc, h = _meta_handle(meta)
    assert rc == 0 and _lib.lib().okv_meta_has_bloom(h) == 1
    try:
        for k in members:
            assert _test(h, k) == 1
        probes = [b"key%06d" % i for i in range(1, 10000, 2)] + [b""] + \
                 [rng.integers(0, 256, int(rng.integers(1, 300)), np.uint8).tobytes()
                  for _ in range(15000)]
        neg = 0
        for k in probes:
            t = _test(h, k)
            assert t == int(f.test(k)), k
            neg += t == 0
        assert neg > len(probes) * 0.99  # a 1e-6 filter rejects almost every non-member
    finally:
        _lib.lib().okv_meta_free(h)


@pytest.mark.parametrize("m,k,length,nwords", [
    (64, 3, 64, 1), (1000, 7, 1000, 16), (10, 2, 0, 0), (100, 0, 100, 2), (129, 4, 200, 4)])
def test_bloom_small_filters(m, k, length, nwords):
    """Hand-built filters (ReadFrom's field order; a bitset length that differs
    from m; k = 0; an empty bitset): both restatements agree on 500 keys."""
    rng = np.random.default_rng(m * 31 + k)
    words = [int(x) for x in rng.integers(0, 2**63, nwords, dtype=np.uint64)]
    bb = struct.pack(f">QQQ{nwords}Q", m, k, length, *words)
    ref = B.BloomFilter.from_bytes(bb)
    rc, h = _meta_handle(_meta_with_bloom(bb))
    assert rc == 0
    try:
        for i in range(500):
            key = b"p%d" % i
            assert _test(h, key) == int(ref.test(key))
    finally:
        _lib.lib().okv_meta_free(h)


@pytest.mark.parametrize("bb", [
    b"", b"\x00" * 23,                                        # m / k / length short
    struct.pack(">QQQ", 64, 3, 65),                           # 2 words needed, 0 present
    struct.pack(">QQQQ", 640, 3, 640, 1),                     # 10 words needed, 1 present
    struct.pack(">QQQ", 64, 3, 2**64 - 1),                    # wordsNeeded overflow guard
])
def test_bloom_read_from_errors(bb):
    """BloomFilter.ReadFrom errors make BytesToMetadata fail (:160-163):
    OKV_M_BLOOM from the product, ErrBloomReadFrom from the oracle."""
    meta = _meta_with_bloom(bb)
    rc, _ = _meta_handle(meta)
    assert rc == -208
    with pytest.raises(P.GoError) as e:
        P.bytes_to_metadata(meta)
    assert e.value.kind == P.ErrBloomReadFrom


def test_bloom_trailing_bytes_and_zero_m():
    """ReadFrom reads no byte past the bitset (trailing bytes are ignored);
    a filter with m == 0 and k > 0 makes Test divide by zero -- Go's runtime
    panic, OKV_R_PANIC from the product."""
    bb = struct.pack(">QQQQ", 64, 2, 64, 2**64 - 1) + b"trailing"
    rc, h = _meta_handle(_meta_with_bloom(bb))
    assert rc == 0
    assert _test(h, b"x") == 1
    _lib.lib().okv_meta_free(h)
    rc, h = _meta_handle(_meta_with_bloom(struct.pack(">QQQQ", 0, 3, 64, 1)))
    assert rc == 0
    assert _test(h, b"x") == -307  # OKV_R_PANIC
    _lib.lib().okv_meta_free(h)
    with pytest.raises(ZeroDivisionError):
        B.BloomFilter.from_bytes(struct.pack(">QQQQ", 0, 3, 64, 1)).test(b"x")
