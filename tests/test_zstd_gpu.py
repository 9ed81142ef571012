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

@pytest.fixture(scope="module")
def one_pass_decoder():
    """A context opened with OKV_OPEN_ZSTD_ONE_PASS: every zstd block through
    the one-wave-per-block kernel."""
    dec = okv.Decoder(0, flags=okv._lib.OPEN_ZSTD_ONE_PASS)
    yield dec
    dec.close()


@pytest.fixture(params=["staged", "one_pass"])
def zdec(request, decoder, one_pass_decoder):
    """Every case through both device paths: the staged decoder (prologue ->
    lane-per-block sequences -> parallel executor, the default) and the
    one-pass kernel (OKV_OPEN_ZSTD_ONE_PASS; also the staged path's fallback
    for the blocks its prologue hands back)."""
    return one_pass_decoder if request.param == "one_pass" else decoder


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
def test_zstd_cases(zdec, case):
    name, seg, descs, _note = case
    got = _check(zdec, seg, descs)
    assert int(got.status.max()) == 0, name
    _check(zdec, seg, descs, index_only=True)  # every block OKV_BLK_UNSUPPORTED


@pytest.mark.parametrize("case", ZC.corrupt_cases(), ids=lambda c: c[0])
def test_zstd_corrupt(zdec, case):
    name, seg, descs = case
    _check(zdec, seg, descs)


def test_zstd_segment_through_product_reader(zdec):
    """RowIter / GetRow / GetRange over a zstd segment (C++ reader mirror)."""
    rows = ZC._rows(21, 2500)
    seg, flen, _meta = ZC.Z.zstd_segment(rows, 3584, 4096, level=7)
    pr = R.SegmentReader(seg, flen, zdec)
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


def test_zstd_bench_shape_blocks(zdec):
    """64 KiB text blocks as bench.py --config cz builds them (libzstd level 3)."""
    from tools.zstd_gen import text_zstd_segment
    seg, descs, _ = text_zstd_segment(24, 9, 3)
    got = _check(zdec, seg.tobytes(), [tuple(int(x) for x in d) for d in descs])
    assert int(got.status.max()) == 0


def test_zstd_long_runs_and_rle_literals(zdec):
    """Matches far longer than the executor's 1 KiB byte map, offset-1 runs,
    and blocks whose literals are RLE."""
    rows = []
    for i in range(120):
        v = bytes([i % 7]) * (4500 + 37 * i) if i % 3 else (b"ab" * 2100 + bytes(range(i % 50)))
        rows.append((b"r%06d" % i, v))
    seg, _, _ = ZC.Z.zstd_segment(rows, 57344, 65536, level=3)
    from oracle import pyoracle as P2
    md = P2.bytes_to_metadata(ZC._meta_of(seg))
    got = _check(zdec, seg, [st.desc() for st in md.entries])
    assert int(got.status.max()) == 0


def test_zstd_dense_short_sequences(zdec):
    """Values of 5-byte words from a vocabulary of 8, each followed by one random
    byte: libzstd emits a short sequence (one literal, one short match) every ~6
    bytes, more per KiB of output than the executor's 128-sequence window holds,
    so chunks end at the window instead of at the byte map."""
    rng = np.random.default_rng(11)
    vocab = [bytes(rng.integers(97, 123, size=5, dtype=np.uint8)) for _ in range(8)]
    rows = []
    for i in range(400):
        n = 200 + (i % 97)
        v = b"".join(vocab[int(t)] + bytes([int(r)])
                     for t, r in zip(rng.integers(0, 8, n), rng.integers(0, 256, n)))
        rows.append((b"d%06d" % i, v))
    seg, _, _ = ZC.Z.zstd_segment(rows, 57344, 65536, level=3)
    from oracle import pyoracle as P2
    md = P2.bytes_to_metadata(ZC._meta_of(seg))
    got = _check(zdec, seg, [st.desc() for st in md.entries])
    assert int(got.status.max()) == 0


def test_zstd_staged_equals_general_under_corruption(decoder, one_pass_decoder):
    """Byte flips in the sequence sections of 48 blocks.  Two-sided against the
    oracle (libzstd as the decoder checker): every block's status must equal
    the oracle's -- a corrupt frame the checker rejects must fail on the
    device too, and vice versa -- and the decoded rows of the blocks that
    succeed must equal its bytes.  Both device paths, and they agree."""
    import random
    from tools.zstd_gen import text_zstd_segment
    seg, descs, _ = text_zstd_segment(48, 13, 3)
    b = bytearray(seg.tobytes())
    rng = random.Random(5)
    for i, d in enumerate(descs):
        off, csz = int(d[0]), int(d[3])
        for _ in range(1 + i % 3):
            b[off + csz - 1 - rng.randrange(min(csz - 20, 3000))] ^= 1 << rng.randrange(8)
    dl = [tuple(int(x) for x in d) for d in descs]
    staged = _check(decoder, bytes(b), dl)
    general = _check(one_pass_decoder, bytes(b), dl)
    assert np.array_equal(staged.status, general.status)
    assert staged.val_arena.tobytes() == general.val_arena.tobytes()
    # the flips must actually exercise both outcomes
    assert 0 < int((staged.status != 0).sum()) < len(dl)


def test_zstd_sequence_section_corruption_wide(decoder, one_pass_decoder):
    """Bit flips in the back 40 % of 256 frames (the sequences section and its
    bitstream, whose first bytes are read last): most such streams overflow,
    so the sequence stage's last stored sequence reads past the stream's start
    and the executor re-reads its extra bits masked (ZBlk::pfix); corrupt
    repeat-offset codes go through the executor's repeat-offset scan.
    Two-sided against libzstd through the oracle (statuses and the rows of the
    blocks that decode), and the one-pass kernel agrees."""
    import random
    from tools.zstd_gen import text_zstd_segment
    seg, descs, _ = text_zstd_segment(256, 29, 3)
    b = bytearray(seg.tobytes())
    rng = random.Random(31)
    for d in descs:
        off, csz = int(d[0]), int(d[3])
        back = max(8, (csz * 2) // 5)
        for _ in range(1 + rng.randrange(2)):
            b[off + csz - 1 - rng.randrange(back)] ^= 1 << rng.randrange(8)
    dl = [tuple(int(x) for x in d) for d in descs]
    staged = _check(decoder, bytes(b), dl)
    general = _check(one_pass_decoder, bytes(b), dl)
    assert np.array_equal(staged.status, general.status)
    bad = int((staged.status != 0).sum())
    assert 0 < bad < len(dl)


def test_zstd_literal_stream_corruption(decoder, one_pass_decoder):
    """Byte flips in the first KiBs of 48 frames -- the Huffman tree and the
    literal streams, which the staged path decodes in its stream stage
    (okv_zstd_huf_kernel, 8 blocks per wave) and the one-pass kernel inline.
    Two-sided against libzstd through the oracle: every block's status equals
    the checker's (a stream that fails its end-marker or bit-count checks fails
    the block; a flip that only changes literal values must give the checker's
    bytes), on both device paths."""
    import random
    from tools.zstd_gen import text_zstd_segment
    seg, descs, _ = text_zstd_segment(48, 17, 3)
    b = bytearray(seg.tobytes())
    rng = random.Random(23)
    for i, d in enumerate(descs):
        off, csz = int(d[0]), int(d[3])
        for _ in range(1 + i % 2):
            b[off + 40 + rng.randrange(min(csz - 60, 4000))] ^= 1 << rng.randrange(8)
    dl = [tuple(int(x) for x in d) for d in descs]
    staged = _check(decoder, bytes(b), dl)
    general = _check(one_pass_decoder, bytes(b), dl)
    assert np.array_equal(staged.status, general.status)
    assert 0 < int((staged.status != 0).sum()) < len(dl)


@pytest.mark.parametrize("case", ZC.past_original_cases(), ids=lambda c: c[0])
def test_zstd_past_original_size(zdec, case):
    """Frames that inflate past OriginalSize decode in full on the device (Go's
    io.Copy, segment_reader.go:320-330) and walk to OriginalSize (:338-352);
    OriginalSize >= 2^63 walks nothing (:340); blocks past Block_Maximum_Size
    (RFC 8878 3.1.1.2.4) and windowLog > 31 fail.  No block ends at
    OKV_BLK_CAPACITY; frames larger than their first output region take the
    regrow pass (OKV_PATH_ZSTD_REGROW), the others do not."""
    name, seg, descs, want, regrow = case
    got = _check(zdec, seg, descs)
    assert [int(x) for x in got.status] == want, name
    assert bool(zdec.last_path() & okv._lib.PATH_ZSTD_REGROW) == regrow, name
