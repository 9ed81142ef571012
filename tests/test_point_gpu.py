"""The host-mode point path (okv_point_kernel: a host-mode call of <= 16
small uncompressed blocks decoded by one workgroup in one launch, reading
and writing a pinned slab) against the oracle, bit-exact, and
GetRow's host bloom probe through the product reader
(segment_reader.go:245-258, :362-404)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import objectkv_amd as okv
from objectkv_amd import _lib
from objectkv_amd import reader as R
from tests.conftest import descs_of, unpack
from oracle import coracle as CO
from tests.test_decode_gpu import _assert_same_as_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nopoint():
    dec = okv.Decoder(0, flags=_lib.OPEN_NO_POINT)
    yield dec
    dec.close()


def _point(decoder, seg, d, comp=0, expect=True):
    got = decoder.decode(bytes(seg), d, comp)
    if expect:
        assert decoder.last_path() == _lib.PATH_POINT, decoder.last_path()
    return got


def _same(a, b):
    for k in ("status", "row_start", "key_base", "val_base", "key_off", "key_len", "val_off",
              "val_len"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    assert a.key_arena.tobytes() == b.key_arena.tobytes()
    assert a.val_arena.tobytes() == b.val_arena.tobytes()


def test_point_golden_writer_cases(decoder, golden):
    """The reference test segments (segment_reader_test.go inputs), in
    batches of <= 16 blocks, through the point path == oracle."""
    for name, case in golden.items():
        if case["kind"] != "writer" or case["compression"] == _lib.COMP_ZSTD:
            continue
        seg = unpack(case["segment_z"])
        d = descs_of(case)
        for b0 in range(0, d.shape[0], 16):
            dd = d[b0:b0 + 16]
            got = _point(decoder, seg, dd, case["compression"])
            _assert_same_as_oracle(got, seg, dd, case["compression"], False)


@pytest.mark.parametrize("comp", [_lib.COMP_NONE, _lib.COMP_LZ4])
def test_point_crafted_edges(decoder, golden, comp):
    """Overrun panics, short reads, EOF, OriginalSize 0, records past
    OriginalSize, nil keys/values, the u16-max key, 600 rows, unaligned
    offsets, Go's int() conversions, the LZ4 flag -- every crafted block that
    stages (BlockSize <= 64 KiB or not readable), one block per call and all
    of them in batches of 16."""
    case = golden["crafted_edges"]
    seg = unpack(case["segment_z"])
    d = descs_of(case)
    for b in range(d.shape[0]):
        one = d[b:b + 1]
        got = decoder.decode(seg, one, comp)
        if decoder.last_path() == _lib.PATH_POINT:
            _assert_same_as_oracle(got, seg, one, comp, False)
    keep = [b for b in range(d.shape[0])
            if comp == _lib.COMP_LZ4 or int(d[b][1]) <= 65536 or int(d[b][0]) >= len(seg)
            or int(d[b][0]) >= 2**63 or int(d[b][1]) > 2**48
            or len(seg) - int(d[b][0]) < int(d[b][1])]
    dd = d[keep]
    for b0 in range(0, dd.shape[0], 16):
        got = _point(decoder, seg, dd[b0:b0 + 16], comp)
        _assert_same_as_oracle(got, seg, dd[b0:b0 + 16], comp, False)


def _blocks(rng, nblk, max_rows=40, corrupt=0.2):
    seg, descs = bytearray(), []
    for _ in range(nblk):
        body = bytearray()
        for _ in range(int(rng.integers(0, max_rows))):
            kl = int(rng.choice([0, 1, 5, 16, 100, 300]))
            vl = int(rng.choice([0, 1, 7, 64, 500, 2000]))
            if len(body) + 6 + kl + vl > 60000:
                break
            body += kl.to_bytes(2, "little") + vl.to_bytes(4, "little")
            body += rng.integers(0, 256, kl + vl, dtype=np.uint8).tobytes()
        orig = len(body)
        if rng.random() < 0.3 and body:
            orig = int(rng.integers(0, len(body) + 1))
        if rng.random() < corrupt and len(body) > 3:
            body[int(rng.integers(0, len(body)))] = int(rng.integers(0, 256))
        bsize = min(65536, len(body) + int(rng.choice([0, 1, 5, 64, 4096])))
        body = body[:bsize]
        off = len(seg) + int(rng.choice([0, 0, 1, 3, 8, 15]))
        seg += bytes(off - len(seg))
        seg += body + bytes(bsize - len(body))
        descs.append((off, bsize, orig, 0))
    return bytes(seg), np.array(descs, np.uint64).reshape(-1, 4)


def test_point_fuzz_against_oracle_and_device_path(decoder, nopoint):
    """60 random batches of 1-16 blocks (corrupt and truncated records, odd
    offsets, OriginalSize inside records, empty blocks, the LZ4 flag): the
    point path == oracle == the device-resident path of a NO_POINT context."""
    rng = np.random.default_rng(515)
    for trial in range(60):
        seg, d = _blocks(rng, int(rng.integers(1, 17)))
        comp = int(rng.choice([0, 0, 0, 2]))
        got = _point(decoder, seg, d, comp)
        _assert_same_as_oracle(got, seg, d, comp, False)
        ref = nopoint.decode(seg, d, comp)
        assert not nopoint.last_path() & _lib.PATH_POINT
        _same(got, ref)


def test_point_many_rows(decoder):
    """Blocks past kFastRows (1024) rows: 1 500 small records, and a 64 KiB
    block of empty records (10 922 rows, the most a staged block can hold),
    beside an ordinary block: the batched re-walk (materialise) == oracle."""
    rng = np.random.default_rng(3)
    body1 = bytearray()
    for _ in range(1500):
        kl, vl = int(rng.integers(0, 12)), int(rng.integers(0, 20))
        body1 += kl.to_bytes(2, "little") + vl.to_bytes(4, "little")
        body1 += rng.integers(0, 256, kl + vl, dtype=np.uint8).tobytes()
    body2 = bytes(65536 // 6 * 6)
    body3 = (5).to_bytes(2, "little") + (9).to_bytes(4, "little") + b"hello" + b"world!!!!"
    seg = bytes(body1) + bytes(body2) + body3 + bytes(7)
    d = np.array([(0, len(body1), len(body1), 0), (len(body1), len(body2), len(body2), 0),
                  (len(body1) + len(body2), len(body3) + 7, len(body3), 0)], np.uint64)
    got = _point(decoder, seg, d)
    ref = _assert_same_as_oracle(got, seg, d, 0, False)
    assert int(got.row_start[-1]) == 1500 + 65536 // 6 + 1
    assert got.block_rows(2) == [(b"hello", b"world!!!!")]
    assert int(ref["row_start"][-1]) == int(got.row_start[-1])


def test_point_c3_blocks(decoder, nopoint):
    """8 C3 (64 KiB Zipf) blocks (512 KiB: the point path's byte cap) and 16 C2
    (4 KiB) blocks: point == device path == oracle; 16 C3 blocks (1 MiB) take
    the device path (measured faster past the cap)."""
    for kind, th, bs, nb in ((okv.sst.SYNTH_ZIPF, 57344, 65536, 8),
                             (okv.sst.SYNTH_FIXED, 3584, 4096, 16)):
        w = okv.synth_segment(kind, 12, nblocks=40, threshold=th, block_size=bs)
        seg, d = w.data(), w.descs()
        for b0 in (0, 16, 23):
            dd = d[b0:b0 + nb].copy()
            base = int(dd[0][0])
            span = seg.tobytes()[base:int(dd[-1][0] + dd[-1][1])]
            dd[:, 0] -= base
            got = _point(decoder, span, dd)
            _assert_same_as_oracle(got, span, dd, 0, False)
            _same(got, nopoint.decode(span, dd))
        if kind == okv.sst.SYNTH_ZIPF:  # past the byte cap: the device path
            dd = d[0:16].copy()
            span = seg.tobytes()[:int(dd[-1][0] + dd[-1][1])]
            got = decoder.decode(span, dd)
            assert not decoder.last_path() & _lib.PATH_POINT, decoder.last_path()
            _assert_same_as_oracle(got, span, dd, 0, False)


def test_point_capacity_error(decoder, golden):
    """A caller capacity below the totals: OKV_E_CAPACITY with the totals set
    (as the device path reports it)."""
    import ctypes as C
    case = golden["ref_read_uncompressed_200"]
    seg = np.frombuffer(unpack(case["segment_z"]), np.uint8)
    d = descs_of(case)
    o = {k: np.zeros(n, t) for k, n, t in [("row_start", 3, np.uint64), ("status", 2, np.int32)]}
    small = _lib.DecodeOut(o["row_start"].ctypes.data, None, None, o["status"].ctypes.data,
                           None, None, None, None, None, None, 0, 0, 0, 0, 0, 0, 0)
    rc = _lib.lib().okv_decode_blocks(decoder._ctx, seg.ctypes.data, seg.size, d.ctypes.data,
                                      2, 0, C.byref(small), 0)
    assert decoder.last_path() == _lib.PATH_POINT
    assert rc == _lib.OKV_E_CAPACITY and small.n_rows == 200


# ---- GetRow: the bloom probe on the host, one GPU call per block read --------

def _bloom_segment(n=4000):
    from oracle.bloom_ref import default_filter
    f = default_filter()
    rows = [(b"k%06d" % i, b"v%06d" % i * (1 + i % 7)) for i in range(0, 2 * n, 2)]
    w = okv.SegmentWriter(3584, 4096, bloom=f)
    for k, v in rows:
        w.WriteRow(k, v)
    flen, meta = w.Close()
    return rows, w.data().tobytes(), flen, meta, f


def test_getrow_bloom_negative_costs_no_gpu_call(decoder):
    """A key the filter rejects returns ErrNoRows without a block read (no
    GPU call); a member costs exactly one call staging one block."""
    rows, data, flen, meta, f = _bloom_segment()
    r = R.SegmentReader(data, flen, decoder)
    r.GetRow(rows[0][0])  # metadata loaded
    absent = [b"k%06d" % i for i in range(1, 8000, 2)]
    absent = [k for k in absent if not f.test(k)][:500]
    before = r.io_stats()
    for k in absent:
        with pytest.raises(R.GoError) as e:
            r.GetRow(k)
        assert e.value.kind == "ErrNoRows"
    assert r.io_stats() == before
    for k, v in rows[::397]:
        b = r.io_stats()
        assert r.GetRow(k).Value == v
        a = r.io_stats()
        assert a["calls"] - b["calls"] == 1 and a["blocks"] - b["blocks"] == 1
        assert decoder.last_path() == _lib.PATH_POINT


def test_getrow_bloom_negative_over_corrupt_block(decoder):
    """Go probes the filter before touching any block (:371-378): a key the
    filter rejects whose floor block is corrupt is ErrNoRows, while a member
    of that block panics in mustReadBytes (:506-512) -- product == oracle."""
    from oracle import pyoracle as P
    rows, data, flen, meta, f = _bloom_segment()
    md = P.bytes_to_metadata(meta)
    ent = sorted(md.entries, key=lambda e: e.FirstKey)
    target = ent[len(ent) // 2]
    bad = bytearray(data)
    # the second record's key length -> past the block: the walk panics there
    kl0 = int.from_bytes(bad[target.Offset:target.Offset + 2], "little")
    vl0 = int.from_bytes(bad[target.Offset + 2:target.Offset + 6], "little")
    p2 = target.Offset + 6 + kl0 + vl0
    bad[p2:p2 + 2] = (65535).to_bytes(2, "little")
    bad = bytes(bad)
    member = target.FirstKey
    nxt = ent[len(ent) // 2 + 1].FirstKey
    absent = next(k for k in (member + b"%03d" % i for i in range(1000))
                  if k < nxt and not f.test(k))
    pr, orr = R.SegmentReader(bad, flen, decoder), P.SegmentReader(bad, flen)
    with pytest.raises(R.GoError) as e:
        pr.GetRow(absent)
    assert e.value.kind == "ErrNoRows"
    with pytest.raises(P.GoError) as e2:
        orr.GetRow(absent)
    assert e2.value.kind == P.ErrNoRows
    with pytest.raises(R.GoPanic):
        pr.GetRow(member)
    with pytest.raises(P.GoPanic):
        orr.GetRow(member)


def _point_get(decoder, seg, desc, comp, key):
    """okv_point_get through ctypes: (status, found, key, value)."""
    L = _lib.lib()
    buf = np.frombuffer(bytes(seg), np.uint8) if len(seg) else np.zeros(1, np.uint8)
    d = _lib.BlockDesc(*[int(x) for x in desc])
    out = _lib.PointRow()
    kb = bytes(key)
    rc = L.okv_point_get(decoder._ctx, buf.ctypes.data, len(seg), C.byref(d), comp, kb, len(kb),
                         C.byref(out))
    assert rc == 0, decoder.error()
    k = C.string_at(out.key, out.key_len) if out.found == 1 and out.key_len else b""
    v = C.string_at(out.val, out.val_len) if out.found == 1 and out.val_len else b""
    return out.status, out.found, k, v


def _expect_get(ref, b, key):
    """GetRow's row loop (segment_reader.go:395-403) on the oracle's rows of block b."""
    st = int(ref["status"][b])
    if st != 0:
        return st, 0, b"", b""
    r0, r1 = int(ref["row_start"][b]), int(ref["row_start"][b + 1])
    ka, va = ref["key_arena"].tobytes(), ref["val_arena"].tobytes()
    for g in range(r0, r1):
        ko, kl = int(ref["key_off"][g]), int(ref["key_len"][g])
        if ka[ko:ko + kl] == bytes(key):
            vo, vl = int(ref["val_off"][g]), int(ref["val_len"][g])
            return 0, 1, ka[ko:ko + kl], va[vo:vo + vl]
    return 0, 0, b"", b""


@pytest.mark.parametrize("comp", [_lib.COMP_NONE, _lib.COMP_LZ4])
def test_point_get_matches_oracle_row_loop(decoder, golden, comp):
    """okv_point_get (GetRow's block step, one row back) == the oracle's
    ReadBlockWithStat + bytes.Equal loop: every key of every stageable
    crafted and writer block (duplicates: the first row), absent keys, the
    empty key, a key one byte longer, and every block status."""
    cases = [golden["crafted_edges"]] + [c for c in golden.values()
                                         if c["kind"] == "writer" and c["compression"] != 2]
    checked = 0
    for case in cases:
        seg = unpack(case["segment_z"])
        d = descs_of(case)
        c = comp if case is golden["crafted_edges"] else case["compression"]
        for b in range(d.shape[0]):
            ref = CO.decode_soa(seg, CO.descs_array([tuple(int(x) for x in d[b])]), c, False)
            keys = [b"", b"\x00", b"no-such-key"]
            r0, r1 = int(ref["row_start"][0]), int(ref["row_start"][1])
            ka = ref["key_arena"].tobytes()
            for g in list(range(r0, r1))[:40] + list(range(max(r0, r1 - 5), r1)):
                ko, kl = int(ref["key_off"][g]), int(ref["key_len"][g])
                keys += [ka[ko:ko + kl], ka[ko:ko + kl] + b"\x01"]
            for key in keys:
                got = _point_get(decoder, seg, d[b], c, key)
                if got[1] == -1:  # not a point-path block (> 64 KiB, > 1 024 rows, key > 8 KiB)
                    continue
                assert got == _expect_get(ref, 0, key), (b, key[:20])
                checked += 1
    assert checked > 200


def test_point_get_reader_rows_and_fallback(decoder, nopoint):
    """GetRow through the product reader takes okv_point_get and agrees with a
    NO_POINT context's reader (full decode + host row loop) on present,
    duplicate-free and absent keys, values (nil for empty) included; blocks of
    more than 1 024 rows (tiny records) fall back to the full decode."""
    from tests.test_reader_gpu import _segment
    for nrows, vmax in ((3000, 300), (5000, 0)):
        rows, data, flen, _meta = _segment(nrows=nrows, vmax=vmax)
        ra = R.SegmentReader(data, flen, decoder)
        rb = R.SegmentReader(data, flen, nopoint)
        keys = [k for k, _v in rows[::97]] + [rows[-1][0], b"", b"\xff" * 9, rows[5][0] + b"\x00"]
        for k in keys:
            out = []
            for rd in (ra, rb):
                try:
                    kv = rd.GetRow(k)
                    out.append((kv.Key, kv.Value))
                except Exception as e:  # noqa: BLE001
                    out.append(type(e).__name__)
            assert out[0] == out[1], (k, out)


def test_getrow_counts_point_launch_before_full_decode(decoder):
    """A block of more than 1 024 rows: okv_point_get walks it (one launch,
    found == -1) and the reader then decodes it in full -- both GPU calls are
    counted in the reader's I/O stats, and the row is Go's."""
    rows = [(b"k%05d" % i, b"") for i in range(1500)]  # 12-byte records
    w = okv.SegmentWriter(60000, 65536)
    for k, v in rows:
        w.WriteRow(k, v)
    flen, _meta = w.Close()
    r = R.SegmentReader(w.data().tobytes(), flen, decoder)
    b = r.io_stats()
    got = r.GetRow(rows[1234][0])
    assert got.Key == rows[1234][0] and not got.Value
    a = r.io_stats()
    assert a["calls"] - b["calls"] == 2 and a["blocks"] - b["blocks"] == 2, (b, a)
