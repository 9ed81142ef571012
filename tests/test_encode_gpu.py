"""GPU parity for the device encode (okv_encode_rows, okv_encode.hip): the
segment bytes -- data blocks, BlockStat index, meta block and trailer -- must
equal the CPU oracle writer's (oracle/okv_oracle.c, a restatement of
segment_writer.go:80-328) and the committed golden segments, bit for bit."""
from __future__ import annotations

import random

import numpy as np
import pytest
import torch

import objectkv_amd as okv
from objectkv_amd import _lib
from oracle import coracle as CO
from oracle import pyoracle as P
from tests import reference_cases as RC
from tests.conftest import descs_of, unpack
from tests.golden.make_golden import writer_inputs
from tests.test_reader_gpu import ProductImpl

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def enc():
    e = okv.Encoder(0)
    yield e
    e.close()


def oracle_segment(rows, threshold=3584, block_size=4096, lz4=False):
    w = CO.Writer(threshold, block_size, 0, lz4)
    for k, v in rows:
        assert w.write_row(k, v) == 0
    return w.close()  # (rc, file bytes, meta bytes)


def test_golden_writer_cases(enc, golden):
    """Every reference test input encodes to the committed golden segment."""
    for name, rows, kw in writer_inputs():
        case = golden[name]
        got = enc.encode(rows, compression=okv.sst.COMP_LZ4 if kw.get("lz4") else 0)
        want = unpack(case["segment_z"])
        assert got.seg.tobytes() == want, name
        assert got.file_bytes == case["file_len"] == len(want)
        assert np.array_equal(got.descs, descs_of(case)), name
        assert [int(h) for h in got.hashes] == [b["hash"] for b in case["blocks"]], name
        assert got.meta() == bytes.fromhex(case["meta"]), name


class GpuWriterImpl(ProductImpl):
    """The reference Go tests with the GPU writer on the write side."""
    encoder = None

    @classmethod
    def write(cls, rows, **kw):
        bloom = None
        if kw.get("BloomFilter") == "default":
            from oracle.bloom_ref import default_filter
            bloom = default_filter()
        w = okv.GpuSegmentWriter(cls.encoder, bloom=bloom)
        for k, v in rows:
            w.WriteRow(k, v)
        flen, meta = w.Close()
        return w.data().tobytes(), flen, meta


@pytest.mark.parametrize("case", RC.CASES, ids=lambda c: c.__name__)
def test_reference_cases_gpu_writer(case, enc, decoder):
    GpuWriterImpl.encoder = enc
    GpuWriterImpl.decoder = decoder
    case(GpuWriterImpl)


def _random_rows(rng, n, kmax, vmax, big_every=0):
    rows = []
    for i in range(n):
        k = b"%08d" % i + bytes(rng.getrandbits(8) for _ in range(rng.randint(0, kmax)))
        vl = rng.randint(0, vmax)
        if big_every and i % big_every == big_every - 1:
            vl = rng.randint(5000, 20000)
        rows.append((k, bytes(rng.getrandbits(8) for _ in range(vl))))
    return rows


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_vs_oracle(enc, seed):
    """Random rows and writer options (incl. DataBlockSize not a multiple of
    16 -> byte path, tiny thresholds, rows larger than a block, LZ4 flag)."""
    rng = random.Random(seed)
    for trial in range(4):
        n = rng.choice([1, 2, 7, 300, 2500])
        rows = _random_rows(rng, n, rng.choice([0, 5, 80]), rng.choice([0, 10, 300]),
                            big_every=rng.choice([0, 97]))
        T = rng.choice([1, 50, 3584, 20000])
        D = rng.choice([4096, 512, 16, 100, 1])
        lz4 = rng.random() < 0.3
        rc, want, meta = oracle_segment(rows, T, D, lz4)
        comp = okv.sst.COMP_LZ4 if lz4 else 0
        if rc:  # the oracle reproduces Go's panic when the last row closed a block (Q1)
            assert rc == _lib.W_NIL_WRITER
            with pytest.raises(okv.OkvError) as e:
                enc.encode(rows, T, D, comp)
            assert e.value.code == _lib.W_NIL_WRITER
            # non-strict: the footer is written normally (host writer, strict_go=0)
            hw = okv.SegmentWriter(T, D, 0, lz4)
            for k, v in rows:
                hw.WriteRow(k, v)
            hw.Close(strict_go=False)
            got = enc.encode(rows, T, D, comp, strict_go=False)
            assert got.seg.tobytes() == hw.data().tobytes(), (seed, trial)
            continue
        got = enc.encode(rows, T, D, comp)
        assert got.seg.tobytes() == want, (seed, trial, n, T, D, lz4)
        assert got.meta() == meta


def test_errors(enc):
    rows = [(b"a", b"1"), (b"b", b""), (b"", b"x"), (b"d", b"2")]
    with pytest.raises(okv.OkvError) as e:
        enc.encode(rows)
    assert e.value.code == _lib.W_INVALID_KEY  # ErrInvalidKey, segment_writer.go:89-91
    with pytest.raises(okv.OkvError) as e:
        enc.encode([])
    assert e.value.code == _lib.W_NIL_WRITER  # Close with nothing open panics (Q1)
    with pytest.raises(okv.OkvError) as e:
        enc.encode([], strict_go=False)
    assert e.value.code == _lib.W_NO_ROWS  # ErrNoRowsWritten (:221-223)
    with pytest.raises(okv.OkvError) as e:
        enc.encode([(b"a", b"b")], compression=okv.sst.COMP_ZSTD)
    assert e.value.code == _lib.W_UNSUPPORTED
    # GpuSegmentWriter validates per row like WriteRow (:80-91)
    w = okv.GpuSegmentWriter(enc)
    for bad, code in ((b"", _lib.W_INVALID_KEY), (b"k" * 65536, _lib.W_KEY_TOO_LARGE)):
        with pytest.raises(okv.OkvError) as e:
            w.WriteRow(bad, b"v")
        assert e.value.code == code


def test_bad_row_reported_device(enc):
    n = 1000
    kl = torch.full((n,), 4, dtype=torch.int16, device="cuda")
    kl[617] = 0
    kl[901] = 0
    rows = dict(key_arena=torch.zeros(4 * n, dtype=torch.uint8, device="cuda"),
                key_off=torch.arange(n, dtype=torch.int64, device="cuda") * 4, key_len=kl,
                val_arena=torch.zeros(16, dtype=torch.uint8, device="cuda"),
                val_off=torch.zeros(n, dtype=torch.int64, device="cuda"),
                val_len=torch.zeros(n, dtype=torch.int32, device="cuda"))
    with pytest.raises(okv.OkvError) as e:
        enc.encode_device(rows, n, {"seg": torch.empty(1 << 20, dtype=torch.uint8,
                                                       device="cuda")})
    assert e.value.code == _lib.W_INVALID_KEY and e.value.out.bad_row == 617


def test_capacity_is_a_size_query(enc):
    rows = [(b"key%03d" % i, b"value%03d" % i) for i in range(200)]
    r = okv.pack_rows(rows)
    dev = {k: torch.from_numpy(v.astype(v.dtype)).cuda() for k, v in r.items()}
    for k in ("key_off", "val_off"):
        dev[k] = dev[k].view(torch.int64)
    with pytest.raises(okv.OkvError) as e:
        enc.encode_device(dev, 200, {"seg": torch.empty(16, dtype=torch.uint8, device="cuda")})
    o = e.value.out
    assert e.value.code == _lib.OKV_E_CAPACITY
    assert (o.n_blocks, o.data_bytes, o.file_bytes) == (2, 8192, 8340)


def _device_rows_from_decode(decoder, seg, descs):
    """Decode a segment on the GPU and hand its SoA straight to the encoder."""
    nblk = descs.shape[0]
    seg_t = torch.from_numpy(seg.copy()).cuda()
    d_t = torch.from_numpy(descs.astype(np.uint64).view(np.int64)).cuda()
    rows, kb, vb = decoder.plan_device(seg_t, seg.size, d_t, nblk)
    out = dict(row_start=torch.empty(nblk + 1, dtype=torch.int64, device="cuda"),
               key_base=torch.empty(nblk, dtype=torch.int64, device="cuda"),
               val_base=torch.empty(nblk, dtype=torch.int64, device="cuda"),
               status=torch.empty(nblk, dtype=torch.int32, device="cuda"),
               key_off=torch.empty(rows, dtype=torch.int64, device="cuda"),
               key_len=torch.empty(rows, dtype=torch.int16, device="cuda"),
               val_off=torch.empty(rows, dtype=torch.int64, device="cuda"),
               val_len=torch.empty(rows, dtype=torch.int32, device="cuda"),
               key_arena=torch.empty(max(kb, 16), dtype=torch.uint8, device="cuda"),
               val_arena=torch.empty(max(vb, 16), dtype=torch.uint8, device="cuda"))
    decoder.decode_device(seg_t, seg.size, d_t, nblk, out)
    return out, rows


@pytest.mark.parametrize("kind,th,bs", [(okv.sst.SYNTH_ZIPF, 57344, 65536),
                                        (okv.sst.SYNTH_FIXED, 3584, 4096)])
def test_decode_encode_round_trip(enc, decoder, kind, th, bs):
    """Size-independent property (the compaction shape): GPU decode of a whole
    segment -> GPU encode of its rows reproduces the segment file exactly."""
    w = okv.synth_segment(kind, 5, nrows=30000 if kind else 100000, threshold=th,
                          block_size=bs)
    seg = w.data()
    descs = w.descs()
    out, n = _device_rows_from_decode(decoder, seg, descs)
    seg_t = torch.zeros(seg.size + 4096, dtype=torch.uint8, device="cuda")
    desc_t = torch.empty((descs.shape[0], 4), dtype=torch.int64, device="cuda")
    hash_t = torch.empty(descs.shape[0], dtype=torch.int64, device="cuda")
    eo = enc.encode_device(out, n, {"seg": seg_t, "desc": desc_t, "hash": hash_t},
                           threshold=th, block_size=bs, strict_go=False)
    assert eo.file_bytes == seg.size
    assert seg_t[:seg.size].cpu().numpy().tobytes() == seg.tobytes()
    assert np.array_equal(desc_t.cpu().numpy().view(np.uint64), descs)
    want_h = np.array([b[2] for b in w.blocks()], np.uint64)
    assert np.array_equal(hash_t.cpu().numpy().view(np.uint64), want_h)


def test_synth_rows_fixed_device(enc):
    n, first = 1000, 5000
    t = dict(key_arena=torch.empty(n * 16, dtype=torch.uint8, device="cuda"),
             key_off=torch.empty(n, dtype=torch.int64, device="cuda"),
             key_len=torch.empty(n, dtype=torch.int16, device="cuda"),
             val_arena=torch.empty(n * 64, dtype=torch.uint8, device="cuda"),
             val_off=torch.empty(n, dtype=torch.int64, device="cuda"),
             val_len=torch.empty(n, dtype=torch.int32, device="cuda"))
    enc.synth_fixed_device(1, first, n, 16, 64, t)
    want = list(P.rows_fixed(first + n, 1))[first:]
    ka, va = t["key_arena"].cpu().numpy().tobytes(), t["val_arena"].cpu().numpy().tobytes()
    for i, (k, v) in enumerate(want):
        assert ka[16 * i:16 * i + 16] == k and va[64 * i:64 * i + 64] == v


def test_c4_shape_property(enc, decoder):
    """C4 shape at 2 M rows (16 B keys, 64 B values): the first blocks equal
    the oracle writer's, every block re-decodes to its input rows, block
    hashes verify, and the metadata parses back to the same index."""
    n = 2_000_000
    t = dict(key_arena=torch.empty(n * 16, dtype=torch.uint8, device="cuda"),
             key_off=torch.empty(n, dtype=torch.int64, device="cuda"),
             key_len=torch.empty(n, dtype=torch.int16, device="cuda"),
             val_arena=torch.empty(n * 64, dtype=torch.uint8, device="cuda"),
             val_off=torch.empty(n, dtype=torch.int64, device="cuda"),
             val_len=torch.empty(n, dtype=torch.int32, device="cuda"))
    enc.synth_fixed_device(1, 0, n, 16, 64, t)
    nb = -(-n // 42)
    seg_t = torch.zeros(nb * 4096 + nb * 70 + 4096, dtype=torch.uint8, device="cuda")
    desc_t = torch.empty((nb, 4), dtype=torch.int64, device="cuda")
    eo = enc.encode_device(t, n, {"seg": seg_t, "desc": desc_t}, strict_go=False)
    assert eo.n_blocks == nb and eo.data_bytes == nb * 4096
    seg = seg_t[:eo.file_bytes].cpu().numpy()
    # oracle writer over the first 42*3 + 5 rows: identical first 3 blocks
    rc, want, _ = oracle_segment(list(P.rows_fixed(42 * 3 + 5, 1)))
    assert rc == 0 and seg[:3 * 4096].tobytes() == want[:3 * 4096]
    md = okv.fetch_metadata(seg, eo.file_bytes)
    assert np.array_equal(md.descs, desc_t.cpu().numpy().view(np.uint64))
    assert md.first_key == bytes(16) and md.last_key == (n - 1).to_bytes(16, "big")
    dec = decoder.decode(seg, md.descs)
    assert int(dec.status.max()) == 0 and dec.key_len.size == n
    assert np.array_equal(dec.key_arena.reshape(-1, 16)[:n], t["key_arena"].cpu().numpy()
                          .reshape(-1, 16))
    assert np.array_equal(dec.val_arena.reshape(-1, 64)[:n], t["val_arena"].cpu().numpy()
                          .reshape(-1, 64))
    h = decoder.hash_blocks(seg, md.descs)
    assert np.array_equal(h, md.hashes)


def test_general_pack_path_vs_oracle(enc):
    """Blocks over 64 KiB (a 150 KB value) and blocks of > 512 rows (7-byte
    records under a 57 344-byte threshold) take the per-block pack kernel."""
    rng = random.Random(11)
    big = [(b"b%06d" % i, bytes(rng.getrandbits(8) for _ in range(150_000 if i % 5 == 2 else 40)))
           for i in range(12)]
    tiny = [(b"%c" % (33 + (i % 90)), b"") for i in range(20_000)]
    for rows, T, D in ((big, 3584, 4096), (tiny, 57344, 65536), (big + tiny, 57344, 4096)):
        rc, want, _ = oracle_segment(rows, T, D)
        if rc:
            continue
        got = enc.encode(rows, T, D)
        assert got.seg.tobytes() == want


def test_c1_round_trip(enc, decoder):
    """BASELINE.json configs[0] (C1): 10 000 rows of 16 B key / 64 B value
    written with the GPU SegmentWriter and read back in full through the
    GPU-backed RowIter; bytes equal the oracle writer's, 239 blocks
    (238 x 42 rows + 4), every row returned in order."""
    from objectkv_amd import reader as R
    rows = list(P.rows_fixed(10_000, seed=1))
    w = okv.GpuSegmentWriter(enc)
    for k, v in rows:
        w.WriteRow(k, v)
    flen, meta = w.Close()
    rc, want, want_meta = oracle_segment(rows)
    assert rc == 0 and w.data().tobytes() == want and meta == want_meta
    assert flen == len(want) and w.result.n_blocks == 239
    r = R.SegmentReader(w.data().tobytes(), flen, decoder)
    it = r.RowIter(R.DirectionAscending)
    got = []
    while True:
        try:
            kv = it.Next()
        except R.GoError as e:
            assert e.kind == "EOF"
            break
        got.append((kv.Key, kv.Value))
    assert got == rows


def test_bloom_pass_through(enc, decoder):
    """DefaultSegmentWriterOptions' bloom filter (segment_writer_option.go:20):
    the caller's WriteTo bytes land in the meta block as [1][u64 len][bytes]
    (segment_writer.go:295-300) through every product writer -- the host C++
    writer, the GPU encoder on host buffers and on device tensors -- byte for
    byte as the oracle writer writes them; the segment decodes and its
    metadata parses past the filter."""
    from oracle.bloom_ref import default_filter
    rng = random.Random(3)
    rows = sorted(_random_rows(rng, 3000, 40, 300))
    f = default_filter()
    for k, _v in rows:
        f.add(k)
    bb = f.to_bytes()
    w = CO.Writer()
    for k, v in rows:
        assert w.write_row(k, v) == 0
    w.set_bloom(bb)
    rc, want, want_meta = w.close()
    assert rc == 0
    # host C++ writer (the filter object is the caller's: add per row)
    hw = okv.SegmentWriter(bloom=default_filter())
    for k, v in rows:
        hw.WriteRow(k, v)
    flen, meta = hw.Close()
    assert hw.data().tobytes() == want and meta == want_meta
    # GPU encoder, host buffers
    got = enc.encode(rows, bloom=bb)
    assert got.seg.tobytes() == want and got.meta() == want_meta
    # GPU encoder, device tensors (the bench path) + Close's meta hash / trailer
    r = okv.sst.pack_rows(rows)
    t = {k: torch.from_numpy((v.view(np.int64) if v.dtype == np.uint64 else
                              v.view(np.int16) if v.dtype == np.uint16 else
                              v.view(np.int32) if v.dtype == np.uint32 else v).copy()).to("cuda")
         for k, v in r.items()}
    seg_t = torch.zeros(len(want) + 4096, dtype=torch.uint8, device="cuda")
    eo = enc.encode_device(t, len(rows), {"seg": seg_t}, bloom=bb,
                           key_arena_bytes=r["key_arena"].size,
                           val_arena_bytes=r["val_arena"].size)
    assert eo.file_bytes == len(want)
    assert seg_t[:eo.file_bytes].cpu().numpy().tobytes() == want
    md = okv.fetch_metadata(want, len(want))
    dec = decoder.decode(want, md.descs)
    assert [(k, v or b"") for b in range(md.descs.shape[0]) for k, v in dec.block_rows(b)] == \
        [(k, v) for k, v in rows]


@pytest.mark.parametrize("T,vmax", [(50, 60), (3584, 120), (9000, 60), (20000, 12), (3584, 3000)])
def test_multi_chunk_encode(enc, T, vmax):
    """Segments of 9 000 - 30 000 rows (5 - 15 scan tiles of 2 048 rows; blocks
    of 1 - 700+ rows) through the product plan (E1-E9, pointer doubling over
    chunks): byte-equal to the oracle writer, and a second encode reusing the
    context's buffers byte-equal to the first.  (The single-pass plan kernel is
    an ablation arm: OKV_PATH_ENC_ONEPASS never set by the product.)"""
    rng = random.Random(T + vmax)
    n = 30000 if vmax <= 120 else 9000
    rows = _random_rows(rng, n, 8, vmax)
    rc, want, meta = oracle_segment(rows, T, 4096)
    strict = rc == 0
    got = enc.encode(rows, T, 4096, strict_go=strict)
    if strict:
        assert got.seg.tobytes() == want and got.meta() == meta
    else:  # the last row closed a block (Q1): compare with the host writer's footer
        hw = okv.SegmentWriter(T, 4096, 0, False)
        for k, v in rows:
            hw.WriteRow(k, v)
        hw.Close(strict_go=False)
        assert got.seg.tobytes() == hw.data().tobytes()
    assert not enc.last_path() & _lib.PATH_ENC_ONEPASS
    # a second encode reuses the context's buffers
    got2 = enc.encode(rows, T, 4096, strict_go=strict)
    assert got2.seg.tobytes() == got.seg.tobytes()


@pytest.mark.parametrize("T", [14, 40, 3584, 5000])
def test_tile_cut_uniform_tiles(enc, T):
    """Tiles whose blocks all hold one row count (fixed 20-byte records: 1,
    2, 180 and 250 rows per block): the cut kernel's arithmetic chains and the
    emit kernel's speculated walk, beside a variable-size stretch (the walks)
    and a short last block -- byte-equal to the oracle writer."""
    rng = random.Random(T)
    rows = [(b"%08d" % i, bytes([i & 255]) * (rng.randint(0, 12) if 12000 <= i < 13000 else 6))
            for i in range(30001)]
    rc, want, meta = oracle_segment(rows, T, 4096)
    got = enc.encode(rows, T, 4096, strict_go=rc == 0)
    if rc == 0:
        assert got.seg.tobytes() == want
        assert got.meta() == meta
    else:  # the last row closed a block (Q1): compare with the host writer's footer
        hw = okv.SegmentWriter(T, 4096, 0, False)
        for k, v in rows:
            hw.WriteRow(k, v)
        hw.Close(strict_go=False)
        assert got.seg.tobytes() == hw.data().tobytes()


@pytest.mark.parametrize("T", [60, 3584, 4400, 5200, 20000])
def test_tile_cut_boundaries_and_general_path(enc, T):
    """The greedy cut across many 2048-row tiles (okv_enc_cut_kernel /
    okv_enc_emit_tile_kernel): small records so blocks hold ~4, ~200, ~250,
    ~290 (past the 256-row lookahead: the general kernels) and ~1 300 rows
    -- every segment byte-equal to the oracle writer."""
    rng = random.Random(T)
    rows = [(b"%08d" % i, bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 8))))
            for i in range(20000)]
    rc, want, meta = oracle_segment(rows, T, 4096)
    got = enc.encode(rows, T, 4096, strict_go=rc == 0)
    if rc == 0:
        assert got.seg.tobytes() == want
        assert got.meta() == meta
