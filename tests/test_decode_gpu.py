"""GPU parity: the HIP decode (libokv_sst.so through the C-ABI) against the
CPU oracle (oracle/) and the committed golden vectors.  Integer/byte work:
every comparison is bit-exact."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import objectkv_amd as okv
from objectkv_amd import _lib
from oracle import coracle as CO
from tests.conftest import descs_of, rowval, unpack

pytestmark = pytest.mark.gpu

SOA = ("row_start", "key_off", "key_len", "val_off", "val_len")


def _assert_same_as_oracle(got: okv.Decoded, seg, descs, comp, index_only):
    ref = CO.decode_soa(seg, CO.descs_array([tuple(int(x) for x in d) for d in descs]), comp,
                        index_only)
    assert np.array_equal(got.status, ref["status"])
    for k in SOA:
        assert np.array_equal(getattr(got, k), ref[k]), k
    if not index_only:
        assert np.array_equal(got.key_base, ref["key_base"])
        assert np.array_equal(got.val_base, ref["val_base"])
        assert got.key_arena.tobytes() == ref["key_arena"].tobytes()
        assert got.val_arena.tobytes() == ref["val_arena"].tobytes()
    return ref


@pytest.mark.parametrize("index_only", [False, True])
def test_golden_writer_cases(decoder, golden, index_only):
    """Reference test segments (segment_reader_test.go inputs) decode to the
    golden rows, including the nil value of TestReadBlankRecordUncompressed."""
    for name, case in golden.items():
        if case["kind"] != "writer":
            continue
        seg = np.frombuffer(unpack(case["segment_z"]), np.uint8)
        d = descs_of(case)
        got = decoder.decode(seg, d, case["compression"], index_only=index_only)
        for b, blk in enumerate(case["blocks"]):
            assert got.status[b] == blk["status"], (name, b)
            rows = got.block_rows(b)
            assert [[rowval(k), rowval(v)] for k, v in rows] == blk["rows"], (name, b)
        _assert_same_as_oracle(got, seg, d, case["compression"], index_only)


def test_reference_known_answers_on_gpu(decoder, golden):
    """TestReadUncompressed's asserted rows, straight from the HIP decode."""
    case = golden["ref_read_uncompressed_200"]
    got = decoder.decode(unpack(case["segment_z"]), descs_of(case))
    r0, r1 = got.block_rows(0), got.block_rows(1)
    assert len(r0) + len(r1) == 200
    assert r0[0] == (b"key000", b"value000") and r1[0] == (b"key180", b"value180")
    assert r1[-1] == (b"key199", b"value199")
    blank = golden["ref_blank_value"]
    got = decoder.decode(unpack(blank["segment_z"]), descs_of(blank))
    assert got.block_rows(1)[-1] == (b"key200", None)  # nil value (Q4)


@pytest.mark.parametrize("comp", [_lib.COMP_NONE, _lib.COMP_LZ4])
@pytest.mark.parametrize("index_only", [False, True])
def test_crafted_edges(decoder, golden, comp, index_only):
    """Overrun panics, short reads, EOF, OriginalSize 0, records past
    OriginalSize, nil keys/values, u16-max key, >64 KiB block (HBM path),
    600-row block (several row-table batches), unaligned offset, LZ4 flag."""
    case = golden["crafted_edges"]
    seg = unpack(case["segment_z"])
    d = descs_of(case)
    got = decoder.decode(seg, d, comp, index_only=index_only)
    for b, blk in enumerate(case["blocks"]):
        want_st = blk["status"] if comp == _lib.COMP_NONE else blk["status_lz4"]
        want_rows = blk["rows"] if comp == _lib.COMP_NONE else blk["rows_lz4"]
        assert got.status[b] == want_st, (b, blk["note"])
        assert [[rowval(k), rowval(v)] for k, v in got.block_rows(b)] == want_rows, blk["note"]
    _assert_same_as_oracle(got, seg, d, comp, index_only)


def _digests(got: okv.Decoded, index_only):
    dig = {"row_start": got.row_start, "status": got.status, "key_off": got.key_off,
           "key_len": got.key_len, "val_off": got.val_off, "val_len": got.val_len}
    if not index_only:
        dig.update(key_base=got.key_base, val_base=got.val_base, key_arena=got.key_arena,
                   val_arena=got.val_arena)
    return {k: hashlib.sha256(v.tobytes()).hexdigest() for k, v in dig.items()}


@pytest.mark.parametrize("name", ["c2_fixed_256x4k", "c3_zipf_8x64k"])
@pytest.mark.parametrize("index_only", [False, True])
def test_golden_synthetic_configs(decoder, golden, name, index_only):
    """C2 (256 x 4 KiB, 16/64) and a C3-shaped sample (8 x 64 KiB Zipf):
    SHA-256 of every output array equals the golden digest."""
    c = golden[name]
    kind = okv.sst.SYNTH_FIXED if c["gen"] == "fixed" else okv.sst.SYNTH_ZIPF
    w = okv.synth_segment(kind, c["seed"], nblocks=c["nblocks"], threshold=c["threshold"],
                          block_size=c["block_size"])
    seg = w.data()
    assert hashlib.sha256(seg.tobytes()).hexdigest() == c["segment_sha256"]
    d = w.descs()[:c["decode_blocks"]]
    got = decoder.decode(seg, d, index_only=index_only)
    want = c["index" if index_only else "full"]
    dig = _digests(got, index_only)
    for k, v in dig.items():
        assert v == want[k], k
    assert int(got.row_start[-1]) == want["n_rows"]


def test_c3_scale_against_c_oracle(decoder):
    """A larger C3-shaped segment (512 x 64 KiB) against the C oracle,
    plus size-independent properties."""
    w = okv.synth_segment(okv.sst.SYNTH_ZIPF, 3, nblocks=512, threshold=57344, block_size=65536)
    seg = w.data()
    d = w.descs()[:512]
    got = decoder.decode(seg, d)
    ref = _assert_same_as_oracle(got, seg, d, 0, False)
    n = int(got.row_start[-1])
    assert n == int(ref["row_start"][-1]) and n > 512 * 20
    # property: re-encoding the decoded rows reproduces the segment bytes
    w2 = okv.SegmentWriter(57344, 65536)
    for b in range(512):
        for k, v in got.block_rows(b):
            w2.WriteRow(k or b"", v or b"")
    w2.Close(strict_go=False)
    assert w2.data().tobytes()[:int(d[-1][0] + d[-1][1])] == \
        seg.tobytes()[:int(d[-1][0] + d[-1][1])]


def test_hash_blocks_matches_writer(decoder, golden):
    """Device XXH64 of each block == BlockStat.Hash written by the writer
    (segment_writer.go:185)."""
    for name in ("ref_read_uncompressed_200", "ref_larger_than_block"):
        case = golden[name]
        h = decoder.hash_blocks(unpack(case["segment_z"]), descs_of(case))
        assert h.tolist() == [b["hash"] for b in case["blocks"]]
    w = okv.synth_segment(okv.sst.SYNTH_ZIPF, 3, nblocks=64, threshold=57344, block_size=65536)
    h = decoder.hash_blocks(w.data(), w.descs())
    assert h.tolist() == [b[2] for b in w.blocks()]


def test_capacity_error_reports_totals(decoder, golden):
    case = golden["ref_read_uncompressed_200"]
    seg = np.frombuffer(unpack(case["segment_z"]), np.uint8)
    d = descs_of(case)
    rows, kb, vb = decoder.plan(seg, d)
    # keys 6 B, values 8 B; per-block regions padded to 16 B: 1080->1088 + 120->128, 1440 + 160
    assert (rows, kb, vb) == (200, 1216, 1600)
    o = {k: np.zeros(n, t) for k, n, t in [("row_start", 3, np.uint64),
                                           ("status", 2, np.int32)]}
    small = _lib.DecodeOut(o["row_start"].ctypes.data, None, None, o["status"].ctypes.data,
                           None, None, None, None, None, None, 0, 0, 0, 0, 0, 0, 0)
    import ctypes as C
    rc = _lib.lib().okv_decode_blocks(decoder._ctx, seg.ctypes.data, seg.size, d.ctypes.data,
                                      2, 0, C.byref(small), 0)
    assert rc == _lib.OKV_E_CAPACITY and small.n_rows == 200


def test_device_pointer_api_torch(decoder):
    """Device-resident mode (the bench path): torch tensors in HBM, async
    enqueue, totals after sync."""
    torch = pytest.importorskip("torch")
    w = okv.synth_segment(okv.sst.SYNTH_ZIPF, 3, nblocks=32, threshold=57344, block_size=65536)
    seg = w.data()
    d = w.descs()[:32]
    dev = torch.device("cuda", 0)
    seg_t = torch.from_numpy(seg).to(dev)
    d_t = torch.from_numpy(d.view(np.int64)).to(dev)
    rows, kb, vb = decoder.plan_device(seg_t, seg.size, d_t, 32)
    out = dict(row_start=torch.zeros(33, dtype=torch.int64, device=dev),
               key_base=torch.zeros(32, dtype=torch.int64, device=dev),
               val_base=torch.zeros(32, dtype=torch.int64, device=dev),
               status=torch.zeros(32, dtype=torch.int32, device=dev),
               key_off=torch.zeros(rows, dtype=torch.int64, device=dev),
               key_len=torch.zeros(rows, dtype=torch.int16, device=dev),
               val_off=torch.zeros(rows, dtype=torch.int64, device=dev),
               val_len=torch.zeros(rows, dtype=torch.int32, device=dev),
               key_arena=torch.zeros(kb, dtype=torch.uint8, device=dev),
               val_arena=torch.zeros(vb, dtype=torch.uint8, device=dev))
    decoder.decode_device(seg_t, seg.size, d_t, 32, out, sync=False)
    decoder.sync()
    host = decoder.decode(seg, d)
    assert np.array_equal(out["row_start"].cpu().numpy().view(np.uint64), host.row_start)
    assert np.array_equal(out["val_len"].cpu().numpy().view(np.uint32), host.val_len)
    assert out["val_arena"].cpu().numpy().tobytes() == host.val_arena.tobytes()
    assert out["key_arena"].cpu().numpy().tobytes() == host.key_arena.tobytes()


def test_bimodal_blocks_with_plan_span(decoder):
    """Alternating 4 KiB / 60 KiB blocks (average 32 KiB): okv_decode_plan
    measures the longest walk and the tile pass of the same batch sizes its
    tiles per block from it (no block left to okv_copy_kernel).  Device-pointer
    decode after the plan == host-mode decode == oracle."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(77)
    parts, descs, off = [], [], 0
    for i in range(1200):
        target = 4096 if i % 2 == 0 else 61440
        body = bytearray()
        while len(body) < target - 3100:
            vl = int(rng.integers(1000, 3000))
            body += (16).to_bytes(2, "little") + vl.to_bytes(4, "little")
            body += rng.integers(0, 256, 16 + vl, dtype=np.uint8).tobytes()
        bsize = (len(body) // 4096 + 1) * 4096
        parts.append(bytes(body) + bytes(bsize - len(body)))
        descs.append((off, bsize, len(body), 0))
        off += bsize
    seg = np.frombuffer(b"".join(parts) + bytes(4096), np.uint8)
    d = np.array(descs, np.uint64)
    n = d.shape[0]
    dev = torch.device("cuda", 0)
    seg_t = torch.from_numpy(seg.copy()).to(dev)
    d_t = torch.from_numpy(d.view(np.int64).copy()).to(dev)
    rows, kb, vb = decoder.plan_device(seg_t, seg.size, d_t, n)
    out = {k: torch.zeros(m, dtype=t, device=dev) for k, m, t in [
        ("row_start", n + 1, torch.int64), ("key_base", n, torch.int64),
        ("val_base", n, torch.int64), ("status", n, torch.int32),
        ("key_off", rows, torch.int64), ("key_len", rows, torch.int16),
        ("val_off", rows, torch.int64), ("val_len", rows, torch.int32),
        ("key_arena", kb, torch.uint8), ("val_arena", vb, torch.uint8)]}
    decoder.decode_device(seg_t, seg.size, d_t, n, out, sync=True)
    assert decoder.last_path() & _lib.PATH_TILE
    host = decoder.decode(seg.tobytes(), d)
    _assert_same_as_oracle(host, seg.tobytes(), d, 0, False)
    assert np.array_equal(out["row_start"].cpu().numpy().view(np.uint64), host.row_start)
    assert np.array_equal(out["val_off"].cpu().numpy().view(np.uint64), host.val_off)
    assert out["val_arena"].cpu().numpy().tobytes() == host.val_arena.tobytes()
    assert out["key_arena"].cpu().numpy().tobytes() == host.key_arena.tobytes()


def test_random_fuzz_against_c_oracle(decoder):
    """Random record streams with truncation/corruption/odd offsets."""
    rng = np.random.default_rng(2024)
    for trial in range(25):
        seg = bytearray()
        descs = []
        for b in range(int(rng.integers(1, 40))):
            body = bytearray()
            for _ in range(int(rng.integers(0, 30))):
                kl = int(rng.choice([0, 1, 5, 16, 100, 300]))
                vl = int(rng.choice([0, 1, 7, 64, 500, 3000]))
                body += kl.to_bytes(2, "little") + vl.to_bytes(4, "little")
                body += rng.integers(0, 256, kl + vl, dtype=np.uint8).tobytes()
            orig = len(body)
            if rng.random() < 0.3 and body:
                orig = int(rng.integers(0, len(body) + 1))
            if rng.random() < 0.2 and len(body) > 3:
                body[int(rng.integers(0, len(body)))] = int(rng.integers(0, 256))
            bsize = len(body) + int(rng.choice([0, 1, 5, 64, 4096]))
            off = len(seg) + int(rng.choice([0, 0, 1, 3, 8]))
            seg += bytes(off - len(seg))
            seg += body + bytes(bsize - len(body))
            descs.append((off, bsize, orig, 0))
        d = np.array(descs, np.uint64).reshape(-1, 4)
        comp = int(rng.choice([0, 0, 2]))
        for index_only in (False, True):
            got = decoder.decode(bytes(seg), d, comp, index_only=index_only)
            _assert_same_as_oracle(got, bytes(seg), d, comp, index_only)


def test_empty_batch(decoder):
    got = decoder.decode(b"\x00" * 32, np.zeros((0, 4), np.uint64))
    assert got.row_start.tolist() == [0]


def _mixed_segment(kinds, seed):
    """Raw record blocks of mixed shapes, back to back at 16-byte offsets:
    's' 4 KiB with 42 rows of 16/64, 'L' 64 KiB with <= 40 rows of 1-3 KiB
    values, 'M' more than kRCap (64) rows (staged path, okv_copy_kernel)."""
    rng = np.random.default_rng(seed)
    seg, descs = bytearray(), []
    for kind in kinds:
        body = bytearray()
        if kind == "s":
            shape = [(16, 64)] * 42
        elif kind == "L":
            shape = [(int(rng.integers(8, 257)), int(rng.integers(1000, 3000)))
                     for _ in range(int(rng.integers(5, 28)))]
        else:
            shape = [(int(rng.integers(1, 20)), int(rng.integers(0, 40)))
                     for _ in range(int(rng.integers(65, 300)))]
        for kl, vl in shape:
            body += kl.to_bytes(2, "little") + vl.to_bytes(4, "little")
            body += rng.integers(0, 256, kl + vl, dtype=np.uint8).tobytes()
        bsize = (len(body) // 4096 + 1) * 4096
        off = len(seg)
        seg += body + bytes(bsize - len(body))
        descs.append((off, bsize, len(body), 0))
    return bytes(seg), np.array(descs, np.uint64).reshape(-1, 4)


@pytest.fixture(scope="module")
def nofused_decoder():
    """A context opened with OKV_OPEN_NO_FUSED (and NO_POINT): small batches
    of small blocks take the three-launch path (count, scan,
    okv_gather_small_kernel)."""
    dec = okv.Decoder(0, flags=_lib.OPEN_NO_FUSED | _lib.OPEN_NO_POINT)
    yield dec
    dec.close()


@pytest.fixture(scope="module")
def nopoint_decoder():
    """A context opened with OKV_OPEN_NO_POINT: host-mode calls of a few small
    blocks are staged to device memory (the fused / tile kernels) instead of
    taking the point path."""
    dec = okv.Decoder(0, flags=_lib.OPEN_NO_POINT)
    yield dec
    dec.close()


# The shipping decode paths.  Which kernels run follows from the call: a
# host-mode call of <= 16 small uncompressed blocks takes the point path
# (okv_point_kernel) unless the context was opened with NO_POINT; otherwise
# the average block span (segment bytes / blocks) picks the small-block
# kernels (<= 16 KiB) or the large-block tile pass; <= 512 small blocks run
# the single-pass fused kernel unless the context was opened with NO_FUSED;
# big blocks (> 64 rows, or past the tile span) go to okv_copy_kernel on either.
PATHS = ["as_given", "fused", "nofused", "large"]


def decode_path(path, decoder, nofused, seg, d, nopoint=None, **kw):
    """Decode (seg, d) through one shipping path; returns (decoded, seg used).
    "as_given": the default context (the point path when the call is
    eligible); "fused": a NO_POINT context; "large": the segment buffer
    padded with zeros so the blocks average more than 16 KiB (a caller
    decoding some blocks of a larger segment), NO_POINT -- every block goes
    through the large-block pass."""
    seg = bytes(seg)
    if path == "large":
        n = max(1, d.shape[0])
        seg = seg + bytes(max(0, 16385 * n - len(seg)) + 4096)
    if path in ("fused", "large"):
        assert nopoint is not None
        dec = nopoint
    else:
        dec = nofused if path == "nofused" else decoder
    got = dec.decode(seg, d, **kw)
    lp = dec.last_path()
    if d.shape[0]:
        if path != "as_given":
            assert not lp & _lib.PATH_POINT, lp
        if path == "nofused":
            assert not lp & _lib.PATH_FUSED, lp
        if path == "large":
            # the large-block pass ran (not the small-block kernels)
            assert not lp & (_lib.PATH_FUSED | _lib.PATH_SMALL), lp
            if not kw.get("index_only"):
                assert lp & (_lib.PATH_TILE | _lib.PATH_SWEEP), lp
    return got, seg


def _wide_segment(seed, nblk=120):
    """Large blocks whose value tiles span far more source than values:
    'W' up to 64 rows of 200-256 B keys and 0-40 B values (a 1 KiB value tile
    spans > 6 KiB of records: global-window fallback), 'V' 200 B keys with
    300-600 B values (a 5-tile span overflows the stage: one-tile retry),
    'L' 1-3 KiB values.  The first block sits at offset 0 (the stage's
    16-byte lead-in would start before the segment), the others at odd
    offsets, and the last block ends at the segment's last byte."""
    rng = np.random.default_rng(seed)
    seg, descs = bytearray(), []
    for b in range(nblk):
        kind = rng.choice(["W", "V", "L"])
        if kind == "W":
            shape = [(int(rng.integers(200, 257)), int(rng.integers(0, 41)))
                     for _ in range(int(rng.integers(40, 65)))]
        elif kind == "V":
            shape = [(200, int(rng.integers(300, 601))) for _ in range(int(rng.integers(30, 64)))]
        else:
            shape = [(int(rng.integers(8, 257)), int(rng.integers(1000, 3000)))
                     for _ in range(int(rng.integers(5, 28)))]
        body = bytearray()
        for kl, vl in shape:
            body += kl.to_bytes(2, "little") + vl.to_bytes(4, "little")
            body += rng.integers(0, 256, kl + vl, dtype=np.uint8).tobytes()
        pad = 0 if b == nblk - 1 else int(rng.choice([0, 1, 3, 8, 13, 4096]))
        off = 0 if b == 0 else len(seg) + int(rng.choice([0, 1, 5, 11]))
        seg += bytes(off - len(seg))
        seg += body + bytes(pad)
        descs.append((off, len(body) + pad, len(body), 0))
    return bytes(seg), np.array(descs, np.uint64).reshape(-1, 4)


@pytest.mark.parametrize("path", PATHS)
def test_wide_spans_all_paths(decoder, nofused_decoder, nopoint_decoder, path):
    """Long keys with tiny values (a value tile spans many records), stage
    overflow, the segment's first and last bytes, odd block offsets: every
    shipping path vs the oracle."""
    for seed in (1, 2):
        seg, d = _wide_segment(seed)
        got, seg2 = decode_path(path, decoder, nofused_decoder, seg, d, nopoint=nopoint_decoder)
        _assert_same_as_oracle(got, seg2, d, 0, False)


@pytest.mark.parametrize("path", PATHS)
def test_mixed_blocks_all_paths(decoder, nofused_decoder, nopoint_decoder, path):
    """A segment mixing 4 KiB blocks, 64 KiB blocks with few rows and blocks
    over kRCap rows, full and index-only, through every shipping path."""
    rng = np.random.default_rng(11)
    kinds = list(rng.choice(["s", "s", "L", "M"], size=300))
    seg, d = _mixed_segment(kinds, 5)
    for index_only in (False, True):
        got, seg2 = decode_path(path, decoder, nofused_decoder, seg, d, index_only=index_only, nopoint=nopoint_decoder)
        _assert_same_as_oracle(got, seg2, d, 0, index_only)


@pytest.mark.parametrize("nblk", [255, 256, 257, 513])
def test_single_tile_and_scan_paths(decoder, nofused_decoder, nopoint_decoder, nblk):
    """<= 256 blocks: pass 1 writes the totals itself (one tile, no scan
    launch, in-kernel big-block counter reset); more: okv_scan_kernel.  Both
    with a block over kRCap rows, through every shipping path, against the
    oracle and each other."""
    kinds = ["s"] * nblk
    kinds[nblk // 2] = "M"
    kinds[-1] = "M"
    seg, d = _mixed_segment(kinds, nblk)
    outs = []
    for path in PATHS:
        got, seg2 = decode_path(path, decoder, nofused_decoder, seg, d, nopoint=nopoint_decoder)
        _assert_same_as_oracle(got, seg2, d, 0, False)
        outs.append(got)
    for got in outs[1:]:
        assert got.val_arena.tobytes() == outs[0].val_arena.tobytes()
    # the same decoder again after a larger call (scratch reuse, counter reset)
    again = decoder.decode(seg, d)
    assert again.val_arena.tobytes() == outs[0].val_arena.tobytes()
    assert np.array_equal(again.row_start, outs[0].row_start)


def _tiny_value_segment(seed, nblk=300):
    """Blocks of <= 64 rows with 0-3 byte values: a 4 KiB value-sweep tile
    holds thousands of rows (past the sweep's LDS row window)."""
    rng = np.random.default_rng(seed)
    seg, descs = bytearray(), []
    for b in range(nblk):
        body = bytearray()
        for _ in range(int(rng.integers(0, 65))):
            kl, vl = int(rng.integers(0, 9)), int(rng.integers(0, 4))
            body += kl.to_bytes(2, "little") + vl.to_bytes(4, "little")
            body += rng.integers(0, 256, kl + vl, dtype=np.uint8).tobytes()
        off = len(seg) + int(rng.choice([0, 1, 7]))
        seg += bytes(off - len(seg)) + body + bytes(int(rng.choice([0, 3, 100])))
        descs.append((off, len(seg) - off, len(body), 0))
    return bytes(seg), np.array(descs, np.uint64).reshape(-1, 4)


@pytest.mark.parametrize("path", PATHS)
def test_tiny_values_fuzz_and_capacity(decoder, nofused_decoder, nopoint_decoder, path):
    """C3 blocks; tiny values (thousands of rows per 4 KiB of values, many
    rows per destination chunk); a fuzz of corrupt / truncated blocks
    (statuses with other blocks' rows around them) -- every shipping path vs
    the oracle.  Then an undersized value arena on the device: the blocks past
    it report OKV_BLK_CAPACITY, the blocks before it match the oracle."""
    w = okv.synth_segment(okv.sst.SYNTH_ZIPF, 7, nblocks=96, threshold=57344, block_size=65536)
    seg, d = w.data(), w.descs()
    got, seg2 = decode_path(path, decoder, nofused_decoder, seg, d, nopoint=nopoint_decoder)
    _assert_same_as_oracle(got, seg2, d, 0, False)
    for seed in (3, 4):
        seg, d = _tiny_value_segment(seed)
        got, seg2 = decode_path(path, decoder, nofused_decoder, seg, d, nopoint=nopoint_decoder)
        _assert_same_as_oracle(got, seg2, d, 0, False)
    rng = np.random.default_rng(77)
    for trial in range(12):
        seg = bytearray()
        descs = []
        for b in range(int(rng.integers(1, 40))):
            body = bytearray()
            for _ in range(int(rng.integers(0, 30))):
                kl = int(rng.choice([0, 1, 5, 16, 100, 300]))
                vl = int(rng.choice([0, 1, 7, 64, 500, 3000, 9000]))
                body += kl.to_bytes(2, "little") + vl.to_bytes(4, "little")
                body += rng.integers(0, 256, kl + vl, dtype=np.uint8).tobytes()
            orig = len(body)
            if rng.random() < 0.3 and body:
                orig = int(rng.integers(0, len(body) + 1))
            if rng.random() < 0.2 and len(body) > 3:
                body[int(rng.integers(0, len(body)))] = int(rng.integers(0, 256))
            bsize = len(body) + int(rng.choice([0, 1, 5, 64, 4096]))
            off = len(seg) + int(rng.choice([0, 0, 1, 3, 8]))
            seg += bytes(off - len(seg))
            seg += body + bytes(bsize - len(body))
            descs.append((off, bsize, orig, 0))
        d = np.array(descs, np.uint64).reshape(-1, 4)
        got, seg2 = decode_path(path, decoder, nofused_decoder, bytes(seg), d, nopoint=nopoint_decoder)
        _assert_same_as_oracle(got, seg2, d, 0, False)
    # device path with an undersized value arena
    import torch
    w = okv.synth_segment(okv.sst.SYNTH_ZIPF, 8, nblocks=64, threshold=57344, block_size=65536)
    seg, d = w.data(), w.descs()[:64]
    dec = nofused_decoder if path == "nofused" else decoder
    ref = dec.decode(seg, d)
    dev = torch.device("cuda", 0)
    seg_t = torch.from_numpy(seg).to(dev)
    d_t = torch.from_numpy(d.view(np.int64)).to(dev)
    rows, kb, vb = dec.plan_device(seg_t, seg.size, d_t, 64)
    out = dict(row_start=torch.zeros(65, dtype=torch.int64, device=dev),
               key_base=torch.zeros(64, dtype=torch.int64, device=dev),
               val_base=torch.zeros(64, dtype=torch.int64, device=dev),
               status=torch.zeros(64, dtype=torch.int32, device=dev),
               key_off=torch.zeros(rows, dtype=torch.int64, device=dev),
               key_len=torch.zeros(rows, dtype=torch.int16, device=dev),
               val_off=torch.zeros(rows, dtype=torch.int64, device=dev),
               val_len=torch.zeros(rows, dtype=torch.int32, device=dev),
               key_arena=torch.zeros(kb, dtype=torch.uint8, device=dev),
               val_arena=torch.zeros(vb // 2, dtype=torch.uint8, device=dev))
    with pytest.raises(Exception):
        dec.decode_device(seg_t, seg.size, d_t, 64, out, sync=True)
    st = out["status"].cpu().numpy()
    assert (st != 0).any() and (st == 0).any()
    arena = out["val_arena"].cpu().numpy()
    vbase = ref.val_base
    for b in range(64):
        if st[b] != 0:
            continue
        lo = int(vbase[b])
        hi = int(vbase[b + 1]) if b + 1 < 64 else vb
        assert arena[lo:hi].tobytes() == ref.val_arena[lo:hi].tobytes()


def test_decode_chain_ring():
    """okv_decode_chain: two decoders chained to each other (each one's pass 3
    after the other's last pass 3) decoding alternate segments on their own
    streams, async; every result == the oracle.  A context cannot chain to
    itself."""
    import torch
    a, b = okv.Decoder(0), okv.Decoder(0)
    try:
        with pytest.raises(Exception):
            a.chain(a)
        a.chain(b)
        b.chain(a)
        dev = torch.device("cuda", 0)
        cases = []
        for seed in (5, 6):
            w = okv.synth_segment(okv.sst.SYNTH_ZIPF, seed, nblocks=384, threshold=57344,
                                  block_size=65536)
            seg, d = w.data(), w.descs()[:384]
            seg_t = torch.from_numpy(seg).to(dev)
            d_t = torch.from_numpy(d.view(np.int64).copy()).to(dev)
            rows, kb, vb = a.plan_device(seg_t, seg.size, d_t, 384)
            cases.append((seg, d, seg_t, d_t, rows, kb, vb))
        outs = []
        for i in range(6):
            dec = (a, b)[i % 2]
            seg, d, seg_t, d_t, rows, kb, vb = cases[i % 2]
            out = dict(row_start=torch.zeros(385, dtype=torch.int64, device=dev),
                       key_base=torch.zeros(384, dtype=torch.int64, device=dev),
                       val_base=torch.zeros(384, dtype=torch.int64, device=dev),
                       status=torch.zeros(384, dtype=torch.int32, device=dev),
                       key_off=torch.zeros(rows, dtype=torch.int64, device=dev),
                       key_len=torch.zeros(rows, dtype=torch.int16, device=dev),
                       val_off=torch.zeros(rows, dtype=torch.int64, device=dev),
                       val_len=torch.zeros(rows, dtype=torch.int32, device=dev),
                       key_arena=torch.zeros(kb, dtype=torch.uint8, device=dev),
                       val_arena=torch.zeros(vb, dtype=torch.uint8, device=dev))
            dec.decode_device(seg_t, seg.size, d_t, 384, out, sync=False)
            outs.append((i % 2, out))
        torch.cuda.synchronize()
        for k, out in outs:
            seg, d = cases[k][0], cases[k][1]
            ref = CO.decode_soa(seg, CO.descs_array([tuple(int(x) for x in r)
                                                     for r in d]))
            for f, rk in (("status", "status"), ("row_start", "row_start"),
                          ("key_len", "key_len"), ("val_len", "val_len")):
                got = out[f].cpu().numpy()
                assert np.array_equal(got.view(ref[rk].dtype) if got.dtype != ref[rk].dtype
                                      else got, ref[rk]), f
            assert out["key_arena"].cpu().numpy().tobytes() == ref["key_arena"].tobytes()
            assert out["val_arena"].cpu().numpy().tobytes() == ref["val_arena"].tobytes()
        a.chain(None)
        b.chain(None)
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("index_only", [False, True])
def test_large_batch_with_big_blocks(decoder, index_only):
    """9 000 large blocks through the tile pass with blocks over kRCap rows at
    both ends, in the middle and around tile-count boundaries (the big-block
    list, okv_copy_kernel): equal to the oracle."""
    n = 9000
    kinds = ["L"] * n
    for i in (0, 3, 1023, 1024, 1025, 4000, n - 1):
        kinds[i] = "M"
    seg, d = _mixed_segment(kinds, 21)
    seg = seg + bytes(4096)
    a = decoder.decode(seg, d, index_only=index_only)
    assert decoder.last_path() & _lib.PATH_BIG
    _assert_same_as_oracle(a, seg, d, 0, index_only)


def test_large_batches_of_small_blocks(decoder, nofused_decoder, golden):
    """More than 512 small blocks: passes 1-3 as three launches (count, scan,
    staged gather) -- 3 000 mixed blocks (4 KiB, over-kRCap blocks for
    okv_copy_kernel), and the crafted edge blocks repeated past 512 -- equal
    to the oracle and to the OKV_OPEN_NO_FUSED context."""
    rng = np.random.default_rng(5)
    kinds = list(rng.choice(["s"] * 12 + ["M"], size=3000))
    seg, d = _mixed_segment(kinds, 8)
    for index_only in (False, True):
        got = decoder.decode(seg, d, index_only=index_only)
        assert decoder.last_path() & (_lib.PATH_SMALL | _lib.PATH_GATHER)
        assert not decoder.last_path() & (_lib.PATH_STREAM | _lib.PATH_FUSED)
        _assert_same_as_oracle(got, seg, d, 0, index_only)
        ref = nofused_decoder.decode(seg, d, index_only=index_only)
        for k in ("status", "row_start", "key_off", "key_len", "val_off", "val_len"):
            assert np.array_equal(getattr(got, k), getattr(ref, k)), k
        if not index_only:
            assert got.val_arena.tobytes() == ref.val_arena.tobytes()
    case = golden["crafted_edges"]
    cseg = unpack(case["segment_z"])
    cd = np.tile(descs_of(case), (60, 1))
    for comp in (_lib.COMP_NONE, _lib.COMP_LZ4):
        got = decoder.decode(cseg, cd, comp)
        assert not decoder.last_path() & (_lib.PATH_STREAM | _lib.PATH_FUSED)
        want = [b["status"] if comp == _lib.COMP_NONE else b["status_lz4"] for b in case["blocks"]]
        assert [int(x) for x in got.status] == want * 60
        _assert_same_as_oracle(got, cseg, cd, comp, False)
