"""GPU parity of the large-block pass (okv_tile_kernel: 16 KiB source tiles,
one short-lived workgroup each) at the edges of its tiling, against the C
oracle.  Every segment here averages more than 16 KiB per block, so the
decode takes the large-block path (okv_count_kernel -> okv_scan_kernel ->
okv_tile_kernel + okv_copy_kernel for big blocks).  Bit-exact."""
from __future__ import annotations

import numpy as np
import pytest

from tests.test_decode_gpu import _assert_same_as_oracle

pytestmark = pytest.mark.gpu

TILE = 16384


def _rec(rng, kl, vl):
    return (kl.to_bytes(2, "little") + vl.to_bytes(4, "little") +
            rng.integers(0, 256, kl + vl, dtype=np.uint8).tobytes())


def _segment(blocks, seed, pad_to=65536, gap=0):
    """blocks: list of record-shape lists [(klen, vlen), ...]; each block is
    padded to a multiple of pad_to (BlockSize) and placed `gap` bytes after
    the previous one."""
    rng = np.random.default_rng(seed)
    seg, descs = bytearray(), []
    for shape in blocks:
        body = b"".join(_rec(rng, kl, vl) for kl, vl in shape)
        bsize = max(pad_to, -(-len(body) // pad_to) * pad_to)
        off = len(seg) + gap
        seg += bytes(off - len(seg)) + body + bytes(bsize - len(body))
        descs.append((off, bsize, len(body), 0))
    return bytes(seg), np.array(descs, np.uint64).reshape(-1, 4)


def _fill_to(target, kl, rng):
    """Record shapes whose framed bytes sum exactly to target (>= 6 + kl)."""
    shape, left = [], target
    while left > 0:
        vl = int(rng.integers(500, 3000))
        if left - (6 + kl + vl) < 6 + kl + 1:
            vl = left - 6 - kl
        shape.append((kl, vl))
        left -= 6 + kl + vl
    return shape


def test_tile_boundaries(decoder):
    """Records whose header, key or value straddles a 16 KiB tile edge, and
    values / whole blocks ending exactly on one (the last tile then owns only
    the 16-byte padding of its regions)."""
    rng = np.random.default_rng(1)
    blocks = []
    for edge in (TILE, 2 * TILE, 3 * TILE):
        for delta in (-7, -6, -3, 0, 1, 3, 6, 9, 40, 200):
            # a first stretch ending `delta` bytes around the edge, then one record across it
            head = _fill_to(edge + delta - (6 + 20 + 1000), 12, rng)
            blocks.append(head + [(20, 1000)] + [(33, 777)] * 3)
    for k in (1, 2, 3, 4):  # blocks ending exactly on a tile edge
        blocks.append(_fill_to(k * TILE, 16, rng))
    seg, d = _segment(blocks, 2)
    got = decoder.decode(seg, d)
    _assert_same_as_oracle(got, seg, d, 0, False)
    assert (got.status == 0).all()


def test_long_keys_and_tiny_values(decoder):
    """A 60 000-byte key spanning four tiles; 64-row blocks of 0-3 byte
    values and 0-8 byte keys (many rows per destination chunk and per 64-byte
    granule of the row lookup); empty keys; a block of empty values only."""
    rng = np.random.default_rng(3)
    blocks = [[(60000, 100), (5, 4000)],
              [(65535 - 10, 0)],
              [(int(rng.integers(0, 9)), int(rng.integers(0, 4))) for _ in range(64)],
              [(0, int(rng.integers(0, 300))) for _ in range(64)],
              [(int(rng.integers(1, 300)), 0) for _ in range(64)],
              [(7, 1)] * 64]
    blocks += [[(int(rng.integers(0, 9)), int(rng.integers(0, 4))) for _ in range(64)]
               for _ in range(40)]
    seg, d = _segment(blocks, 4)
    got = decoder.decode(seg, d)
    _assert_same_as_oracle(got, seg, d, 0, False)


def test_odd_offsets_and_segment_edges(decoder):
    """Blocks at unaligned offsets (the tile stage's lead-in line starts
    before the block; the first block's before the segment), and the last
    block ending at the segment's last byte."""
    rng = np.random.default_rng(5)
    blocks = [_fill_to(int(rng.integers(30000, 65000)), int(rng.integers(8, 200)), rng)
              for _ in range(60)]
    for gap in (1, 3, 5, 13):
        seg, d = _segment(blocks, 6, pad_to=65536, gap=gap)
        d[-1, 1] = len(seg) - d[-1, 0]  # ends exactly at the segment end
        got = decoder.decode(seg, d)
        _assert_same_as_oracle(got, seg, d, 0, False)


def test_blocks_past_the_tile_span_and_over_64_rows(decoder):
    """Big blocks mixed into a 64 KiB segment: a 128 KiB block with few rows
    (its walk ends past tiles-per-block x 16 KiB: okv_copy_kernel), blocks of
    more than kRCap (64) rows, and statuses (short, EOF, overrun) beside them."""
    rng = np.random.default_rng(7)
    blocks = []
    for i in range(48):
        if i % 7 == 3:
            blocks.append(_fill_to(100000, 40, rng))  # BlockSize 128 KiB, ~40 rows
        elif i % 7 == 5:
            blocks.append([(8, int(rng.integers(0, 200))) for _ in range(300)])
        else:
            blocks.append(_fill_to(int(rng.integers(40000, 62000)), 24, rng))
    seg, d = _segment(blocks, 8)
    d = d.copy()
    d[10, 2] += 5000  # OriginalSize past the records: the walk overruns -> panic status
    d[20, 0] = len(seg) + 10  # past the segment: EOF
    d[30, 1] = len(seg) - d[30, 0] + 1  # BlockSize past the segment end: short read
    got = decoder.decode(seg, d)
    _assert_same_as_oracle(got, seg, d, 0, False)
    assert got.status[20] == 1 and got.status[30] == 2  # EOF, short read


def test_capacity_statuses_device(decoder):
    """Device outputs sized below the totals: the blocks that do not fit
    report OKV_BLK_CAPACITY, the others are complete and equal the oracle's."""
    torch = pytest.importorskip("torch")
    import objectkv_amd as okv
    w = okv.synth_segment(okv.sst.SYNTH_ZIPF, 9, nblocks=64, threshold=57344, block_size=65536)
    seg, d = w.data(), w.descs()[:64]
    ref = decoder.decode(seg, d)
    dev = torch.device("cuda", 0)
    seg_t = torch.from_numpy(seg).to(dev)
    d_t = torch.from_numpy(d.view(np.int64)).to(dev)
    rows, kb, vb = decoder.plan_device(seg_t, seg.size, d_t, 64)
    for cut in ("val", "key", "rows"):
        out = dict(row_start=torch.zeros(65, dtype=torch.int64, device=dev),
                   key_base=torch.zeros(64, dtype=torch.int64, device=dev),
                   val_base=torch.zeros(64, dtype=torch.int64, device=dev),
                   status=torch.zeros(64, dtype=torch.int32, device=dev),
                   key_off=torch.zeros(rows // 2 if cut == "rows" else rows, dtype=torch.int64,
                                       device=dev),
                   key_len=torch.zeros(rows, dtype=torch.int16, device=dev),
                   val_off=torch.zeros(rows, dtype=torch.int64, device=dev),
                   val_len=torch.zeros(rows, dtype=torch.int32, device=dev),
                   key_arena=torch.zeros(kb // 2 if cut == "key" else kb, dtype=torch.uint8,
                                         device=dev),
                   val_arena=torch.zeros(vb // 2 if cut == "val" else vb, dtype=torch.uint8,
                                         device=dev))
        with pytest.raises(Exception):
            decoder.decode_device(seg_t, seg.size, d_t, 64, out, sync=True)
        st = out["status"].cpu().numpy()
        assert (st == 5).any() and (st == 0).any(), cut
        first_bad = int(np.argmax(st != 0))
        assert (st[first_bad:] == 5).all()  # capacity failures are a suffix
        for b in range(first_bad):
            r0, r1 = int(ref.row_start[b]), int(ref.row_start[b + 1])
            assert np.array_equal(out["val_len"][r0:r1].cpu().numpy().view(np.uint32),
                                  ref.val_len[r0:r1])
            if cut != "val":
                lo, hi = int(ref.val_base[b]), int(ref.val_base[b + 1])
                assert out["val_arena"][lo:hi].cpu().numpy().tobytes() == \
                    ref.val_arena[lo:hi].tobytes()
