"""zstd decode cases shared by the CPU oracle test and the GPU parity test.
Every block is a libzstd frame set (oracle/zstd_ref.py); see DESIGN.md for why
libzstd is the checker (klauspost v1.17.9 is not available offline)."""
from __future__ import annotations

import random
import struct

from oracle import zstd_ref as Z


def _rows(seed, n, kmax=40, vmax=300, text=True):
    rng = random.Random(seed)
    words = [b"alpha", b"beta", b"gamma", b"delta", b"kv", b"segment", b"block", b"zstd"]
    out = []
    for i in range(n):
        k = b"k%07d" % i + bytes(rng.getrandbits(8) for _ in range(rng.randint(0, kmax)))
        if text:
            v = b" ".join(rng.choice(words) for _ in range(rng.randint(0, vmax // 6)))
        else:
            v = bytes(rng.getrandbits(8) for _ in range(rng.randint(0, vmax)))
        out.append((k, v))
    return out


def cases():
    """[(name, segment bytes, descs [(off, bsize, orig, csize)], note)]"""
    from oracle import pyoracle as P
    out = []

    def add(name, seg, note):
        md = P.bytes_to_metadata(_meta_of(seg))
        out.append((name, seg, [st.desc() for st in md.entries], note))

    for lvl in (1, 3, 9, 19):
        seg, _, _ = Z.zstd_segment(_rows(lvl, 1500), 3584, 4096, level=lvl)
        add(f"text_l{lvl}", seg, "Huffman literals, FSE sequences, repeat offsets")
    seg, _, _ = Z.zstd_segment(_rows(7, 400, vmax=4000, text=False), 57344, 65536, level=3)
    add("random_64k", seg, "incompressible: raw blocks")
    seg, _, _ = Z.zstd_segment(_rows(8, 3000, vmax=2000), 57344, 65536, level=5,
                               checksum=False, content_size=False)
    add("text_64k_nocsum_nofcs", seg, "no checksum, no frame content size")
    zeros = [(b"z%06d" % i, bytes(1000)) for i in range(300)]
    seg, _, _ = Z.zstd_segment(zeros, 57344, 65536, level=3)
    add("zeros", seg, "RLE blocks / long matches")
    seg, _, _ = Z.zstd_segment(_rows(9, 2000, vmax=600), 57344, 65536, level=19)
    add("text_64k_l19", seg, "level 19")

    def multi(raw, i):  # two frames + a skippable frame per block
        h = len(raw) // 2
        return Z.compress(raw[:h], 3) + Z.skippable_frame(b"skip%d" % i, i) + \
            Z.compress(raw[h:], 1, checksum=False)
    seg, _, _ = Z.zstd_segment(_rows(10, 600), 3584, 4096, frame_fn=multi)
    add("multi_frame_skippable", seg, "concatenated frames + skippable frame")
    return out


def _meta_of(seg: bytes) -> bytes:
    meta_off, = struct.unpack_from("<Q", seg, len(seg) - 25)
    return seg[meta_off:len(seg) - 25]


def corrupt_cases():
    """Blocks whose zstd decode fails, or whose descriptor breaks Go's slice."""
    rows = _rows(11, 300)
    seg, _, _ = Z.zstd_segment(rows, 3584, 4096, level=3)
    from oracle import pyoracle as P
    md = P.bytes_to_metadata(_meta_of(seg))
    d0 = md.entries[0]
    base = list(d0.desc())
    b = bytearray(seg)
    b[d0.Offset + d0.CompressedSize // 2] ^= 0x5A  # payload corruption
    trunc = list(base)
    trunc[3] = base[3] - 7  # truncated frame
    big = list(base)
    big[3] = base[1] + 1  # CompressedSize > BlockSize: slice bounds panic
    empty = list(base)
    empty[2], empty[3] = 0, 0  # no frames, nothing to read
    empty_rows = list(base)
    empty_rows[3] = 0  # no frames, OriginalSize > 0: mustReadBytes panic
    return [("payload_flip", bytes(b), [tuple(base)]),
            ("truncated", seg, [tuple(trunc)]),
            ("csize_gt_bsize", seg, [tuple(big)]),
            ("empty_ok", seg, [tuple(empty)]),
            ("empty_panics", seg, [tuple(empty_rows)])]
