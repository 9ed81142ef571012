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


# ---- hand-made frames (RFC 8878 3.1) ----------------------------------------

def frame(blocks, fcs=None, single=False, wlog=20):
    """A zstd frame around `blocks` (already encoded block bytes): optional
    8-byte Frame_Content_Size; a Window_Descriptor of 2^wlog unless single."""
    fhd = (0x20 if single else 0) | ((3 << 6) if fcs is not None else 0)
    hdr = bytes([fhd])
    if not single:
        hdr += bytes([(wlog - 10) << 3])
    if fcs is not None:
        hdr += struct.pack("<Q", fcs)
    return struct.pack("<I", 0xFD2FB528) + hdr + b"".join(blocks)


def _bh(last, btype, size):
    return struct.pack("<I", last | (btype << 1) | (size << 3))[:3]


def rle_block(size, byte=0, last=1):
    return _bh(last, 1, size) + bytes([byte])


def raw_block(data, last=1):
    return _bh(last, 0, len(data)) + bytes(data)


def long_match_block(nseq, lits=b"\0" * 16, mlx=0xFFFF, last=1):
    """A compressed block of `nseq` sequences, each 8 literals + one match of
    ML code 52 (65 539 + mlx bytes) at offset 5, all three symbol tables in
    RLE_Mode, literals raw: the block's output is 8 + nseq * (8 + 65 539 + mlx)
    bytes from a few bytes of input."""
    body = bytes([(len(lits) << 3) | 0]) + bytes(lits)  # Raw_Literals_Block, 1-byte header
    body += bytes([nseq]) + bytes([(1 << 6) | (1 << 4) | (1 << 2)]) + bytes([8, 3, 52])
    acc, n = 0, 0
    for _ in range(nseq):  # written low to high = read last to first
        for v, nb in ((0, 0), (mlx, 16), (0, 3)):  # LL extra, ML extra, OF extra (ofv 8)
            acc |= (v & ((1 << nb) - 1)) << n
            n += nb
    acc |= 1 << n
    body += acc.to_bytes((n + 8) // 8, "little")
    return _bh(last, 2, len(body)) + body


def _frames_segment(frames_origs):
    """A zstd segment whose blocks hold the given frame bytes with the given
    OriginalSize each (padded to 4 KiB multiples as the writer pads, Q2)."""
    from oracle import pyoracle as P
    seg, index = bytearray(), []
    for i, (fr, orig) in enumerate(frames_origs):
        padded = fr + bytes(4096 - len(fr) % 4096)
        st = P.BlockStat(b"b%04d" % i, len(seg), len(padded), orig, len(fr))
        st.Hash = P.xxh64(padded)
        index.append(st)
        seg += padded
    meta = bytearray()
    fk, lk = index[0].FirstKey, index[-1].FirstKey
    meta += struct.pack("<H", len(fk)) + fk + struct.pack("<H", len(lk)) + lk
    meta += bytes([0, 1, 0]) + struct.pack("<Q", len(index))
    for st in index:
        meta += st.to_bytes()
    meta_off = len(seg)
    seg += meta
    seg += struct.pack("<QQBQ", meta_off, P.xxh64(bytes(meta)), 1, P.MAGIC)
    return bytes(seg), [st.desc() for st in index]


def past_original_cases():
    """Frames that decompress past OriginalSize (Go's io.Copy inflates the
    whole frame set, segment_reader.go:320-330, then walks records to
    OriginalSize, :338-352), OriginalSize values past Go's int() conversion
    (:340), and Block_Maximum_Size / window violations (RFC 8878 3.1.1.2.4).
    [(name, segment, descs, expected statuses or None, needs the regrow)]"""
    rows = _rows(31, 60)
    rawb = b"".join(struct.pack("<HI", len(k), len(v)) + k + v for k, v in rows)
    tail = bytes(range(256)) * 1200  # 300 KiB after the records
    big = Z.compress(rawb + tail, 3)
    half = len(rawb) // 2
    out = []
    out.append(("inflate_past_orig", *_frames_segment([(big, len(rawb))]), [0], True))
    # OriginalSize inside a record: the record is decoded from bytes past it (Q5)
    out.append(("orig_inside_record", *_frames_segment([(big, half)]), [0], True))
    out.append(("orig_zero", *_frames_segment([(big, 0)]), [0], True))
    out.append(("orig_2^63", *_frames_segment([(big, 1 << 63)]), [0], False))
    out.append(("orig_2^64-1", *_frames_segment([(Z.compress(rawb, 1), (1 << 64) - 1)]), [0], False))
    # the frame ends before OriginalSize: mustReadBytes panics
    out.append(("orig_2^40_short_frame", *_frames_segment([(Z.compress(rawb, 1), 1 << 40)]), [3],
                False))
    # 10 RLE blocks of 128 KiB (Block_Maximum_Size exactly): 1.25 MiB of zero
    # records (klen 0, vlen 0) from 44 bytes of frame
    rle10 = frame([rle_block(128 << 10, 0, last=0) for _ in range(9)] + [rle_block(128 << 10)])
    out.append(("rle_10x128k", *_frames_segment([(rle10, 600)]), [0], True))
    # two compressed blocks of exactly 128 KiB each (16 literals + one match of
    # 131 056 bytes): at the limit
    ok2 = frame([long_match_block(1, mlx=0xFFFF - 18, last=0), long_match_block(1, mlx=0xFFFF - 18)])
    out.append(("long_matches_2_blocks", *_frames_segment([(ok2, 64)]), [0], True))
    # Block_Maximum_Size violations: each is a decode error
    out.append(("rle_128k_plus_1", *_frames_segment([(frame([rle_block((128 << 10) + 1)]), 60)]),
                [6], False))
    out.append(("raw_129k", *_frames_segment([(frame([raw_block(bytes(129 << 10))]), 60)]),
                [6], False))
    out.append(("match_block_over_128k", *_frames_segment([(frame([long_match_block(2)]), 60)]),
                [6], False))
    out.append(("rle_2k_window_1k", *_frames_segment([(frame([rle_block(2048)], wlog=10), 60)]),
                [6], False))
    out.append(("window_log_41", *_frames_segment([(frame([rle_block(1024)], wlog=41), 60)]),
                [6], False))
    # several blocks in one segment: regrown, failing and plain blocks together
    mix = [(big, len(rawb)), (Z.compress(rawb, 1), len(rawb)), (rle10, 6000),
           (frame([rle_block((128 << 10) + 1)]), 60), (big, 100)]
    out.append(("mixed", *_frames_segment(mix), [0, 0, 0, 6, 0], True))
    return out
