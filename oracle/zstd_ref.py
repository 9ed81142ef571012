"""zstd checker and fixture builder (test infrastructure only).

The reference decodes zstd blocks with github.com/klauspost/compress v1.17.9
(go.mod:10): `zstd.NewReader(bytes.NewReader(rawBlockBytes[:CompressedSize]))`
then `io.Copy` (sst/segment_reader.go:320-330), i.e. standard RFC 8878 frame
decoding of every frame in the slice.  That library is not available offline;
the checker here is the system libzstd (1.4.8, the RFC's reference
implementation), called through ctypes.  Frames are produced with libzstd too
(klauspost *encoder* output is parity-unpinned), so decode
parity is pinned on standard frames: identical decompressed bytes.
"""
from __future__ import annotations

import ctypes as C
import ctypes.util
import struct

_L = None

# ZSTD_cParameter values (zstd.h, stable API since 1.4.0)
C_LEVEL, C_WINDOWLOG = 100, 101
C_CONTENTSIZE, C_CHECKSUM, C_DICTID = 200, 201, 202
ERR_DST_TOO_SMALL = 70


def lib():
    global _L
    if _L is None:
        path = ctypes.util.find_library("zstd") or "libzstd.so.1"
        L = C.CDLL(path)
        sz, p = C.c_size_t, C.c_void_p
        L.ZSTD_versionNumber.restype = C.c_uint
        L.ZSTD_compressBound.restype = sz
        L.ZSTD_compressBound.argtypes = [sz]
        L.ZSTD_createCCtx.restype = p
        L.ZSTD_freeCCtx.argtypes = [p]
        L.ZSTD_CCtx_setParameter.restype = sz
        L.ZSTD_CCtx_setParameter.argtypes = [p, C.c_int, C.c_int]
        L.ZSTD_compress2.restype = sz
        L.ZSTD_compress2.argtypes = [p, p, sz, p, sz]
        L.ZSTD_decompress.restype = sz
        L.ZSTD_decompress.argtypes = [p, sz, p, sz]
        L.ZSTD_isError.restype = C.c_uint
        L.ZSTD_isError.argtypes = [sz]
        L.ZSTD_getErrorCode.restype = C.c_int
        L.ZSTD_getErrorCode.argtypes = [sz]
        L.ZSTD_createDCtx.restype = p
        L.ZSTD_freeDCtx.argtypes = [p]
        L.ZSTD_decompressBegin.restype = sz
        L.ZSTD_decompressBegin.argtypes = [p]
        L.ZSTD_getFrameHeader.restype = sz
        L.ZSTD_getFrameHeader.argtypes = [p, p, sz]
        L.ZSTD_nextSrcSizeToDecompress.restype = sz
        L.ZSTD_nextSrcSizeToDecompress.argtypes = [p]
        L.ZSTD_nextInputType.restype = C.c_int
        L.ZSTD_nextInputType.argtypes = [p]
        L.ZSTD_decompressContinue.restype = sz
        L.ZSTD_decompressContinue.argtypes = [p, p, sz, p, sz]
        _L = L
    return _L


def version() -> int:
    return lib().ZSTD_versionNumber()


def compress(data: bytes, level: int = 3, checksum: bool = True, content_size: bool = True,
             window_log: int = 0) -> bytes:
    """One zstd frame of `data` (libzstd)."""
    L = lib()
    cctx = L.ZSTD_createCCtx()
    try:
        for prm, val in ((C_LEVEL, level), (C_CHECKSUM, int(checksum)),
                         (C_CONTENTSIZE, int(content_size))):
            assert not L.ZSTD_isError(L.ZSTD_CCtx_setParameter(cctx, prm, val))
        if window_log:
            assert not L.ZSTD_isError(L.ZSTD_CCtx_setParameter(cctx, C_WINDOWLOG, window_log))
        cap = L.ZSTD_compressBound(len(data))
        dst = C.create_string_buffer(cap)
        src = C.create_string_buffer(bytes(data), max(len(data), 1))
        n = L.ZSTD_compress2(cctx, dst, cap, src, len(data))
        assert not L.ZSTD_isError(n), "ZSTD_compress2"
        return dst.raw[:n]
    finally:
        L.ZSTD_freeCCtx(cctx)


def _oneshot(L, frames: bytes, hint: int):
    src = C.create_string_buffer(bytes(frames), max(len(frames), 1))
    cap = max(min(hint, 1 << 24), 64) + 65536
    while True:
        dst = C.create_string_buffer(cap)
        n = L.ZSTD_decompress(dst, cap, src, len(frames))
        if not L.ZSTD_isError(n):
            return dst.raw[:n]
        if L.ZSTD_getErrorCode(n) != ERR_DST_TOO_SMALL or cap > (1 << 31):
            return None
        cap *= 2


class _FrameHeader(C.Structure):  # ZSTD_frameHeader (zstd.h, 1.4.x)
    _fields_ = [("frameContentSize", C.c_ulonglong), ("windowSize", C.c_ulonglong),
                ("blockSizeMax", C.c_uint), ("frameType", C.c_int), ("headerSize", C.c_uint),
                ("dictID", C.c_uint), ("checksumFlag", C.c_uint)]


NIT_BLOCK, NIT_LAST_BLOCK = 2, 3  # ZSTD_nextInputType_e


def _blocks_within_max(L, frames: bytes, out_len: int) -> bool:
    """Replays the frames block by block (ZSTD_decompressContinue) and checks
    every block's decompressed size against its frame's Block_Maximum_Size =
    min(Window_Size, 128 KiB) (RFC 8878 3.1.1.2.3-4; ZSTD_frameHeader.blockSizeMax).
    libzstd 1.4.8's one-shot decoder does not enforce that limit (an RLE block
    of 200 KiB decodes); the device decoder does, as the RFC -- and newer
    libzstd -- require.  Also False for input the block-wise API rejects
    (e.g. the legacy v0.5-v0.7 frames 1.4.8's one-shot path still accepts)."""
    d = L.ZSTD_createDCtx()
    try:
        src = bytes(frames)
        sbuf = C.create_string_buffer(src, max(len(src), 1))
        dst = C.create_string_buffer(out_len + 64)
        at = pos = 0
        while at < len(src):
            fh = _FrameHeader()
            r = L.ZSTD_getFrameHeader(C.byref(fh), C.byref(sbuf, at), len(src) - at)
            if L.ZSTD_isError(r) or r != 0:
                return False
            bmax = fh.blockSizeMax
            if L.ZSTD_isError(L.ZSTD_decompressBegin(d)):
                return False
            while True:
                need = L.ZSTD_nextSrcSizeToDecompress(d)
                if need == 0:
                    break
                if need > len(src) - at:
                    return False
                kind = L.ZSTD_nextInputType(d)
                n = L.ZSTD_decompressContinue(d, C.byref(dst, pos), out_len + 64 - pos,
                                              C.byref(sbuf, at), need)
                if L.ZSTD_isError(n):
                    return False
                if kind in (NIT_BLOCK, NIT_LAST_BLOCK) and fh.frameType == 0 and n > bmax:
                    return False
                at += need
                pos += n
        return pos == out_len
    finally:
        L.ZSTD_freeDCtx(d)


def decompress(frames: bytes, hint: int = 0):
    """All frames of `frames` -> bytes, or None on a decode error (Go: the
    io.Copy error of segment_reader.go:326-330).  libzstd's one-shot decode,
    plus RFC 8878's Block_Maximum_Size rule (_blocks_within_max).  The whole
    frame set is inflated whatever the caller's OriginalSize (`hint` only
    sizes the first buffer): Go's io.Copy does the same before its record walk."""
    L = lib()
    out = _oneshot(L, frames, hint)
    if out is None or not _blocks_within_max(L, frames, len(out)):
        return None
    return out


def skippable_frame(payload: bytes, nibble: int = 0) -> bytes:
    """RFC 8878 §3.1.2 skippable frame."""
    return struct.pack("<II", 0x184D2A50 | (nibble & 15), len(payload)) + payload


def zstd_segment(rows, threshold=3584, block_size=4096, level=3, checksum=True,
                 content_size=True, frame_fn=None):
    """A segment whose blocks are zstd frames, laid out as segment_writer.go
    lays out compressed blocks (CompressedSize = frame bytes, zero padding to
    a multiple of DataBlockSize (Q2), Hash over the padded block, meta
    compression byte 1).  The cut uses the raw block length; the Go writer cuts
    on the klauspost encoder's buffered output length (Q6), which is not
    reproducible offline.  frame_fn(raw, block_index) -> frame bytes overrides
    the compressor (multi-frame / skippable-frame blocks).
    Returns (segment bytes, file length, meta bytes)."""
    from oracle import pyoracle as P
    blocks, cur = [], []
    raw = 0
    for k, v in rows:
        cur.append((k, v))
        raw += 6 + len(k) + len(v)
        if raw >= threshold:
            blocks.append(cur)
            cur, raw = [], 0
    if cur:
        blocks.append(cur)
    seg = bytearray()
    index = []
    for i, blk in enumerate(blocks):
        rawb = b"".join(struct.pack("<HI", len(k), len(v)) + k + v for k, v in blk)
        frame = frame_fn(rawb, i) if frame_fn else compress(rawb, level, checksum, content_size)
        padded = frame + bytes(block_size - len(frame) % block_size)
        st = P.BlockStat(blk[0][0], len(seg), len(padded), len(rawb), len(frame))
        st.Hash = P.xxh64(padded)
        index.append(st)
        seg += padded
    meta = bytearray()
    fk, lk = blocks[0][0][0], blocks[-1][-1][0]
    meta += struct.pack("<H", len(fk)) + fk + struct.pack("<H", len(lk)) + lk
    meta += bytes([0, 1, 0]) + struct.pack("<Q", len(index))
    for st in index:
        meta += st.to_bytes()
    meta_off = len(seg)
    seg += meta
    seg += struct.pack("<QQBQ", meta_off, P.xxh64(bytes(meta)), 1, P.MAGIC)
    return bytes(seg), len(seg), bytes(meta)
