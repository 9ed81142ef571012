"""Synthetic zstd segments for the benchmark (workload generator, not a
checker): C3-shaped 64 KiB blocks whose values are slices of a word corpus
(compressible: Huffman literals, FSE sequences, repeat offsets), each block one
libzstd frame laid out as segment_writer.go lays out compressed blocks
(CompressedSize = frame bytes, zero padding to a DataBlockSize multiple)."""
from __future__ import annotations

import ctypes as C
import ctypes.util

import numpy as np

_L = None


def _lib():
    global _L
    if _L is None:
        L = C.CDLL(ctypes.util.find_library("zstd") or "libzstd.so.1")
        L.ZSTD_compressBound.restype = C.c_size_t
        L.ZSTD_compressBound.argtypes = [C.c_size_t]
        L.ZSTD_compress.restype = C.c_size_t
        L.ZSTD_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int]
        L.ZSTD_isError.restype = C.c_uint
        L.ZSTD_isError.argtypes = [C.c_size_t]
        _L = L
    return _L


def _corpus(rng, nbytes=4 << 20):
    words = [bytes(rng.integers(97, 123, size=int(k), dtype=np.uint8))
             for k in rng.integers(2, 10, size=400)]
    idx = rng.zipf(1.3, size=nbytes // 4) % len(words)
    return b" ".join(words[i] for i in idx)[:nbytes]


def text_zstd_segment(nblocks, seed=5, level=3, threshold=57344, block_size=65536):
    """-> (segment uint8 array, descs uint64 [nblocks, 4], original bytes)"""
    rng = np.random.default_rng(seed)
    corpus = _corpus(rng)
    L = _lib()
    cap = L.ZSTD_compressBound(threshold + 8192)
    dst = C.create_string_buffer(cap)
    parts, descs = [], []
    off = 0
    row = 0
    orig_total = 0
    for _ in range(nblocks):
        recs, raw = [], 0
        while raw < threshold:
            vl = int(rng.integers(0, 4097))
            vo = int(rng.integers(0, len(corpus) - vl))
            key = row.to_bytes(8, "big") + rng.bytes(8)
            val = corpus[vo:vo + vl]
            recs.append(len(key).to_bytes(2, "little") + vl.to_bytes(4, "little") + key + val)
            raw += 6 + len(key) + vl
            row += 1
        body = b"".join(recs)
        n = L.ZSTD_compress(dst, cap, body, len(body), level)
        assert not L.ZSTD_isError(n)
        pad = block_size - n % block_size
        parts.append(dst.raw[:n] + bytes(pad))
        descs.append((off, n + pad, len(body), n))
        off += n + pad
        orig_total += len(body)
    seg = np.frombuffer(b"".join(parts), np.uint8)
    return seg, np.array(descs, np.uint64), orig_total
