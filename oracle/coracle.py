"""coracle -- TEST INFRASTRUCTURE ONLY: ctypes binding of the C restatement
(oracle/okv_oracle.c -> oracle/build/liboref.so).  Used by tests/ as the
checker, by __graft_entry__.smoke(), and by bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboref.so")
_lib = None


class BlockDesc(C.Structure):
    _fields_ = [("offset", C.c_uint64), ("block_size", C.c_uint64),
                ("original_size", C.c_uint64), ("compressed_size", C.c_uint64)]


DESC_DTYPE = np.dtype([("offset", "<u8"), ("block_size", "<u8"), ("original_size", "<u8"),
                       ("compressed_size", "<u8")])


class Meta(C.Structure):
    _fields_ = [("first_key", C.c_void_p), ("first_key_len", C.c_uint64),
                ("last_key", C.c_void_p), ("last_key_len", C.c_uint64),
                ("has_bloom", C.c_int), ("bloom_off", C.c_uint64), ("bloom_len", C.c_uint64),
                ("compression", C.c_int), ("n_entries", C.c_uint64),
                ("entry_key", C.POINTER(C.c_void_p)), ("entry_key_len", C.POINTER(C.c_uint64)),
                ("entry_offset", C.POINTER(C.c_uint64)),
                ("entry_block_size", C.POINTER(C.c_uint64)),
                ("entry_original_size", C.POINTER(C.c_uint64)),
                ("entry_compressed_size", C.POINTER(C.c_uint64)),
                ("entry_hash", C.POINTER(C.c_uint64))]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        u64, p = C.c_uint64, C.c_void_p
        L.oref_xxh64.restype = u64
        L.oref_xxh64.argtypes = [p, C.c_size_t, u64]
        L.oref_writer_new.restype = p
        L.oref_writer_new.argtypes = [u64, u64, C.c_int, C.c_int]
        L.oref_writer_write_row.argtypes = [p, p, C.c_size_t, p, C.c_size_t]
        L.oref_writer_close.argtypes = [p, C.POINTER(p), C.POINTER(u64), C.POINTER(p),
                                        C.POINTER(u64)]
        L.oref_writer_bytes.restype = p
        L.oref_writer_bytes.argtypes = [p, C.POINTER(u64)]
        L.oref_writer_num_blocks.restype = u64
        L.oref_writer_num_blocks.argtypes = [p]
        L.oref_writer_free.argtypes = [p]
        L.oref_writer_set_bloom.argtypes = [p, p, u64]
        L.oref_parse_meta.argtypes = [p, u64, C.POINTER(Meta)]
        L.oref_fetch_meta.argtypes = [p, u64, C.c_int64, C.POINTER(Meta), C.POINTER(u64),
                                      C.POINTER(u64)]
        L.oref_meta_free.argtypes = [C.POINTER(Meta)]
        L.oref_encode_go.restype = C.c_int
        L.oref_encode_go.argtypes = [p, p, p, p, p, p, u64, u64, u64, C.c_int, C.c_int,
                                     C.POINTER(u64)]
        L.oref_encode_soa.restype = p
        L.oref_encode_soa.argtypes = [p, p, p, p, p, p, u64, u64, u64, C.POINTER(C.c_int)]
        L.oref_roundtrip_go.restype = u64
        L.oref_roundtrip_go.argtypes = [p, p, p, p, p, p, u64, u64, u64, C.c_int,
                                        C.POINTER(u64)]
        L.oref_compact_go.restype = u64
        L.oref_compact_go.argtypes = [C.c_int, p, p, p, p, u64, u64, C.c_int, C.POINTER(u64)]
        L.oref_decode_range_go.restype = u64
        L.oref_decode_range_go.argtypes = [p, u64, p, u64, C.c_int, C.c_int, C.POINTER(u64)]
        L.oref_block_counts.argtypes = [p, u64, p, u64, C.c_int, p, p, p, p]
        L.oref_decode_soa.argtypes = [p, u64, p, u64, C.c_int, C.c_int] + [p] * 10
        L.oref_arena_trim.argtypes = []
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


def xxh64(data: bytes, seed: int = 0) -> int:
    buf = np.frombuffer(data, np.uint8) if len(data) else np.zeros(1, np.uint8)
    return lib().oref_xxh64(_ptr(buf), len(data), seed)


class Writer:
    def __init__(self, threshold=3584, block_size=4096, zstd_level=0, lz4=False):
        self.h = lib().oref_writer_new(threshold, block_size, zstd_level, int(lz4))

    def set_bloom(self, data: bytes):
        """BloomFilter != nil: the meta block carries these WriteTo bytes."""
        buf = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
        lib().oref_writer_set_bloom(self.h, _ptr(buf), len(data))

    def write_row(self, key: bytes, val: bytes) -> int:
        return lib().oref_writer_write_row(self.h, key, len(key), val, len(val))

    def close(self):
        f, fl, m, ml = C.c_void_p(), C.c_uint64(), C.c_void_p(), C.c_uint64()
        rc = lib().oref_writer_close(self.h, C.byref(f), C.byref(fl), C.byref(m), C.byref(ml))
        if rc:
            return rc, None, None
        return 0, C.string_at(f, fl.value), C.string_at(m, ml.value)

    def num_blocks(self):
        return lib().oref_writer_num_blocks(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oref_writer_free(self.h)
            self.h = None


def _meta_dict(m: Meta, base):
    n = m.n_entries
    ents = []
    for i in range(n):
        kl = m.entry_key_len[i]
        key = C.string_at(m.entry_key[i], kl) if kl else b""
        ents.append(dict(first_key=key, offset=m.entry_offset[i],
                         block_size=m.entry_block_size[i],
                         original_size=m.entry_original_size[i],
                         compressed_size=m.entry_compressed_size[i], hash=m.entry_hash[i]))
    return dict(first_key=C.string_at(m.first_key, m.first_key_len) if m.first_key_len else b"",
                last_key=C.string_at(m.last_key, m.last_key_len) if m.last_key_len else b"",
                has_bloom=bool(m.has_bloom), compression=m.compression, entries=ents)


def parse_meta(meta: bytes):
    buf = C.create_string_buffer(meta, len(meta))
    m = Meta()
    rc = lib().oref_parse_meta(buf, len(meta), C.byref(m))
    if rc:
        return rc, None
    d = _meta_dict(m, buf)
    lib().oref_meta_free(C.byref(m))
    return 0, d


def fetch_meta(data: bytes, file_bytes: int):
    buf = C.create_string_buffer(data, len(data))
    m = Meta()
    off, ln = C.c_uint64(), C.c_uint64()
    rc = lib().oref_fetch_meta(buf, len(data), file_bytes, C.byref(m), C.byref(off),
                               C.byref(ln))
    if rc:
        return rc, None
    d = _meta_dict(m, buf)
    lib().oref_meta_free(C.byref(m))
    return 0, d


def descs_array(descs) -> np.ndarray:
    a = np.zeros(len(descs), DESC_DTYPE)
    for i, d in enumerate(descs):
        a[i] = tuple(d) + (0,) * (4 - len(d))
    return a


def _seg_array(seg):
    if isinstance(seg, np.ndarray):
        return seg
    return np.frombuffer(seg, np.uint8) if len(seg) else np.zeros(1, np.uint8)


def block_counts(seg, descs: np.ndarray, compression=0):
    s = _seg_array(seg)
    n = len(descs)
    st = np.zeros(n, np.int32)
    rows, kb, vb = (np.zeros(n, np.uint64) for _ in range(3))
    lib().oref_block_counts(_ptr(s), len(seg), _ptr(descs), n, compression, _ptr(st),
                            _ptr(rows), _ptr(kb), _ptr(vb))
    return st, rows, kb, vb


def decode_soa(seg, descs: np.ndarray, compression=0, index_only=False):
    """Oracle output in the product layout (numpy arrays)."""
    s = _seg_array(seg)
    st, rows, kb, vb = block_counts(seg, descs, compression)
    n = len(descs)
    total = int(rows.sum())
    ka_n = int(sum((int(x) + 15) // 16 * 16 for x in kb))
    va_n = int(sum((int(x) + 15) // 16 * 16 for x in vb))
    out = dict(row_start=np.zeros(n + 1, np.uint64), key_base=np.zeros(n, np.uint64),
               val_base=np.zeros(n, np.uint64), key_off=np.zeros(total, np.uint64),
               key_len=np.zeros(total, np.uint16), val_off=np.zeros(total, np.uint64),
               val_len=np.zeros(total, np.uint32), key_arena=np.zeros(ka_n, np.uint8),
               val_arena=np.zeros(va_n, np.uint8), status=np.zeros(n, np.int32))
    if index_only:
        out["key_arena"] = out["val_arena"] = None
    o = out
    lib().oref_decode_soa(_ptr(s), len(seg), _ptr(descs), n, compression, int(index_only),
                          _ptr(o["row_start"]), _ptr(o["key_base"]), _ptr(o["val_base"]),
                          _ptr(o["key_off"]), _ptr(o["key_len"]), _ptr(o["val_off"]),
                          _ptr(o["val_len"]), _ptr(o["key_arena"]), _ptr(o["val_arena"]),
                          _ptr(o["status"]))
    rows_out = int(out["row_start"][-1])  # index-only zstd blocks yield no rows
    for k in ("key_off", "key_len", "val_off", "val_len"):
        out[k] = out[k][:rows_out]
    return out


def arena_trim():
    """Free the baseline arena's pooled chunks (after a CPU baseline sweep)."""
    lib().oref_arena_trim()


def decode_go(seg, descs: np.ndarray, compression=0, threads=1):
    """CPU baseline: Go allocation semantics; returns (rows, payload bytes)."""
    s = _seg_array(seg)
    pay = C.c_uint64()
    rows = lib().oref_decode_range_go(_ptr(s), len(seg), _ptr(descs), len(descs), compression,
                                      threads, C.byref(pay))
    return rows, pay.value


def _view(ptr, n):
    """numpy uint8 view of n bytes at ptr (no copy; owner keeps it alive)."""
    if not n:
        return np.zeros(0, np.uint8)
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(n,))


class SoaSegment:
    """oref_encode_soa result: .file / .meta are views into the writer."""

    def __init__(self, rows: dict, n, threshold, block_size):
        rc = C.c_int()
        self.h = lib().oref_encode_soa(_ptr(rows["key_arena"]), _ptr(rows["key_off"]),
                                       _ptr(rows["key_len"]), _ptr(rows["val_arena"]),
                                       _ptr(rows["val_off"]), _ptr(rows["val_len"]), n,
                                       threshold, block_size, C.byref(rc))
        self.rc = rc.value
        self.file = self.meta = None
        if self.rc == 0:
            f, fl, m, ml = C.c_void_p(), C.c_uint64(), C.c_void_p(), C.c_uint64()
            self.rc = lib().oref_writer_close(self.h, C.byref(f), C.byref(fl), C.byref(m),
                                              C.byref(ml))
            if self.rc == 0:
                self.file, self.meta = _view(f.value, fl.value), _view(m.value, ml.value)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oref_writer_free(self.h)
            self.h = None


def encode_soa(rows: dict, n, threshold=3584, block_size=4096) -> SoaSegment:
    """One segment from SoA numpy rows, single-threaded (the oracle writer)."""
    return SoaSegment(rows, n, threshold, block_size)


def encode_go(rows: dict, n, threshold=3584, block_size=4096, lz4=False, threads=1):
    """CPU encode baseline over SoA numpy arrays (okv_rows layout); returns the
    total segment bytes written by `threads` key-range shards."""
    fb = C.c_uint64()
    rc = lib().oref_encode_go(_ptr(rows["key_arena"]), _ptr(rows["key_off"]),
                              _ptr(rows["key_len"]), _ptr(rows["val_arena"]),
                              _ptr(rows["val_off"]), _ptr(rows["val_len"]), n, threshold,
                              block_size, int(lz4), threads, C.byref(fb))
    if rc:
        raise RuntimeError(f"oref_encode_go: {rc}")
    return fb.value


def roundtrip_go(rows: dict, n, threshold=3584, block_size=4096, threads=1):
    """CPU baseline of C1 (write + full ascending read, Go semantics) on
    `threads` concurrent copies; returns (rows read, segment bytes) summed."""
    fb = C.c_uint64()
    r = lib().oref_roundtrip_go(_ptr(rows["key_arena"]), _ptr(rows["key_off"]),
                                _ptr(rows["key_len"]), _ptr(rows["val_arena"]),
                                _ptr(rows["val_off"]), _ptr(rows["val_len"]), n, threshold,
                                block_size, threads, C.byref(fb))
    return r, fb.value


def compact_go(segs, threshold=3584, block_size=4096, threads=1):
    """CPU baseline of one compaction step: segs = [(segment bytes (numpy),
    descs (DESC_DTYPE array)), ...] newest first; `threads` concurrent copies.
    Returns (merged rows of one compaction, output bytes summed)."""
    k = len(segs)
    sp = (C.c_void_p * k)(*[s.ctypes.data for s, _ in segs])
    ln = (C.c_uint64 * k)(*[s.nbytes for s, _ in segs])
    dp = (C.c_void_p * k)(*[d.ctypes.data for _, d in segs])
    nb = (C.c_uint64 * k)(*[len(d) for _, d in segs])
    ob = C.c_uint64()
    r = lib().oref_compact_go(k, sp, ln, dp, nb, threshold, block_size, threads, C.byref(ob))
    return r, ob.value
