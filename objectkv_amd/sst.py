"""Python host side of the MI355X SST decode path.

Mirrors the Go ``sst`` API surface the hot path sits under
(/root/reference/sst): ``SegmentWriter`` (segment_writer.go:35-328),
metadata loading (segment_reader.go:91-238) and the batched
``ReadBlockWithStat`` (segment_reader.go:295-355) executed by the HIP kernels
in libokv_sst.so.  ``objectkv_amd.reader`` builds ``SegmentReader`` /
``RowIter`` on top of this.

Descriptor arrays are numpy ``uint64`` arrays of shape (nblk, 4):
``(Offset, BlockSize, OriginalSize, CompressedSize)`` == ``okv_block_desc``.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import (BLK_OK, COMP_LZ4, COMP_NONE, COMP_ZSTD, F_ASYNC, F_DEVICE_PTRS,  # noqa: F401
                   F_INDEX_ONLY, OKV_E_CAPACITY, OKV_OK, SYNTH_FIXED, SYNTH_ZIPF, BlockDesc,
                   DecodeOut, lib)


class OkvError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__(f"okv error {code}: {msg}")
        self.code = code


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data if a.size else None
    return a.data_ptr()  # torch tensor


def _bytes_array(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return b
    return np.frombuffer(bytes(b), np.uint8)


def xxh64(data, seed: int = 0) -> int:
    a = _bytes_array(data)
    return lib().okv_xxh64(_ptr(a), a.size, seed)


# ---- SegmentWriter -------------------------------------------------------------


class SegmentWriter:
    """Host C++ SegmentWriter (okv_writer_*); raises OkvError with the Go
    sentinel codes of include/okv_host.h.  bloom: the caller's filter object
    (SegmentWriterOptions.BloomFilter) with add(key) and to_bytes() -- add runs
    per row as in WriteRow (segment_writer.go:133-136), Close serialises
    to_bytes() into the meta block (:295-300); the library treats the bytes
    as opaque."""

    def __init__(self, threshold=3584, block_size=4096, zstd_level=0, lz4=False, _handle=None,
                 bloom=None):
        L = lib()
        self._h = _handle or L.okv_writer_new(threshold, block_size, zstd_level, int(lz4))
        if not self._h:
            raise OkvError(-1, "okv_writer_new")
        self.bloom = bloom

    def WriteRow(self, key: bytes, val: bytes):
        rc = lib().okv_writer_write_row(self._h, key, len(key), val, len(val))
        if rc:
            raise OkvError(rc, "WriteRow")
        if self.bloom is not None:
            self.bloom.add(bytes(key))

    def Close(self, strict_go=True):
        if self.bloom is not None:
            b = np.frombuffer(self.bloom.to_bytes(), np.uint8)
            lib().okv_writer_set_bloom(self._h, _ptr(b), b.size)
        fl, ml = C.c_uint64(), C.c_uint64()
        rc = lib().okv_writer_close(self._h, int(strict_go), C.byref(fl), C.byref(ml))
        if rc:
            raise OkvError(rc, "Close")
        return fl.value, self.meta()

    def data_view(self) -> np.ndarray:
        """Zero-copy view of the segment bytes (valid while the writer lives)."""
        n = C.c_uint64()
        p = lib().okv_writer_data(self._h, C.byref(n))
        if not n.value:
            return np.zeros(0, np.uint8)
        return np.ctypeslib.as_array((C.c_uint8 * n.value).from_address(p))

    def data(self) -> np.ndarray:
        n = C.c_uint64()
        p = lib().okv_writer_data(self._h, C.byref(n))
        if not n.value:
            return np.zeros(0, np.uint8)
        return np.ctypeslib.as_array((C.c_uint8 * n.value).from_address(p)).copy()

    def meta(self) -> bytes:
        n = C.c_uint64()
        p = lib().okv_writer_meta(self._h, C.byref(n))
        return C.string_at(p, n.value) if n.value else b""

    def num_blocks(self) -> int:
        return lib().okv_writer_num_blocks(self._h)

    def blocks(self):
        """[(first_key, (offset, block_size, original_size, compressed_size), hash)]"""
        out = []
        d, h, fk, fl = BlockDesc(), C.c_uint64(), C.c_void_p(), C.c_uint64()
        for i in range(self.num_blocks()):
            lib().okv_writer_block(self._h, i, C.byref(d), C.byref(h), C.byref(fk), C.byref(fl))
            key = C.string_at(fk, fl.value) if fl.value else b""
            out.append((key, (d.offset, d.block_size, d.original_size, d.compressed_size),
                        h.value))
        return out

    def descs(self) -> np.ndarray:
        return np.array([b[1] for b in self.blocks()], np.uint64).reshape(-1, 4)

    def __del__(self):
        h = getattr(self, "_h", None)
        L = _lib._lib
        if h and L is not None:
            L.okv_writer_free(h)
            self._h = None


def synth_segment(kind: int, seed: int, nrows: int = 0, nblocks: int = 0,
                  threshold: int = 3584, block_size: int = 4096) -> SegmentWriter:
    """Deterministic synthetic segment, closed."""
    h = lib().okv_synth_segment(kind, seed, nrows, nblocks, threshold, block_size)
    if not h:
        raise OkvError(-1, "okv_synth_segment")
    return SegmentWriter(_handle=h)


# ---- metadata ------------------------------------------------------------------


@dataclass
class Metadata:
    """SegmentMetadata (segment_reader.go:43-55) plus the index in file order."""

    first_key: bytes
    last_key: bytes
    compression: int
    first_keys: list  # per index entry, file order
    descs: np.ndarray  # (n, 4) uint64, file order
    hashes: np.ndarray  # (n,) uint64


def _meta_from_handle(h) -> Metadata:
    L = lib()
    try:
        n = L.okv_meta_num_blocks(h)
        ln = C.c_uint64()
        p = L.okv_meta_first_key(h, C.byref(ln))
        fk = C.string_at(p, ln.value) if ln.value else b""
        p = L.okv_meta_last_key(h, C.byref(ln))
        lk = C.string_at(p, ln.value) if ln.value else b""
        descs = np.zeros((n, 4), np.uint64)
        hashes = np.zeros(n, np.uint64)
        keys = []
        d, hh, kp, kl = BlockDesc(), C.c_uint64(), C.c_void_p(), C.c_uint64()
        for i in range(n):
            L.okv_meta_block(h, i, C.byref(d), C.byref(hh), C.byref(kp), C.byref(kl))
            descs[i] = (d.offset, d.block_size, d.original_size, d.compressed_size)
            hashes[i] = hh.value
            keys.append(C.string_at(kp, kl.value) if kl.value else b"")
        return Metadata(fk, lk, L.okv_meta_compression(h), keys, descs, hashes)
    finally:
        L.okv_meta_free(h)


def bytes_to_metadata(meta: bytes) -> Metadata:
    """BytesToMetadata (segment_reader.go:147-181)."""
    h = C.c_void_p()
    buf = C.create_string_buffer(bytes(meta), len(meta))
    rc = lib().okv_meta_parse(buf, len(meta), C.byref(h))
    if rc:
        raise OkvError(rc, "BytesToMetadata")
    return _meta_from_handle(h)


def fetch_metadata(data, file_bytes: int) -> Metadata:
    """FetchAndLoadMetadata (segment_reader.go:91-141)."""
    a = _bytes_array(data)
    h = C.c_void_p()
    rc = lib().okv_meta_fetch(_ptr(a), a.size, file_bytes, C.byref(h))
    if rc:
        raise OkvError(rc, "FetchAndLoadMetadata")
    return _meta_from_handle(h)


# ---- batched decode ------------------------------------------------------------


@dataclass
class Decoded:
    """Host copy of an okv_decode_out (see include/okv_sst.h)."""

    status: np.ndarray
    row_start: np.ndarray
    key_base: np.ndarray | None
    val_base: np.ndarray | None
    key_off: np.ndarray
    key_len: np.ndarray
    val_off: np.ndarray
    val_len: np.ndarray
    key_arena: np.ndarray | None
    val_arena: np.ndarray | None
    index_only: bool
    seg: np.ndarray | None = None

    def block_rows(self, b):
        """Rows of block b as [(key|None, value|None)] (None = Go nil, Q4)."""
        src_k = self.seg if self.index_only else self.key_arena
        src_v = self.seg if self.index_only else self.val_arena
        out = []
        for g in range(int(self.row_start[b]), int(self.row_start[b + 1])):
            kl, vl = int(self.key_len[g]), int(self.val_len[g])
            ko, vo = int(self.key_off[g]), int(self.val_off[g])
            out.append((src_k[ko:ko + kl].tobytes() if kl else None,
                        src_v[vo:vo + vl].tobytes() if vl else None))
        return out


class Decoder:
    """One okv_ctx bound to a GPU (HIP device ordinal)."""

    def __init__(self, device: int = 0, stream=None, flags: int = 0):
        """flags: okv_open_opts.flags (OPEN_NO_FUSED, OPEN_ZSTD_ONE_PASS, OPEN_NO_POINT)."""
        L = lib()
        if flags:
            opts = _lib.OpenOpts(C.sizeof(_lib.OpenOpts), flags)
            self._ctx = L.okv_open_ex(device, stream, C.byref(opts))
        else:
            self._ctx = (L.okv_open_on_stream(device, stream) if stream is not None
                         else L.okv_open(device))
        if not self._ctx:
            raise OkvError(_lib.OKV_E_NODEV, f"okv_open({device}) failed (no GPU?)")
        self.device = device

    def close(self):
        L = _lib._lib
        if getattr(self, "_ctx", None) and L is not None:
            L.okv_close(self._ctx)
            self._ctx = None

    __del__ = close

    def error(self) -> str:
        return (lib().okv_last_error(self._ctx) or b"").decode()

    def _check(self, rc, what):
        if rc:
            raise OkvError(rc, f"{what}: {self.error()}")

    @property
    def stream(self):
        return lib().okv_stream(self._ctx)

    def sync(self):
        self._check(lib().okv_sync(self._ctx), "okv_sync")

    def profile(self, enable=True):
        """Per-pass HIP-event timing on the context stream (okv_profile)."""
        self._check(lib().okv_profile(self._ctx, int(enable)), "okv_profile")

    def profile_read(self):
        """-> ({'count', 'scan', 'copy' (pass 3 gather), 'zstd'}: ms summed over
        the timed calls, number of calls)"""
        ms = (C.c_double * 4)()
        n = C.c_uint64()
        self._check(lib().okv_profile_read(self._ctx, ms, C.byref(n)), "okv_profile_read")
        return {"count": ms[0], "scan": ms[1], "copy": ms[2], "zstd": ms[3]}, n.value

    def chain(self, after: "Decoder | None") -> None:
        """okv_decode_chain: this decoder's pass 3 waits for `after`'s last
        pass 3 (consecutive-segment pipelining on two decoders); None unchains."""
        self._check(lib().okv_decode_chain(self._ctx, after._ctx if after else None),
                    "okv_decode_chain")

    def last_path(self) -> int:
        """OKV_PATH_* bits: the pass-3 kernels the last decode call launched."""
        return int(lib().okv_last_path(self._ctx))

    # -- host-pointer API ------------------------------------------------------
    def plan(self, seg, descs: np.ndarray, compression=COMP_NONE, index_only=False):
        s = _bytes_array(seg)
        d = np.ascontiguousarray(descs, np.uint64).reshape(-1, 4)
        r, k, v = C.c_uint64(), C.c_uint64(), C.c_uint64()
        flags = F_INDEX_ONLY if index_only else 0
        self._check(lib().okv_decode_plan(self._ctx, _ptr(s), s.size, _ptr(d), d.shape[0],
                                          compression, flags, C.byref(r), C.byref(k),
                                          C.byref(v)), "okv_decode_plan")
        return r.value, k.value, v.value

    def decode(self, seg, descs: np.ndarray, compression=COMP_NONE,
               index_only=False) -> Decoded:
        """Batched ReadBlockWithStat over host buffers (H2D, kernels, D2H)."""
        s = _bytes_array(seg)
        d = np.ascontiguousarray(descs, np.uint64).reshape(-1, 4)
        n = d.shape[0]
        rows, kb, vb = self.plan(s, d, compression, index_only)
        o = dict(status=np.zeros(n, np.int32), row_start=np.zeros(n + 1, np.uint64),
                 key_base=None if index_only else np.zeros(n, np.uint64),
                 val_base=None if index_only else np.zeros(n, np.uint64),
                 key_off=np.zeros(rows, np.uint64), key_len=np.zeros(rows, np.uint16),
                 val_off=np.zeros(rows, np.uint64), val_len=np.zeros(rows, np.uint32),
                 key_arena=None if index_only else np.zeros(kb, np.uint8),
                 val_arena=None if index_only else np.zeros(vb, np.uint8))
        out = DecodeOut(_ptr(o["row_start"]), _ptr(o["key_base"]), _ptr(o["val_base"]),
                        _ptr(o["status"]), _ptr(o["key_off"]), _ptr(o["key_len"]),
                        _ptr(o["val_off"]), _ptr(o["val_len"]), _ptr(o["key_arena"]),
                        _ptr(o["val_arena"]), rows, kb, vb, 0, 0, 0, 0)
        flags = F_INDEX_ONLY if index_only else 0
        self._check(lib().okv_decode_blocks(self._ctx, _ptr(s), s.size, _ptr(d), n, compression,
                                            C.byref(out), flags), "okv_decode_blocks")
        return Decoded(index_only=index_only, seg=s if index_only else None, **o)

    def hash_blocks(self, seg, descs: np.ndarray) -> np.ndarray:
        s = _bytes_array(seg)
        d = np.ascontiguousarray(descs, np.uint64).reshape(-1, 4)
        h = np.zeros(d.shape[0], np.uint64)
        self._check(lib().okv_hash_blocks(self._ctx, _ptr(s), s.size, _ptr(d), d.shape[0],
                                          _ptr(h), 0), "okv_hash_blocks")
        return h

    # -- device-pointer API (torch tensors on this device) ---------------------
    def decode_device(self, seg_t, seg_bytes, descs_t, nblk, out: dict, compression=COMP_NONE,
                      index_only=False, sync=True) -> DecodeOut:
        """Device-resident decode into caller-allocated torch tensors.

        ``out`` keys: row_start, key_base, val_base, status, key_off, key_len,
        val_off, val_len, key_arena, val_arena (arenas/bases unused when
        index_only).  With sync=False the call only enqueues (OKV_F_ASYNC).
        """
        g = out.get
        o = DecodeOut(_ptr(g("row_start")), _ptr(g("key_base")), _ptr(g("val_base")),
                      _ptr(g("status")), _ptr(g("key_off")), _ptr(g("key_len")),
                      _ptr(g("val_off")), _ptr(g("val_len")), _ptr(g("key_arena")),
                      _ptr(g("val_arena")), g("key_off").numel(),
                      0 if index_only else g("key_arena").numel(),
                      0 if index_only else g("val_arena").numel(), 0, 0, 0, 0)
        flags = F_DEVICE_PTRS | (F_INDEX_ONLY if index_only else 0) | (0 if sync else F_ASYNC)
        rc = lib().okv_decode_blocks(self._ctx, _ptr(seg_t), seg_bytes, _ptr(descs_t), nblk,
                                     compression, C.byref(o), flags)
        self._check(rc, "okv_decode_blocks(device)")
        return o

    def merge_device(self, srcs, mode, direction, limit=0, bound=None, drop_tombstones=False,
                     out: dict | None = None, key_base=0, val_base=0, row_cap=0):
        """okv_merge_rows over decoded device segments.

        srcs: [(soa dict of torch tensors key_arena/key_off/key_len/val_arena/
        val_off/val_len, row_lo, row_hi, level)] in priority order.  out: torch
        tensors src (int32), row (int64) and optionally key_off, key_len,
        val_off, val_len (relative to key_base / val_base).  Returns the filled
        okv_merge_out."""
        arr = (_lib.MergeSrc * max(1, len(srcs)))()
        for i, (t, lo, hi, level) in enumerate(srcs):
            arr[i] = _lib.MergeSrc(_ptr(t["key_arena"]), _ptr(t["key_off"]), _ptr(t["key_len"]),
                                   _ptr(t["val_arena"]), _ptr(t["val_off"]), _ptr(t["val_len"]),
                                   int(lo), int(hi), int(level), 0)
        b = None if bound is None else np.frombuffer(bytes(bound), np.uint8)
        o = _lib.MergeOpts(mode, direction, int(drop_tombstones), 0, int(limit),
                           _ptr(b) if b is not None and b.size else None,
                           0 if b is None else int(b.size))
        g = (out or {}).get
        mo = _lib.MergeOut(_ptr(g("src")), _ptr(g("row")), _ptr(g("key_off")),
                           _ptr(g("key_len")), _ptr(g("val_off")), _ptr(g("val_len")),
                           key_base or None, val_base or None, int(row_cap), 0, 0, 0, 0)
        rc = lib().okv_merge_rows(self._ctx, arr, len(srcs), C.byref(o), C.byref(mo),
                                  F_DEVICE_PTRS)
        if rc and rc != _lib.OKV_E_CAPACITY:
            self._check(rc, "okv_merge_rows")
        if rc:
            err = OkvError(rc, "okv_merge_rows: output capacity")
            err.out = mo
            raise err
        return mo

    def plan_device(self, seg_t, seg_bytes, descs_t, nblk, compression=COMP_NONE,
                    index_only=False):
        r, k, v = C.c_uint64(), C.c_uint64(), C.c_uint64()
        flags = F_DEVICE_PTRS | (F_INDEX_ONLY if index_only else 0)
        self._check(lib().okv_decode_plan(self._ctx, _ptr(seg_t), seg_bytes, _ptr(descs_t), nblk,
                                          compression, flags, C.byref(r), C.byref(k),
                                          C.byref(v)), "okv_decode_plan(device)")
        return r.value, k.value, v.value


# ---- device encode (okv_encode_rows) ----------------------------------------------


@dataclass
class Encoded:
    """Result of one GPU encode: the segment file bytes and the block index
    (BlockStat order).  ``first_row[b]`` is the row whose key is FirstKey."""
    seg: np.ndarray          # uint8[file_bytes]
    file_bytes: int
    data_bytes: int
    meta_bytes: int
    meta_hash: int
    first_row: np.ndarray    # uint64[n_blocks + 1]
    descs: np.ndarray        # uint64[n_blocks, 4]
    hashes: np.ndarray       # uint64[n_blocks]

    @property
    def n_blocks(self):
        return self.descs.shape[0]

    def meta(self) -> bytes:
        return self.seg[self.data_bytes:self.data_bytes + self.meta_bytes].tobytes()


def pack_rows(rows):
    """[(key, value), ...] -> SoA numpy arrays (okv_rows layout)."""
    keys = [bytes(k) for k, _ in rows]
    vals = [bytes(v) if v is not None else b"" for _, v in rows]
    kl = np.array([len(k) for k in keys], np.uint16)
    vl = np.array([len(v) for v in vals], np.uint32)
    ko = np.zeros(len(keys), np.uint64)
    vo = np.zeros(len(vals), np.uint64)
    if len(keys):
        ko[1:] = np.cumsum(kl[:-1], dtype=np.uint64)
        vo[1:] = np.cumsum(vl[:-1], dtype=np.uint64)
    ka = np.frombuffer(b"".join(keys) + b"\0" * 16, np.uint8)
    va = np.frombuffer(b"".join(vals) + b"\0" * 16, np.uint8)
    return dict(key_arena=ka, key_off=ko, key_len=kl, val_arena=va, val_off=vo, val_len=vl)


class Encoder(Decoder):
    """GPU SegmentWriter batch encode on one okv_ctx (shares the Decoder's
    context management)."""

    def profile_read_encode(self):
        """-> ({'cut', 'pack', 'hash', 'meta'} ms summed, calls)"""
        ms = (C.c_double * 4)()
        n = C.c_uint64()
        self._check(lib().okv_encode_profile_read(self._ctx, ms, C.byref(n)),
                    "okv_encode_profile_read")
        return {"cut": ms[0], "pack": ms[1], "hash": ms[2], "meta": ms[3]}, n.value

    def profile_reset_encode(self):
        self._check(lib().okv_encode_profile_reset(self._ctx), "okv_encode_profile_reset")

    @staticmethod
    def _opts(threshold, block_size, compression, strict_go, bloom=None):
        """bloom: BloomFilter.WriteTo bytes (kept alive on the returned struct)."""
        o = _lib.EncodeOpts(threshold, block_size, compression, int(strict_go), None, 0)
        if bloom is not None:
            o._bloom = np.frombuffer(bytes(bloom), np.uint8) if len(bloom) else \
                np.zeros(1, np.uint8)
            o.bloom, o.bloom_len = o._bloom.ctypes.data, len(bloom)
        return o

    def encode(self, rows, threshold=3584, block_size=4096, compression=COMP_NONE,
               strict_go=True, bloom=None) -> Encoded:
        """Host-buffer encode: rows is a list of (key, value) pairs or the dict
        of SoA arrays from pack_rows().  bloom: the filter's WriteTo bytes."""
        r = rows if isinstance(rows, dict) else pack_rows(rows)
        n = int(r["key_len"].size)
        R = _lib.Rows(_ptr(r["key_arena"]), _ptr(r["key_off"]), _ptr(r["key_len"]),
                      _ptr(r["val_arena"]), _ptr(r["val_off"]), _ptr(r["val_len"]), n,
                      int(r["key_arena"].size), int(r["val_arena"].size))
        o = self._opts(threshold, block_size, compression, strict_go, bloom)
        out = _lib.EncodeOut()
        rc = lib().okv_encode_rows(self._ctx, C.byref(R), C.byref(o), C.byref(out), 0)
        if rc != OKV_E_CAPACITY:
            self._check(rc, "okv_encode_rows(size)")
        nb = out.n_blocks
        seg = np.zeros(out.file_bytes, np.uint8)
        first = np.zeros(nb + 1, np.uint64)
        descs = np.zeros((nb, 4), np.uint64)
        hashes = np.zeros(nb, np.uint64)
        out = _lib.EncodeOut(_ptr(seg), seg.size, _ptr(first), _ptr(descs), _ptr(hashes), nb)
        rc = lib().okv_encode_rows(self._ctx, C.byref(R), C.byref(o), C.byref(out), 0)
        self._check(rc, "okv_encode_rows")
        return Encoded(seg, out.file_bytes, out.data_bytes, out.meta_bytes, out.meta_hash,
                       first, descs, hashes)

    def encode_device(self, rows: dict, n_rows: int, out: dict, threshold=3584,
                      block_size=4096, compression=COMP_NONE, strict_go=True, close=True,
                      key_arena_bytes=0, val_arena_bytes=0, bloom=None):
        """Device-resident encode.  rows: torch tensors key_arena, key_off,
        key_len, val_arena, val_off, val_len; out: torch tensors seg (uint8),
        optional first_row, desc (int64 [cap, 4]), hash.  Returns the filled
        okv_encode_out (raises OkvError, e.g. OKV_E_CAPACITY with sizes in
        .out)."""
        R = _lib.Rows(_ptr(rows["key_arena"]), _ptr(rows["key_off"]), _ptr(rows["key_len"]),
                      _ptr(rows["val_arena"]), _ptr(rows["val_off"]), _ptr(rows["val_len"]),
                      n_rows, key_arena_bytes, val_arena_bytes)
        o = self._opts(threshold, block_size, compression, strict_go, bloom)
        g = out.get
        caps = [t.shape[0] for t in (g("first_row"), g("desc"), g("hash")) if t is not None]
        blk_cap = min([caps[0] - 1 if g("first_row") is not None else caps[0]] + caps[1:]) \
            if caps else 0
        eo = _lib.EncodeOut(_ptr(g("seg")), g("seg").numel() if g("seg") is not None else 0,
                            _ptr(g("first_row")), _ptr(g("desc")), _ptr(g("hash")), blk_cap)
        flags = F_DEVICE_PTRS | (0 if close else _lib.F_NO_CLOSE)
        rc = lib().okv_encode_rows(self._ctx, C.byref(R), C.byref(o), C.byref(eo), flags)
        if rc:
            err = OkvError(rc, f"okv_encode_rows(device): {self.error()}")
            err.out = eo
            raise err
        return eo

    def close_device(self, eo):
        """okv_encode_close on a device segment (meta XXH64 on the host)."""
        self._check(lib().okv_encode_close(self._ctx, C.byref(eo), F_DEVICE_PTRS),
                    "okv_encode_close")
        return eo

    def synth_fixed_device(self, seed, first_row, n, key_len, val_len, t: dict):
        """Fill torch tensors (key_arena, key_off, key_len, val_arena, val_off,
        val_len) with rows_fixed rows first_row .. first_row + n - 1."""
        self._check(lib().okv_synth_rows_fixed(
            self._ctx, seed, first_row, n, key_len, val_len, _ptr(t["key_arena"]),
            _ptr(t["key_off"]), _ptr(t["key_len"]), _ptr(t["val_arena"]), _ptr(t["val_off"]),
            _ptr(t["val_len"])), "okv_synth_rows_fixed")


class GpuSegmentWriter:
    """sst.SegmentWriter (segment_writer.go:35-328) whose Close encodes on the
    GPU.  WriteRow validates each row exactly as Go does (:80-91) and buffers
    it; Close runs okv_encode_rows over the buffered rows and returns
    (file length, meta block bytes).  ``data()`` is what the Go writer's sink
    holds afterwards.  bloom: as SegmentWriter's (add per row, WriteTo bytes
    into the meta block)."""

    def __init__(self, encoder: Encoder, threshold=3584, block_size=4096, zstd_level=0,
                 lz4=False, strict_go=True, bloom=None):
        self._enc = encoder
        self.bloom = bloom
        self._opts = dict(threshold=threshold, block_size=block_size,
                          compression=COMP_ZSTD if zstd_level > 0 else
                          (COMP_LZ4 if lz4 else COMP_NONE), strict_go=strict_go)
        self._rows = []
        self._closed = False
        self.result = None

    def WriteRow(self, key, val):
        key = b"" if key is None else bytes(key)
        val = b"" if val is None else bytes(val)
        if len(key) > 0xFFFF:
            raise OkvError(_lib.W_KEY_TOO_LARGE, "ErrKeyTooLarge")
        if len(val) > 0xFFFFFFFF:
            raise OkvError(_lib.W_VALUE_TOO_LARGE, "ErrValueTooLarge")
        if self._closed:
            raise OkvError(_lib.W_CLOSED, "ErrWriterClosed")
        if not key:
            raise OkvError(_lib.W_INVALID_KEY, "key cannot be empty: ErrInvalidKey")
        self._rows.append((key, val))
        if self.bloom is not None:
            self.bloom.add(key)

    def Close(self):
        if self._closed:  # Go: blockWriter is nil after the first Close -> panic (Q1)
            raise OkvError(_lib.W_NIL_WRITER, "Close on a closed writer")
        bloom = self.bloom.to_bytes() if self.bloom is not None else None
        self.result = self._enc.encode(self._rows, bloom=bloom, **self._opts)
        self._closed = True
        return self.result.file_bytes, self.result.meta()

    def data(self) -> np.ndarray:
        return self.result.seg
