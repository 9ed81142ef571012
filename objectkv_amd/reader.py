"""Go-shaped SegmentReader / RowIter over the GPU decode (objectkv_amd/csrc/okv_reader.cpp).

Mirrors /root/reference/sst/segment_reader.go and segment_row_iter.go:
method names, argument meaning, row order and error behaviour.  Errors carry
the Go sentinel name in ``.kind`` (ErrNoRows, EOF, ErrAlreadyClosed, ...);
Go panics raise ``GoPanic``.  Every block read is a batched okv_decode_blocks
call on the GPU, bounded as the cgo shim's ReadBlocks (one block for GetRow,
the selected set for GetRange, a 256-block window for RowIter) -- there is no
CPU decode path.
"""
from __future__ import annotations

import ctypes as C

from . import _lib
from ._lib import Row, lib
from .sst import Decoder, bytes_to_metadata

DirectionAscending, DirectionDescending = 0, 1  # segment_row_iter.go:22-25
UnboundStart = None  # segment_reader.go:60
UnboundEnd = b"\xff"  # segment_reader.go:62

_KIND = {
    -101: "ErrKeyTooLarge", -102: "ErrValueTooLarge", -103: "ErrWriterClosed",
    -104: "ErrInvalidKey", -201: "ErrInvalidMagicNumber", -202: "ErrUnknownSegmentVersion",
    -203: "ErrMismatchedMetaBlockHash", -204: "ErrInvalidMetaBlock", -206: "ErrIO",
    -301: "ErrNoRows", -302: "EOF", -303: "ErrClosed", -304: "ErrAlreadyClosed",
    -305: "EOF", -306: "ErrUnexpectedBytesRead", -308: "ErrUnsupported", -309: "ErrGPU",
    -310: "ErrZstd", -208: "ErrBloomReadFrom",
}
_PANIC = {-105, -205, -207, -307}
FATAL = {"ErrInvalidMagicNumber", "ErrUnknownSegmentVersion", "ErrMismatchedMetaBlockHash",
         "ErrInvalidMetaBlock"}  # wrap FatalError (segment_reader.go:80-85)


class GoError(Exception):
    def __init__(self, code):
        self.code = code
        self.kind = _KIND.get(code, f"code{code}")
        super().__init__(self.kind)


class GoPanic(Exception):
    def __init__(self, code):
        self.code = code
        super().__init__(f"panic (code {code})")


def _check(rc):
    if rc == 0:
        return
    if rc in _PANIC:
        raise GoPanic(rc)
    raise GoError(rc)


class KVPair:
    """segment_reader.go:285-288; None is Go's nil slice (Q4)."""

    __slots__ = ("Key", "Value")

    def __init__(self, Key, Value):
        self.Key, self.Value = Key, Value

    def __repr__(self):
        return f"KVPair({self.Key!r}, {self.Value!r})"


def _pair(row: Row) -> KVPair:
    k = C.string_at(row.key, row.key_len) if row.key else None
    v = C.string_at(row.val, row.val_len) if row.val else None
    return KVPair(k, v)


def _buf(b):
    b = b or b""
    return C.create_string_buffer(bytes(b), len(b)), len(b)


class SegmentReader:
    """NewSegmentReader(reader, fileBytes) (segment_reader.go:65) over bytes."""

    def __init__(self, data, file_bytes: int, decoder: Decoder):
        self._dec = decoder
        raw = bytes(data)
        self._h = lib().okv_reader_open(decoder._ctx, raw, len(raw), file_bytes)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib._lib is not None:
            _lib._lib.okv_reader_free(h)
            self._h = None

    def FetchAndLoadMetadata(self):
        _check(lib().okv_reader_fetch_metadata(self._h))

    def BytesToMetadata(self, meta: bytes):
        md = bytes_to_metadata(meta)  # raises OkvError on a malformed block
        md._raw = bytes(meta)
        return md

    def LoadCachedMetadata(self, md):
        raw = md._raw
        _check(lib().okv_reader_load_metadata(self._h, raw, len(raw)))

    def NumBlocks(self) -> int:
        n = C.c_uint64()
        _check(lib().okv_reader_num_blocks(self._h, C.byref(n)))
        return n.value

    def ReadBlock(self, i: int):
        """ReadBlockWithStat of the i-th block index entry in FirstKey order."""
        rows, n = C.POINTER(Row)(), C.c_uint64()
        _check(lib().okv_reader_read_block(self._h, i, C.byref(rows), C.byref(n)))
        return [_pair(rows[j]) for j in range(n.value)] or None

    def GetRow(self, key: bytes) -> KVPair:
        kb, kl = _buf(key)
        out = Row()
        _check(lib().okv_reader_get_row(self._h, kb, kl, C.byref(out)))
        return _pair(out)

    def GetRange(self, start, end):
        sb, sl = _buf(start)
        eb, el = _buf(end)
        rows, n = C.POINTER(Row)(), C.c_uint64()
        _check(lib().okv_reader_get_range(self._h, sb, sl, eb, el, C.byref(rows), C.byref(n)))
        return [_pair(rows[j]) for j in range(n.value)]

    def RowIter(self, direction: int) -> "RowIter":
        h = lib().okv_reader_row_iter(self._h, direction)
        if not h:
            self.FetchAndLoadMetadata()  # raises the metadata error
        return RowIter(self, h)

    def Close(self):
        _check(lib().okv_reader_close(self._h))

    def io_stats(self) -> dict:
        """GPU decode calls, blocks decoded and storage bytes staged so far."""
        io = _lib.ReaderIO()
        _check(lib().okv_reader_io_stats(self._h, C.byref(io)))
        return {"calls": io.calls, "blocks": io.blocks, "bytes_staged": io.bytes_staged}


class RowIter:
    """segment_row_iter.go:11-212."""

    def __init__(self, reader: SegmentReader, h):
        self._r = reader  # keeps the reader (and its rows) alive
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib._lib is not None:
            _lib._lib.okv_iter_free(h)
            self._h = None

    def Next(self) -> KVPair:
        out = Row()
        _check(lib().okv_iter_next(self._h, C.byref(out)))
        return _pair(out)

    def Seek(self, key):
        kb, kl = _buf(key)
        _check(lib().okv_iter_seek(self._h, kb, kl))

    def CloseReader(self):
        self._r.Close()


__all__ = ["SegmentReader", "RowIter", "KVPair", "GoError", "GoPanic", "DirectionAscending",
           "DirectionDescending", "UnboundStart", "UnboundEnd", "FATAL"]
