"""ctypes binding of libokv_sst.so (include/okv_sst.h, include/okv_host.h).

The product path: every decode goes through the HIP kernels in this library.
There is no CPU fallback -- if the library is missing or no GPU is present,
the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# The product library; OKV_ABLATE=1 loads the ablation build instead (the
# measured alternative kernel forms and their OKV_* knobs, tools/ablate*.py);
# OKV_ZTRACE=1 the product configuration with the zstd exit-line recorder
# (`make ztrace`).
LIB_PATH = os.path.join(_HERE, "libokv_sst_ablate.so" if os.environ.get("OKV_ABLATE") == "1"
                        else "libokv_sst_ztrace.so" if os.environ.get("OKV_ZTRACE") == "1"
                        else "libokv_sst.so")
# OKV_LIB=<path>: another build of the library (A/B runs of two builds on one
# box, tools/gpu_*ab*.sh); never set by the product or the tests
if os.environ.get("OKV_LIB"):
    LIB_PATH = os.path.abspath(os.environ["OKV_LIB"])

# ---- constants (include/okv_sst.h) -------------------------------------------
OKV_OK, OKV_E_ARG, OKV_E_HIP, OKV_E_CAPACITY, OKV_E_NOMEM, OKV_E_NODEV = 0, -1, -2, -3, -4, -5
BLK_OK, BLK_EOF, BLK_SHORT, BLK_PANIC, BLK_UNSUPPORTED, BLK_CAPACITY = 0, 1, 2, 3, 4, 5
COMP_NONE, COMP_ZSTD, COMP_LZ4 = 0, 1, 2
F_DEVICE_PTRS, F_INDEX_ONLY, F_ASYNC, F_NO_CLOSE = 1, 2, 4, 8
OPEN_NO_FUSED, OPEN_ZSTD_ONE_PASS, OPEN_NO_POINT = 1, 2, 4
# okv_last_path bits (include/okv_sst.h OKV_PATH_*)
PATH_FUSED, PATH_SMALL, PATH_TILE, PATH_SWEEP = 1, 2, 4, 8
PATH_STAGED, PATH_GATHER, PATH_BIG, PATH_ZSTD = 16, 32, 64, 128
PATH_ZSTD_REGROW, PATH_ENC_ONEPASS, PATH_STREAM = 256, 512, 1024
PATH_POINT, PATH_GROUP = 2048, 4096
# SegmentWriter sentinels (okv_sst.h OKV_W_*)
W_KEY_TOO_LARGE, W_VALUE_TOO_LARGE, W_CLOSED, W_INVALID_KEY = -101, -102, -103, -104
W_NIL_WRITER, W_UNSUPPORTED, W_NO_ROWS = -105, -106, -107
SYNTH_FIXED, SYNTH_ZIPF = 0, 1
MERGE_GETRANGE, MERGE_ALL = 0, 1
DIR_ASC, DIR_DESC = 0, 1
M_EOF = 1

# exported symbols declared by include/*.h (checked by tests/test_abi.py)
SYMBOLS = [
    "okv_open", "okv_open_on_stream", "okv_open_ex", "okv_close", "okv_last_error", "okv_stream", "okv_sync",
    "okv_abi_version", "okv_decode_plan", "okv_decode_blocks", "okv_decode_totals",
    "okv_point_get",
    "okv_xxh64", "okv_hash_blocks", "okv_device_alloc", "okv_device_free", "okv_host_alloc",
    "okv_host_free", "okv_memcpy", "okv_profile", "okv_profile_read", "okv_last_path",
    "okv_decode_chain",
    "okv_encode_rows", "okv_encode_close", "okv_encode_profile_read", "okv_encode_profile_reset",
    "okv_synth_rows_fixed", "okv_merge_rows",
    "okv_writer_new", "okv_writer_write_row", "okv_writer_close", "okv_writer_data",
    "okv_writer_meta", "okv_writer_num_blocks", "okv_writer_block", "okv_writer_free",
    "okv_writer_set_bloom",
    "okv_meta_fetch", "okv_meta_parse", "okv_meta_num_blocks", "okv_meta_compression",
    "okv_meta_descs", "okv_meta_first_key", "okv_meta_last_key", "okv_meta_block",
    "okv_meta_free", "okv_meta_has_bloom", "okv_meta_bloom_test", "okv_synth_segment",
    "okv_reader_open", "okv_reader_fetch_metadata", "okv_reader_load_metadata",
    "okv_reader_num_blocks", "okv_reader_read_block", "okv_reader_get_row",
    "okv_reader_get_range", "okv_reader_close", "okv_reader_free", "okv_reader_row_iter",
    "okv_iter_next", "okv_iter_seek", "okv_iter_free", "okv_reader_io_stats",
]


class OpenOpts(C.Structure):
    _fields_ = [("size", C.c_uint32), ("flags", C.c_uint32)]


class Row(C.Structure):
    _fields_ = [("key", C.c_void_p), ("key_len", C.c_uint64), ("val", C.c_void_p),
                ("val_len", C.c_uint64)]


class ReaderIO(C.Structure):
    _fields_ = [("calls", C.c_uint64), ("blocks", C.c_uint64), ("bytes_staged", C.c_uint64)]


class PointRow(C.Structure):
    """okv_point_row (include/okv_sst.h, ABI 6)."""
    _fields_ = [("status", C.c_int32), ("found", C.c_int32), ("key", C.c_void_p),
                ("key_len", C.c_uint64), ("val", C.c_void_p), ("val_len", C.c_uint64)]


class BlockDesc(C.Structure):
    _fields_ = [("offset", C.c_uint64), ("block_size", C.c_uint64),
                ("original_size", C.c_uint64), ("compressed_size", C.c_uint64)]


class DecodeOut(C.Structure):
    _fields_ = [("row_start", C.c_void_p), ("key_base", C.c_void_p), ("val_base", C.c_void_p),
                ("blk_status", C.c_void_p), ("key_off", C.c_void_p), ("key_len", C.c_void_p),
                ("val_off", C.c_void_p), ("val_len", C.c_void_p), ("key_arena", C.c_void_p),
                ("val_arena", C.c_void_p), ("row_cap", C.c_uint64), ("key_cap", C.c_uint64),
                ("val_cap", C.c_uint64), ("n_rows", C.c_uint64), ("key_bytes", C.c_uint64),
                ("val_bytes", C.c_uint64), ("n_bad_blocks", C.c_uint64)]


class Rows(C.Structure):
    _fields_ = [("key_arena", C.c_void_p), ("key_off", C.c_void_p), ("key_len", C.c_void_p),
                ("val_arena", C.c_void_p), ("val_off", C.c_void_p), ("val_len", C.c_void_p),
                ("n_rows", C.c_uint64), ("key_arena_bytes", C.c_uint64),
                ("val_arena_bytes", C.c_uint64)]


class EncodeOpts(C.Structure):
    _fields_ = [("threshold_bytes", C.c_uint64), ("block_size", C.c_uint64),
                ("compression", C.c_int), ("strict_go", C.c_int), ("bloom", C.c_void_p),
                ("bloom_len", C.c_uint64)]


class EncodeOut(C.Structure):
    _fields_ = [("seg", C.c_void_p), ("seg_cap", C.c_uint64), ("blk_first_row", C.c_void_p),
                ("blk_desc", C.c_void_p), ("blk_hash", C.c_void_p), ("blk_cap", C.c_uint64),
                ("n_blocks", C.c_uint64), ("data_bytes", C.c_uint64),
                ("meta_bytes", C.c_uint64), ("file_bytes", C.c_uint64),
                ("meta_hash", C.c_uint64), ("bad_row", C.c_uint64)]


class MergeSrc(C.Structure):
    _fields_ = [("key_arena", C.c_void_p), ("key_off", C.c_void_p), ("key_len", C.c_void_p),
                ("val_arena", C.c_void_p), ("val_off", C.c_void_p), ("val_len", C.c_void_p),
                ("row_lo", C.c_uint64), ("row_hi", C.c_uint64), ("level", C.c_int32),
                ("pad", C.c_int32)]


class MergeOpts(C.Structure):
    _fields_ = [("mode", C.c_int), ("direction", C.c_int), ("drop_tombstones", C.c_int),
                ("pad", C.c_int), ("limit", C.c_uint64), ("bound", C.c_void_p),
                ("bound_len", C.c_uint64)]


class MergeOut(C.Structure):
    _fields_ = [("src", C.c_void_p), ("row", C.c_void_p), ("key_off", C.c_void_p),
                ("key_len", C.c_void_p), ("val_off", C.c_void_p), ("val_len", C.c_void_p),
                ("key_base", C.c_void_p), ("val_base", C.c_void_p), ("row_cap", C.c_uint64),
                ("n_rows", C.c_uint64), ("n_unique", C.c_uint64), ("status", C.c_int32),
                ("pad", C.c_int32)]


_lib = None


def build(ablate=True):
    """Compile libokv_sst.so (and the ablation build) for gfx950 (hipcc) in-tree."""
    import subprocess
    subprocess.run(["make", "-s", "-j4", "-C", os.path.join(_HERE, "csrc")] +
                   (["ablate"] if ablate else []), check=True)


def lib():
    """Load libokv_sst.so (raises if it is missing: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run objectkv_amd._lib.build() "
                          "(or __graft_entry__.build())")
    # PyTorch-ROCm ships its own libamdhip64.so with the same soname
    # (libamdhip64.so.7) as /opt/rocm's.  Loading torch first makes our
    # DT_NEEDED resolve to the copy already in the process, so one HIP runtime
    # serves both (torch tensors and our kernels); loading ours first would put
    # two runtimes in the process and torch would then see no GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    p, u64, i32, u32 = C.c_void_p, C.c_uint64, C.c_int, C.c_uint32
    sig = {
        "okv_open": (p, [i32]),
        "okv_open_on_stream": (p, [i32, p]),
        "okv_open_ex": (p, [i32, p, C.POINTER(OpenOpts)]),
        "okv_close": (None, [p]),
        "okv_last_error": (C.c_char_p, [p]),
        "okv_stream": (p, [p]),
        "okv_sync": (i32, [p]),
        "okv_abi_version": (i32, []),
        "okv_decode_plan": (i32, [p, p, u64, p, u32, i32, u32, C.POINTER(u64), C.POINTER(u64),
                                  C.POINTER(u64)]),
        "okv_decode_blocks": (i32, [p, p, u64, p, u32, i32, C.POINTER(DecodeOut), u32]),
        "okv_decode_totals": (i32, [p, C.POINTER(DecodeOut)]),
        "okv_point_get": (i32, [p, p, u64, C.POINTER(BlockDesc), i32, p, u64,
                                C.POINTER(PointRow)]),
        "okv_xxh64": (u64, [p, C.c_size_t, u64]),
        "okv_hash_blocks": (i32, [p, p, u64, p, u32, p, u32]),
        "okv_device_alloc": (p, [p, C.c_size_t]),
        "okv_device_free": (None, [p, p]),
        "okv_host_alloc": (p, [C.c_size_t]),
        "okv_host_free": (None, [p]),
        "okv_memcpy": (i32, [p, p, p, C.c_size_t, i32]),
        "okv_profile": (i32, [p, i32]),
        "okv_profile_read": (i32, [p, C.POINTER(C.c_double), C.POINTER(u64)]),
        "okv_last_path": (C.c_uint32, [p]),
        "okv_decode_chain": (i32, [p, p]),
        "okv_encode_rows": (i32, [p, C.POINTER(Rows), C.POINTER(EncodeOpts),
                                  C.POINTER(EncodeOut), u32]),
        "okv_encode_close": (i32, [p, C.POINTER(EncodeOut), u32]),
        "okv_encode_profile_read": (i32, [p, C.POINTER(C.c_double), C.POINTER(u64)]),
        "okv_encode_profile_reset": (i32, [p]),
        "okv_synth_rows_fixed": (i32, [p, u64, u64, u64, u32, u32, p, p, p, p, p, p]),
        "okv_merge_rows": (i32, [p, C.POINTER(MergeSrc), u32, C.POINTER(MergeOpts),
                                 C.POINTER(MergeOut), u32]),
        "okv_writer_new": (p, [u64, u64, i32, i32]),
        "okv_writer_write_row": (i32, [p, p, C.c_size_t, p, C.c_size_t]),
        "okv_writer_close": (i32, [p, i32, C.POINTER(u64), C.POINTER(u64)]),
        "okv_writer_data": (p, [p, C.POINTER(u64)]),
        "okv_writer_meta": (p, [p, C.POINTER(u64)]),
        "okv_writer_num_blocks": (u64, [p]),
        "okv_writer_block": (i32, [p, u64, C.POINTER(BlockDesc), C.POINTER(u64),
                                   C.POINTER(p), C.POINTER(u64)]),
        "okv_writer_free": (None, [p]),
        "okv_writer_set_bloom": (None, [p, p, u64]),
        "okv_meta_fetch": (i32, [p, u64, C.c_int64, C.POINTER(p)]),
        "okv_meta_parse": (i32, [p, u64, C.POINTER(p)]),
        "okv_meta_has_bloom": (i32, [p]),
        "okv_meta_bloom_test": (i32, [p, p, C.c_size_t]),
        "okv_meta_num_blocks": (u64, [p]),
        "okv_meta_compression": (i32, [p]),
        "okv_meta_descs": (p, [p]),
        "okv_meta_first_key": (p, [p, C.POINTER(u64)]),
        "okv_meta_last_key": (p, [p, C.POINTER(u64)]),
        "okv_meta_block": (i32, [p, u64, C.POINTER(BlockDesc), C.POINTER(u64), C.POINTER(p),
                                 C.POINTER(u64)]),
        "okv_meta_free": (None, [p]),
        "okv_synth_segment": (p, [i32, u64, u64, u64, u64, u64]),
        "okv_reader_open": (p, [p, p, u64, C.c_int64]),
        "okv_reader_fetch_metadata": (i32, [p]),
        "okv_reader_load_metadata": (i32, [p, p, u64]),
        "okv_reader_num_blocks": (i32, [p, C.POINTER(u64)]),
        "okv_reader_read_block": (i32, [p, u64, C.POINTER(C.POINTER(Row)), C.POINTER(u64)]),
        "okv_reader_get_row": (i32, [p, p, C.c_size_t, C.POINTER(Row)]),
        "okv_reader_get_range": (i32, [p, p, C.c_size_t, p, C.c_size_t,
                                       C.POINTER(C.POINTER(Row)), C.POINTER(u64)]),
        "okv_reader_close": (i32, [p]),
        "okv_reader_free": (None, [p]),
        "okv_reader_row_iter": (p, [p, i32]),
        "okv_iter_next": (i32, [p, C.POINTER(Row)]),
        "okv_iter_seek": (i32, [p, p, C.c_size_t]),
        "okv_iter_free": (None, [p]),
        "okv_reader_io_stats": (i32, [p, C.POINTER(ReaderIO)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L
