"""Generate tests/golden/golden.json from the Python restatement
(oracle/pyoracle.py).

The Go reference cannot run in this image (no Go toolchain, no module cache;
SURVEY.md §8c), so these vectors come from the restatement; the restatement
itself is pinned against every known answer the reference's own tests assert
(tests/test_oracle.py::test_reference_known_answers_*).  Each case records the
inputs (or the deterministic generator that makes them) and the expected
outputs: block index entries, decoded rows and, for the larger synthetic
cases, SHA-256 digests of the product-layout SoA arrays.

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import base64
import hashlib
import json
import os
import struct
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import pyoracle as P  # noqa: E402


def hx(b):
    return None if b is None else bytes(b).hex()


def rowval(b):
    """Row key/value as hex (<= 64 bytes) or "sha256:<digest>:<len>"."""
    if b is None:
        return None
    b = bytes(b)
    return b.hex() if len(b) <= 64 else f"sha256:{hashlib.sha256(b).hexdigest()}:{len(b)}"


def packed(b):
    """Segment bytes as base64(zlib(bytes))."""
    return base64.b64encode(zlib.compress(bytes(b), 9)).decode()


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def soa_digests(seg, descs, comp, index_only):
    import numpy as np
    o = P.decode_soa(seg, descs, comp, index_only)
    dig = {"row_start": sha(np.array(o["row_start"], np.uint64).tobytes()),
           "status": sha(np.array(o["status"], np.int32).tobytes()),
           "key_off": sha(np.array(o["key_off"], np.uint64).tobytes()),
           "key_len": sha(np.array(o["key_len"], np.uint16).tobytes()),
           "val_off": sha(np.array(o["val_off"], np.uint64).tobytes()),
           "val_len": sha(np.array(o["val_len"], np.uint32).tobytes()),
           "n_rows": o["row_start"][-1]}
    if not index_only:
        dig.update(key_base=sha(np.array(o["key_base"], np.uint64).tobytes()),
                   val_base=sha(np.array(o["val_base"], np.uint64).tobytes()),
                   key_arena=sha(o["key_arena"]), val_arena=sha(o["val_arena"]),
                   key_bytes=len(o["key_arena"]), val_bytes=len(o["val_arena"]))
    return dig


def writer_case(name, rows, threshold=3584, block_size=4096, lz4=False):
    w = P.SegmentWriter(P.SegmentWriterOptions(threshold, block_size, LZ4Compression=lz4))
    for k, v in rows:
        w.WriteRow(k, v)
    flen, meta = w.Close()
    seg = bytes(w.external)
    md = P.bytes_to_metadata(meta)
    blocks = []
    for st in md.entries:
        status, rws = P.read_block(seg, st.desc(), md.compression)
        blocks.append({"first_key": hx(st.FirstKey), "desc": list(st.desc()), "hash": st.Hash,
                       "status": status,
                       "rows": [[rowval(r.Key), rowval(r.Value)] for r in (rws or [])]})
    return {"name": name, "kind": "writer",
            "options": {"threshold": threshold, "block_size": block_size, "lz4": lz4},
            "file_len": flen, "segment_z": packed(seg), "meta": hx(meta), "compression": md.compression,
            "first_key": hx(md.FirstKey), "last_key": hx(md.LastKey), "blocks": blocks}


def synth_case(name, gen, seed, nblocks, threshold, block_size):
    rows = P.rows_fixed(10 ** 12, seed) if gen == "fixed" else P.rows_zipf(seed)
    seg, meta, w = P.build_segment(rows, nblocks_target=nblocks, threshold=threshold,
                                   block_size=block_size)
    md = P.bytes_to_metadata(meta)
    descs = [st.desc() for st in md.entries][:nblocks]
    return {"name": name, "kind": "synth", "gen": gen, "seed": seed, "nblocks": nblocks,
            "threshold": threshold, "block_size": block_size, "segment_sha256": sha(seg),
            "segment_len": len(seg), "meta_sha256": sha(meta), "n_index": len(md.entries),
            "hashes_first": [st.Hash for st in md.entries[:4]],
            "decode_blocks": nblocks,
            "full": soa_digests(seg, descs, md.compression, False),
            "index": soa_digests(seg, descs, md.compression, True)}


def rec(k, v, klen=None, vlen=None):
    klen = len(k) if klen is None else klen
    vlen = len(v) if vlen is None else vlen
    return struct.pack("<HI", klen, vlen) + k + v


def crafted_case():
    """Hand-made blocks exercising the decode loop's edge semantics
    (segment_reader.go:295-355, :489-512) in one buffer."""
    blocks = []
    seg = bytearray()

    def add(body, block_size, orig, note, pad_to=None):
        off = len(seg)
        data = bytes(body) + bytes(block_size - len(body))
        seg.extend(data)
        blocks.append({"note": note, "desc": [off, block_size, orig, 0]})

    # 0: normal two records
    b = rec(b"k1", b"v1") + rec(b"k22", b"value22")
    add(b, 64, len(b), "two records")
    # 1: empty value (nil, Q4) and empty key (decoder allows it)
    b = rec(b"key", b"") + rec(b"", b"val") + rec(b"", b"")
    add(b, 64, len(b), "nil key/value")
    # 2: last record runs past OriginalSize into padding (Q5) -- still decoded
    b = rec(b"a", b"b") + rec(b"long", b"x" * 20)
    add(b, 64, 8, "record past OriginalSize")
    # 3: value overruns the buffer -> mustReadBytes panic
    b = rec(b"a", b"", vlen=100)
    add(b, 32, len(b), "value overrun (panic)")
    # 4: header truncated at the buffer end -> panic
    b = rec(b"abc", b"de")
    add(b + b"\x01\x00", len(b) + 2, len(b) + 2, "truncated header (panic)")
    # 5: OriginalSize 0 -> no rows
    add(rec(b"zz", b"yy"), 32, 0, "OriginalSize 0")
    # 6: key length 0xFFFF within a large block
    b = rec(b"K" * 65535, b"V" * 3)
    add(b, 65536 + 64, len(b), "max u16 key")
    # 7: block larger than the 64 KiB LDS stage (global path)
    b = rec(b"big", b"Z" * 70000) + rec(b"next", b"n")
    add(b, 72000, len(b), "block > 64 KiB")
    # 8: many tiny records (more rows than one row-table batch)
    b = b"".join(rec(bytes([i % 251 + 1]), b"") for i in range(600))
    add(b, 8192, len(b), "600 tiny records")
    # 8b: more rows than the fast path holds (> 1024): general batched path
    b = b"".join(rec(bytes([i % 7 + 1]) * (i % 3), bytes([i % 5]) * (i % 4)) for i in range(1500))
    add(b, 16384, len(b), "1500 records (> fast-path rows)")
    # 9: unaligned block offset (offset % 16 == 3)
    seg.extend(b"\xAA" * 3)
    b = rec(b"unaligned", b"offset!") + rec(b"k2", b"v" * 37)
    add(b, 80, len(b), "unaligned offset")
    # 10: short read (block extends past the segment end) -> Go error
    blocks.append({"note": "short read", "desc": [len(seg) - 10, 64, 10, 0]})
    # 11: offset beyond the segment -> io.EOF error
    blocks.append({"note": "offset past end", "desc": [len(seg) + 100, 16, 4, 0]})
    # 12: zero-length block at a valid offset, OriginalSize 0
    blocks.append({"note": "empty block", "desc": [0, 0, 0, 0]})
    # Go's int() conversions (segment_reader.go:303-340)
    # 13/14: int(OriginalSize) < 0 -> the loop runs no iteration: nil rows, no error
    blocks.append({"note": "OriginalSize 2^63", "desc": [0, 64, 1 << 63, 0]})
    blocks.append({"note": "OriginalSize 2^64-1", "desc": [0, 64, (1 << 64) - 1, 0]})
    # 15/16: make([]byte, BlockSize) above maxAlloc (2^48) / negative as int -> panic
    blocks.append({"note": "BlockSize 2^48+1 (makeslice panic)", "desc": [0, (1 << 48) + 1, 8, 0]})
    blocks.append({"note": "BlockSize 2^63 (makeslice panic)", "desc": [0, 1 << 63, 8, 0]})
    # 17: BlockSize == maxAlloc is allocatable: the read is short
    blocks.append({"note": "BlockSize 2^48 (short)", "desc": [0, 1 << 48, 8, 0]})
    # 18: make panics before the read would see io.EOF
    blocks.append({"note": "past end, BlockSize 2^50", "desc": [len(seg) + 7, 1 << 50, 4, 0]})
    # 19: the Seek error (negative int64 Offset) comes before make
    blocks.append({"note": "Offset 2^63+1, BlockSize 2^60", "desc": [(1 << 63) + 1, 1 << 60, 4, 0]})
    seg_b = bytes(seg)
    for bl in blocks:
        st, rws = P.read_block(seg_b, bl["desc"], P.COMP_NONE)
        bl["status"] = st
        bl["rows"] = [[rowval(r.Key), rowval(r.Value)] for r in (rws or [])]
        st_lz4, rws_lz4 = P.read_block(seg_b, bl["desc"], P.COMP_LZ4)
        bl["status_lz4"] = st_lz4
        bl["rows_lz4"] = [[rowval(r.Key), rowval(r.Value)] for r in (rws_lz4 or [])]
    return {"name": "crafted_edges", "kind": "crafted", "segment_z": packed(seg_b), "blocks": blocks}


def writer_inputs():
    """(name, rows, writer options) of the reference test inputs
    (sst/segment_reader_test.go, segment_writer_test.go, segment_row_iter_test.go);
    also the device-encode parity inputs (tests/test_encode_gpu.py)."""
    r200 = [(b"key%03d" % i, b"value%03d" % i) for i in range(200)]
    big = [(b"a" * 511, b"b" * 10000)] + [(b"key%d" % i, b"value%d" % i) for i in range(200)]
    return [
        ("ref_read_uncompressed_200", r200, {}),  # segment_reader_test.go:12-269
        ("ref_blank_value", r200 + [(b"key200", b"")], {}),  # :271-326
        ("ref_single_row", r200[:1], {}),  # :328-511
        ("ref_larger_than_block", big, {}),  # segment_writer_test.go:73-112
        ("ref_writer_no_compression",
         [(b"key%d" % i, b"value%d" % i) for i in range(200)], {}),  # :12-40
        ("ref_rollover_no_bloom",
         [(b"key%03d" % i, b"value%03d-I-SHOULD-NOT-SHOW" % i) for i in range(1, 200, 2)]
         + [(b"key900", b"value900")], {}),  # segment_row_iter_test.go:380-450
        ("lz4_flag_200", r200, {"lz4": True}),  # Q7
    ]


def main(out_path=os.path.join(HERE, "golden.json")):
    cases = []
    # reference test inputs (sst/segment_reader_test.go, segment_writer_test.go,
    # segment_row_iter_test.go)
    for name, rows, kw in writer_inputs():
        cases.append(writer_case(name, rows, **kw))
    cases.append(synth_case("c2_fixed_256x4k", "fixed", 1, 256, 3584, 4096))
    cases.append(synth_case("c3_zipf_8x64k", "zipf", 3, 8, 57344, 65536))
    cases.append(crafted_case())
    with open(out_path, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (oracle/pyoracle.py)",
                   "cases": cases}, f, indent=1)
    print("wrote", len(cases), "cases")


if __name__ == "__main__":
    main(*sys.argv[1:2])
