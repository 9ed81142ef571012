"""CPU-side checks of the product library (no GPU calls): it loads, exports
every symbol include/*.h declares, and its host-side code (XXH64, the C++
SegmentWriter mirror, metadata parsing, synthetic workloads) matches the
oracle byte for byte."""
from __future__ import annotations

import os
import re
import subprocess

import numpy as np
import pytest

import objectkv_amd as okv
from objectkv_amd import _lib
from oracle import coracle as CO
from oracle import pyoracle as P
from tests.conftest import ROOT, unpack


def _declared_symbols():
    names = set()
    for h in ("okv_sst.h", "okv_host.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(okv_[a-z0-9_]+)\s*\(", src):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    declared = _declared_symbols()
    assert declared, "no declarations parsed"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = declared - exported
    assert not missing, missing
    assert set(_lib.SYMBOLS) == declared
    L = _lib.lib()
    for name in declared:
        assert getattr(L, name)
    assert L.okv_abi_version() == 6


def test_library_has_gfx950_code_object():
    """The .so embeds an HIP fat binary with a gfx950 code object."""
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"okv_copy_kernel" in data and b"okv_count_kernel" in data


def test_product_xxh64_matches_oracle():
    rng = np.random.default_rng(5)
    for n in [0, 1, 3, 4, 7, 8, 31, 32, 33, 64, 100, 4096, 65536 + 7]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for seed in (0, 1, 2 ** 64 - 1):
            assert okv.xxh64(d, seed) == CO.xxh64(d, seed) == P.xxh64(d, seed)


def test_product_writer_matches_oracle(golden):
    for name, case in golden.items():
        if case["kind"] != "writer":
            continue
        md = P.bytes_to_metadata(bytes.fromhex(case["meta"]))
        seg = unpack(case["segment_z"])
        # rebuild the rows from the oracle decode of the golden segment
        rows = []
        for st in md.entries:
            _, rws = P.read_block(seg, st.desc(), P.COMP_NONE)
            rows += [(P._b(r.Key), P._b(r.Value)) for r in rws or []]
        opts = case["options"]
        w = okv.SegmentWriter(opts["threshold"], opts["block_size"], 0, opts["lz4"])
        for k, v in rows:
            w.WriteRow(k, v)
        flen, meta = w.Close(strict_go=True)
        assert flen == case["file_len"] and meta == bytes.fromhex(case["meta"]), name
        assert w.data().tobytes() == seg, name
        assert [list(b[1]) for b in w.blocks()] == [b["desc"] for b in case["blocks"]]
        assert [b[2] for b in w.blocks()] == [b["hash"] for b in case["blocks"]]


def test_product_writer_go_errors():
    w = okv.SegmentWriter()
    for (k, v), code in [((b"", b""), -104), ((b"k" * 65536, b""), -101)]:
        with pytest.raises(okv.OkvError) as e:
            w.WriteRow(k, v)
        assert e.value.code == code
    with pytest.raises(okv.OkvError) as e:  # Q1: strict Go semantics panic in Close
        okv.SegmentWriter().Close(strict_go=True)
    assert e.value.code == -105
    with pytest.raises(okv.OkvError) as e:  # documented divergence: no rows at all
        okv.SegmentWriter().Close(strict_go=False)
    assert e.value.code == -107
    # flush on the last row: strict -> Go panic; non-strict -> footer written
    w1, w2 = okv.SegmentWriter(threshold=10), okv.SegmentWriter(threshold=10)
    for w in (w1, w2):
        w.WriteRow(b"abcd", b"efgh")  # 14 B >= 10 -> flushed
    with pytest.raises(okv.OkvError):
        w1.Close(strict_go=True)
    flen, meta = w2.Close(strict_go=False)
    md = okv.fetch_metadata(w2.data(), flen)
    assert md.first_key == md.last_key == b"abcd" and md.descs.shape == (1, 4)
    with pytest.raises(okv.OkvError) as e:
        w2.WriteRow(b"x", b"y")
    assert e.value.code == -103


def test_product_metadata_matches_oracle(golden):
    case = golden["ref_larger_than_block"]
    seg = unpack(case["segment_z"])
    md = okv.fetch_metadata(seg, case["file_len"])
    assert md.first_key == b"a" * 511 and md.last_key == b"key199"
    assert md.descs.tolist() == [b["desc"] for b in case["blocks"]]
    assert md.hashes.tolist() == [b["hash"] for b in case["blocks"]]
    md2 = okv.bytes_to_metadata(bytes.fromhex(case["meta"]))
    assert md2.descs.tolist() == md.descs.tolist() and md2.first_keys == md.first_keys
    # corruption outcomes match the reference tests (segment_reader_test.go:727-830)
    with pytest.raises(okv.OkvError) as e:
        okv.fetch_metadata(seg + b"\x01" * 10, case["file_len"])
    assert e.value.code == -201
    shifted = b"\x07" * 10 + seg
    with pytest.raises(okv.OkvError) as e:
        okv.fetch_metadata(shifted, case["file_len"])
    assert e.value.code == -203


@pytest.mark.parametrize("gen,nb,th,bs", [("fixed", 30, 3584, 4096), ("zipf", 5, 57344, 65536)])
def test_synthetic_generator_matches_oracle(gen, nb, th, bs):
    kind = okv.sst.SYNTH_FIXED if gen == "fixed" else okv.sst.SYNTH_ZIPF
    seed = 1 if gen == "fixed" else 3
    w = okv.synth_segment(kind, seed, nblocks=nb, threshold=th, block_size=bs)
    rows = P.rows_fixed(10 ** 12, seed) if gen == "fixed" else P.rows_zipf(seed)
    seg, meta, pw = P.build_segment(rows, nblocks_target=nb, threshold=th, block_size=bs)
    assert w.data().tobytes() == seg
    assert w.meta() == meta
    assert w.num_blocks() == nb + 1
