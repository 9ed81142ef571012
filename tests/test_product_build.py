"""The product library ships only the kernels the product paths launch and reads
no environment (the measured alternatives and their OKV_* knobs live in the
ablation build, -DOKV_ABLATE).  Checked on the built files, no GPU needed:
kernel symbol names of the embedded gfx950 code object and the string
literals of the host code are plain bytes in the shared object."""
from __future__ import annotations

import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRODUCT = os.path.join(ROOT, "objectkv_amd", "libokv_sst.so")
ABLATE = os.path.join(ROOT, "objectkv_amd", "libokv_sst_ablate.so")

# kernels of the measured alternative forms: ablation build only
ABLATION_ONLY = [b"okv_value_sweep_kernel", b"okv_rows_kernel", b"okv_gather_staged_kernel",
                 b"okv_gather_kernel", b"okv_tile_kernel_w7", b"okv_scan_kernel",
                 b"okv_tile_kernel_diag",
                 # round 4's measured-and-not-kept forms
                 b"okv_decode_stream_kernel", b"okv_enc_plan_kernel", b"fused_prefix_lookback",
                 # round 6's
                 b"okv_group_kernel", b"okv_tile_kernel_skip"]
KNOBS = [b"OKV_GATHER_THREADS", b"OKV_GATHER_GRID", b"OKV_DECODE_FUSED", b"OKV_GATHER_STAGED",
         b"OKV_VALUE_SWEEP", b"OKV_TILE", b"OKV_ZSTD_GENERAL", b"OKV_ZSTD_PROF",
         b"OKV_ENC_VARIANT", b"OKV_ENC_IMAGE", b"OKV_DECODE_PIECES", b"OKV_DECODE_STREAM",
         b"OKV_SMALL_PIECE_MB", b"OKV_COUNT_PREFETCH", b"OKV_ENC_ONEPASS", b"OKV_ENC_META_FUSED",
         b"OKV_ZSTD_HUF_BLOCKS", b"OKV_DECODE_GROUP"]


def _bytes(path):
    if not os.path.exists(path):
        pytest.skip(f"{os.path.basename(path)} not built")
    with open(path, "rb") as f:
        return f.read()


def test_product_ships_one_tile_pass_form():
    data = _bytes(PRODUCT)
    forms = set(re.findall(rb"_ZN3okv15okv_tile_kernelI[A-Za-z0-9_]+", data))
    assert forms == {b"_ZN3okv15okv_tile_kernelILj16384ELj256ELb1EEEvNS_10CopyParamsEjj"}, forms
    for name in ABLATION_ONLY:
        assert name not in data, name
    # the shipping kernels are all there
    for name in (b"okv_count_kernel", b"okv_gather_small_kernel", b"okv_decode_fused_kernel",
                 b"okv_copy_kernel", b"okv_index_kernel", b"okv_hash_kernel",
                 b"okv_enc_pack_lds_kernel", b"okv_zstd_seq_kernel", b"okv_zstd_exec_kernel",
                 b"okv_merge_rank"):
        assert name in data, name


def test_product_source_holds_only_product_kernels():
    """The shipped source is the shipped code: the measured alternatives and
    the tile pass's diagnostic arms live in okv_decode_ablate.inc, which
    okv_decode.hip includes only under -DOKV_ABLATE."""
    src = open(os.path.join(ROOT, "objectkv_amd", "csrc", "okv_decode.hip")).read()
    for name in ("okv_value_sweep_kernel", "okv_rows_kernel", "okv_gather_staged_kernel",
                 "okv_gather_kernel", "tile_pass_diag", "okv_tile_kernel_diag"):
        assert not re.search(r"void\s+" + name + r"\s*\(", src), name
    for arm in ("kProbe", "kDirect", "kChunk", "kDiag == 1", "kDiag == 4", "kDiag == 5"):
        assert arm not in src, arm
    for inc_name in ("okv_decode_ablate.inc", "okv_decode_ablate_host.inc",
                     "okv_decode_ablate_lb.inc"):
        inc = src.index(f'#include "{inc_name}"')
        assert src.rfind("#ifdef OKV_ABLATE", 0, inc) > src.rfind("#endif", 0, inc), inc_name
    # round 4's arms are in the includes, not in the product translation units
    for name in ("okv_decode_stream_kernel", "launch_plan_pieces", "launch_count_piece",
                 "piece_params", "okv_group_kernel", "ensure_group"):
        assert not re.search(r"\b" + name + r"\s*\([^;]*\)\s*\{", src), name
    enc = open(os.path.join(ROOT, "objectkv_amd", "csrc", "okv_encode.hip")).read()
    for name in ("okv_enc_plan_kernel", "enc_plan_fast"):
        assert not re.search(r"\b" + name + r"\s*\([^;]*\)\s*\{", enc), name
    for inc_name in ("okv_encode_ablate.inc", "okv_encode_ablate_host.inc"):
        inc = enc.index(f'#include "{inc_name}"')
        assert enc.rfind("#ifdef OKV_ABLATE", 0, inc) > enc.rfind("#endif", 0, inc), inc_name


def test_product_reads_no_environment():
    data = _bytes(PRODUCT)
    for knob in KNOBS:
        assert knob not in data, knob
    dyn = subprocess.run(["nm", "-D", "--undefined-only", PRODUCT], capture_output=True,
                         text=True, check=True).stdout
    assert not re.search(r"\bgetenv\b", dyn), "the product library imports getenv"


def test_ablation_build_carries_the_alternatives():
    data = _bytes(ABLATE)
    for name in (b"okv_value_sweep_kernel", b"okv_gather_staged_kernel", b"okv_tile_kernel_w7",
                 b"okv_decode_stream_kernel", b"okv_enc_plan_kernel"):
        assert name in data, name
    for knob in (b"OKV_VALUE_SWEEP", b"OKV_TILE", b"OKV_ZSTD_PROF"):
        assert knob in data, knob
