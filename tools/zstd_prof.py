"""zstd decode diagnostics on the CZ workload: phase cycle counters
(OKV_ZSTD_PROF).  ZP_LIB=<path to a libokv_sst build> times that build instead."""
import os as _os
_os.environ.setdefault("OKV_ABLATE", "1")  # the ablation build (its OKV_* knobs)

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("ZP_LIB"):  # A/B of library builds: one process per build
    from objectkv_amd import _lib  # noqa: E402
    _lib.LIB_PATH = os.path.abspath(os.environ["ZP_LIB"])
import objectkv_amd as okv  # noqa: E402
from tools.zstd_gen import text_zstd_segment  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
seg, descs, orig = text_zstd_segment(n, 5)
dec = okv.Decoder(0)
for stage in ("1",):
    os.environ.pop("OKV_ZSTD_GENERAL", None)
    os.environ.pop("OKV_ZSTD_PROF", None)
    dec.profile(True)
    got = dec.decode(seg, descs, compression=okv.sst.COMP_ZSTD)
    ms, calls = dec.profile_read()
    assert int(got.status.max()) == 0
    print(f"stage={stage}: zstd+count {ms['count']:.2f} ms, gather {ms['copy']:.2f} ms, "
          f"{orig / ms['count'] / 1e6:.1f} GB/s decompressed", flush=True)
for stage in ("1",):
    os.environ.pop("OKV_ZSTD_GENERAL", None)
    os.environ["OKV_ZSTD_PROF"] = "1"
    print("stage", stage, flush=True)
    dec.decode(seg, descs, compression=okv.sst.COMP_ZSTD)
