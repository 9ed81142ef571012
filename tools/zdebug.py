"""Diagnostics (ablation build made with `make ablate ZTRACE=1`): decode the zstd test cases through the
one-pass kernel and print each case's statuses with the last corrupt-input
exit line the kernel recorded (okv_debug_zstd_err)."""
import ctypes as C
import os
import sys

os.environ.setdefault("OKV_ABLATE", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import objectkv_amd as okv  # noqa: E402
from objectkv_amd import _lib  # noqa: E402
from oracle import pyoracle as P  # noqa: E402
from tests import zstd_cases as ZC  # noqa: E402

lib = C.CDLL(_lib.LIB_PATH)
lib.okv_debug_zstd_err.argtypes = [C.POINTER(C.c_int)]
args = sys.argv[1:]
staged = "--staged" in args
args = [a for a in args if a != "--staged"]
dec = okv.Decoder(0, flags=0 if staged else _lib.OPEN_ZSTD_ONE_PASS)
want = args or None
for name, seg, descs, _note in ZC.cases():
    if want and name not in want:
        continue
    d = np.array(descs, np.uint64).reshape(-1, 4)
    h = (C.c_int * 4)()
    lib.okv_debug_zstd_err(h)
    got = dec.decode(np.frombuffer(seg, np.uint8), d, P.COMP_ZSTD)
    lib.okv_debug_zstd_err(h)
    st = np.bincount(got.status, minlength=8)
    print(f"{name:28s} statuses {st.tolist()} last err line {h[0]} exits {h[1]} inner {h[2]} outer {h[3]}", flush=True)
dec.close()
