"""Host-mode decodes of small batches (GetRange / RowIter-window shapes):
the point path (one okv_point_kernel launch reading and writing the pinned
slab) against a context opened with OKV_OPEN_NO_POINT (device staging: H2D,
count + pass 3, D2H).  ADVICE r5: the point path is the default for every
host-mode call of up to 16 blocks / 1 MiB; this measures 1, 4 and 16 blocks
of 64 KiB (C3 Zipf rows) and of 4 KiB (C2 fixed rows).

usage: python tools/point_batch_ab.py [calls]     prints one JSON line per shape
Median wall time per okv_decode_blocks call (outputs preallocated, host
buffers), both contexts on one stream-less device, alternating; each batch's
outputs compared equal between the two contexts first."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import objectkv_amd as okv  # noqa: E402
from objectkv_amd import _lib  # noqa: E402
from objectkv_amd.sst import DecodeOut, _ptr  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 300
L = _lib.lib()


def batch(kind, bs, th, nb, seed=3):
    w = okv.synth_segment(kind, seed, nblocks=64, threshold=th, block_size=bs)
    seg = np.frombuffer(w.data_view(), np.uint8)
    d = w.descs()[:64].astype(np.uint64)
    b0 = 7
    sub = d[b0:b0 + nb].copy()
    lo, hi = int(sub[0, 0]), int(sub[-1, 0] + sub[-1, 1])
    sub[:, 0] -= lo
    return seg[lo:hi].copy(), np.ascontiguousarray(sub)  # (copies: w owns seg)


def outputs(s, d):
    n = d.shape[0]
    R = int(d[:, 1].sum()) // 6 + 1
    A = int(d[:, 1].sum()) + 16 * n + 16
    o = dict(status=np.zeros(n, np.int32), row_start=np.zeros(n + 1, np.uint64),
             key_base=np.zeros(n, np.uint64), val_base=np.zeros(n, np.uint64),
             key_off=np.zeros(R, np.uint64), key_len=np.zeros(R, np.uint16),
             val_off=np.zeros(R, np.uint64), val_len=np.zeros(R, np.uint32),
             key_arena=np.zeros(A, np.uint8), val_arena=np.zeros(A, np.uint8))
    out = DecodeOut(_ptr(o["row_start"]), _ptr(o["key_base"]), _ptr(o["val_base"]),
                    _ptr(o["status"]), _ptr(o["key_off"]), _ptr(o["key_len"]),
                    _ptr(o["val_off"]), _ptr(o["val_len"]), _ptr(o["key_arena"]),
                    _ptr(o["val_arena"]), R, A, A, 0, 0, 0, 0)
    return o, out


decs = {"point": okv.Decoder(0), "no_point": okv.Decoder(0, flags=_lib.OPEN_NO_POINT)}
for name, kind, bs, th in (("64KiB_zipf", 1, 65536, 57344), ("4KiB_fixed", 0, 4096, 3584)):
    for nb in (1, 4, 16):
        s, d = batch(kind, bs, th, nb)
        res, got, outs = {}, {}, {}
        for k, dec in decs.items():
            o, out = outputs(s, d)
            rc = L.okv_decode_blocks(dec._ctx, _ptr(s), s.size, _ptr(d), d.shape[0], 0,
                                     C.byref(out), 0)
            assert rc == 0, (k, rc)
            got[k] = (o, out.n_rows, out.key_bytes, out.val_bytes)
            outs[k] = out
            res[k] = []
        a, b = got["point"], got["no_point"]
        assert a[1:] == b[1:], (a[1:], b[1:])
        n = a[1]
        for f in ("status", "key_len", "val_len", "key_off", "val_off"):
            m = d.shape[0] if f == "status" else n
            assert np.array_equal(a[0][f][:m], b[0][f][:m]), f
        assert bytes(a[0]["val_arena"][:a[3]]) == bytes(b[0]["val_arena"][:b[3]])
        for _ in range(calls):
            for k, dec in decs.items():
                t0 = time.perf_counter()
                rc = L.okv_decode_blocks(dec._ctx, _ptr(s), s.size, _ptr(d), d.shape[0], 0,
                                         C.byref(outs[k]), 0)
                res[k].append((time.perf_counter() - t0) * 1e6)
                assert rc == 0
        med = {k: round(float(np.median(v)), 1) for k, v in res.items()}
        print(json.dumps({"shape": name, "blocks": nb, "bytes": int(s.size),
                          "median_us": med, "calls": calls}), flush=True)
