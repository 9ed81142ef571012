"""Time one C3-style decode configuration with a given build of the library
(A/B of two builds: run this alternately for each .so, one process per run,
so that both builds see the same box).

usage: python tools/ab_lib.py <path to libokv_sst*.so> [label]
env:   ABL_NBLK (65536), ABL_ROUNDS (5), ABL_STEPS (10), ABL_KIND (1), ABL_BS (65536),
       ABL_TH (57344), ABL_FLAGS (okv_open_opts.flags, 0)
Prints one JSON line: per-pass ms (HIP events, median over rounds), the
one-at-a-time decode step (host clock, median) and its roofline fraction.
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from objectkv_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
label = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(sys.argv[1])
import objectkv_amd as okv  # noqa: E402

nblk = int(os.environ.get("ABL_NBLK", "65536"))
rounds = int(os.environ.get("ABL_ROUNDS", "5"))
steps = int(os.environ.get("ABL_STEPS", "10"))
kind = int(os.environ.get("ABL_KIND", "1"))
bs = int(os.environ.get("ABL_BS", "65536"))
th = int(os.environ.get("ABL_TH", "57344"))
w = okv.synth_segment(kind, 3, nblocks=nblk, threshold=th, block_size=bs)
seg = w.data_view()
d = w.descs()[:nblk]
dev = torch.device("cuda", 0)
dec = okv.Decoder(0, stream=torch.cuda.current_stream(dev).cuda_stream,
                  flags=int(os.environ.get("ABL_FLAGS", "0")))
seg_t = torch.empty(seg.nbytes + 64, dtype=torch.uint8, device=dev)
seg_t[:seg.nbytes].copy_(torch.from_numpy(seg))
d_t = torch.from_numpy(d.view(np.int64).copy()).to(dev)
rows, kb, vb = dec.plan_device(seg_t, seg.nbytes, d_t, nblk)
out = {k: torch.empty(n, dtype=t, device=dev) for k, n, t in [
    ("row_start", nblk + 1, torch.int64), ("key_base", nblk, torch.int64),
    ("val_base", nblk, torch.int64), ("status", nblk, torch.int32),
    ("key_off", rows, torch.int64), ("key_len", rows, torch.int16),
    ("val_off", rows, torch.int64), ("val_len", rows, torch.int32),
    ("key_arena", kb, torch.uint8), ("val_arena", vb, torch.uint8)]}
for _ in range(3):
    dec.decode_device(seg_t, seg.nbytes, d_t, nblk, out, sync=True)
res = []
for r in range(rounds):
    dec.profile(True)
    for _ in range(5):
        dec.decode_device(seg_t, seg.nbytes, d_t, nblk, out, sync=False)
    ms, n = dec.profile_read()
    dec.profile(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        dec.decode_device(seg_t, seg.nbytes, d_t, nblk, out, sync=False)
    torch.cuda.synchronize()
    res.append(((ms["count"] + ms["scan"]) / n, ms["copy"] / n,
                (time.perf_counter() - t0) * 1e3 / steps))
alg = int(d[:, 2].sum()) + kb + vb + rows * 22 + nblk * 28
med = [sorted(x[k] for x in res)[len(res) // 2] for k in range(3)]
print(json.dumps({"lib": label, "count_scan_ms": round(med[0], 4), "pass3_ms": round(med[1], 4),
                  "step_ms": round(med[2], 4), "step_min_ms": round(min(x[2] for x in res), 4),
                  "frac_pass3": round(alg / med[1] / 1e6 / 8000, 4),
                  "frac_step": round(alg / med[2] / 1e6 / 8000, 4)}), flush=True)
