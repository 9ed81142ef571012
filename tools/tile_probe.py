"""Phase timing of okv_tile_kernel (diagnostic arm OKV_TILE=<form>d3): every
256th workgroup records s_memrealtime (100 MHz) at its start, after the
metadata trip, after issuing its DMA, after the row table, after the stage
barrier, after its own chunk pass, after the workgroup's chunk pass, and
after its stores drain.  Prints per-phase medians / p90 in microseconds.

usage: python tools/tile_probe.py [tile form, default 16x]
"""
import os as _os
_os.environ.setdefault("OKV_ABLATE", "1")  # the ablation build (its OKV_* knobs)

import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import objectkv_amd as okv  # noqa: E402
from objectkv_amd import _lib  # noqa: E402

form = sys.argv[1] if len(sys.argv) > 1 else "16xd3"
os.environ["OKV_VALUE_SWEEP"] = "8"
os.environ["OKV_TILE"] = form
nblk = int(os.environ.get("ABL_NBLK", "65536"))
w = okv.synth_segment(1, 3, nblocks=nblk, threshold=57344, block_size=65536)
seg, d = w.data_view(), w.descs()[:nblk]
dev = torch.device("cuda", 0)
dec = okv.Decoder(0, stream=torch.cuda.current_stream(dev).cuda_stream)
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
L = _lib.lib()
L.okv_debug_probe.restype = C.c_int
L.okv_debug_probe.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
tpb = 4 if form.startswith("16") else 2
n = nblk * tpb // 256
buf = np.zeros(n * 8, np.uint64)
assert L.okv_debug_probe(dec._ctx, buf.ctypes.data, buf.nbytes) == 0
T = buf.reshape(n, 8).astype(np.int64)
T = T[T[:, 0] > 0]
t0 = T[:, 0].min()
names = ["meta", "dma issue", "row table", "stage wait+barrier", "own chunks", "wg chunks",
         "stores drain"]
print(f"form {form}: {len(T)} sampled workgroups, kernel span "
      f"{(T[:, 7].max() - t0) / 100:.1f} us (first start -> last drained)")
for k, nm in enumerate(names):
    dt = (T[:, k + 1] - T[:, k]) / 100.0
    print(f"  {nm:20s} median {np.median(dt):7.2f} us  p90 {np.percentile(dt, 90):7.2f}  "
          f"max {dt.max():7.2f}")
life = (T[:, 7] - T[:, 0]) / 100.0
print(f"  {'lifetime':20s} median {np.median(life):7.2f} us  p90 {np.percentile(life, 90):7.2f}")
starts = (T[:, 0] - t0) / 100.0
print(f"  start times: p10 {np.percentile(starts, 10):.1f}  p50 {np.percentile(starts, 50):.1f}  "
      f"p90 {np.percentile(starts, 90):.1f} us")
