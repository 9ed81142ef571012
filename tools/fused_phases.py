"""Phase breakdown of the single-pass small-block decode (okv_decode_fused_kernel)
on C2 (256 x 4 KiB blocks of 16 B / 64 B rows), from the ablation build's
per-block wall-clock stamps (okv_debug_fused_times; 100 MHz ticks).

usage: python tools/fused_phases.py        env: ABL_NBLK (256), ABL_KIND (0), ABL_BS (4096), ABL_TH (3584)
Prints, over the timed calls, the median across blocks of each phase's
duration and of each phase's end relative to the call's first block start.
"""
import ctypes
import os
import sys

os.environ.setdefault("OKV_ABLATE", "1")
import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import objectkv_amd as okv  # noqa: E402
from objectkv_amd import _lib  # noqa: E402

nblk = int(os.environ.get("ABL_NBLK", "256"))
kind = int(os.environ.get("ABL_KIND", "0"))
bs = int(os.environ.get("ABL_BS", "4096"))
th = int(os.environ.get("ABL_TH", "3584"))
w = okv.synth_segment(kind, 1, nblocks=nblk, threshold=th, block_size=bs)
seg = w.data_view()
d = w.descs()[:nblk]
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
fn = _lib.lib().okv_debug_fused_times
fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
buf = np.zeros(nblk * 8, dtype=np.uint64)
names = ["staged", "walked", "prefix", "gathered"]
dur, end = [], []
for it in range(40):
    dec.decode_device(seg_t, seg.nbytes, d_t, nblk, out, sync=True)
    if it < 5:
        continue
    assert fn(buf.ctypes.data, nblk) == 0
    t = buf.reshape(nblk, 8)[:, :5].astype(np.int64)
    t0 = t[:, 0].min()
    dur.append(np.diff(t, axis=1))
    end.append(t - t0)
dur = np.concatenate(dur) * 10 / 1000.0  # ticks -> us
end = np.concatenate(end) * 10 / 1000.0
print(f"path {dec.last_path()}  blocks {nblk}  rows {rows}  (us, median over blocks x calls)")
for i, n in enumerate(names):
    print(f"  {n:9s} phase {np.median(dur[:, i]):6.2f}  p90 {np.percentile(dur[:, i], 90):6.2f}"
          f"   ends at {np.median(end[:, i + 1]):6.2f} (max {np.percentile(end[:, i + 1], 99):6.2f})")
print(f"  block start: median {np.median(end[:, 0]):.2f} us after the first, p99 {np.percentile(end[:, 0], 99):.2f}")
