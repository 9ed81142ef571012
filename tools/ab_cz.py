"""Time the CZ decode (16 384 x 64 KiB-raw zstd blocks, libzstd level 3) with a
given build of the library: A/B of two builds, run alternately, one process
per run, so both see the same box.  Device-resident, one decode at a time,
HIP events per pass (zstd stage = the 'zstd' slot of okv_profile_read).

usage: python tools/ab_cz.py <libokv_sst*.so> [label]
Prints one JSON line."""
import json
import os
import statistics
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
from tools.zstd_gen import text_zstd_segment  # noqa: E402

nblk = int(os.environ.get("ABZ_NBLK", "16384"))
seg, descs, orig = text_zstd_segment(nblk, 5)
dev = torch.device("cuda", 0)
dec = okv.Decoder(0, stream=torch.cuda.current_stream(dev).cuda_stream)
seg_np = np.asarray(seg)
seg_t = torch.empty(seg_np.nbytes + 64, dtype=torch.uint8, device=dev)
seg_t[:seg_np.nbytes].copy_(torch.from_numpy(seg_np))
d = np.ascontiguousarray(descs, np.uint64).reshape(-1, 4)
d_t = torch.from_numpy(d.view(np.int64).copy()).to(dev)
rows, kb, vb = dec.plan_device(seg_t, seg_np.nbytes, d_t, nblk, compression=okv.sst.COMP_ZSTD)
out = {k: torch.empty(n, dtype=t, device=dev) for k, n, t in [
    ("row_start", nblk + 1, torch.int64), ("key_base", nblk, torch.int64),
    ("val_base", nblk, torch.int64), ("status", nblk, torch.int32),
    ("key_off", rows, torch.int64), ("key_len", rows, torch.int16),
    ("val_off", rows, torch.int64), ("val_len", rows, torch.int32),
    ("key_arena", kb, torch.uint8), ("val_arena", vb, torch.uint8)]}
kw = dict(compression=okv.sst.COMP_ZSTD)
for _ in range(3):
    dec.decode_device(seg_t, seg_np.nbytes, d_t, nblk, out, sync=True, **kw)
assert int(out["status"].max()) == 0
stage, step = [], []
for r in range(5):
    dec.profile(True)
    for _ in range(4):
        dec.decode_device(seg_t, seg_np.nbytes, d_t, nblk, out, sync=True, **kw)
    ms, n = dec.profile_read()
    dec.profile(False)
    stage.append(ms["zstd"] / n)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(4):
        dec.decode_device(seg_t, seg_np.nbytes, d_t, nblk, out, sync=True, **kw)
    torch.cuda.synchronize()
    step.append((time.perf_counter() - t0) / 4 * 1e3)
print(json.dumps({"lib": label, "zstd_stage_ms": round(statistics.median(stage), 4),
                  "step_ms": round(statistics.median(step), 4),
                  "stage_all": [round(x, 4) for x in stage]}), flush=True)
