"""Diagnostic: interleaved A/B of okv_gather_kernel variants in ONE process
(cdna_hip_programming.md §5.4 rule 24).  Usage: python tools/ablate.py 3 5 6
Variant = OKV_COPY_VARIANT value, optional ":grid" suffix for a persistent grid."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import objectkv_amd as okv  # noqa: E402

variants = sys.argv[1:] or ["3"]
nblk = int(os.environ.get("ABL_NBLK", "65536"))
rounds = int(os.environ.get("ABL_ROUNDS", "5"))
w = okv.synth_segment(1, 3, nblocks=nblk, threshold=57344, block_size=65536)
seg = w.data_view()
d = w.descs()[:nblk]
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev).cuda_stream
decs = {}
for v in variants:
    var, _, grid = v.partition(":")
    os.environ["OKV_COPY_VARIANT"] = var
    os.environ["OKV_GATHER_GRID"] = grid or "0"
    decs[v] = okv.Decoder(0, stream=stream)
seg_t = torch.empty(seg.nbytes + 64, dtype=torch.uint8, device=dev)
seg_t[:seg.nbytes].copy_(torch.from_numpy(seg))
d_t = torch.from_numpy(d.view(np.int64).copy()).to(dev)
first = decs[variants[0]]
rows, kb, vb = first.plan_device(seg_t, seg.nbytes, d_t, nblk)
out = {k: torch.empty(n, dtype=t, device=dev) for k, n, t in [
    ("row_start", nblk + 1, torch.int64), ("key_base", nblk, torch.int64),
    ("val_base", nblk, torch.int64), ("status", nblk, torch.int32),
    ("key_off", rows, torch.int64), ("key_len", rows, torch.int16),
    ("val_off", rows, torch.int64), ("val_len", rows, torch.int32),
    ("key_arena", kb, torch.uint8), ("val_arena", vb, torch.uint8)]}
res = {v: [] for v in variants}
for v, dec in decs.items():  # warm up
    for _ in range(2):
        dec.decode_device(seg_t, seg.nbytes, d_t, nblk, out, sync=False)
torch.cuda.synchronize()
for r in range(rounds):
    for v, dec in decs.items():
        dec.profile(True)
        for _ in range(5):
            dec.decode_device(seg_t, seg.nbytes, d_t, nblk, out, sync=False)
        ms, n = dec.profile_read()
        dec.profile(False)
        res[v].append((ms["copy"] / n, ms["count"] / n))
for v in variants:
    cp = sorted(x[0] for x in res[v])
    ct = sorted(x[1] for x in res[v])
    print(f"variant={v} copy_ms median={cp[len(cp) // 2]:.4f} min={cp[0]:.4f} "
          f"count_ms median={ct[len(ct) // 2]:.4f}", flush=True)
