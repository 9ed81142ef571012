"""Diagnostic A/B of pass-3 launch forms, interleaved in ONE process
(cdna_hip_programming.md §5.4 rule 24), with a bit-equality check of every
output array between the arms.

usage: python tools/ablate.py [arm ...]     arm = <threads>[:<grid>[:<staged>]]  (staged = OKV_GATHER_STAGED: 0 = global-window pass 3)
  fused = OKV_DECODE_FUSED (0: small blocks decode in 3 launches)  arm = <t>:<grid>:<staged>:<fused>
  threads = 64 | 256 | auto (OKV_GATHER_THREADS), grid = OKV_GATHER_GRID (0: one per block)
env:   ABL_NBLK (65536), ABL_ROUNDS (5), ABL_KIND (1 = Zipf C3, 0 = fixed C2),
       ABL_BS (65536), ABL_TH (57344)
"""
import os as _os
_os.environ.setdefault("OKV_ABLATE", "1")  # the ablation build (its OKV_* knobs)

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import objectkv_amd as okv  # noqa: E402

arms = sys.argv[1:] or ["auto", "64"]
nblk = int(os.environ.get("ABL_NBLK", "65536"))
rounds = int(os.environ.get("ABL_ROUNDS", "5"))
kind = int(os.environ.get("ABL_KIND", "1"))
bs = int(os.environ.get("ABL_BS", "65536"))
th = int(os.environ.get("ABL_TH", "57344"))
w = okv.synth_segment(kind, 3, nblocks=nblk, threshold=th, block_size=bs)
seg = w.data_view()
d = w.descs()[:nblk]
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev).cuda_stream
decs = {}
for a in arms:
    thr, _, rest = a.partition(":")
    grid, _, rest = rest.partition(":")
    staged, _, fused = rest.partition(":")
    if fused:
        os.environ["OKV_DECODE_FUSED"] = fused
    else:
        os.environ.pop("OKV_DECODE_FUSED", None)
    os.environ["OKV_GATHER_GRID"] = grid or "0"
    if staged:
        os.environ["OKV_GATHER_STAGED"] = staged
    else:
        os.environ.pop("OKV_GATHER_STAGED", None)
    if thr in ("64", "256"):
        os.environ["OKV_GATHER_THREADS"] = thr
    else:
        os.environ.pop("OKV_GATHER_THREADS", None)
    decs[a] = okv.Decoder(0, stream=stream)
seg_t = torch.empty(seg.nbytes + 64, dtype=torch.uint8, device=dev)
seg_t[:seg.nbytes].copy_(torch.from_numpy(seg))
d_t = torch.from_numpy(d.view(np.int64).copy()).to(dev)
first = decs[arms[0]]
rows, kb, vb = first.plan_device(seg_t, seg.nbytes, d_t, nblk)


def new_out():
    return {k: torch.full((n,), 0x5A, dtype=t, device=dev) for k, n, t in [
        ("row_start", nblk + 1, torch.int64), ("key_base", nblk, torch.int64),
        ("val_base", nblk, torch.int64), ("status", nblk, torch.int32),
        ("key_off", rows, torch.int64), ("key_len", rows, torch.int16),
        ("val_off", rows, torch.int64), ("val_len", rows, torch.int32),
        ("key_arena", kb, torch.uint8), ("val_arena", vb, torch.uint8)]}


outs = {a: new_out() for a in arms}
for a, dec in decs.items():  # warm up + equality between arms
    for _ in range(2):
        dec.decode_device(seg_t, seg.nbytes, d_t, nblk, outs[a], sync=False)
torch.cuda.synchronize()
ref = outs[arms[0]]
for a in arms[1:]:
    bad = [k for k in ref if not torch.equal(ref[k], outs[a][k])]
    print(f"arm {a} vs {arms[0]}: {'EQUAL' if not bad else 'DIFFER ' + ','.join(bad)}",
          flush=True)
del outs
out = new_out()
res = {a: [] for a in arms}
for r in range(rounds):
    for a, dec in decs.items():
        dec.profile(True)
        for _ in range(5):
            dec.decode_device(seg_t, seg.nbytes, d_t, nblk, out, sync=False)
        ms, n = dec.profile_read()
        dec.profile(False)
        res[a].append((ms["copy"] / n, ms["count"] / n))
alg = int(d[:, 2].sum()) + kb + vb + rows * 22 + nblk * 28
for a in arms:
    cp = sorted(x[0] for x in res[a])
    ct = sorted(x[1] for x in res[a])
    med = cp[len(cp) // 2]
    print(f"arm={a:16s} gather_ms median={med:.4f} min={cp[0]:.4f} "
          f"count_ms median={ct[len(ct) // 2]:.4f} sum={med + ct[len(ct) // 2]:.4f}  alg {alg / med / 1e6:.0f} GB/s "
          f"frac {alg / med / 1e6 / 8000:.3f}", flush=True)
