"""A/B of the large-block pass-3 forms, interleaved in ONE process, with a
bit-equality check of every output array between the arms (and against the
oracle for the first arm when ABL_VERIFY=1).

usage: python tools/ablate_tile.py [arm ...]
  arm = <value_sweep>[:<tile>]   value_sweep = OKV_VALUE_SWEEP (7 = round-2 row pass +
                                 value sweep, 8 = okv_tile_kernel); tile = OKV_TILE
                                 (4 | 8 | 16 KiB, suffix x = XCD-grouped tiles)
env:   ABL_NBLK (65536), ABL_ROUNDS (5), ABL_KIND (1 = Zipf C3), ABL_BS (65536),
       ABL_TH (57344), ABL_STEPS (10)
Prints per arm: pass-3 ms (HIP events), count + scan ms, and the whole
one-at-a-time decode step (host clock, no events) with its roofline fraction.
"""
import os as _os
_os.environ.setdefault("OKV_ABLATE", "1")  # the ablation build (its OKV_* knobs)

import os
import re
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import objectkv_amd as okv  # noqa: E402

arms = sys.argv[1:] or ["7", "8:16x"]
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
stream = torch.cuda.current_stream(dev).cuda_stream
decs = {}
for a in arms:
    vs, _, tile = a.partition(":")
    os.environ["OKV_VALUE_SWEEP"] = vs
    if tile:
        os.environ["OKV_TILE"] = tile
    else:
        os.environ.pop("OKV_TILE", None)
    decs[a] = okv.Decoder(0, stream=stream)
for k in ("OKV_VALUE_SWEEP", "OKV_TILE"):
    os.environ.pop(k, None)
seg_t = torch.empty(seg.nbytes + 64, dtype=torch.uint8, device=dev)
seg_t[:seg.nbytes].copy_(torch.from_numpy(seg))
d_t = torch.from_numpy(d.view(np.int64).copy()).to(dev)
first = decs[arms[0]]
rows, kb, vb = first.plan_device(seg_t, seg.nbytes, d_t, nblk)


def new_out(fill):
    return {k: torch.full((n,), fill, dtype=t, device=dev) for k, n, t in [
        ("row_start", nblk + 1, torch.int64), ("key_base", nblk, torch.int64),
        ("val_base", nblk, torch.int64), ("status", nblk, torch.int32),
        ("key_off", rows, torch.int64), ("key_len", rows, torch.int16),
        ("val_off", rows, torch.int64), ("val_len", rows, torch.int32),
        ("key_arena", kb, torch.uint8), ("val_arena", vb, torch.uint8)]}


ref = None
for i, (a, dec) in enumerate(decs.items()):  # every arm on poisoned outputs, compared
    o = new_out(0x5A if i % 2 else 0x3C)
    for _ in range(2):
        dec.decode_device(seg_t, seg.nbytes, d_t, nblk, o, sync=True)
    if ref is None:
        ref = o
        if os.environ.get("ABL_CLASSES") == "1":  # output-class bytes (write attribution arms)
            vo = o["val_off"].cpu().numpy().astype(np.uint64)
            vl = o["val_len"].cpu().numpy().view(np.uint32).astype(np.uint64)
            e = (vo + vl)[(vl > 0) & ((vo + vl) % 16 != 0)]
            nb = int(np.unique(e // 16).size)
            print(f"classes soa={rows * 22} blocks={nblk * 28} keys={kb} vals={vb} "
                  f"bnd_chunks={nb} bnd_bytes={nb * 16} runs_bytes~={vb - nb * 16} "
                  f"read_orig={int(d[:, 2].sum())}", flush=True)
        if os.environ.get("ABL_VERIFY") == "1":
            sys.path.insert(0, ROOT)
            from bench import verify_decode
            print(verify_decode(o, seg, d, 0, False, True, torch), flush=True)
        continue
    if re.search(r"d([1-5]|3[3-9]|[4-6][0-9])$", a):
        print(f"arm {a}: diagnostic (outputs not compared)", flush=True)
        del o
        continue
    bad = [k for k in ref if not torch.equal(ref[k], o[k])]
    print(f"arm {a} vs {arms[0]}: {'EQUAL' if not bad else 'DIFFER ' + ','.join(bad)}",
          flush=True)
    del o
del ref
out = new_out(0)
res = {a: [] for a in arms}
for r in range(rounds):
    for a, dec in decs.items():
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
        step = (time.perf_counter() - t0) * 1e3 / steps
        res[a].append((ms["copy"] / n, (ms["count"] + ms["scan"]) / n, step))
alg = int(d[:, 2].sum()) + kb + vb + rows * 22 + nblk * 28
for a in arms:
    med = [sorted(x[k] for x in res[a])[len(res[a]) // 2] for k in range(3)]
    print(f"arm={a:8s} pass3_ms={med[0]:.4f} count+scan_ms={med[1]:.4f} "
          f"step_ms={med[2]:.4f} (min {min(x[2] for x in res[a]):.4f})  "
          f"pass3 frac {alg / med[0] / 1e6 / 8000:.3f}  step frac {alg / med[2] / 1e6 / 8000:.3f}",
          flush=True)
