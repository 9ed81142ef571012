"""Interleaved encode ablations in one process (OKV_ENC_VARIANT), C4 rows.

    python tools/ablate_enc.py [--rows N] [--reps R] [--variants 0,1,2]
"""
import os as _os
_os.environ.setdefault("OKV_ABLATE", "1")  # the ablation build (its OKV_* knobs)

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import objectkv_amd as okv  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=100_000_000)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--variants", default="0,1,2")
ap.add_argument("--images", default="32768", help="OKV_ENC_IMAGE values to interleave")
args = ap.parse_args()
n = args.rows
dev = torch.device("cuda", 0)
enc = okv.Encoder(0, stream=torch.cuda.current_stream(dev).cuda_stream)
rows = dict(key_arena=torch.empty(n * 16, dtype=torch.uint8, device=dev),
            key_off=torch.empty(n, dtype=torch.int64, device=dev),
            key_len=torch.empty(n, dtype=torch.int16, device=dev),
            val_arena=torch.empty(n * 64, dtype=torch.uint8, device=dev),
            val_off=torch.empty(n, dtype=torch.int64, device=dev),
            val_len=torch.empty(n, dtype=torch.int32, device=dev))
enc.synth_fixed_device(1, 0, n, 16, 64, rows)
nb = -(-n // 42) + 1
out = dict(seg=torch.empty(nb * 4096 + nb * 60 + 4096, dtype=torch.uint8, device=dev))
variants = [(int(v), int(i)) for v in args.variants.split(",") for i in args.images.split(",")]
res = {v: [] for v in variants}
ref = None
for rep in range(args.reps):
    for v in variants:
        os.environ["OKV_ENC_VARIANT"] = str(v[0])
        os.environ["OKV_ENC_IMAGE"] = str(v[1])
        enc.profile(True)
        enc.profile_reset_encode()
        eo = enc.encode_device(rows, n, out, strict_go=False, close=False)
        if rep == 0 and v[0] in (0, 7):  # product-equivalent variants: the same file bytes
            fb = int(eo.data_bytes + eo.meta_bytes)
            if ref is None:
                ref = out["seg"][:fb].clone()
            else:
                print(f"variant {v}: {'EQUAL' if torch.equal(ref, out['seg'][:fb]) else 'DIFFER'} "
                      f"to variant {variants[0]}", flush=True)
        ph, _ = enc.profile_read_encode()
        if rep:
            res[v].append(ph)
for v in variants:
    avg = {k: sum(p[k] for p in res[v]) / len(res[v]) for k in res[v][0]}
    print(f"variant {v}: " + " ".join(f"{k}={x:.3f}" for k, x in avg.items()), flush=True)
