"""Diagnostic: time okv_copy_kernel ablations on the C3 workload.
V=0 stage only, 1 + chase, 2 + SoA index, 3 full.  Prints copy-kernel ms."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    import objectkv_amd as okv
    nblk = int(os.environ.get("ABL_NBLK", "65536"))
    w = okv.synth_segment(1, 3, nblocks=nblk, threshold=57344, block_size=65536)
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
    for _ in range(3):
        dec.decode_device(seg_t, seg.nbytes, d_t, nblk, out, sync=False)
    torch.cuda.synchronize()
    dec.profile(True)
    for _ in range(10):
        dec.decode_device(seg_t, seg.nbytes, d_t, nblk, out, sync=False)
    ms, n = dec.profile_read()
    print(f"variant={os.environ.get('OKV_COPY_VARIANT', '3')} copy_ms={ms['copy'] / n:.4f} "
          f"count_ms={ms['count'] / n:.4f}", flush=True)
else:
    for v in sys.argv[1:] or ["0", "1", "2", "3"]:
        env = dict(os.environ, OKV_COPY_VARIANT=v)
        subprocess.run([sys.executable, __file__, "child"], env=env, check=True, timeout=300)
