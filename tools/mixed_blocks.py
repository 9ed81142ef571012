"""Bimodal block sizes through the large-block decode (the tile
pass sizes its per-block tile count from the call's AVERAGE block span; a
block whose records run past tpb x 16 KiB goes to okv_copy_kernel).

Segments of N blocks whose BlockSize alternates 4 KiB / 60 KiB (records of
16 B keys and 1-3 KiB values, written by the C++ host writer's framing), and
of N uniform 32 KiB blocks of the same records, device-resident, one decode at
a time: per-pass HIP-event ms, GB/s of input, and the path taken.
usage: python tools/mixed_blocks.py [N]  -> JSON lines"""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import objectkv_amd as okv  # noqa: E402
from objectkv_amd import _lib  # noqa: E402


def segment(sizes, seed):
    rng = np.random.default_rng(seed)
    parts, descs, off = [], [], 0
    for target in sizes:
        body = bytearray()
        while len(body) < target - 3100:
            vl = int(rng.integers(1000, 3000))
            body += (16).to_bytes(2, "little") + vl.to_bytes(4, "little")
            body += rng.integers(0, 256, 16 + vl, dtype=np.uint8).tobytes()
        bsize = (len(body) // 4096 + 1) * 4096
        parts.append(bytes(body) + bytes(bsize - len(body)))
        descs.append((off, bsize, len(body), 0))
        off += bsize
    return np.frombuffer(b"".join(parts) + bytes(4096), np.uint8), np.array(descs, np.uint64)


def run(name, seg, d):
    dev = torch.device("cuda", 0)
    dec = okv.Decoder(0, stream=torch.cuda.current_stream(dev).cuda_stream)
    n = d.shape[0]
    seg_t = torch.empty(seg.nbytes + 64, dtype=torch.uint8, device=dev)
    seg_t[:seg.nbytes].copy_(torch.from_numpy(seg))
    d_t = torch.from_numpy(d.view(np.int64).copy()).to(dev)
    rows, kb, vb = dec.plan_device(seg_t, seg.nbytes, d_t, n)
    out = {k: torch.empty(m, dtype=t, device=dev) for k, m, t in [
        ("row_start", n + 1, torch.int64), ("key_base", n, torch.int64),
        ("val_base", n, torch.int64), ("status", n, torch.int32),
        ("key_off", rows, torch.int64), ("key_len", rows, torch.int16),
        ("val_off", rows, torch.int64), ("val_len", rows, torch.int32),
        ("key_arena", kb, torch.uint8), ("val_arena", vb, torch.uint8)]}
    for _ in range(3):
        dec.decode_device(seg_t, seg.nbytes, d_t, n, out, sync=True)
    assert int(out["status"].max()) == 0
    lp = dec.last_path()
    dec.profile(True)
    for _ in range(10):
        dec.decode_device(seg_t, seg.nbytes, d_t, n, out, sync=True)
    ms, calls = dec.profile_read()
    dec.profile(False)
    t = []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dec.decode_device(seg_t, seg.nbytes, d_t, n, out, sync=True)
        t.append((time.perf_counter() - t0) * 1e3)
    step = statistics.median(t)
    blk = int(d[:, 1].sum())
    print(json.dumps({"segment": name, "blocks": n, "block_bytes": blk,
                      "pass3_ms": round(ms["copy"] / calls, 4),
                      "count_ms": round(ms["count"] / calls, 4), "step_ms": round(step, 4),
                      "GiB_s": round(blk / step / 1e-3 / 2**30, 1),
                      "big_block_path": bool(lp & _lib.PATH_BIG)}), flush=True)
    dec.close()


N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
run("bimodal_4k_60k", *segment([4096 if i % 2 else 61440 for i in range(N)], 1))
run("uniform_32k", *segment([32768] * N, 1))
