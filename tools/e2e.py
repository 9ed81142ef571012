"""End-to-end decode rate with host-resident input and output (PCIe both ways).

The segment arrives in pinned host memory (as from S3 / the local disk cache
tier) and the decoded SoA + arenas must land back in pinned host memory (for
the Go caller).  Blocks are processed in chunks; chunk i's H2D copy, chunk
i-1's decode and chunk i-2's D2H copies run on three streams so PCIe in both
directions overlaps the kernels.  bench.py --e2e calls run_e2e(); standalone
it prints one JSON line.

    python tools/e2e.py [--config c3] [--chunk-mib 256]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_e2e(config="c3", chunk_mib=256, reps=3, torch=None):
    if torch is None:
        import torch
    import objectkv_amd as okv
    from bench import CONFIGS
    kind, seed, nblk, th, bs, desc = CONFIGS[config]
    w = okv.synth_segment(kind, seed, nblocks=nblk, threshold=th, block_size=bs)
    seg_np = w.data_view()
    descs = w.descs()[:nblk]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)

    # chunking: contiguous block ranges of ~chunk-mib bytes
    per = max(1, (chunk_mib << 20) // bs)
    chunks = [(b, min(b + per, nblk)) for b in range(0, nblk, per)]

    seg_h = torch.empty(seg_np.nbytes, dtype=torch.uint8).pin_memory()
    seg_h.numpy()[:] = seg_np
    dec0 = okv.Decoder(0)
    # sizes per chunk (plan on the host copy once, outside the timed region)
    plans = []
    for b0, b1 in chunks:
        d = descs[b0:b1].copy()
        plans.append(dec0.plan(seg_np, d))
    dec0.close()

    s_h2d, s_cmp, s_d2h = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    dec = okv.Decoder(0, stream=s_cmp.cuda_stream)
    NB = 2  # device buffer sets
    max_chunk_bytes = max(int(descs[b1 - 1][0] + descs[b1 - 1][1] - descs[b0][0]) for b0, b1 in chunks)
    max_rows = max(p[0] for p in plans)
    max_kb = max(p[1] for p in plans)
    max_vb = max(p[2] for p in plans)
    max_nb = max(b1 - b0 for b0, b1 in chunks)


    def dev_set():
        return dict(seg=torch.empty(max_chunk_bytes + 64, dtype=torch.uint8, device=dev),
                    descs=torch.empty((max_nb, 4), dtype=torch.int64, device=dev),
                    row_start=torch.empty(max_nb + 1, dtype=torch.int64, device=dev),
                    key_base=torch.empty(max_nb, dtype=torch.int64, device=dev),
                    val_base=torch.empty(max_nb, dtype=torch.int64, device=dev),
                    status=torch.empty(max_nb, dtype=torch.int32, device=dev),
                    key_off=torch.empty(max_rows, dtype=torch.int64, device=dev),
                    key_len=torch.empty(max_rows, dtype=torch.int16, device=dev),
                    val_off=torch.empty(max_rows, dtype=torch.int64, device=dev),
                    val_len=torch.empty(max_rows, dtype=torch.int32, device=dev),
                    key_arena=torch.empty(max(max_kb, 16), dtype=torch.uint8, device=dev),
                    val_arena=torch.empty(max(max_vb, 16), dtype=torch.uint8, device=dev))


    dsets = [dev_set() for _ in range(NB)]
    # pinned host outputs for the whole segment
    tot_rows = sum(p[0] for p in plans)
    host = dict(key_off=torch.empty(tot_rows, dtype=torch.int64).pin_memory(),
                key_len=torch.empty(tot_rows, dtype=torch.int16).pin_memory(),
                val_off=torch.empty(tot_rows, dtype=torch.int64).pin_memory(),
                val_len=torch.empty(tot_rows, dtype=torch.int32).pin_memory(),
                key_arena=torch.empty(sum(p[1] for p in plans) + 16, dtype=torch.uint8).pin_memory(),
                val_arena=torch.empty(sum(p[2] for p in plans) + 16, dtype=torch.uint8).pin_memory(),
                status=torch.empty(nblk, dtype=torch.int32).pin_memory())
    # per-chunk descriptors rebased to the chunk's first byte, pinned
    cdescs = []
    for b0, b1 in chunks:
        d = descs[b0:b1].copy()
        d[:, 0] -= descs[b0][0]
        cdescs.append(torch.from_numpy(d.view(np.int64)).pin_memory())


    def run_once():
        ev_h2d = [torch.cuda.Event() for _ in chunks]
        ev_cmp = [torch.cuda.Event() for _ in chunks]
        ev_d2h = [torch.cuda.Event() for _ in chunks]
        r0 = k0 = v0 = 0
        for i, (b0, b1) in enumerate(chunks):
            D = dsets[i % NB]
            off0 = int(descs[b0][0])
            nbytes = int(descs[b1 - 1][0] + descs[b1 - 1][1]) - off0
            rows, kb, vb = plans[i]
            with torch.cuda.stream(s_h2d):
                if i >= NB:
                    s_h2d.wait_event(ev_d2h[i - NB])  # buffer set free again
                D["seg"][:nbytes].copy_(seg_h[off0:off0 + nbytes], non_blocking=True)
                D["descs"][:b1 - b0].copy_(cdescs[i], non_blocking=True)
                ev_h2d[i].record(s_h2d)
            s_cmp.wait_event(ev_h2d[i])
            outs = {k: (v if k in ("seg", "descs") else v) for k, v in D.items()}
            dec.decode_device(D["seg"], nbytes, D["descs"], b1 - b0,
                              {k: outs[k] for k in ("row_start", "key_base", "val_base", "status",
                                                    "key_off", "key_len", "val_off", "val_len",
                                                    "key_arena", "val_arena")}, sync=False)
            ev_cmp[i].record(s_cmp)
            with torch.cuda.stream(s_d2h):
                s_d2h.wait_event(ev_cmp[i])
                host["key_off"][r0:r0 + rows].copy_(D["key_off"][:rows], non_blocking=True)
                host["key_len"][r0:r0 + rows].copy_(D["key_len"][:rows], non_blocking=True)
                host["val_off"][r0:r0 + rows].copy_(D["val_off"][:rows], non_blocking=True)
                host["val_len"][r0:r0 + rows].copy_(D["val_len"][:rows], non_blocking=True)
                host["key_arena"][k0:k0 + kb].copy_(D["key_arena"][:kb], non_blocking=True)
                host["val_arena"][v0:v0 + vb].copy_(D["val_arena"][:vb], non_blocking=True)
                host["status"][b0:b1].copy_(D["status"][:b1 - b0], non_blocking=True)
                ev_d2h[i].record(s_d2h)
            r0 += rows
            k0 += kb
            v0 += vb
        torch.cuda.synchronize()


    run_once()  # warm-up
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        run_once()
        times.append(time.perf_counter() - t0)
    t = sorted(times)[len(times) // 2]
    in_bytes = int(descs[:, 1].sum())
    out_bytes = sum(p[1] + p[2] for p in plans) + tot_rows * 22 + nblk * 4
    assert int(host["status"].sum()) == 0
    return {"e2e_GiB_s": round(in_bytes / t / 2**30, 2), "ms": round(t * 1e3, 2),
                      "rows_per_s": round(tot_rows / t), "h2d_bytes": in_bytes,
                      "d2h_bytes": int(out_bytes),
                      "pcie_GB_s_each_way": round(max(in_bytes, out_bytes) / t / 1e9, 2),
                      "chunks": len(chunks), "chunk_MiB": chunk_mib, "config": desc,
                      "note": "pinned host in/out, 3 streams (H2D / decode / D2H), 2 device "
                              "buffer sets"}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--chunk-mib", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    print(json.dumps(run_e2e(a.config, a.chunk_mib, a.reps)), flush=True)
