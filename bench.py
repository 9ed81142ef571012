#!/usr/bin/env python3
"""bench.py -- device-resident SST block decode throughput (BASELINE.json).

One "step" = one batched ReadBlockWithStat over the whole per-GPU workload
(okv_decode_blocks: count + scan + copy kernels), inputs already resident in
HBM.  Default workload = BASELINE.json configs[2] (C3): 65 536 x 64 KiB
blocks, Zipf key 8-256 B / value 0-4096 B, full decode (keys and values
materialised into packed arenas + SoA row index: Go's fresh-copy semantics).

Multi-GPU (launched by torch.distributed.run): one process per GPU, each
decodes its own segment (seed 3 + rank) -- blocks/segments are independent,
so there is no data-path collective (weak scaling).  Timing: barrier +
synchronize on both sides of K steps, max over ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2]
                    [--mode full|index] [--no-cpu] [--e2e]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident SST block decode + M rows/s, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec

CONFIGS = {
    # name: (synth kind, seed, nblocks, threshold, block size, description)
    "c3": (1, 3, 65536, 57344, 65536,
           "C3: 65536 x 64 KiB blocks, Zipf key 8-256 B / value 0-4096 B"),
    "c2": (0, 1, 256, 3584, 4096, "C2: 256 x 4 KiB blocks, fixed 16 B key / 64 B value"),
    "c5": (1, 3, 16384, 57344, 65536,
           "C5: 1 GiB segment per GPU (16384 x 64 KiB C3-style blocks)"),
    # zstd: 1 GiB of text-like rows in 64 KiB blocks, one libzstd level-3 frame per block
    "cz": ("zstd", 5, 16384, 57344, 65536,
           "CZ: 16384 x 64 KiB-raw blocks, zstd level 3 frames (text-like values 0-4096 B)"),
    # encode: total rows (split across ranks by key range), key/value bytes
    "c4": ("encode", 1, 100_000_000, 3584, 4096,
           "C4: encode 100 M sorted pairs (16 B key / 64 B value) into 4 KiB blocks + "
           "BlockStat index + meta block on device, key-range shards across GPUs"),
    # compaction: K overlapping L0 segments of n rows each -> one segment
    "cm": ("compact", 11, 16_000_000, 3584, 4096,
           "CM: compaction of 4 overlapping L0 segments x 16 M rows (16 B key / 64 B value, "
           "each overlapping the next by half): decode -> newest-wins merge -> encode, on device"),
}
ENC_METRIC = "GiB/s device-resident segment encode (data blocks written) + M rows/s"
CMP_METRIC = "GiB/s device-resident compaction (input segment bytes) + M rows/s"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="full", choices=["full", "index"])
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--e2e", action="store_true", help="also time the host-buffer path")
    ap.add_argument("--dist-backend", default="nccl",
                    help="control-plane backend (barrier, max time); gloo for rehearsals")
    ap.add_argument("--device-mod", type=int, default=0,
                    help="rehearsal only: map LOCAL_RANK -> LOCAL_RANK %% N (ranks share a GPU)")
    args = ap.parse_args()

    import torch

    import objectkv_amd as okv

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.device_mod:
        local %= args.device_mod
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local)

    if args.config == "c4":
        return run_encode(args, torch, okv, dist, world, rank, local, dev)
    if args.config == "cm":
        return run_compact(args, torch, okv, dist, world, rank, local, dev)
    kind, seed0, nblk, th, bs, desc = CONFIGS[args.config]
    seed = seed0 + rank
    t0 = time.time()
    comp = 0
    if kind == "zstd":
        from tools.zstd_gen import text_zstd_segment
        seg, descs, _ = text_zstd_segment(nblk, seed, 3, th, bs)
        comp = okv.sst.COMP_ZSTD
        if args.mode == "index":
            raise SystemExit("index-only decode does not apply to zstd blocks")
    else:
        w = okv.synth_segment(kind, seed, nblocks=nblk, threshold=th, block_size=bs)
        seg = w.data_view()
        descs = w.descs()[:nblk]
    log(f"[rank {rank}] generated {seg.nbytes / 2**30:.2f} GiB segment "
        f"({nblk} blocks) in {time.time() - t0:.1f}s")
    in_bytes = int(descs[:, 1].sum())  # sum BlockSize (headline GiB/s numerator)
    orig_bytes = int(descs[:, 2].sum())

    # ---- device-resident inputs ---------------------------------------------
    stream = torch.cuda.current_stream(dev)
    dec = okv.Decoder(local, stream=stream.cuda_stream)
    seg_t = torch.empty(seg.nbytes + 64, dtype=torch.uint8, device=dev)
    seg_t[:seg.nbytes].copy_(torch.from_numpy(seg))
    d_t = torch.from_numpy(descs.view(np.int64).copy()).to(dev)
    index_only = args.mode == "index"
    rows, kb, vb = dec.plan_device(seg_t, seg.nbytes, d_t, nblk, compression=comp,
                                   index_only=index_only)
    out = dict(row_start=torch.empty(nblk + 1, dtype=torch.int64, device=dev),
               key_base=torch.empty(nblk, dtype=torch.int64, device=dev),
               val_base=torch.empty(nblk, dtype=torch.int64, device=dev),
               status=torch.empty(nblk, dtype=torch.int32, device=dev),
               key_off=torch.empty(rows, dtype=torch.int64, device=dev),
               key_len=torch.empty(rows, dtype=torch.int16, device=dev),
               val_off=torch.empty(rows, dtype=torch.int64, device=dev),
               val_len=torch.empty(rows, dtype=torch.int32, device=dev),
               key_arena=torch.empty(max(kb, 16), dtype=torch.uint8, device=dev),
               val_arena=torch.empty(max(vb, 16), dtype=torch.uint8, device=dev))
    payload = int(kb + vb)  # padded arena bytes written

    def step(sync=False):
        return dec.decode_device(seg_t, seg.nbytes, d_t, nblk, out, compression=comp,
                                 index_only=index_only, sync=sync)

    # correctness guard on the bench path itself (totals + statuses)
    o = step(sync=True)
    assert o.n_rows == rows and o.n_bad_blocks == 0, (o.n_rows, rows, o.n_bad_blocks)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    # ---- timed region ----------------------------------------------------------
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dec.profile(True)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    t_elapsed = time.perf_counter() - t_start
    if dist:
        dist.barrier()
    kern_ms, calls = dec.profile_read()
    dec.profile(False)
    t_max = t_elapsed
    if dist:
        tdev = dev if args.dist_backend == "nccl" else "cpu"
        tt = torch.tensor([t_elapsed], dtype=torch.float64, device=tdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
    ms_per_step = 1e3 * t_max / args.steps

    # ---- roofline for the dominant kernel (pass 3) ------------------------------
    copy_ms = kern_ms["copy"] / max(calls, 1)
    count_ms = kern_ms["count"] / max(calls, 1)
    scan_ms = kern_ms["scan"] / max(calls, 1)
    if index_only:
        # index mode reads only the record headers: 6 B per row (+ the descs)
        alg = rows * 6 + rows * 22 + nblk * 12
    else:
        # read OriginalSize per block; write payload (padded arenas) + 22 B/row
        # SoA (u64 key_off, u16 key_len, u64 val_off, u32 val_len) + 28 B/block
        alg = orig_bytes + payload + rows * 22 + nblk * 28
    achieved = alg / (copy_ms * 1e-3) / 1e9
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_{args.config}_{args.mode}.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            traffic = json.load(f).get("copy_kernel_hbm_bytes_per_launch")

    # ---- CPU baseline (rank 0, N = 1 only) ---------------------------------------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        from oracle import coracle
        threads = min(16, os.cpu_count() or 1)
        cd = coracle.descs_array([tuple(int(x) for x in d) for d in descs])
        res = {}
        for nth in (1, threads):
            # bounded sample: whole passes over the first blocks until the budget is spent
            sample = nblk if args.config not in ("c3", "cz") else 4096 * nth
            sample = min(sample, nblk)
            n_pass, t_cpu, nrows_cpu = 0, 0.0, 0
            budget = args.cpu_seconds / 2
            while t_cpu < budget:
                t1 = time.perf_counter()
                r_, _pay = coracle.decode_go(seg, cd[:sample], comp, nth)
                t_cpu += time.perf_counter() - t1
                n_pass += 1
                nrows_cpu += r_
            sbytes = int(descs[:sample, 1].sum()) * n_pass
            res[nth] = (sbytes / t_cpu / 2**30, nrows_cpu / t_cpu, sample, n_pass, t_cpu)
        v1, vN = res[1], res[threads]
        cpu = {"value": round(vN[0], 4), "unit": "GiB/s", "cores": threads, "kind": "port",
               "rows_per_s": round(vN[1]), "single_thread_value": round(v1[0], 4),
               "single_thread_rows_per_s": round(v1[1]),
               "sample": (f"{vN[2]} of {nblk} blocks x {vN[3]} passes ({vN[4]:.1f}s) on "
                          f"{threads} threads; 1 thread: {v1[2]} blocks x {v1[3]} passes "
                          f"({v1[4]:.1f}s); C restatement of Go ReadBlockWithStat with Go "
                          f"allocation semantics (Go toolchain unavailable); host CPU: "
                          f"{cpu_model()}, nproc={os.cpu_count()}")}

    # ---- optional end-to-end (host buffers, PCIe both ways) -----------------------
    e2e = None
    if args.e2e and rank == 0:
        t1 = time.perf_counter()
        n_e2e = 3
        for _ in range(n_e2e):
            got = dec.decode(seg, descs, compression=comp, index_only=index_only)
        t_e2e = (time.perf_counter() - t1) / n_e2e
        e2e = {"GiB_s": round(in_bytes / t_e2e / 2**30, 3), "ms": round(t_e2e * 1e3, 2),
               "note": "pageable host buffers, H2D + plan + decode + D2H, synchronous"}
        del got

    total_in = in_bytes * world
    total_rows = rows * world
    value = total_in / (t_max / args.steps) / 2**30
    line = {
        "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": desc + (", full decode (arenas + SoA)" if not index_only
                                       else ", index-only spans"),
                   "blocks_per_gpu": nblk, "segment_bytes_per_gpu": int(seg.nbytes),
                   "block_bytes_per_gpu": in_bytes, "original_bytes_per_gpu": orig_bytes,
                   "rows_per_gpu": int(rows), "mode": args.mode,
                   "parallelism": f"{world} independent segments (no collective)"},
        "rows_per_s": round(total_rows / (t_max / args.steps)),
        "mrows_per_s": round(total_rows / (t_max / args.steps) / 1e6, 3),
        "original_GiB_s": round(orig_bytes * world / (t_max / args.steps) / 2**30, 3),
        "kernel_ms": {"count": round(count_ms, 4), "scan": round(scan_ms, 4),
                      "copy": round(copy_ms, 4)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel": "okv_gather_kernel" if not index_only
                     else "okv_gather_kernel (index)", "algorithmic_bytes_per_launch": int(alg)},
        "cpu_baseline": cpu,
    }
    if e2e:
        line["e2e"] = e2e
    if rank == 0:
        print(json.dumps(line), flush=True)
    dec.close()
    if dist:
        dist.destroy_process_group()


def run_encode(args, torch, okv, dist, world, rank, local, dev):
    """C4: okv_encode_rows over rows resident in HBM.  One step = the whole
    device encode of this rank's key-range shard (cut + pack + block hash +
    meta block, OKV_F_NO_CLOSE); the meta XXH64 + trailer (one sequential hash,
    host) is timed separately as `close_ms`.  Total rows fixed across N:
    strong scaling."""
    _, seed, total_rows, th, bs, desc = CONFIGS["c4"]
    KL, VL = 16, 64
    lo, hi = total_rows * rank // world, total_rows * (rank + 1) // world
    n = hi - lo
    stream = torch.cuda.current_stream(dev)
    enc = okv.Encoder(local, stream=stream.cuda_stream)
    t0 = time.time()
    rows = dict(key_arena=torch.empty(n * KL, dtype=torch.uint8, device=dev),
                key_off=torch.empty(n, dtype=torch.int64, device=dev),
                key_len=torch.empty(n, dtype=torch.int16, device=dev),
                val_arena=torch.empty(n * VL, dtype=torch.uint8, device=dev),
                val_off=torch.empty(n, dtype=torch.int64, device=dev),
                val_len=torch.empty(n, dtype=torch.int32, device=dev))
    enc.synth_fixed_device(seed, lo, n, KL, VL, rows)
    rec = 6 + KL + VL
    per_block = -(-th // rec)  # rows per block (fixed-size records)
    nb = -(-n // per_block)
    cap_blk = nb + 1
    seg_cap = nb * bs + cap_blk * (42 + KL) + 4096
    out = dict(seg=torch.empty(seg_cap, dtype=torch.uint8, device=dev),
               first_row=torch.empty(cap_blk + 1, dtype=torch.int64, device=dev),
               desc=torch.empty((cap_blk, 4), dtype=torch.int64, device=dev),
               hash=torch.empty(cap_blk, dtype=torch.int64, device=dev))
    log(f"[rank {rank}] generated {n} rows ({n * (KL + VL) / 2**30:.2f} GiB payload) "
        f"in {time.time() - t0:.1f}s")

    # correctness guard: full encode with close; block count/sizes; the first
    # blocks against the CPU writer; every block hash re-verified on device
    eo = enc.encode_device(rows, n, out, threshold=th, block_size=bs, strict_go=False)
    assert eo.n_blocks == nb and eo.data_bytes == nb * bs, (eo.n_blocks, nb)
    from oracle import coracle
    w = coracle.Writer(th, bs)
    nchk = min(n, 3 * per_block + 1)
    ka = rows["key_arena"][:nchk * KL].cpu().numpy().tobytes()
    va = rows["val_arena"][:nchk * VL].cpu().numpy().tobytes()
    for i in range(nchk):
        assert w.write_row(ka[i * KL:(i + 1) * KL], va[i * VL:(i + 1) * VL]) == 0
    _, want, _ = w.close()
    nfull = min(3, nb - 1)
    assert out["seg"][:nfull * bs].cpu().numpy().tobytes() == want[:nfull * bs]
    hv = torch.empty(nb, dtype=torch.int64, device=dev)
    enc._check(okv._lib.lib().okv_hash_blocks(enc._ctx, out["seg"].data_ptr(), eo.data_bytes,
                                               out["desc"].data_ptr(), nb, hv.data_ptr(),
                                               okv._lib.F_DEVICE_PTRS), "hash")
    assert torch.equal(hv, out["hash"][:nb])
    data_bytes, meta_bytes = eo.data_bytes, eo.meta_bytes

    def step():
        return enc.encode_device(rows, n, out, threshold=th, block_size=bs, strict_go=False,
                                 close=False)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    enc.profile(True)
    enc.profile_reset_encode()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        eo = step()
    torch.cuda.synchronize(dev)
    t_elapsed = time.perf_counter() - t_start
    if dist:
        dist.barrier()
    ph, calls = enc.profile_read_encode()
    enc.profile(False)
    t1 = time.perf_counter()
    enc.close_device(eo)
    close_ms = (time.perf_counter() - t1) * 1e3
    t_max = t_elapsed
    if dist:
        tdev = dev if args.dist_backend == "nccl" else "cpu"
        tt = torch.tensor([t_elapsed], dtype=torch.float64, device=tdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
    t_step = t_max / args.steps
    ph = {k: v / max(calls, 1) for k, v in ph.items()}
    # pack kernel: read payload (16+64 B/row) + SoA (22 B/row), write the padded blocks
    alg = n * (KL + VL) + n * 22 + data_bytes
    achieved = alg / (ph["pack"] * 1e-3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        threads = min(16, os.cpu_count() or 1)
        sample = min(n, 8_000_000)
        host = {k: rows[k][:sample].cpu().numpy() for k in ("key_off", "key_len", "val_off",
                                                             "val_len")}
        host["key_off"] = host["key_off"].view(np.uint64)
        host["val_off"] = host["val_off"].view(np.uint64)
        host["key_len"] = host["key_len"].view(np.uint16)
        host["val_len"] = host["val_len"].view(np.uint32)
        host["key_arena"] = rows["key_arena"][:sample * KL].cpu().numpy()
        host["val_arena"] = rows["val_arena"][:sample * VL].cpu().numpy()
        res = {}
        for nth, ns in ((1, min(sample, 1_000_000)), (threads, sample)):
            n_pass, t_cpu, fb = 0, 0.0, 0
            while t_cpu < args.cpu_seconds / 2:
                t2 = time.perf_counter()
                fb += coracle.encode_go(host, ns, th, bs, False, nth)
                t_cpu += time.perf_counter() - t2
                n_pass += 1
            res[nth] = (ns * n_pass / t_cpu, fb / t_cpu / 2**30, ns, n_pass, t_cpu)
        v1, vN = res[1], res[threads]
        cpu = {"value": round(vN[1], 4), "unit": "GiB/s", "cores": threads, "kind": "port",
               "rows_per_s": round(vN[0]), "single_thread_value": round(v1[1], 4),
               "single_thread_rows_per_s": round(v1[0]),
               "sample": (f"{vN[2]} rows x {vN[3]} passes ({vN[4]:.1f}s) as {threads} "
                          f"key-range segments on {threads} threads; 1 thread: {v1[2]} rows x "
                          f"{v1[3]} passes ({v1[4]:.1f}s); C restatement of Go "
                          f"WriteRow+Close with per-row rowBuf allocation (Go toolchain "
                          f"unavailable); host CPU: {cpu_model()}")}

    line = {
        "metric": ENC_METRIC, "value": round(data_bytes * world / t_step / 2**30, 3),
        "unit": "GiB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": desc, "rows_total": total_rows, "rows_per_gpu": n,
                   "blocks_per_gpu": nb, "data_bytes_per_gpu": data_bytes,
                   "meta_bytes_per_gpu": meta_bytes, "threshold": th, "block_size": bs,
                   "parallelism": f"{world} key-range shards, one segment each (no collective)"},
        "rows_per_s": round(total_rows / t_step),
        "mrows_per_s": round(total_rows / t_step / 1e6, 3),
        "kernel_ms": {k: round(v, 4) for k, v in ph.items()},
        "close_ms": round(close_ms, 3),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "okv_enc_pack_lds_kernel (pack + block XXH64)",
                     "algorithmic_bytes_per_launch": int(alg)},
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    enc.close()
    if dist:
        dist.destroy_process_group()


def _fixed_vals(seed, r0, n, vl=64):
    """Values of rows r0 .. r0 + n - 1 of rows_fixed(seed) (splitmix64 words
    drawn in row order; okv_synth_rows_fixed), for the guard below."""
    w = np.arange(r0 * (vl // 8), (r0 + n) * (vl // 8), dtype=np.uint64) + np.uint64(1)
    z = np.uint64(seed) + w * np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8).reshape(n, vl)


def run_compact(args, torch, okv, dist, world, rank, local, dev):
    """CM: one compaction step on device-resident segments -- the compactor the
    reference leaves as a stub (sst/compactor.go:3-6) over its own merge rule
    (GetRange: newest L0 segment owns a key, snapshot_reader.go:294-331).
    K input segments (segment s = rows [s n/2, s n/2 + n) of seed + s, written
    once by the device encoder) -> K batched decodes (okv_decode_blocks) ->
    okv_merge_rows (OKV_MERGE_ALL, newest first) -> okv_encode_rows of the
    merged rows straight from the decoded arenas (no close: the meta hash is
    one host XXH64, as in C4).  Each rank compacts its own segment set (weak
    scaling, no collective)."""
    from objectkv_amd import _lib
    from objectkv_amd.snapshot import _Addr
    _, seed0, n, th, bs, desc = CONFIGS["cm"]
    K, KL, VL = 4, 16, 64
    seed0 += 100 * rank
    stream = torch.cuda.current_stream(dev)
    enc = okv.Encoder(local, stream=stream.cuda_stream)
    per_block = -(-th // (6 + KL + VL))

    def out_for(rows):
        nb = -(-rows // per_block)
        return dict(seg=torch.empty(nb * bs + (nb + 1) * (42 + KL) + 4096, dtype=torch.uint8,
                                    device=dev),
                    first_row=torch.empty(nb + 2, dtype=torch.int64, device=dev),
                    desc=torch.empty((nb + 1, 4), dtype=torch.int64, device=dev),
                    hash=torch.empty(nb + 1, dtype=torch.int64, device=dev))

    t0 = time.time()
    segs = []  # (seg tensor, file bytes, desc tensor, n_blocks)
    for s in range(K):
        rows = dict(key_arena=torch.empty(n * KL, dtype=torch.uint8, device=dev),
                    key_off=torch.empty(n, dtype=torch.int64, device=dev),
                    key_len=torch.empty(n, dtype=torch.int16, device=dev),
                    val_arena=torch.empty(n * VL, dtype=torch.uint8, device=dev),
                    val_off=torch.empty(n, dtype=torch.int64, device=dev),
                    val_len=torch.empty(n, dtype=torch.int32, device=dev))
        enc.synth_fixed_device(seed0 + s, s * n // 2, n, KL, VL, rows)
        out = out_for(n)
        eo = enc.encode_device(rows, n, out, threshold=th, block_size=bs, strict_go=False)
        segs.append((out["seg"], int(eo.file_bytes), out["desc"][:eo.n_blocks].contiguous(),
                     int(eo.n_blocks)))
        del rows
    in_bytes = sum(f for _s, f, _d, _nb in segs)
    # decode outputs (SoA + arenas) per input segment
    douts = []
    for seg_t, fb, d_t, nb in segs:
        r, kb, vb = enc.plan_device(seg_t, fb, d_t, nb)
        douts.append(dict(row_start=torch.empty(nb + 1, dtype=torch.int64, device=dev),
                          key_base=torch.empty(nb, dtype=torch.int64, device=dev),
                          val_base=torch.empty(nb, dtype=torch.int64, device=dev),
                          status=torch.empty(nb, dtype=torch.int32, device=dev),
                          key_off=torch.empty(r, dtype=torch.int64, device=dev),
                          key_len=torch.empty(r, dtype=torch.int16, device=dev),
                          val_off=torch.empty(r, dtype=torch.int64, device=dev),
                          val_len=torch.empty(r, dtype=torch.int32, device=dev),
                          key_arena=torch.empty(max(kb, 16), dtype=torch.uint8, device=dev),
                          val_arena=torch.empty(max(vb, 16), dtype=torch.uint8, device=dev),
                          rows=r))
    n_in = sum(d["rows"] for d in douts)
    order = list(range(K - 1, -1, -1))  # newest (highest s) first
    kb0 = min(douts[s]["key_arena"].data_ptr() for s in order)
    vb0 = min(douts[s]["val_arena"].data_ptr() for s in order)
    kspan = max(d["key_arena"].data_ptr() + d["key_arena"].numel() for d in douts) - kb0
    vspan = max(d["val_arena"].data_ptr() + d["val_arena"].numel() for d in douts) - vb0
    mout = dict(key_off=torch.empty(n_in, dtype=torch.int64, device=dev),
                key_len=torch.empty(n_in, dtype=torch.int16, device=dev),
                val_off=torch.empty(n_in, dtype=torch.int64, device=dev),
                val_len=torch.empty(n_in, dtype=torch.int32, device=dev))
    n_uniq = (K - 1) * n // 2 + n
    eout = out_for(n_uniq)
    mrows = dict(key_arena=_Addr(kb0), key_off=mout["key_off"], key_len=mout["key_len"],
                 val_arena=_Addr(vb0), val_off=mout["val_off"], val_len=mout["val_len"])
    log(f"[rank {rank}] built {K} segments ({in_bytes / 2**30:.2f} GiB, {n_in} rows) "
        f"in {time.time() - t0:.1f}s")

    def step(ph=None):
        # stage times (diagnostic): host clock around each stage, the context
        # stream drained at each boundary (the merge syncs internally anyway)
        t = time.perf_counter()
        for (seg_t, fb, d_t, nb), d in zip(segs, douts):
            enc.decode_device(seg_t, fb, d_t, nb, d, sync=False)
        if ph is not None:
            enc.sync()
            t, ph[0] = time.perf_counter(), ph[0] + time.perf_counter() - t
        mo = enc.merge_device([(douts[s], 0, douts[s]["rows"], 0) for s in order],
                              _lib.MERGE_ALL, _lib.DIR_ASC, 0, None, True, out=mout,
                              key_base=kb0, val_base=vb0, row_cap=n_in)
        if ph is not None:
            enc.sync()
            t, ph[1] = time.perf_counter(), ph[1] + time.perf_counter() - t
        eo = enc.encode_device(mrows, int(mo.n_rows), eout, threshold=th, block_size=bs,
                               strict_go=False, close=False, key_arena_bytes=kspan,
                               val_arena_bytes=vspan)
        if ph is not None:
            enc.sync()
            ph[2] += time.perf_counter() - t
        return mo, eo

    # correctness guard: every key once, the newest segment's value, output
    # blocks in the overlaps byte-equal to the CPU writer over the expected rows
    mo, eo = step()
    torch.cuda.synchronize(dev)
    assert int(mo.n_rows) == n_uniq == int(mo.n_unique), (mo.n_rows, n_uniq)
    from oracle import coracle
    for b0 in (0, (n // 2) // per_block + 3, (n + n // 4) // per_block, n_uniq // per_block - 4):
        r0 = b0 * per_block
        w = coracle.Writer(th, bs)
        for r in range(r0, r0 + 3 * per_block + 1):  # +1: not Q1
            s_new = min(K - 1, r // (n // 2))  # newest segment holding row r
            assert w.write_row(r.to_bytes(KL, "big"),
                               _fixed_vals(seed0 + s_new, r, 1)[0].tobytes()) == 0
        _, want, _ = w.close()
        got = eout["seg"][b0 * bs:(b0 + 3) * bs].cpu().numpy().tobytes()
        assert got == want[:3 * bs], b0
    out_bytes = int(eo.data_bytes)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    t_elapsed = time.perf_counter() - t_start
    if dist:
        dist.barrier()
    t_max = t_elapsed
    if dist:
        tdev = dev if args.dist_backend == "nccl" else "cpu"
        tt = torch.tensor([t_elapsed], dtype=torch.float64, device=tdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
    t_step = t_max / args.steps
    ph = np.zeros(3)  # untimed diagnostic pass: per-stage wall time
    for _ in range(2):
        step(ph)
    ph *= 1e3 / 2
    line = {
        "metric": CMP_METRIC, "value": round(in_bytes * world / t_step / 2**30, 3),
        "unit": "GiB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": desc, "segments_per_gpu": K, "rows_in_per_gpu": n_in,
                   "rows_out_per_gpu": n_uniq, "input_bytes_per_gpu": in_bytes,
                   "output_data_bytes_per_gpu": out_bytes,
                   "parallelism": f"{world} independent compactions (no collective)"},
        "rows_per_s": round(n_in * world / t_step),
        "mrows_per_s": round(n_in * world / t_step / 1e6, 3),
        "stage_ms": {"decode": round(ph[0], 4), "merge": round(ph[1], 4),
                     "encode": round(ph[2], 4)},
        "roofline": None, "cpu_baseline": None,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    enc.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
