#!/usr/bin/env python3
"""bench.py -- device-resident SST block decode throughput (BASELINE.json).

One "step" = one batched ReadBlockWithStat over the whole per-GPU workload
(okv_decode_blocks: count + scan + gather kernels), inputs already resident
in HBM.  Default workload = BASELINE.json configs[2] (C3): 65 536 x 64 KiB
blocks, Zipf key 8-256 B / value 0-4096 B, full decode (keys and values
materialised into packed arenas + SoA row index: Go's fresh-copy semantics).

Multi-GPU: one process per GPU, each decoding its own segment (seed 3 +
rank) -- blocks/segments are independent, so there is no data-path
collective (weak scaling).  `--gpus N` without a launcher spawns the N rank
processes itself (before anything touches HIP); under torch.distributed.run
WORLD_SIZE must equal N.  Timing: barrier + synchronize on both sides of K
steps, max over ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--config c3|c2|c5|cz|c4|cm|c1] [--mode full|index]
                    [--no-cpu] [--no-verify] [--e2e]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident SST block decode + M rows/s, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
PMC_ROUND = "r6"  # profiles/<round>/pmc_<config>_<mode>.json (FETCH/WRITE_SIZE passes)

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
           "BlockStat index + meta block + trailer (Close) on device, key-range shards across "
           "GPUs"),
    # compaction: K overlapping L0 segments of n rows each -> one segment
    "cm": ("compact", 11, 16_000_000, 3584, 4096,
           "CM: compaction of 4 overlapping L0 segments x 16 M rows (16 B key / 64 B value, "
           "each overlapping the next by half): decode -> newest-wins merge -> encode, on device"),
    # C1: one segment round trip of 10 000 rows (write + full ascending read)
    "c1": ("roundtrip", 1, 10_000, 3584, 4096,
           "C1: single segment round trip, 10 000 x 16 B key / 64 B value: write (WriteRow x n "
           "+ Close) + full ascending read"),
}
ALLOC_NOTE = ("; allocations from a per-thread bump arena (the analogue of Go's per-P mcache "
              "fast path: glibc malloc contended past 16 threads), reset every 4 MiB")
ENC_METRIC = "GiB/s device-resident segment encode (data blocks written, Close included) + M rows/s"
CMP_METRIC = "GiB/s device-resident compaction (input segment bytes) + M rows/s"
RT_METRIC = "MB/s segment round trip (write + full ascending read, segment bytes) + rows/s"
DECODE_SOURCES = ("objectkv_amd/csrc/okv_decode.hip", "objectkv_amd/csrc/okv_kernels.hpp",
                  "objectkv_amd/csrc/okv_ctx.hpp")
ENCODE_SOURCES = ("objectkv_amd/csrc/okv_encode.hip", "objectkv_amd/csrc/okv_kernels.hpp",
                  "objectkv_amd/csrc/okv_ctx.hpp")
ZSTD_SOURCES = DECODE_SOURCES + ("objectkv_amd/csrc/okv_zstd.hip",)


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


def host_cores():
    """Cores this process may run on (the CPU baseline's thread count)."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def thread_counts():
    """CPU baseline thread counts: 1, 16, 64 and every core this process may
    use.  Memory-allocation-heavy Go-semantics code can scale past its best
    count into allocator contention, so the reported value is the best of
    the sweep (with its thread count) and the all-cores figure is kept."""
    c = host_cores()
    return sorted({1, min(16, c), min(64, c), c})


def sweep(run_once, budget_s):
    """{threads: (units per second, passes, seconds)} for run_once(threads) ->
    units done, each count run in whole passes until budget_s is spent."""
    res = {}
    for nth in thread_counts():
        n_pass, t_cpu, units = 0, 0.0, 0.0
        while t_cpu < budget_s:
            t1 = time.perf_counter()
            units += run_once(nth)
            t_cpu += time.perf_counter() - t1
            n_pass += 1
        res[nth] = (units / t_cpu, n_pass, t_cpu)
    from oracle import coracle
    coracle.arena_trim()  # the arena pool back to the OS after the sweep
    return res


def sweep_summary(res, scale, unit, kind, sample):
    """cpu_baseline entry: the best thread count's rate as value."""
    best = max(res, key=lambda k: res[k][0])
    allc = max(res)
    return {"value": round(res[best][0] * scale, 4), "unit": unit, "cores": best, "kind": kind,
            "single_thread_value": round(res[1][0] * scale, 4),
            "all_cores": {"cores": allc, "value": round(res[allc][0] * scale, 4)},
            "by_threads": {str(k): round(v[0] * scale, 4) for k, v in sorted(res.items())},
            # (rounds 1-4 allocated with glibc malloc: their CPU lines are not
            # comparable with these)
            "allocator": "per-thread bump arena (Go per-P mcache analogue), since round 5",
            "sample": sample + f"; host CPU: {cpu_model()}, nproc={os.cpu_count()}, "
                               f"affinity={host_cores()}"}


def source_sha(paths=DECODE_SOURCES):
    h = hashlib.sha256()
    for p in paths:
        with open(os.path.join(ROOT, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def pmc_traffic(config, mode, kernel, sources=DECODE_SOURCES):
    """HBM bytes per launch of `kernel` from profiles/<PMC_ROUND>/pmc_<config>_<mode>.json
    -- used only if it was collected from the kernel sources being timed
    (same source_sha); else None."""
    path = os.path.join(ROOT, "profiles", PMC_ROUND, f"pmc_{config}_{mode}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    if d.get("source_sha") != source_sha(sources):
        return None, "stale (kernel sources changed since the PMC run)"
    names = (kernel,) if isinstance(kernel, str) else tuple(kernel)
    # per launch, times the launches one step makes of it (a two-piece decode
    # launches the tile pass twice; pmc_summary averages over launches)
    per = d.get("launches_per_step", {})
    hits = [k["hbm_bytes"] * next((m for p, m in per.items() if p in name), 1)
            for name, k in d.get("kernels", {}).items() if any(n in name for n in names)]
    if hits:  # per launch, summed over the kernels of the pass
        return sum(hits), os.path.relpath(path, ROOT)
    return None, None


def trace_roofline(config, alg, sources=DECODE_SOURCES):
    """The rocprofv3 kernel-trace average of the roofline kernel from
    profiles/<PMC_ROUND>/trace_<config>.json (tools/trace_summary.py), and the
    roofline fraction it implies for `alg` bytes -- attached only if the trace
    was taken of the kernel sources being timed (same source_sha)."""
    path = os.path.join(ROOT, "profiles", PMC_ROUND, f"trace_{config}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    if d.get("source_sha") != source_sha(sources):
        return {"source": os.path.relpath(path, ROOT),
                "stale": "kernel sources changed since the trace"}
    ms = d["avg_ns_timed"] / 1e6
    out = {"kernel": d["kernel"], "avg_ms": round(ms, 4), "steps": d["timed_launches"],
           "launches_per_step": d.get("launches_per_step", 1),
           "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "source": os.path.relpath(path, ROOT)}
    if d.get("bench_event_ms_same_process"):
        out["event_ms_same_process"] = round(d["bench_event_ms_same_process"], 4)
        out["event_over_trace_same_process"] = round(d["bench_event_vs_trace"], 4)
    return out


# ---- process launch ---------------------------------------------------------------


def spawn_ranks(args, cmd=None):
    """`--gpus N` without a launcher: start N rank processes (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_*) running this script with the same arguments, and
    wait.  Runs before this process imports torch or touches HIP; only rank 0
    prints the result line.  Returns the worst exit status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = cmd or [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


class Dist:
    """Rank layout + the control-plane collectives (barrier, max and gather of
    elapsed times).  No data-path collective exists: each rank owns its
    segment(s)."""

    def __init__(self, args, torch):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != args.gpus:
            raise SystemExit(f"WORLD_SIZE={self.world} but --gpus {args.gpus}")
        if args.device_mod:
            self.local %= args.device_mod
        self.torch = torch
        self.backend = args.dist_backend
        torch.cuda.set_device(self.local)
        self.dev = torch.device("cuda", self.local)
        self.dist = None
        if self.world > 1 or getattr(args, "dist_always", False):
            import torch.distributed as dist
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=self.dev)
            else:
                dist.init_process_group(self.backend)
            assert dist.get_world_size() == self.world, (dist.get_world_size(), self.world)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def gather(self, x: float):
        """x from every rank (rank order)."""
        if not self.dist:
            return [x]
        torch = self.torch
        tdev = self.dev if self.backend == "nccl" else "cpu"
        t = torch.tensor([x], dtype=torch.float64, device=tdev)
        out = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [float(o.item()) for o in out]

    def timed(self, step, steps):
        """Barrier + synchronize, K steps, synchronize + barrier; returns
        (max over ranks of the elapsed seconds, per-rank seconds)."""
        torch = self.torch
        self.barrier()
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize(self.dev)
        el = time.perf_counter() - t0
        self.barrier()
        per = self.gather(el)
        return max(per), per

    def info(self):
        return {"world_size": self.dist.get_world_size() if self.dist else 1,
                "dist_backend": self.backend if self.dist else None}

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="full", choices=["full", "index"])
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the oracle comparison of the bench outputs")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--c4-inflight", type=int, default=3,
                    help="c4: segments in flight (the Closes of two overlap the next's kernels)")
    ap.add_argument("--decode-inflight", type=int, default=None,
                    help="decode configs: whole-segment decodes in flight, each on its own "
                         "context, stream, segment copy and output buffers (later decodes' "
                         "pass 1 under the current pass 3); 1 = one at a time.  Default 4 for "
                         "C3 (one box: 2 / 3 / 4 in flight 2694 / 2765 / 2789 GiB/s), 2 for the "
                         "others (C2 at 4: 48.3 vs 55.3 GiB/s; DESIGN.md 13.11)")
    ap.add_argument("--e2e", action="store_true",
                    help="also time the pinned, pipelined host-buffer path (PCIe both ways)")
    ap.add_argument("--dist-backend", default="gloo",
                    help="control-plane backend (barrier, gather of the ranks' times).  The "
                         "data path has no collective (each rank owns its segments), so the "
                         "default keeps the control plane on the host: gloo, after "
                         "torch.cuda.synchronize.  nccl (RCCL) is covered by "
                         "tests/test_bench_gpu.py::test_rccl_control_plane_world1")
    ap.add_argument("--pass3-chain", choices=["auto", "on", "off"], default="auto",
                    help="decodes in flight: chain each pass 3 behind the previous decode's "
                         "(auto: large uncompressed blocks)")
    ap.add_argument("--dist-always", action="store_true",
                    help="initialise the process group at world size 1 too (tests)")
    ap.add_argument("--device-mod", type=int, default=0,
                    help="rehearsal only: map LOCAL_RANK -> LOCAL_RANK %% N (ranks share a GPU)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args)

    import torch

    import objectkv_amd as okv

    D = Dist(args, torch)
    kind = CONFIGS[args.config][0]
    try:
        if kind == "encode":
            return run_encode(args, torch, okv, D)
        if kind == "compact":
            return run_compact(args, torch, okv, D)
        if kind == "roundtrip":
            return run_roundtrip(args, torch, okv, D)
        return run_decode(args, torch, okv, D)
    finally:
        D.close()


def emit(D, line):
    if D.rank == 0:
        print(json.dumps(line), flush=True)


# ---- decode (C2 / C3 / C5 / CZ) ---------------------------------------------------


def verify_decode(dec_out, seg, descs, comp, index_only, full, torch):
    """The bench path's own outputs against the C oracle (oracle/coracle.py):
    full = every output array; else the totals + 64 blocks spread over the
    segment (their rows, lengths and arena bytes)."""
    from oracle import coracle as CO
    d = np.ascontiguousarray(descs, np.uint64)
    host = {k: v.cpu().numpy() for k, v in dec_out.items()}
    for k, dt in (("row_start", np.uint64), ("key_base", np.uint64), ("val_base", np.uint64),
                  ("key_off", np.uint64), ("val_off", np.uint64), ("key_len", np.uint16),
                  ("val_len", np.uint32)):
        host[k] = host[k].view(dt)
    nblk = d.shape[0]
    if full:
        ref = CO.decode_soa(seg, d.view(CO.DESC_DTYPE).reshape(-1), comp, index_only)
        rows = int(ref["row_start"][-1])
        keys = ["status", "row_start", "key_off", "key_len", "val_off", "val_len"]
        if not index_only:
            keys += ["key_base", "val_base"]
        for k in keys:
            got = host[k][:rows] if k in ("key_off", "key_len", "val_off", "val_len") else host[k]
            assert np.array_equal(got, ref[k]), f"bench output {k} differs from the oracle"
        if not index_only:
            for k in ("key_arena", "val_arena"):
                n = ref[k].size
                assert np.array_equal(host[k][:n], ref[k]), f"bench output {k} differs"
        return {"verified": "all output arrays == oracle (oref_decode_soa)", "rows": rows}
    pick = np.unique(np.linspace(0, nblk - 1, min(64, nblk)).astype(np.int64))
    for b in pick:
        ref = CO.decode_soa(seg, d[b:b + 1].view(CO.DESC_DTYPE).reshape(-1), comp, index_only)
        r0, r1 = int(host["row_start"][b]), int(host["row_start"][b + 1])
        assert r1 - r0 == int(ref["row_start"][-1]) and host["status"][b] == ref["status"][0]
        assert np.array_equal(host["key_len"][r0:r1], ref["key_len"])
        assert np.array_equal(host["val_len"][r0:r1], ref["val_len"])
        if not index_only:
            kb, vb = int(host["key_base"][b]), int(host["val_base"][b])
            assert np.array_equal(host["key_arena"][kb:kb + ref["key_arena"].size],
                                  ref["key_arena"])
            assert np.array_equal(host["val_arena"][vb:vb + ref["val_arena"].size],
                                  ref["val_arena"])
    return {"verified": f"{len(pick)} sampled blocks == oracle", "rows": None}


def run_decode(args, torch, okv, D):
    kind, seed0, nblk, th, bs, desc = CONFIGS[args.config]
    rank, world, dev = D.rank, D.world, D.dev
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
    comp_bytes = int(descs[:, 3].sum())

    # ---- device-resident inputs ---------------------------------------------
    stream = torch.cuda.current_stream(dev)
    dec = okv.Decoder(D.local, stream=stream.cuda_stream)
    seg_t = torch.empty(seg.nbytes + 64, dtype=torch.uint8, device=dev)
    seg_t[:seg.nbytes].copy_(torch.from_numpy(seg))
    d_t = torch.from_numpy(descs.view(np.int64).copy()).to(dev)
    index_only = args.mode == "index"
    rows, kb, vb = dec.plan_device(seg_t, seg.nbytes, d_t, nblk, compression=comp,
                                   index_only=index_only)
    def new_out():
        return dict(row_start=torch.empty(nblk + 1, dtype=torch.int64, device=dev),
                    key_base=torch.empty(nblk, dtype=torch.int64, device=dev),
                    val_base=torch.empty(nblk, dtype=torch.int64, device=dev),
                    status=torch.empty(nblk, dtype=torch.int32, device=dev),
                    key_off=torch.empty(rows, dtype=torch.int64, device=dev),
                    key_len=torch.empty(rows, dtype=torch.int16, device=dev),
                    val_off=torch.empty(rows, dtype=torch.int64, device=dev),
                    val_len=torch.empty(rows, dtype=torch.int32, device=dev),
                    key_arena=torch.empty(max(kb, 16), dtype=torch.uint8, device=dev),
                    val_arena=torch.empty(max(vb, 16), dtype=torch.uint8, device=dev))
    out = new_out()
    payload = int(kb + vb)  # padded arena bytes written

    def step(sync=False):
        return dec.decode_device(seg_t, seg.nbytes, d_t, nblk, out, compression=comp,
                                 index_only=index_only, sync=sync)

    # correctness guard on the bench path itself: totals, statuses, and the
    # outputs against the oracle (every array on rank 0, sampled blocks elsewhere)
    o = step(sync=True)
    assert o.n_rows == rows and o.n_bad_blocks == 0, (o.n_rows, rows, o.n_bad_blocks)
    ver = None
    if not args.no_verify:
        t1 = time.time()
        ver = verify_decode(out, seg, descs, comp, index_only, rank == 0, torch)
        ver["seconds"] = round(time.time() - t1, 1)
        log(f"[rank {rank}] {ver['verified']} ({ver['seconds']} s)")
    # Throughput: a reader decoding consecutive segments (a compaction feed, a
    # scan over many segments) keeps `inflight` whole-segment decodes in flight,
    # each with its own context, stream and output buffers, so one decode's
    # latency-bound pass 1 overlaps another's bandwidth-bound pass 3.  Every
    # step is still one whole-segment decode; the one-at-a-time latency is
    # reported beside it.
    # Each in-flight decode reads its own copy of the segment (consecutive
    # segments of a reader are different bytes: two decodes of one buffer
    # could share its lines in the caches).
    inflight = max(1, args.decode_inflight if args.decode_inflight is not None
                   else (4 if args.config == "c3" else 2))
    decs, outs, streams, segs = [dec], [out], [], [seg_t]
    for i in range(1, inflight):
        streams.append(torch.cuda.Stream(dev))
        decs.append(okv.Decoder(D.local, stream=streams[-1].cuda_stream))
        outs.append(new_out())
        segs.append(seg_t.clone())
        torch.cuda.synchronize(dev)  # the copy (current stream) before the decode (its stream)
        decs[i].decode_device(segs[i], seg.nbytes, d_t, nblk, outs[i], compression=comp,
                              index_only=index_only, sync=True)
        for k, v in out.items():  # each context's outputs == the verified ones
            if index_only and k in ("key_arena", "val_arena", "key_base", "val_base"):
                continue
            assert torch.equal(outs[i][k], v), k
    # pass 3 of each decode waits for the previous decode's pass 3 (ring of
    # contexts, okv_decode_chain): one decode's header walk (pass 1) runs under
    # the previous decode's pass 3, while the bandwidth-bound pass-3 kernels of
    # two segments never share the HBM (measured: sharing it is slower).  Only
    # for large blocks: small-block and zstd decodes are latency-bound and gain
    # from running side by side.
    chained = inflight > 1 and bs >= 32768 and kind != "zstd"
    if args.pass3_chain != "auto":
        chained = inflight > 1 and args.pass3_chain == "on"
    if chained:
        for i in range(inflight):
            decs[i].chain(decs[i - 1])
    turn = [0]

    def step_inflight(sync=False):
        i = turn[0] % inflight
        turn[0] += 1
        return decs[i].decode_device(segs[i], seg.nbytes, d_t, nblk, outs[i], compression=comp,
                                     index_only=index_only, sync=sync)

    for _ in range(max(args.warmup, inflight)):
        step_inflight()
    torch.cuda.synchronize(dev)

    # ---- timed region (no instrumentation: per-pass events cost ~5 us each in
    # the stream, 40 % of a C2 step) -----------------------------------------------
    t_max, per = D.timed(step_inflight, args.steps)
    ms_per_step = 1e3 * t_max / args.steps
    if chained:
        for d in decs:
            d.chain(None)
    t_one, _ = D.timed(step, args.steps) if inflight > 1 else (t_max, per)
    for d in decs[1:]:
        d.close()
    # per-pass kernel times from a second, event-instrumented run of the same steps
    dec.profile(True)
    D.timed(step, args.steps)
    kern_ms, calls = dec.profile_read()
    dec.profile(False)

    # ---- roofline for the dominant kernel ------------------------------------------
    ms = {k: v / max(calls, 1) for k, v in kern_ms.items()}
    if index_only:
        # index mode reads only the record headers: 6 B per row (+ the descs)
        alg = rows * 6 + rows * 22 + nblk * 12
        roof_kernel, roof_ms = "okv_gather_kernel (index)", ms["copy"]
    elif comp:
        # the zstd stage dominates: compressed frames in, decompressed blocks out
        alg = comp_bytes + orig_bytes
        roof_kernel, roof_ms = "zstd stage (okv_zstd_* kernels)", ms["zstd"]
    else:
        # read OriginalSize per block; write payload (padded arenas) + 22 B/row
        # SoA (u64 key_off, u16 key_len, u64 val_off, u32 val_len) + 28 B/block
        alg = orig_bytes + payload + rows * 22 + nblk * 28
        roof_kernel = path_kernels(okv, dec.last_path())
        roof_ms = ms["copy"]
    achieved = alg / (roof_ms * 1e-3) / 1e9
    pass3 = tuple(w for w in roof_kernel.replace("(", " ").split() if w.startswith("okv_"))
    if comp:  # the zstd stage: its kernels' bytes per decode, summed (zstd sources)
        traffic, traffic_src = pmc_traffic(args.config, args.mode, ("okv_zstd_",), ZSTD_SOURCES)
    else:
        traffic, traffic_src = pmc_traffic(args.config, args.mode, pass3)

    # ---- CPU baseline (rank 0, after every rank's timing has finished) ------------
    cpu = None
    if rank == 0 and not args.no_cpu:
        cpu = cpu_decode_baseline(args, seg, descs, nblk, comp)
        if world > 1:
            cpu["sample"] += f"; run on rank 0 of {world} after the timed region"

    e2e = None
    if args.e2e and rank == 0 and world == 1:
        from tools.e2e import run_e2e
        dec.close()
        e2e = run_e2e(args.config, torch=torch)

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
        "per_rank_ms_per_step": [round(1e3 * p / args.steps, 4) for p in per],
        "decodes_in_flight": inflight,
        "pass3_chained": chained,
        "latency_ms_per_step": round(1e3 * t_one / args.steps, 4),
        "kernel_ms": {k: round(v, 4) for k, v in ms.items()},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     # the same algorithmic bytes over the whole decode (count + scan +
                     # pass 3 + launch gaps): one decode at a time, and per step with
                     # `decodes_in_flight` decodes overlapping (the `value` clock)
                     "frac_pass3": round(achieved / HBM_PEAK_GBS, 4),
                     "frac_step": round(alg / (t_one / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
                     "frac_step_inflight": round(alg / (t_max / args.steps) / 1e9 /
                                                 HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel": roof_kernel,
                     "algorithmic_bytes_per_launch": int(alg),
                     "timing": "HIP events around the kernel on its stream, averaged over a "
                               "second run of the same steps (the timed run carries no events)",
                     "traffic_source": traffic_src, "decode_source_sha": source_sha(),
                     # the same kernel's rocprofv3 trace average (another process, maybe
                     # another box) and the event time the traced process measured itself
                     # (one GPU alone: omitted when ranks share the box's GPUs)
                     "trace": (trace_roofline(args.config, alg,
                                              ZSTD_SOURCES if comp else DECODE_SOURCES)
                               if world == 1 else None)},
        "cpu_baseline": cpu,
        "verify": ver,
        "dist": D.info(),
    }
    if e2e:
        line["e2e"] = e2e
    emit(D, line)
    if not e2e:
        dec.close()


def path_kernels(okv, lp):
    """The pass-3 kernels the last decode launched (okv_last_path bits)."""
    L = okv._lib
    names = [(L.PATH_FUSED, "okv_decode_fused_kernel (passes 1-3)"),
             (L.PATH_GROUP, "okv_group_kernel (passes 1-3)"),
             (L.PATH_STREAM, "okv_decode_stream_kernel (passes 1-3)"),
             (L.PATH_SMALL, "okv_gather_small_kernel"), (L.PATH_TILE, "okv_tile_kernel"),
             (L.PATH_SWEEP, "okv_rows_kernel + okv_value_sweep_kernel"),
             (L.PATH_STAGED, "okv_gather_staged_kernel"), (L.PATH_GATHER, "okv_gather_kernel")]
    # (the big-block kernel of these paths, okv_copy_kernel, runs before the
    # pass-3 interval since round 6: after the count, ahead of the chain wait)
    return " + ".join(n for bit, n in names if lp & bit) or "none"


def cpu_decode_baseline(args, seg, descs, nblk, comp):
    """The C restatement of ReadBlockWithStat with Go's allocation semantics
    (per-block buffer copy, per-row key/value heap copies), swept over thread
    counts (thread t decodes a contiguous block range of the sample)."""
    from oracle import coracle
    cd = np.ascontiguousarray(descs, np.uint64).view(coracle.DESC_DTYPE).reshape(-1)
    big = args.config in ("c3", "cz", "c5")
    samples = {}

    def once(nth):
        sample = min(nblk, 4096 * nth if big else nblk)
        samples[nth] = sample
        coracle.decode_go(seg, cd[:sample], comp, nth)
        return int(descs[:sample, 1].sum())
    res = sweep(once, args.cpu_seconds / len(thread_counts()))
    return sweep_summary(res, 1 / 2**30, "GiB/s", "port",
                         f"first min({nblk}, 4096 x threads) blocks per pass (all {nblk} at "
                         f"{max(res)} threads), whole passes for "
                         f"{args.cpu_seconds / len(thread_counts()):.1f} s per thread count; C "
                         f"restatement of Go ReadBlockWithStat with Go allocation semantics (Go "
                         f"toolchain unavailable)" + ALLOC_NOTE)


# ---- encode (C4) ------------------------------------------------------------------


def run_encode(args, torch, okv, D):
    """C4: okv_encode_rows over rows resident in HBM.  One step = the whole
    encode of this rank's key-range shard, Close included: cut + pack + block
    hash + meta block on device, then the meta block's XXH64 and the 25-byte
    trailer (one sequential hash over the meta block, on the host).  Total
    rows fixed across N: strong scaling."""
    _, seed, total_rows, th, bs, desc = CONFIGS["c4"]
    rank, world, dev = D.rank, D.world, D.dev
    KL, VL = 16, 64
    lo, hi = total_rows * rank // world, total_rows * (rank + 1) // world
    n = hi - lo
    stream = torch.cuda.current_stream(dev)
    enc = okv.Encoder(D.local, stream=stream.cuda_stream)
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

    def step():
        return enc.encode_device(rows, n, out, threshold=th, block_size=bs, strict_go=False)

    def new_out():
        return {k: torch.empty_like(v) for k, v in out.items()}

    # correctness guard: the whole segment file against the oracle writer on
    # rank 0 (tests/test_full_size_gpu.py does the same at 100 M rows); block
    # count/sizes and device-rehashed blocks on every rank
    eo = step()
    assert eo.n_blocks == nb and eo.data_bytes == nb * bs, (eo.n_blocks, nb)
    hv = torch.empty(nb, dtype=torch.int64, device=dev)
    enc._check(okv._lib.lib().okv_hash_blocks(enc._ctx, out["seg"].data_ptr(), eo.data_bytes,
                                               out["desc"].data_ptr(), nb, hv.data_ptr(),
                                               okv._lib.F_DEVICE_PTRS), "hash")
    assert torch.equal(hv, out["hash"][:nb])  # the fused block hashes == a separate rehash
    ver = None
    if rank == 0 and not args.no_verify:
        from oracle import coracle
        t1 = time.time()
        host = {k: v.cpu().numpy() for k, v in rows.items()}
        for k, dt in (("key_off", np.uint64), ("val_off", np.uint64), ("key_len", np.uint16),
                      ("val_len", np.uint32)):
            host[k] = host[k].view(dt)
        want = coracle.encode_soa(host, n, th, bs)
        assert want.rc == 0 and want.file.size == eo.file_bytes
        step_b = 1 << 28
        for i in range(0, want.file.size, step_b):
            j = min(want.file.size, i + step_b)
            assert np.array_equal(out["seg"][i:j].cpu().numpy(), want.file[i:j]), (i, j)
        del host, want
        ver = {"verified": "whole segment file == oracle writer (oref_encode_soa)",
               "seconds": round(time.time() - t1, 1)}
        log(f"[rank {rank}] {ver['verified']} ({ver['seconds']} s)")
    data_bytes, meta_bytes, file_bytes = eo.data_bytes, eo.meta_bytes, eo.file_bytes

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    enc.profile(True)
    enc.profile_reset_encode()
    t_lat, per_lat = D.timed(step, args.steps)  # one segment at a time: encode + Close latency
    ph, calls = enc.profile_read_encode()
    enc.profile(False)
    ph = {k: v / max(calls, 1) for k, v in ph.items()}
    # device-only step (no Close), for reference
    t_dev, _ = D.timed(lambda: enc.encode_device(rows, n, out, threshold=th, block_size=bs,
                                                 strict_go=False, close=False), args.steps)
    # Throughput: a writer producing consecutive segments keeps `inflight` of
    # them open -- segment k's Close (meta-block D2H + its single sequential
    # XXH64 on a host core) runs while segment k+1's cut/pack/hash/meta kernels
    # run.  Each in-flight segment has its own context, stream and output
    # buffers; a token serialises the device phases; every timed step is one
    # whole segment file, Close included.
    inflight = max(1, args.c4_inflight)
    t_step, per = t_lat / args.steps, per_lat
    if inflight > 1:
        import threading
        from concurrent.futures import ThreadPoolExecutor
        streams = [torch.cuda.Stream(dev) for _ in range(inflight - 1)]  # kept alive
        encs = [enc] + [okv.Encoder(D.local, stream=st.cuda_stream) for st in streams]
        outs = [out] + [new_out() for _ in range(inflight - 1)]
        gpu = threading.Lock()

        def worker(i, nseg):
            for _ in range(nseg):
                with gpu:
                    eo_i = encs[i].encode_device(rows, n, outs[i], threshold=th, block_size=bs,
                                                 strict_go=False, close=False)
                encs[i].close_device(eo_i)

        def pipeline(nseg):
            with ThreadPoolExecutor(inflight) as ex:
                futs = [ex.submit(worker, i, nseg // inflight + (i < nseg % inflight))
                        for i in range(inflight)]
                for f in futs:
                    f.result()
        pipeline(2 * inflight)  # warm the extra contexts
        for i in range(1, inflight):  # every in-flight buffer holds the same file
            assert torch.equal(outs[i]["seg"][:file_bytes], out["seg"][:file_bytes])
        t_pipe, per = D.timed(lambda: pipeline(args.steps), 1)
        t_step = t_pipe / args.steps
        for e_ in encs[1:]:
            e_.close()
        del outs
    # pack kernel: read payload (16+64 B/row) + SoA (22 B/row), write the padded blocks
    alg = n * (KL + VL) + n * 22 + data_bytes
    achieved = alg / (ph["pack"] * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic("c4", "encode", "okv_enc_pack_lds_kernel", ENCODE_SOURCES)

    # ---- CPU baseline (rank 0, after every rank's timing has finished) ------------
    cpu = None
    if rank == 0 and not args.no_cpu:
        cpu = cpu_encode_baseline(args, rows, n, th, bs)
        if world > 1:
            cpu["sample"] += f"; run on rank 0 of {world} after the timed region"

    line = {
        "metric": ENC_METRIC, "value": round(data_bytes * world / t_step / 2**30, 3),
        "unit": "GiB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": desc, "rows_total": total_rows, "rows_per_gpu": n,
                   "blocks_per_gpu": nb, "data_bytes_per_gpu": data_bytes,
                   "meta_bytes_per_gpu": meta_bytes, "file_bytes_per_gpu": file_bytes,
                   "threshold": th, "block_size": bs,
                   "parallelism": f"{world} key-range shards, one segment each (no collective)"},
        "rows_per_s": round(total_rows / t_step),
        "mrows_per_s": round(total_rows / t_step / 1e6, 3),
        "per_rank_ms_per_step": [round(1e3 * p / args.steps, 4) for p in per],
        "segments_in_flight": inflight,
        "latency_ms_per_segment": round(1e3 * t_lat / args.steps, 4),
        "device_only_ms_per_step": round(1e3 * t_dev / args.steps, 4),
        "kernel_ms": {k: round(v, 4) for k, v in ph.items()},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "okv_enc_pack_lds_kernel (pack + block XXH64)",
                     "algorithmic_bytes_per_launch": int(alg),
                     "encode_source_sha": source_sha(ENCODE_SOURCES)},
        "cpu_baseline": cpu,
        "verify": ver,
        "dist": D.info(),
    }
    emit(D, line)
    enc.close()


def cpu_encode_baseline(args, rows, n, th, bs):
    """The C writer restatement with Go's per-row rowBuf allocation, threads
    writing key-range shards as separate segments."""
    from oracle import coracle
    sample = min(n, 8_000_000)
    host = {k: rows[k][:sample].cpu().numpy() for k in ("key_off", "key_len", "val_off",
                                                         "val_len")}
    host["key_off"] = host["key_off"].view(np.uint64)
    host["val_off"] = host["val_off"].view(np.uint64)
    host["key_len"] = host["key_len"].view(np.uint16)
    host["val_len"] = host["val_len"].view(np.uint32)
    host["key_arena"] = rows["key_arena"][:sample * 16].cpu().numpy()
    host["val_arena"] = rows["val_arena"][:sample * 64].cpu().numpy()

    def once(nth):
        ns = min(sample, 1_000_000 * nth)
        return coracle.encode_go(host, ns, th, bs, False, nth)
    res = sweep(once, args.cpu_seconds / len(thread_counts()))
    return sweep_summary(res, 1 / 2**30, "GiB/s", "port",
                         f"min({sample}, 1 M x threads) rows per pass as one key-range segment "
                         f"per thread; C restatement of Go WriteRow+Close with per-row rowBuf "
                         f"allocation (Go toolchain unavailable); segment bytes written / s"
                         + ALLOC_NOTE)


# ---- compaction (CM) -----------------------------------------------------------------


def _fixed_vals(seed, r0, n, vl=64):
    """Values of rows r0 .. r0 + n - 1 of rows_fixed(seed) (splitmix64 words
    drawn in row order; okv_synth_rows_fixed), for the guard below."""
    w = np.arange(r0 * (vl // 8), (r0 + n) * (vl // 8), dtype=np.uint64) + np.uint64(1)
    z = np.uint64(seed) + w * np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8).reshape(n, vl)


def run_compact(args, torch, okv, D):
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
    rank, world, dev = D.rank, D.world, D.dev
    K, KL, VL = 4, 16, 64
    seed0 += 100 * rank
    stream = torch.cuda.current_stream(dev)
    enc = okv.Encoder(D.local, stream=stream.cuda_stream)
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
                          rows=r, kb=kb, vb=vb))
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
    seg_t0, fb0, d_t0, nb0 = segs[0]  # which decode kernels the stage runs
    enc.decode_device(seg_t0, fb0, d_t0, nb0, douts[0], sync=True)
    dec_kernels = path_kernels(okv, enc.last_path())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    t_max, per = D.timed(step, args.steps)  # uninstrumented
    t_step = t_max / args.steps
    enc.profile(True)  # per-pass event timing in a second run
    D.timed(step, args.steps)
    kern_ms, calls = enc.profile_read()  # the K decodes of every step
    enc.profile(False)
    ph = np.zeros(3)  # untimed diagnostic pass: per-stage wall time
    for _ in range(2):
        step(ph)
    ph *= 1e3 / 2
    # roofline of the decode stage's pass-3 kernel (okv_group_kernel: passes
    # 1-3 in one launch, since round 6): per step K launches over all input blocks
    gather_ms = kern_ms["copy"] / max(calls, 1) * K
    orig = 0
    for seg_t, fb, d_t, nb in segs:
        orig += int(d_t[:, 2].sum().item())
    alg = orig + sum(d["kb"] + d["vb"] for d in douts) + n_in * 22 + \
        sum(nb for *_x, nb in segs) * 28
    achieved = alg / (gather_ms * 1e-3) / 1e9

    cpu = None
    if rank == 0 and not args.no_cpu:  # (after every rank's timing)
        cpu = cpu_compact_baseline(args, segs, n, per_block, th, bs, K)
        if world > 1:
            cpu["sample"] += f"; run on rank 0 of {world} after the timed region"

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
        "per_rank_ms_per_step": [round(1e3 * p / args.steps, 4) for p in per],
        "stage_ms": {"decode": round(ph[0], 4), "merge": round(ph[1], 4),
                     "encode": round(ph[2], 4)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": f"{dec_kernels} (decode stage, {K} launches per step)",
                     "algorithmic_bytes_per_launch": int(alg / K),
                     "kernel_ms_per_step": round(gather_ms, 4)},
        "cpu_baseline": cpu,
        "dist": D.info(),
    }
    emit(D, line)
    enc.close()


def cpu_compact_baseline(args, segs, n, per_block, th, bs, K):
    """The compaction step on the host: every sampled block of the K segments
    decoded with ReadBlockWithStat's semantics, merged newest-first, written
    with the Go writer (oref_compact_go).  Sample: the blocks of each segment
    that hold global rows [n/2 + n/8, n/2 + n/8 + m) -- a key range covered
    by two or three segments, so the merge resolves real overlaps."""
    from oracle import coracle
    m = 200_000
    x0 = n // 2 + n // 8
    host = []
    for s in range(K - 1, -1, -1):  # newest first
        seg_t, fb, d_t, nb = segs[s]
        lo_row = s * n // 2
        r0, r1 = max(x0, lo_row), min(x0 + m, lo_row + n)
        if r0 >= r1:
            continue
        b0, b1 = (r0 - lo_row) // per_block, -(-(r1 - lo_row) // per_block)
        d = d_t[b0:b1].cpu().numpy().view(np.uint64).copy()
        base = int(d[0, 0])
        end = int(d[-1, 0] + d[-1, 1])
        part = seg_t[base:end].cpu().numpy()
        d[:, 0] -= base
        host.append((part, d.view(coracle.DESC_DTYPE).reshape(-1)))
    in_b = sum(int(d["block_size"].sum()) for _p, d in host)
    out_rows = {}

    def once(nth):
        out_rows[nth] = coracle.compact_go(host, th, bs, nth)
        return in_b * nth
    res = sweep(once, args.cpu_seconds / len(thread_counts()))
    n_out, ob = out_rows[1]
    q1 = ("; Go's Close panics after the last WriteRow flushes (SURVEY Q1): the rows are "
          "written first and counted" if n_out and not ob else "")
    return sweep_summary(res, 1 / 2**30, "GiB/s", "port",
                         f"{len(host)} segments' blocks holding rows [{x0}, {x0 + m}) "
                         f"({in_b} B in, {n_out} rows merged and written{q1}) per compaction, one "
                         f"independent compaction per thread; C restatement: "
                         f"ReadBlockWithStat per block, newest-wins merge, Go writer (the "
                         f"reference's compactor is a stub)" + ALLOC_NOTE)


# ---- C1 round trip ---------------------------------------------------------------------


def run_roundtrip(args, torch, okv, D):
    """C1: 10 000 16/64 rows -> one segment -> a full ascending read.  GPU: the
    rows resident in HBM, okv_encode_rows (Close included) then okv_decode_blocks
    of every block of the new segment (a batched RowIter's reads); CPU: the C
    restatement of WriteRow/Close + ReadBlockWithStat with Go's allocations, on
    1 thread and as independent round trips on every core.  Segment bytes
    (992 878 B) are the MB/s numerator."""
    _, seed, n, th, bs, desc = CONFIGS["c1"]
    rank, world, dev = D.rank, D.world, D.dev
    stream = torch.cuda.current_stream(dev)
    enc = okv.Encoder(D.local, stream=stream.cuda_stream)
    rows = dict(key_arena=torch.empty(n * 16, dtype=torch.uint8, device=dev),
                key_off=torch.empty(n, dtype=torch.int64, device=dev),
                key_len=torch.empty(n, dtype=torch.int16, device=dev),
                val_arena=torch.empty(n * 64, dtype=torch.uint8, device=dev),
                val_off=torch.empty(n, dtype=torch.int64, device=dev),
                val_len=torch.empty(n, dtype=torch.int32, device=dev))
    enc.synth_fixed_device(seed, 0, n, 16, 64, rows)
    nb = -(-n // 42)
    out = dict(seg=torch.empty(nb * bs + (nb + 1) * 58 + 4096, dtype=torch.uint8, device=dev),
               desc=torch.empty((nb + 1, 4), dtype=torch.int64, device=dev))
    eo = enc.encode_device(rows, n, out, threshold=th, block_size=bs, strict_go=True)
    fb = int(eo.file_bytes)
    r, kb, vb = enc.plan_device(out["seg"], fb, out["desc"], nb)
    dout = dict(row_start=torch.empty(nb + 1, dtype=torch.int64, device=dev),
                key_base=torch.empty(nb, dtype=torch.int64, device=dev),
                val_base=torch.empty(nb, dtype=torch.int64, device=dev),
                status=torch.empty(nb, dtype=torch.int32, device=dev),
                key_off=torch.empty(r, dtype=torch.int64, device=dev),
                key_len=torch.empty(r, dtype=torch.int16, device=dev),
                val_off=torch.empty(r, dtype=torch.int64, device=dev),
                val_len=torch.empty(r, dtype=torch.int32, device=dev),
                key_arena=torch.empty(max(kb, 16), dtype=torch.uint8, device=dev),
                val_arena=torch.empty(max(vb, 16), dtype=torch.uint8, device=dev))

    def step():
        e = enc.encode_device(rows, n, out, threshold=th, block_size=bs, strict_go=True)
        enc.decode_device(out["seg"], int(e.file_bytes), out["desc"], nb, dout, sync=False)

    step()
    torch.cuda.synchronize(dev)
    assert r == n and torch.equal(dout["key_arena"][:n * 16], rows["key_arena"])
    assert torch.equal(dout["val_arena"][:n * 64], rows["val_arena"])
    from oracle import coracle
    host = {k: v.cpu().numpy() for k, v in rows.items()}
    for k, dt in (("key_off", np.uint64), ("val_off", np.uint64), ("key_len", np.uint16),
                  ("val_len", np.uint32)):
        host[k] = host[k].view(dt)
    want = coracle.encode_soa(host, n, th, bs)
    assert want.rc == 0 and out["seg"][:fb].cpu().numpy().tobytes() == want.file.tobytes()
    for _ in range(args.warmup):
        step()
    t_max, per = D.timed(step, args.steps)
    t_step = t_max / args.steps

    cpu = None
    if rank == 0 and not args.no_cpu:  # (after every rank's timing)
        def once(nth):
            _r, b_ = coracle.roundtrip_go(host, n, th, bs, nth)
            return b_
        res = sweep(once, args.cpu_seconds / len(thread_counts()))
        cpu = sweep_summary(res, 1e-6, "MB/s", "port",
                            "the whole C1 round trip per pass, one independent segment per "
                            "thread; C restatement of Go WriteRow/Close + ReadBlockWithStat "
                            "with Go allocations" + ALLOC_NOTE)
        if world > 1:
            cpu["sample"] += f"; run on rank 0 of {world} after the timed region"
    line = {
        "metric": RT_METRIC, "value": round(fb * world / t_step / 1e6, 3), "unit": "MB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": desc, "rows": n, "blocks": nb, "file_bytes": fb,
                   "parallelism": f"{world} independent round trips (no collective)"},
        "rows_per_s": round(n * world / t_step),
        "per_rank_ms_per_step": [round(1e3 * p / args.steps, 4) for p in per],
        "roofline": None,
        "cpu_baseline": cpu,
        "verify": {"verified": "segment == oracle writer; decoded arenas == input rows"},
        "dist": D.info(),
    }
    emit(D, line)
    enc.close()


if __name__ == "__main__":
    sys.exit(main())
