"""World-size-2 gloo test of the multi-GPU decode partitioning (no GPU):
each rank takes a contiguous byte-balanced block range, decodes it with the
CPU oracle (standing in for its GPU), and the ranks agree on global row ids
through one control-plane all_gather -- concatenated, they equal the
single-process decode."""
from __future__ import annotations

import os
import tempfile

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from objectkv_amd.shard import global_row_base, partition_blocks
from oracle import coracle as CO
from oracle import pyoracle as P


def _segment():
    seg, meta, w = P.build_segment(P.rows_zipf(3), nblocks_target=12, threshold=57344,
                                   block_size=65536)
    descs = np.array([st.desc() for st in P.bytes_to_metadata(meta).entries], np.uint64)
    return seg, descs


def _worker(rank, world, initf, outdir):
    dist.init_process_group("gloo", init_method=f"file://{initf}", rank=rank,
                            world_size=world)
    seg, descs = _segment()
    b0, b1 = partition_blocks(descs, world, rank)
    o = CO.decode_soa(seg, CO.descs_array([tuple(int(x) for x in d) for d in descs[b0:b1]]))
    base, total = global_row_base(int(o["row_start"][-1]))
    np.savez(os.path.join(outdir, f"r{rank}.npz"), b0=b0, b1=b1, base=base, total=total,
             key_len=o["key_len"], val_len=o["val_len"])
    dist.barrier()
    dist.destroy_process_group()


def test_partition_covers_all_blocks():
    _, descs = _segment()
    for world in (1, 2, 3, 4, 8):
        ranges = [partition_blocks(descs, world, r) for r in range(world)]
        assert ranges[0][0] == 0 and ranges[-1][1] == len(descs)
        for (a0, a1), (c0, c1) in zip(ranges, ranges[1:]):
            assert a1 == c0 and a0 <= a1


def test_gloo_world2_global_rows():
    world = 2
    with tempfile.TemporaryDirectory() as td:
        initf = os.path.join(td, "init")
        mp.spawn(_worker, args=(world, initf, td), nprocs=world, join=True)
        seg, descs = _segment()
        full = CO.decode_soa(seg, CO.descs_array([tuple(int(x) for x in d) for d in descs]))
        parts = [np.load(os.path.join(td, f"r{r}.npz")) for r in range(world)]
        assert parts[0]["base"] == 0
        assert parts[1]["base"] == len(parts[0]["key_len"])
        assert all(int(p["total"]) == int(full["row_start"][-1]) for p in parts)
        assert np.array_equal(np.concatenate([p["key_len"] for p in parts]), full["key_len"])
        assert np.array_equal(np.concatenate([p["val_len"] for p in parts]), full["val_len"])
