"""Multi-GPU partitioning for the decode.

Blocks and segments are independent, so the data path needs no collective:
each rank decodes its own blocks.  The only cross-rank step is control
plane -- turning per-rank row counts into global row ids (an exclusive scan
of `world` integers), done here with one all_gather on any
torch.distributed backend (gloo on CPU, nccl=RCCL on GPU).
"""
from __future__ import annotations

import numpy as np


def partition_blocks(descs: np.ndarray, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block range [b0, b1) for `rank`, balanced by BlockSize bytes."""
    d = np.asarray(descs, dtype=np.uint64).reshape(-1, 4)
    n = d.shape[0]
    if n == 0:
        return 0, 0
    cum = np.cumsum(d[:, 1].astype(np.float64))
    total = cum[-1]

    def cut(k):
        if k <= 0:
            return 0
        if k >= world:
            return n
        return int(np.searchsorted(cum, total * k / world, side="left")) + 1

    b0, b1 = cut(rank), cut(rank + 1)
    return min(b0, n), min(max(b1, b0), n)


def global_row_base(local_rows: int, group=None) -> tuple[int, int]:
    """(first global row id of this rank, total rows) from per-rank counts."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else "cpu"
    mine = torch.tensor([local_rows], dtype=torch.int64, device=dev)
    allc = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(allc, mine, group=group)
    counts = [int(x.item()) for x in allc]
    return sum(counts[:rank]), sum(counts)
