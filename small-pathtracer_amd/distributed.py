"""Multi-GPU assembly of row-tile shards: one gather of each rank's fp32 rows to
rank 0 — RCCL over xGMI when the process group backend is "nccl", gloo on CPU in tests.

Rank k renders the rows spt_shard_rows(params with shard_index=k) into a compact (rows, w, 3)
buffer; shards are padded to the largest shard so one fixed-size gather moves them all; rank 0
scatters each shard's rows back into the full image (device-side index_copy). No reduction is
needed: pixels are disjoint.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np


def shard_row_lists(height: int, tile_rows: int, world: int) -> List[np.ndarray]:
    """Rows owned by every rank (tile t -> rank t % world), the same rule as spt_shard_rows()."""
    out = []
    for k in range(world):
        rows = [r for t in range(k, (height + tile_rows - 1) // tile_rows, world)
                for r in range(t * tile_rows, min(t * tile_rows + tile_rows, height))]
        out.append(np.asarray(rows, dtype=np.int64))
    return out


def gather_rows(shard, rows_of: Sequence[np.ndarray], full=None, gather_list=None, group=None):
    """Gather `shard` ((max_rows, w, 3), this rank's rows first) from every rank to rank 0 and
    de-interleave into `full` ((h, w, 3)) there. `gather_list` may be passed pre-allocated on
    rank 0 to keep allocations out of a timed loop. Returns `full` on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if rank == 0:
        if gather_list is None:
            gather_list = [torch.empty_like(shard) for _ in range(world)]
        dist.gather(shard, gather_list, dst=0, group=group)
        for k in range(world):
            idx = torch.as_tensor(rows_of[k], dtype=torch.long, device=shard.device)
            full.index_copy_(0, idx, gather_list[k][: len(rows_of[k])])
        return full
    dist.gather(shard, None, dst=0, group=group)
    return None


def max_rows(rows_of: Sequence[np.ndarray]) -> int:
    return max(len(r) for r in rows_of)


__all__ = ["shard_row_lists", "gather_rows", "max_rows"]
