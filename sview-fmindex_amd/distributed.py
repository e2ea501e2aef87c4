"""Multi-GPU helpers: one process per GPU, patterns sharded, blob replicated.

Pattern batches are independent: rank r takes a contiguous
slab of the global batch, runs it on its own GPU against its own replica of
the blob, and the per-rank results are concatenated afterwards with
all-gathers (RCCL over xGMI on MI355X nodes, gloo on CPU for tests).  No
collective runs inside the query path.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


def shard(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous slab [start, end) of n_total patterns for `rank`
    (sizes differ by at most one)."""
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def allgather_ragged(t, group=None) -> list:
    """All-gather 1-D tensors of different lengths (pad to the max, trim)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes) if sizes else 0
    padded = torch.zeros(max(mx, 1), dtype=t.dtype, device=t.device)
    padded[:t.numel()] = t
    outs = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(outs, padded, group=group)
    return [o[:s] for o, s in zip(outs, sizes)]


def concat_results(loc_offsets, locations, group=None):
    """Concatenate per-rank (offsets[n_r+1], locations) into the global
    (offsets[N+1], locations) in rank order — the result of running the whole
    batch on one device."""
    import torch
    offs = allgather_ragged(loc_offsets, group)
    locs = allgather_ragged(locations, group)
    out_off: List = [torch.zeros(1, dtype=loc_offsets.dtype, device=loc_offsets.device)]
    base = 0
    for o in offs:
        out_off.append(o[1:] + base)
        base += int(o[-1].item()) if o.numel() else 0
    return torch.cat(out_off), torch.cat(locs)


def max_over_ranks(x: float, device=None, group=None) -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def slab_patterns(data: np.ndarray, offsets: np.ndarray, start: int, end: int):
    """Sub-batch [start, end) of a packed (bytes, offsets) batch, rebased."""
    b0, b1 = int(offsets[start]), int(offsets[end])
    return data[b0:b1], (offsets[start:end + 1] - offsets[start]).astype(np.uint64)
