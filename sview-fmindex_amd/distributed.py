"""Multi-GPU helpers: one process per GPU, patterns sharded, blob replicated.

Pattern batches are independent: rank r takes a contiguous
slab of the global batch, runs it on its own GPU against its own replica of
the blob, and the per-rank results are concatenated with all-gathers (RCCL
over xGMI on MI355X nodes, gloo on CPU for tests).  No collective runs inside
the query path itself; the gather of one launch's results can run on a
communication stream while the next launch computes (`ShardGather`).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def shard(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous slab [start, end) of n_total patterns for `rank`
    (sizes differ by at most one)."""
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_sizes(n_total: int, world: int) -> List[int]:
    return [e - s for s, e in (shard(n_total, world, r) for r in range(world))]


class SlabGather:
    """All-gather of per-rank locate results with no host round trip.

    Each rank owns `slots` result slots of fixed shape: `batch` counts (P-wide)
    and `loc_cap` locations — the kernels write a batch's counts and
    locations straight into a slot (`counts_slot(j)`, `locs_slot(j)`), and
    loc_cap is a bound every batch's total stays under (checked when the batch
    first runs).  Everything is fixed-size, so `gather()` is two all-gathers
    with no size exchange, enqueued on the current stream (issue it on a
    communication stream to overlap it with the next launch).  `result(r, j,
    n)` reads back slot j of rank r's first n patterns as (offsets,
    locations) on the device."""

    def __init__(self, world: int, slots: int, batch: int, loc_cap: int, count_dtype, loc_dtype, device,
                 group=None):
        import torch
        self.world, self.slots, self.batch, self.loc_cap = world, slots, batch, int(loc_cap)
        self.group = group
        self.counts_in = torch.zeros(slots * batch, dtype=count_dtype, device=device)
        self.locs_in = torch.zeros(slots * self.loc_cap, dtype=loc_dtype, device=device)
        self.counts_all = torch.zeros(world * slots * batch, dtype=count_dtype, device=device)
        self.locs_all = torch.zeros(world * slots * self.loc_cap, dtype=loc_dtype, device=device)

    def counts_slot(self, j: int):
        return self.counts_in[j * self.batch:(j + 1) * self.batch]

    def locs_slot(self, j: int):
        return self.locs_in[j * self.loc_cap:(j + 1) * self.loc_cap]

    def gather(self, async_op: bool = False):
        w1 = _all_gather_flat(self.counts_all, self.counts_in, self.group, async_op)
        w2 = _all_gather_flat(self.locs_all, self.locs_in, self.group, async_op)
        return (w1, w2) if async_op else None

    def result(self, r: int, j: int, n: int):
        """(offsets int64[n+1], locations[total]) of rank r's slot j."""
        import torch
        c0 = (r * self.slots + j) * self.batch
        counts = self.counts_all[c0:c0 + n].to(torch.int64)
        offsets = torch.zeros(n + 1, dtype=torch.int64, device=counts.device)
        torch.cumsum(counts, 0, out=offsets[1:])
        l0 = (r * self.slots + j) * self.loc_cap
        total = int(offsets[-1].item()) if n else 0
        return offsets, self.locs_all[l0:l0 + total]

    def bytes_per_gather(self) -> int:
        return (self.counts_all.numel() * self.counts_all.element_size()
                + self.locs_all.numel() * self.locs_all.element_size())


def concat(parts):
    """Concatenate per-rank (offsets, locations) results in rank order into
    the (offsets, locations) one device would have produced for the union."""
    import torch
    offs, locs, base = [parts[0][0][:1]], [], 0
    for o, l in parts:
        offs.append(o[1:] + base)
        locs.append(l)
        base = base + o[-1]
    return torch.cat(offs), torch.cat(locs)


def _all_gather_flat(out, inp, group, async_op):
    """all_gather_into_tensor (one flat output, rank-major); backends without
    it (older gloo) get the list form copied into `out`."""
    import torch.distributed as dist
    try:
        return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)
    except (RuntimeError, NotImplementedError):
        parts = list(out.view(-1, inp.numel()).unbind(0))
        dist.all_gather(parts, inp, group=group)
        return None


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
