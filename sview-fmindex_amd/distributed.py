"""Multi-GPU helpers: one process per GPU, patterns sharded, blob replicated.

Pattern batches are independent: every rank answers its
share of a job against its own replica of the blob, and the per-rank results
are concatenated with all-gathers (RCCL over xGMI on MI355X nodes, gloo on
CPU for tests).  No collective runs inside the query path itself.

- `JobPlan` deals a job of `total` patterns out: rank r takes the contiguous
  slab `shard(total, world, r)`, cut into `nb` near-equal batches — `nb` the
  same on every rank and a multiple of the launch-group size — so every rank
  runs the same launches and per-rank pattern counts differ by at most one.
- `JobGather` collects a sharded job's results with ONE all-gather per launch
  group: each rank's counts and locations of the group's batches are packed
  into one slab (counts first, then the locations of every batch back to
  back), sized exactly from the batches' location totals, so the kernels
  write their outputs straight into the slab and nothing is padded beyond
  the largest rank's share.  `assemble()` concatenates the gathered slabs on
  the device into the job's flat (offsets, locations) — the answer one
  device would give for the whole job — with no host round trip per slot.
- `ShardedLocate` is the same for one global batch as a call: every rank
  passes the batch, locates its shard, one packed all-gather, and every rank
  gets the batch's (offsets, locations).
- `replicate_blob` broadcasts rank 0's blob to every rank (RCCL over xGMI).
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


class JobPlan:
    """How a job of `total` patterns runs on `world` ranks in launch groups of
    `group` batches of about `batch_target` patterns.

    Rank r owns the global patterns shard(total, world, r); its slab is cut
    into `nb` batches with shard(slab, nb, j) (sizes differ by at most one),
    where nb = group * ceil(ceil(max slab / batch_target) / group) is the same
    on every rank.  So every rank issues nb / group launches of about the
    same size, and the ranks' pattern counts differ by at most one — the
    round-robin deal of fixed 100 k batches it replaces gave 8-GPU C5 a 2:1
    imbalance (10 batches over 8 ranks).

    min_groups: at least this many launch groups per rank (nb = group *
    max(ceil(per / group), min_groups)) — bench.py's gathered strong runs
    use one per stream, so that one group's all-gather runs under another
    group's search instead of after the rank's only launch."""

    def __init__(self, total: int, world: int, batch_target: int, group: int, min_groups: int = 1):
        if total < 0 or world < 1 or batch_target < 1 or group < 1 or min_groups < 1:
            raise ValueError("JobPlan: total >= 0, world >= 1, batch_target >= 1, group >= 1, min_groups >= 1")
        self.total, self.world, self.group = int(total), int(world), int(group)
        slab_max = -(-self.total // self.world)
        per = max(1, -(-slab_max // int(batch_target)))
        self.nb = max(-(-per // self.group), int(min_groups)) * self.group
        self.spans = [shard(self.total, self.world, r) for r in range(self.world)]

    @property
    def groups(self) -> int:
        return self.nb // self.group

    def batches(self, rank: int) -> List[Tuple[int, int]]:
        """Global pattern ranges [start, end) of rank's nb batches, in order."""
        s, e = self.spans[rank]
        return [(s + a, s + b) for a, b in (shard(e - s, self.nb, j) for j in range(self.nb))]

    def sizes(self) -> np.ndarray:
        """Patterns per batch, int64[world, nb]."""
        return np.array([[b - a for a, b in self.batches(r)] for r in range(self.world)], dtype=np.int64)

    def max_batch(self) -> int:
        return int(self.sizes().max()) if self.total else 0


class JobGather:
    """One all-gather per launch group of a sharded job's results, into
    exact-size slabs, assembled on the device.

    `sizes[r][j]` / `needs[r][j]`: patterns / locations of rank r's batch j
    (needs come from a sizing pass — bench.py's warm-up — exchanged once with
    `all_gather_ints`).  Group g holds batches [g*group, (g+1)*group).  Rank
    r's part of group g's slab is [its counts of those batches, in order]
    [their locations, back to back]; every rank's part is padded to the
    largest one, so the gather is one all_gather_into_tensor with no size
    exchange in the loop.  `counts_slot(j)` / `locs_slot(j)` are the views the
    kernels write batch j's counts and locations into (locations capacity =
    needs[rank][j] exactly)."""

    def __init__(self, sizes, needs, group: int, rank: int, dtype, device, pg=None, collective=None):
        """collective: gather over the process group even with one rank (a
        one-GPU run that drives the RCCL path: bench.py with FMX_BENCH_DIST=1);
        default: only with several ranks."""
        import torch
        self.sizes = np.asarray(sizes, dtype=np.int64)
        self.needs = np.asarray(needs, dtype=np.int64)
        if self.sizes.shape != self.needs.shape or self.sizes.ndim != 2:
            raise ValueError("JobGather: sizes and needs must both be [world, nb]")
        self.world, self.nb = self.sizes.shape
        self.group, self.rank, self.pg = int(group), int(rank), pg
        self.ngroups = -(-self.nb // self.group)
        self.elt = torch.empty(0, dtype=dtype).element_size()
        self.cnt = np.zeros((self.world, self.ngroups), np.int64)  # counts of rank r in group g
        self.loc = np.zeros((self.world, self.ngroups), np.int64)  # locations of rank r in group g
        for g in range(self.ngroups):
            sl = slice(g * self.group, min(self.nb, (g + 1) * self.group))
            self.cnt[:, g] = self.sizes[:, sl].sum(axis=1)
            self.loc[:, g] = self.needs[:, sl].sum(axis=1)
        self.slab = [max(1, int((self.cnt[:, g] + self.loc[:, g]).max())) for g in range(self.ngroups)]
        self.inp = [torch.zeros(s, dtype=dtype, device=device) for s in self.slab]
        self.collective = self.world > 1 if collective is None else bool(collective)
        # no collective (one rank): the slab is its own result
        self.out = [torch.zeros(self.world * s, dtype=dtype, device=device)
                    for s in self.slab] if self.collective else self.inp
        self.outc = [None] * self.ngroups  # the `counts` gathers' slabs (made on first use)

    def _where(self, j: int):
        g = j // self.group
        return g, g * self.group

    def counts_slot(self, j: int):
        g, j0 = self._where(j)
        o = int(self.sizes[self.rank, j0:j].sum())
        return self.inp[g][o:o + int(self.sizes[self.rank, j])]

    def locs_slot(self, j: int):
        g, j0 = self._where(j)
        o = int(self.cnt[self.rank, g] + self.needs[self.rank, j0:j].sum())
        return self.inp[g][o:o + int(self.needs[self.rank, j])]

    def counts_max(self, g: int) -> int:
        """Group g's count part on the largest rank (the `counts` gather's slab)."""
        return max(1, int(self.cnt[:, g].max()))

    def gather(self, g: int, async_op: bool = False, part: str = "all"):
        """Group g's all-gather (enqueue it on a communication stream to
        overlap it with the next launch); None with one rank.  part "all":
        the whole slab (counts and locations); "counts": the counts alone
        (every rank's first counts_max(g) words, into a slab of their own —
        the job's offsets on every rank; the locations stay where they were
        computed until a later "all" gather)."""
        if not self.collective:
            return None
        if part == "counts":
            import torch
            c = self.counts_max(g)
            if self.outc[g] is None:
                self.outc[g] = torch.zeros(self.world * c, dtype=self.inp[g].dtype, device=self.inp[g].device)
            return _all_gather_flat(self.outc[g], self.inp[g][:c], self.pg, async_op)
        if part != "all":
            raise ValueError(f"JobGather.gather: part {part!r} (all | counts)")
        return _all_gather_flat(self.out[g], self.inp[g], self.pg, async_op)

    def gather_all(self):
        for g in range(self.ngroups):
            self.gather(g)

    def assemble_offsets(self):
        """The job's offsets int64[total+1] from the `counts` gathers alone."""
        import torch
        cnts = []
        for r in range(self.world):
            for g in range(self.ngroups):
                src = self.outc[g] if self.collective else self.inp[g]
                b = r * self.counts_max(g) if self.collective else 0
                cnts.append(src[b:b + int(self.cnt[r, g])])
        counts = torch.cat(cnts).to(torch.int64)
        offsets = torch.zeros(counts.numel() + 1, dtype=torch.int64, device=counts.device)
        torch.cumsum(counts, 0, out=offsets[1:])
        return offsets

    def assemble(self):
        """The job's (offsets int64[total+1], locations) on the device, ranks
        in order, then groups, then batches (= global pattern order for a
        JobPlan)."""
        import torch
        cnts, locs = [], []
        for r in range(self.world):
            for g in range(self.ngroups):
                b = r * self.slab[g]
                c, l = int(self.cnt[r, g]), int(self.loc[r, g])
                cnts.append(self.out[g][b:b + c])
                locs.append(self.out[g][b + c:b + c + l])
        counts = torch.cat(cnts).to(torch.int64)
        offsets = torch.zeros(counts.numel() + 1, dtype=torch.int64, device=counts.device)
        torch.cumsum(counts, 0, out=offsets[1:])
        return offsets, torch.cat(locs)

    def bytes_per_pass(self, part: str = "all") -> int:
        """Bytes every rank receives per pass over the job (all groups), by
        gather part ("all": whole slabs; "counts": the count slabs alone)."""
        if part == "counts":
            return sum(self.world * self.counts_max(g) for g in range(self.ngroups)) * self.elt
        return sum(self.world * s for s in self.slab) * self.elt

    def result_bytes(self) -> int:
        """The job's own result bytes: every count and every location once."""
        return int((self.cnt + self.loc).sum()) * self.elt


class ShardedLocate:
    """`FmIndex.locate_batch` for one global batch over every rank of a
    process group — the north star's "pattern batches shard across the GPUs,
    blob replicated, one all-gather concatenates the results" as a call.

    Every rank passes the same batch (device bytes + int64 offsets[n+1]);
    rank r locates the contiguous shard `shard(n, world, r)` on its own GPU
    against its own replica of the index, writing its counts and locations
    into one packed slab [counts | locations]; after a 16-byte size exchange
    one all_gather_into_tensor moves every rank's slab, and the batch's flat
    (offsets int64[n+1], locations) is assembled on the device — identical on
    every rank and equal to one device's answer for the whole batch.

    `locate_fn(d_bytes, d_offsets, m, counts_out, locs_out, cap) -> needed`
    runs the shard (FmIndex by default: fmx_locate_batch_async on `stream`,
    else on the caller's current stream — the stream the shard's inputs and
    output buffers were made on, so the launch is ordered after them; a
    given stream, or the stream of its own that stands in for torch's null
    default stream (null means the index's own stream to the ABI), first
    waits for the current one); if the shard has more
    occurrences than the first guess of room, it runs again with exactly
    enough.  Host round trips per call: the shard's byte range, its location
    total and the size exchange."""

    def __init__(self, ix=None, dtype=None, device=None, group=None, locate_fn=None, stream=None):
        import torch
        import torch.distributed as dist
        self.dist_on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.dist_on else 1
        self.rank = dist.get_rank(group) if self.dist_on else 0
        self.group, self.device, self.stream = group, device, stream
        self.ix = ix
        self.dtype = dtype or (torch.int32 if ix is None or ix.position.nbytes == 4 else torch.int64)
        self.locate_fn = locate_fn or self._index_locate
        self._ws = None
        self._own = None
        self.last = {}

    def _index_locate(self, d_bytes, d_offsets, m, counts, locs, cap):
        import torch
        ws = self.ix.locate_workspace_size(max(m, 1))
        if self._ws is None or self._ws.numel() < ws:
            self._ws = torch.zeros(ws, dtype=torch.uint8, device=d_offsets.device)
        loff = torch.zeros(m + 1, dtype=torch.int64, device=d_offsets.device)
        need = torch.zeros(1, dtype=torch.int64, device=d_offsets.device)
        cur = torch.cuda.current_stream(d_offsets.device)
        run_on = self.stream
        if run_on is None and cur.cuda_stream == 0:
            # torch's default stream is the null stream, and a null stream
            # means the index's own (unordered) stream to the ABI: run on a
            # stream of ours that waits for it instead
            if self._own is None:
                self._own = torch.cuda.Stream(device=d_offsets.device)
            run_on = self._own
        if run_on is not None:  # ordered after everything the current stream made
            run_on.wait_stream(cur)
        st = (run_on or cur).cuda_stream
        self.ix.locate_batch_async(d_bytes.data_ptr() if d_bytes.numel() else 0, d_offsets.data_ptr(), m,
                                   loff.data_ptr(), locs.data_ptr() if cap else 0, cap, need.data_ptr(),
                                   self._ws.data_ptr(), self._ws.numel(), d_counts=counts.data_ptr() if m else 0,
                                   stream=st)
        self.ix.sync(st)
        return int(need.item())

    def locate(self, d_bytes, d_offsets):
        import torch
        n = int(d_offsets.numel()) - 1
        s, e = shard(n, self.world, self.rank)
        m = e - s
        dev = d_offsets.device
        b = d_offsets[[s, e]].cpu().tolist() if n >= 0 else [0, 0]
        sub_off = (d_offsets[s:e + 1] - b[0]).contiguous()
        sub_bytes = d_bytes[b[0]:b[1]]
        cap = m + m // 8 + 4096
        slab = torch.zeros(m + cap, dtype=self.dtype, device=dev)
        need = self.locate_fn(sub_bytes, sub_off, m, slab[:m], slab[m:], cap)
        if need > cap:  # more occurrences than guessed: run again with room for all of them
            slab = torch.zeros(m + need, dtype=self.dtype, device=dev)
            got = self.locate_fn(sub_bytes, sub_off, m, slab[:m], slab[m:], need)
            if got != need:
                raise RuntimeError(f"ShardedLocate: location total changed between runs ({need} -> {got})")
        parts = all_gather_ints([m, need], device=dev, pg=self.group)  # [world, 2]
        S = max(1, int((parts[:, 0] + parts[:, 1]).max()))
        if slab.numel() < S:
            slab = torch.cat([slab, torch.zeros(S - slab.numel(), dtype=self.dtype, device=dev)])
        inp = slab[:S].contiguous()
        if self.world == 1:
            out = inp
        else:
            out = torch.zeros(self.world * S, dtype=self.dtype, device=dev)
            _all_gather_flat(out, inp, self.group, False)
        cnts = [out[r * S:r * S + int(parts[r, 0])] for r in range(self.world)]
        locs = [out[r * S + int(parts[r, 0]):r * S + int(parts[r, 0] + parts[r, 1])] for r in range(self.world)]
        counts = torch.cat(cnts).to(torch.int64)
        offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        torch.cumsum(counts, 0, out=offsets[1:])
        self.last = {"patterns": n, "shard": (s, e), "bytes_gathered": self.world * S * inp.element_size(),
                     "result_bytes": int((parts[:, 0] + parts[:, 1]).sum()) * inp.element_size()}
        return offsets, torch.cat(locs)


def workspace_bytes(n: int, pos_bytes: int) -> int:
    """fmx_locate_workspace_size for n patterns, from the library itself
    (fmx_workspace_bytes, ABI 8: the same arithmetic as the index's, no
    index needed) — so the per-rank accounting follows any build's key
    counters, batch table (FMX_MAX_MEGA) and record sizes."""
    import ctypes as C
    from . import _native as _n
    out = C.c_uint64()
    st = _n.lib().fmx_workspace_bytes(int(n), int(pos_bytes), C.byref(out))
    if st != 0:
        raise ValueError(f"fmx_workspace_bytes({n}, {pos_bytes}): status {st}")
    return int(out.value)


def hbm_per_rank(*, blob: int, records: int, text: int, batch_sizes: Sequence[int], m: int, pos_bytes: int,
                 world: int, group: int, loc_cap: Sequence[int], gather: bool) -> dict:
    """HBM one rank of bench.py holds (bytes), by part: the replicated blob and
    its interleaved occ records; the synthetic text the patterns are cut from;
    per batch its patterns (m B each), offsets and output offsets (8 B per
    pattern + 8), counts (P), locations (loc_cap[j] x P) and workspace; with
    gathers (several ranks, or the RCCL path at one rank) the JobGather slabs —
    per launch group this rank's part (its counts + locations) and the
    gathered output, world x the largest rank's part (taken as this rank's:
    random patterns make the parts near-equal)."""
    P = int(pos_bytes)
    sizes = [int(b) for b in batch_sizes]
    caps = [int(c) for c in loc_cap]
    batches = sum(b * m + 2 * 8 * (b + 1) + 8 + b * P + c * P + workspace_bytes(b, P) for b, c in zip(sizes, caps))
    slabs = 0
    if gather:
        for g in range(0, len(sizes), group):
            part = (sum(sizes[g:g + group]) + sum(caps[g:g + group])) * P
            slabs += part + world * part
    parts = {"blob": int(blob), "occ_records": int(records), "text": int(text), "batches": batches,
             "gather_slabs": slabs}
    parts["total"] = sum(parts.values())
    return parts


def all_gather_ints(values: Sequence[int], device=None, pg=None) -> np.ndarray:
    """Every rank's int vector (same length on every rank) -> int64[world, len]."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.int64, device=device)
    if not (dist.is_available() and dist.is_initialized()):
        return t.cpu().numpy()[None, :]
    out = torch.zeros(dist.get_world_size(pg) * t.numel(), dtype=torch.int64, device=device)
    _all_gather_flat(out, t, pg, False)
    return out.view(-1, t.numel()).cpu().numpy()


def replicate_blob(d_blob, src: int = 0, group=None) -> dict:
    """Broadcast rank src's blob (a uint8 tensor of the same size on every
    rank) to every rank — SURVEY §8(e)'s replicated blob, over RCCL/xGMI —
    then compare a checksum of every rank's copy.  Returns the broadcast's
    seconds (barrier to barrier) and whether all copies are identical."""
    import time

    import torch
    import torch.distributed as dist
    def sync():
        if d_blob.is_cuda:
            torch.cuda.synchronize()

    dist.barrier(group=group)
    sync()
    t0 = time.perf_counter()
    dist.broadcast(d_blob, src=src, group=group)
    sync()
    dist.barrier(group=group)
    sec = time.perf_counter() - t0
    n8 = d_blob.numel() // 8 * 8
    words = d_blob[:n8].view(torch.int64)
    # two position-weighted sums (wrapping int64): equal on every rank iff
    # the copies agree (up to a checksum collision)
    w = torch.arange(1, words.numel() + 1, dtype=torch.int64, device=d_blob.device)
    ck = torch.stack([words.sum(), (words * w).sum(), d_blob[n8:].to(torch.int64).sum()])
    lo, hi = ck.clone(), ck.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    return {"how": f"built on rank {src}, broadcast to every rank", "seconds": sec,
            "bytes": int(d_blob.numel()), "identical": bool(torch.equal(lo, hi))}


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
