"""The shipped launch shapes at their full width, against the oracle.

  * ONE grouped launch of 1,024 batches: the headline's
    shape — four kernel-argument groups of 256, the launch's batch table
    (GroupTab) full at kMaxMega entries and staged in LDS by the kernels that
    see the whole launch — at the shipped defaults (no FMX_GROUPED forcing,
    no refine pass, no device-side check): ~3.3 M fixed-length patterns, so the
    engine's own threshold groups it.  Every batch's counts, offsets, total
    and locations against the oracle (with_slice.rs:21-33, locate/mod.rs:14-37).
  * Fused launches (k_locate) on two streams at once, each launch over more
    tiles than the chip holds resident (a workgroup must only wait
    on tiles that are already running — the per-batch tickets): every result
    against the oracle, every launch fused.
The path each launch took is asserted through fmx_index_info's counters."""
import numpy as np
import pytest

from _util import table_from_symbols
from test_gpu import gpu_build

pytestmark = pytest.mark.gpu

ACGTN = [b"A", b"C", b"G", b"T", b"N"]


def dna_case(pkg, n_text, seed):
    rng = np.random.default_rng(seed)
    table = table_from_symbols(ACGTN)
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=n_text).astype(np.uint8)
    blob = gpu_build(pkg, text.tobytes(), 5, 4, 3, 64, 3, 2, table)
    return rng, text, blob


class Batches:
    """Many batches in a few large device tensors (one H2D / D2H each): batch j
    = patterns of fixed length m_j, its bytes 16-B aligned in `data`, its own
    offsets, outputs, counts and a workspace full of random bytes."""

    def __init__(self, torch, ix, rng, text, sizes, lengths, reversed_every=3):
        dev = torch.device("cuda:0")
        win = {m: np.lib.stride_tricks.sliding_window_view(text, m) for m in set(lengths)}
        self.fwd, self.rev, self.n, self.m = [], [], list(sizes), list(lengths)
        chunks, offs, doff, ooff = [], [], [], []
        pos = 0
        for j, (n, m) in enumerate(zip(sizes, lengths)):
            starts = rng.integers(0, text.size - m + 1, size=n)
            pats = win[m][starts]                        # (n, m) forward patterns
            rev = reversed_every and j % reversed_every == reversed_every - 1
            self.fwd.append(pats)
            self.rev.append(bool(rev))
            b = (pats[:, ::-1] if rev else pats).reshape(-1)
            pad = (-b.size) % 16 + 16
            chunks.append(np.concatenate([b, np.zeros(pad, np.uint8)]))
            doff.append(pos)
            pos += b.size + pad
            offs.append(np.arange(n + 1, dtype=np.int64) * m)
        self.d_data = torch.from_numpy(np.concatenate(chunks)).to(dev)
        self.off_at = np.concatenate([[0], np.cumsum([n + 1 for n in sizes])])
        self.d_off = torch.from_numpy(np.concatenate(offs)).to(dev)
        self.loff = torch.randint(0, 2**62, (int(self.off_at[-1]),), dtype=torch.int64, device=dev)
        self.cnt_at = np.concatenate([[0], np.cumsum(sizes)])
        self.cnt = torch.randint(0, 2**31 - 1, (int(self.cnt_at[-1]),), dtype=torch.int32, device=dev)
        self.need = torch.zeros(len(sizes), dtype=torch.int64, device=dev)
        self.doff = doff
        self.ws_bytes = [ix.locate_workspace_size(n) for n in sizes]
        self.ws_at = np.concatenate([[0], np.cumsum([(w + 255) // 256 * 256 for w in self.ws_bytes])])
        self.ws = torch.randint(0, 256, (int(self.ws_at[-1]),), dtype=torch.uint8, device=dev)
        self.ix, self.torch = ix, torch

    def oracle(self, orc, threads=8):
        """The oracle's (offsets, locations) of every batch (one oracle call)."""
        allp = np.concatenate([p.reshape(-1) for p in self.fwd])
        lens = np.concatenate([np.full(n, m, np.uint64) for n, m in zip(self.n, self.m)])
        offs = np.zeros(lens.size + 1, dtype=np.uint64)
        offs[1:] = np.cumsum(lens)
        ooff, olocs = orc.locate_batch(allp, offs, threads=threads)
        self.want = []
        for j in range(len(self.n)):
            a, b = int(self.cnt_at[j]), int(self.cnt_at[j + 1])
            o = ooff[a:b + 1]
            self.want.append((o - o[0], olocs[int(o[0]):int(o[-1])]))
        self.cap = [int(w[1].size) + 8 for w in self.want]
        self.locs_at = np.concatenate([[0], np.cumsum(self.cap)])
        self.locs = self.torch.randint(0, 2**31 - 1, (int(self.locs_at[-1]),), dtype=self.torch.int32,
                                       device=self.d_data.device)

    def queue(self, stream=0):
        ix, jobs = self.ix, []
        ptr = lambda t, i, es: t.data_ptr() + int(i) * es  # noqa: E731
        for j, (n, m) in enumerate(zip(self.n, self.m)):
            jobs.append(ix.locate_job(self.d_data.data_ptr() + self.doff[j], ptr(self.d_off, self.off_at[j], 8), n,
                                      ptr(self.loff, self.off_at[j], 8), ptr(self.locs, self.locs_at[j], 4),
                                      self.cap[j], ptr(self.need, j, 8), ptr(self.ws, self.ws_at[j], 1),
                                      self.ws_bytes[j], d_counts=ptr(self.cnt, self.cnt_at[j], 4), stream=stream,
                                      reversed=self.rev[j], stage_kb=max(1, -(-256 * m // 1024)), fixed_len=m))
        return ix.job_queue(jobs)

    def check(self, what):
        loff = self.loff.cpu().numpy().view(np.uint64)
        locs = self.locs.cpu().numpy().view(np.uint32)
        cnt = self.cnt.cpu().numpy().view(np.uint32)
        need = self.need.cpu().numpy()
        for j, (wo, wl) in enumerate(self.want):
            go = loff[self.off_at[j]:self.off_at[j + 1]]
            assert np.array_equal(go, wo), f"{what}: batch {j} (m={self.m[j]}, rev={self.rev[j]}): offsets"
            assert int(need[j]) == wl.size, f"{what}: batch {j}: total"
            gl = locs[self.locs_at[j]:self.locs_at[j] + wl.size]
            assert np.array_equal(gl, wl), f"{what}: batch {j} (m={self.m[j]}, rev={self.rev[j]}): locations"
            assert np.array_equal(cnt[self.cnt_at[j]:self.cnt_at[j + 1]], np.diff(wo).astype(np.uint32)), \
                f"{what}: batch {j}: counts"


def test_grouped_launch_1024_batches(pkg, O):
    """One fmx_locate_group_async call of 1,024 batches (3,100-3,300 patterns
    of 12-32 bp each, every third reversed; 3.28 M patterns) on a 4 Mbp ACGT
    index (u32/Block3<u64>, sr 2, k 3) at the shipped defaults: the launch is
    grouped by the engine's own threshold (3 x 2^20 patterns), as ONE launch over
    four kernel-argument groups; two rounds on the same random-byte
    workspaces, every batch against the oracle."""
    import torch
    rng, text, blob = dna_case(pkg, 4_000_000, 61)
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=1)
    info = ix.info()
    assert info["group_key_len"] > 0 and info["grouped_min"] == 3 << 20, info
    sizes = [int(x) for x in rng.integers(3100, 3301, size=1024)]
    lengths = [12 + (j * 7) % 21 for j in range(1024)]
    assert sum(sizes) >= info["grouped_min"]
    bt = Batches(torch, ix, rng, text, sizes, lengths)
    # the index's workspace size = the host-only fmx_workspace_bytes (per-rank HBM accounting)
    assert bt.ws_bytes == [pkg.distributed.workspace_bytes(n, 4) for n in sizes]
    bt.oracle(orc)
    q = bt.queue()
    torch.cuda.synchronize()
    for rep in range(2):
        before = ix.info()
        ix.locate_group_async(q)
        ix.sync()
        after = ix.info()
        assert after["launches_grouped"] - before["launches_grouped"] == 1, (before, after)
        assert after["launches_ordered"] == before["launches_ordered"], (before, after)
        assert after["launches_grouped_raw"] == before["launches_grouped_raw"]
        bt.check(f"round {rep}")
    ix.close()


def test_fused_two_streams_over_residency(pkg, O, monkeypatch):
    """Two streams, each running fused group launches (k_locate, launch order:
    FMX_GROUPED=0) of 4 x 200,000 x 20 bp = 3,128 tiles — more workgroups
    than the chip keeps resident (256 CUs x 8) — at the same time, three
    rounds: every batch against the oracle; every launch fused."""
    import torch
    rng, text, blob = dna_case(pkg, 2_000_000, 62)
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    monkeypatch.setenv("FMX_GROUPED", "0")
    monkeypatch.setenv("FMX_FUSED", "1")
    ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=1)
    sides = []
    for s in range(2):
        bt = Batches(torch, ix, rng, text, [200_000] * 4, [20] * 4, reversed_every=2)
        bt.oracle(orc)
        stream = torch.cuda.Stream()
        sides.append((bt, stream, bt.queue(stream.cuda_stream)))
    torch.cuda.synchronize()
    before = ix.info()["launches_fused"]
    for rep in range(3):
        for bt, stream, q in sides:
            bt.loff.fill_(-1)
            bt.locs.fill_(-1)
        torch.cuda.synchronize()
        for bt, stream, q in sides:
            ix.locate_group_async(q, stream=stream.cuda_stream)
        for bt, stream, q in sides:
            ix.sync(stream.cuda_stream)
        for s, (bt, stream, q) in enumerate(sides):
            bt.check(f"round {rep} stream {s}")
    assert ix.info()["launches_fused"] - before == 6
    for bt, stream, q in sides:
        ix.release_stream(stream.cuda_stream)
    ix.close()
