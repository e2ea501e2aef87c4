"""The fused launch (k_locate: search, tile counts handed from workgroup to
workgroup inside the launch, offsets and locations — one kernel instead of
k_search + k_emit) on the GPU.  Launches in launch order of fixed-length
batches of at most kFoldTiles tiles take it by default (FMX_FUSED=0: never).

  * every layout: fused and two-kernel answers equal, and equal to the oracle;
  * C2's single batch (100k x 20 bp) on a 16 Mbp index, 40 launches on one
    workspace through the device API: every launch's outputs against the
    oracle (a tag left by an earlier launch never passes for a later one's);
  * under uneven load (cdna_hip_programming.md Guideline 16, Pitfall 3): the
    fused launches run on one stream while another stream runs a heavy
    two-kernel launch on the same GPU — every fused result against the oracle;
  * group launches of 1-8-tile batches on workspaces full of random bytes;
  * grouped launches ended by k_emit_chain (the same hand-off after the
    grouped search) and by k_group_tiles + k_emit.
The path each launch took is asserted through fmx_index_info's counters."""
import numpy as np
import pytest

from _util import ALL_LAYOUTS, rand_chr_list, rand_pattern, rand_text, table_from_symbols
from test_gpu import block_of, gpu_build, pos_of

pytestmark = pytest.mark.gpu


def load(pkg, blob, pb, planes, vb, occ, fused, monkeypatch):
    monkeypatch.setenv("FMX_FUSED", "1" if fused else "0")
    ix = pkg.FmIndex.load(blob, pos_of(pkg, pb), block_of(pkg, planes, vb), options=occ)
    monkeypatch.delenv("FMX_FUSED")
    return ix


@pytest.mark.parametrize("pb,planes,vb", ALL_LAYOUTS)
def test_fused_every_layout(pkg, O, pb, planes, vb, monkeypatch):
    rng = np.random.default_rng(pb * 131 + planes * 17 + vb)
    sigma = min(1 << planes, 20) - 1
    chars = rand_chr_list(rng, sigma)
    table = table_from_symbols([bytes([c]) for c in chars])
    text = rand_text(rng, chars, 60_000, 60_000)
    blob = O.build(text, sigma + 1, O.layout(pb, planes, vb), 3, 2, table)
    orc = O.OracleIndex(blob, O.layout(pb, planes, vb, 0))
    for occ in (0, 1):
        ixf = load(pkg, blob, pb, planes, vb, occ, True, monkeypatch)
        ixs = load(pkg, blob, pb, planes, vb, occ, False, monkeypatch)
        for m in (2, 5, 21):
            pats = [rand_pattern(rng, text, m, m) for _ in range(300 if m == 2 else 3000)]
            pats = [p for p in pats if len(p) == m]
            pats += [bytes(rng.choice(np.frombuffer(chars, np.uint8), size=m)) for _ in range(200)]
            data, offsets = pkg.pack_patterns(pats)
            ooff, olocs = orc.locate_batch(data, offsets)
            for ix, name in ((ixf, "fused"), (ixs, "split")):
                goff, glocs = ix.locate_batch((data, offsets))
                assert np.array_equal(goff, ooff), f"{name} m={m} occ={occ}: offsets"
                assert np.array_equal(glocs, olocs), f"{name} m={m} occ={occ}: locations"
                roff, rlocs = ix.locate_batch([p[::-1] for p in pats], reversed=True)
                assert np.array_equal(roff, ooff) and np.array_equal(rlocs, olocs), f"{name} m={m}: reversed"
        fi, si = ixf.info(), ixs.info()
        assert fi["launches_fused"] == fi["launches_ordered"] >= 6, fi
        assert si["launches_fused"] == 0 and si["launches_ordered"] >= 6, si
        ixf.close()
        ixs.close()


def c2_like(pkg, O, n_text, seed):
    rng = np.random.default_rng(seed)
    table = table_from_symbols([b"A", b"C", b"G", b"T"])
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=n_text).astype(np.uint8)
    blob = gpu_build(pkg, text.tobytes(), 4, 4, 3, 64, 3, 2, table)
    return rng, text, blob


def test_fused_c2_single_batch_repeated(pkg, O, monkeypatch):
    """C2's single batch shape (100k x 20 bp, u32/Block3<u64>, SA sampling 2,
    k-mer 3) on a 16 Mbp text: 40 fused launches on one workspace and one set
    of outputs (filled with -1 before each), every launch's offsets, total and
    locations against the oracle."""
    import torch
    rng, text, blob = c2_like(pkg, O, 16_000_000, 51)
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    ix = load(pkg, blob, 4, 3, 64, 1, True, monkeypatch)
    dev = torch.device("cuda:0")
    starts = rng.integers(0, text.size - 20, size=100_000)
    pats = [text[s:s + 20].tobytes() for s in starts]
    data, offsets = pkg.pack_patterns(pats)
    ooff, olocs = orc.locate_batch(data, offsets)
    n, cap = len(pats), int(olocs.size) + 64
    d_data = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(offsets.view(np.int64).copy()).to(dev)
    loff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    locs = torch.empty(cap, dtype=torch.int32, device=dev)
    need = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = ix.locate_workspace_size(n)
    d_ws = torch.randint(0, 256, (ws,), dtype=torch.uint8, device=dev)
    before = ix.info()["launches_fused"]
    for rep in range(40):
        loff.fill_(-1)
        locs.fill_(-1)
        torch.cuda.synchronize()
        ix.locate_batch_async(d_data.data_ptr(), d_off.data_ptr(), n, loff.data_ptr(), locs.data_ptr(), cap,
                              need.data_ptr(), d_ws.data_ptr(), ws, stage_kb=5, fixed_len=20)
        ix.sync()
        assert np.array_equal(loff.cpu().numpy().view(np.uint64), ooff), f"launch {rep}: offsets"
        assert int(need.item()) == olocs.size, f"launch {rep}: total"
        assert np.array_equal(locs.cpu().numpy()[:olocs.size].view(np.uint32), olocs), f"launch {rep}: locations"
    assert ix.info()["launches_fused"] - before == 40
    ix.close()


def test_fused_under_uneven_load(pkg, O, monkeypatch):
    """Fused launches (single 100k batches, one stream) while a second stream
    runs two-kernel launches of 2M patterns on the same GPU (another index
    object on the same blob): the hand-off's producers and consumers are
    busy unevenly and their L1s hold lines of earlier launches (each fused
    launch reuses one workspace).  Every fused result against the oracle."""
    import torch
    rng, text, blob = c2_like(pkg, O, 16_000_000, 52)
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    ixf = load(pkg, blob, 4, 3, 64, 1, True, monkeypatch)
    ixs = load(pkg, blob, 4, 3, 64, 1, False, monkeypatch)
    dev = torch.device("cuda:0")
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    # the fused side: 4 batches of 100k x 20, outputs per launch
    fb = []
    for j in range(4):
        starts = rng.integers(0, text.size - 20, size=100_000)
        pats = [text[s:s + 20].tobytes() for s in starts]
        data, offsets = pkg.pack_patterns(pats)
        ooff, olocs = orc.locate_batch(data, offsets)
        fb.append(dict(want=(ooff, olocs), n=len(pats), cap=int(olocs.size) + 64,
                       data=torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).to(dev),
                       off=torch.from_numpy(offsets.view(np.int64).copy()).to(dev)))
    ws = ixf.locate_workspace_size(100_000)
    d_ws = torch.randint(0, 256, (ws,), dtype=torch.uint8, device=dev)
    # the heavy side: 2M x 20 bp in launch order on the two-kernel path (k_search, k_scan, k_emit)
    hs = rng.integers(0, text.size - 20, size=2_000_000)
    hbytes = np.lib.stride_tricks.sliding_window_view(text, 20)[hs].reshape(-1).copy()
    hoff = (np.arange(2_000_001, dtype=np.int64) * 20)
    d_hb = torch.from_numpy(np.concatenate([hbytes, np.zeros(16, np.uint8)])).to(dev)
    d_ho = torch.from_numpy(hoff).to(dev)
    hws = ixs.locate_workspace_size(2_000_000)
    d_hws = torch.zeros(hws, dtype=torch.uint8, device=dev)
    h_loff = torch.zeros(2_000_001, dtype=torch.int64, device=dev)
    h_cap = 2_200_000
    h_locs = torch.zeros(h_cap, dtype=torch.int32, device=dev)
    h_need = torch.zeros(1, dtype=torch.int64, device=dev)
    outs = []
    torch.cuda.synchronize()
    for rep in range(6):
        ixs.locate_batch_async(d_hb.data_ptr(), d_ho.data_ptr(), 2_000_000, h_loff.data_ptr(), h_locs.data_ptr(),
                               h_cap, h_need.data_ptr(), d_hws.data_ptr(), hws, stream=sb.cuda_stream)
        for j, b in enumerate(fb):
            loff = torch.full((b["n"] + 1,), -1, dtype=torch.int64, device=dev)
            locs = torch.full((b["cap"],), -1, dtype=torch.int32, device=dev)
            need = torch.zeros(1, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()  # (the fills ran on torch's stream)
            ixf.locate_batch_async(b["data"].data_ptr(), b["off"].data_ptr(), b["n"], loff.data_ptr(),
                                   locs.data_ptr(), b["cap"], need.data_ptr(), d_ws.data_ptr(), ws,
                                   stream=sa.cuda_stream, stage_kb=5, fixed_len=20)
            ixf.sync(sa.cuda_stream)
            outs.append((j, loff.cpu().numpy(), locs.cpu().numpy(), int(need.item())))
        ixs.sync(sb.cuda_stream)
    for k, (j, loff, locs, need) in enumerate(outs):
        ooff, olocs = fb[j]["want"]
        assert np.array_equal(loff.view(np.uint64), ooff), f"fused launch {k} (batch {j}): offsets"
        assert need == olocs.size and np.array_equal(locs[:olocs.size].view(np.uint32), olocs), \
            f"fused launch {k} (batch {j}): locations"
    assert ixf.info()["launches_fused"] == 24
    assert ixs.info()["launches_fused"] == 0
    ixf.release_stream(sa.cuda_stream)
    ixs.release_stream(sb.cuda_stream)
    ixf.close()
    ixs.close()


def test_fused_group_launches(pkg, O, monkeypatch):
    """Group launches in launch order (fmx_locate_group_async) of 300
    fixed-length batches of 1-2,000 patterns (two launches: 256 + 44),
    lengths 1..40, every third reversed, workspaces and outputs full of random
    bytes, three rounds on the same workspaces: every batch's counts, offsets,
    total and locations against the oracle; both launches fused."""
    import torch
    rng, text, blob = c2_like(pkg, O, 2_000_000, 53)
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    ix = load(pkg, blob, 4, 3, 64, 1, True, monkeypatch)
    monkeypatch.setenv("FMX_GROUPED", "0")
    dev = torch.device("cuda:0")
    sizes = [int(x) for x in np.random.default_rng(9).integers(1, 2000, size=300)]
    bats, jobs = [], []
    for bi, n in enumerate(sizes):
        rev, m = bi % 3 == 2, 1 + (bi * 7) % 40
        starts = rng.integers(0, text.size - m, size=n)
        pats = [text[s:s + m].tobytes() for s in starts]
        data, offsets = pkg.pack_patterns(pats)
        want = orc.locate_batch(data, offsets)
        q = [p[::-1] for p in pats] if rev else pats
        data, offsets = pkg.pack_patterns(q)
        cap = int(want[1].size) + 8
        ws = ix.locate_workspace_size(n)
        b = dict(want=want, data=torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).to(dev),
                 off=torch.from_numpy(offsets.view(np.int64).copy()).to(dev),
                 loff=torch.randint(0, 2**62, (n + 1,), dtype=torch.int64, device=dev),
                 locs=torch.randint(0, 2**31 - 1, (cap,), dtype=torch.int32, device=dev),
                 need=torch.zeros(1, dtype=torch.int64, device=dev),
                 cnt=torch.randint(0, 2**31 - 1, (n,), dtype=torch.int32, device=dev),
                 ws=torch.randint(0, 256, (ws,), dtype=torch.uint8, device=dev))
        jobs.append(ix.locate_job(b["data"].data_ptr(), b["off"].data_ptr(), n, b["loff"].data_ptr(),
                                  b["locs"].data_ptr(), cap, b["need"].data_ptr(), b["ws"].data_ptr(), ws,
                                  d_counts=b["cnt"].data_ptr(), reversed=rev, stage_kb=max(1, -(-256 * m // 1024)),
                                  fixed_len=m))
        bats.append(b)
    q = ix.job_queue(jobs)
    torch.cuda.synchronize()
    before = ix.info()["launches_fused"]
    for rep in range(3):
        ix.locate_group_async(q)
        ix.sync()
        for bi, b in enumerate(bats):
            wo, wl = b["want"]
            assert np.array_equal(b["loff"].cpu().numpy().view(np.uint64), wo), f"rep {rep} batch {bi}: offsets"
            assert int(b["need"].item()) == wl.size, f"rep {rep} batch {bi}: total"
            assert np.array_equal(b["locs"].cpu().numpy()[:wl.size].view(np.uint32), wl), \
                f"rep {rep} batch {bi}: locations"
            assert np.array_equal(b["cnt"].cpu().numpy().view(np.uint32), np.diff(wo).astype(np.uint32))
    assert ix.info()["launches_fused"] - before == 6
    ix.close()


@pytest.mark.parametrize("chain", ["1", "0"])
def test_chained_grouped_launches(pkg, O, monkeypatch, chain):
    """Grouped group launches (FMX_GROUPED=1) ended by k_emit_chain (tile
    counts handed from tile to tile inside the kernel; FMX_EMIT_CHAIN=0: the
    k_group_tiles + k_emit pair): 300 fixed-length batches of 1-3,000
    patterns, lengths 8..28, every third reversed, random-byte workspaces and
    outputs, three rounds (each one grouped launch over two kernel-argument
    groups): every batch against the oracle, and the launch counters show
    which ending ran."""
    import torch
    rng, text, blob = c2_like(pkg, O, 4_000_000, 54)
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    monkeypatch.setenv("FMX_GROUPED", "1")
    monkeypatch.setenv("FMX_EMIT_CHAIN", chain)
    ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=1)
    dev = torch.device("cuda:0")
    sizes = [int(x) for x in np.random.default_rng(10).integers(1, 3000, size=300)]
    bats, jobs = [], []
    for bi, n in enumerate(sizes):
        rev, m = bi % 3 == 2, 8 + (bi * 5) % 21  # (from 8: a 4 Mbp text gives a 1-mer ~10^6 locations)
        starts = rng.integers(0, text.size - m, size=n)
        pats = [text[s:s + m].tobytes() for s in starts]
        data, offsets = pkg.pack_patterns(pats)
        want = orc.locate_batch(data, offsets)
        q = [p[::-1] for p in pats] if rev else pats
        data, offsets = pkg.pack_patterns(q)
        cap = int(want[1].size) + 8
        ws = ix.locate_workspace_size(n)
        b = dict(want=want, data=torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).to(dev),
                 off=torch.from_numpy(offsets.view(np.int64).copy()).to(dev),
                 loff=torch.randint(0, 2**62, (n + 1,), dtype=torch.int64, device=dev),
                 locs=torch.randint(0, 2**31 - 1, (cap,), dtype=torch.int32, device=dev),
                 need=torch.zeros(1, dtype=torch.int64, device=dev),
                 cnt=torch.randint(0, 2**31 - 1, (n,), dtype=torch.int32, device=dev),
                 ws=torch.randint(0, 256, (ws,), dtype=torch.uint8, device=dev))
        jobs.append(ix.locate_job(b["data"].data_ptr(), b["off"].data_ptr(), n, b["loff"].data_ptr(),
                                  b["locs"].data_ptr(), cap, b["need"].data_ptr(), b["ws"].data_ptr(), ws,
                                  d_counts=b["cnt"].data_ptr(), reversed=rev, stage_kb=max(1, -(-256 * m // 1024)),
                                  fixed_len=m))
        bats.append(b)
    q = ix.job_queue(jobs)
    torch.cuda.synchronize()
    for rep in range(3):
        ix.locate_group_async(q)
        ix.sync()
        for bi, b in enumerate(bats):
            wo, wl = b["want"]
            assert np.array_equal(b["loff"].cpu().numpy().view(np.uint64), wo), f"rep {rep} batch {bi}: offsets"
            assert int(b["need"].item()) == wl.size, f"rep {rep} batch {bi}: total"
            assert np.array_equal(b["locs"].cpu().numpy()[:wl.size].view(np.uint32), wl), \
                f"rep {rep} batch {bi}: locations"
            assert np.array_equal(b["cnt"].cpu().numpy().view(np.uint32), np.diff(wo).astype(np.uint32))
    info = ix.info()
    # (300 batches: ONE grouped launch per round, over two kernel-argument groups)
    assert info["launches_grouped"] == 3 and info["launches_ordered"] == 0, info
    assert info["launches_chained"] == (3 if chain == "1" else 0), info
    ix.close()
