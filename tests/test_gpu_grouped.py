"""Grouped launches (fmx_internal.hpp kWsHeader): a launch's
patterns searched in the order of their last symbols instead of the order
given.  A launch is grouped when its batches are fixed-length with
patterns that pack into 96 bits (by default from 2^20 patterns, with a key
of at least 5 symbols); FMX_GROUPED=1 groups every such launch, however
small, so the parity tests below run the key / sorted-order / grouped-search
/ count kernels on fixed-length batches of every layout and alphabet size,
forward and reversed, with absent, wildcard and out-of-alphabet symbols,
several batches per launch and many launches on one workspace — each result
against the oracle (or the host API with grouping off).  FMX_GROUP_REFINE_MIN=1
runs the per-key refine sort (k_group_refine) on all of them too, and
FMX_GROUP_CHECK=1 checks every launch's sorted order on the device before its
search (each pattern placed once, under its own key, with its own symbols;
a violation is FMX_E_DEVICE)."""
import numpy as np
import pytest

import test_gpu as T
from _util import ALL_LAYOUTS, rand_chr_list, rand_pattern, rand_text, table_from_symbols

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["shipped", "refine_check"])
def grouped(request, monkeypatch):
    """Every grouped test twice: with the kernel sequence users get (grouping
    forced on, otherwise the shipped defaults: refine off, check off,
    in-workgroup sort on) and with the refine sort and the device check on."""
    monkeypatch.setenv("FMX_GROUPED", "1")
    for k in ("FMX_GROUP_REFINE_MIN", "FMX_GROUP_REFINE", "FMX_GROUP_CHECK", "FMX_GROUPED_WSORT",
              "FMX_GROUPED_RAW", "FMX_GROUPED_MIN", "FMX_GROUPED_PAIR", "FMX_GROUPED_XCD"):
        monkeypatch.delenv(k, raising=False)
    if request.param == "refine_check":
        monkeypatch.setenv("FMX_GROUP_REFINE_MIN", "1")  # k_group_refine on every grouped launch, however small
        monkeypatch.setenv("FMX_GROUP_CHECK", "1")  # the device-side check of the sorted order (k_group_check_*)
    monkeypatch.setenv("FMX_DEBUG", "1")  # (an FMX_E_DEVICE names its cause on stderr)
    return request.param


def pack_bits(sigma):
    return int(sigma).bit_length()  # ceil(log2(sigma + 1))


@pytest.mark.parametrize("pb,planes,vb", ALL_LAYOUTS)
def test_every_layout_grouped(pkg, O, grouped, pb, planes, vb):
    rng = np.random.default_rng(pb * 31 + planes * 7 + vb)
    for sigma in sorted({2, 3, (1 << planes) // 2 + 1, 1 << planes}):
        chars = rand_chr_list(rng, sigma)
        table = table_from_symbols([bytes([c]) for c in chars])
        text = rand_text(rng, chars, 300, 4000)
        k, sr = int(rng.integers(1, 5)), int(rng.integers(1, 5))
        if (sigma + 1) ** k > 1 << 20:
            k = 2
        blob = T.gpu_build(pkg, text, sigma, pb, planes, vb, k, sr, table)
        top = 96 // pack_bits(sigma)
        for m in sorted({1, 2, k, 7, top}):
            pats = [rand_pattern(rng, text, m, m) for _ in range(400)]
            pats = [p for p in pats if len(p) == m]
            pats += [bytes(rng.choice(np.frombuffer(chars, np.uint8), size=m)) for _ in range(40)]
            pats += [b"\x00" * m, chars[:1] * m, chars[-1:] * m]   # wildcard byte, single-symbol runs
            for occ in (0, 1):
                T.check_parity(pkg, O, blob, pb, planes, vb, 0, pats, occ, expect_path="grouped")


@pytest.mark.parametrize("m", [1, 3, 20, 32])
def test_fixed_len_grouped(pkg, O, grouped, m):
    """Group launches of fixed-length batches (sizes 1..2049, forward and
    reversed, counts output), a contradicting hint reported (FMX_E_ARG)."""
    T.test_fixed_len_hint(pkg, O, m)


def test_group_launch_many_batches_grouped(pkg, O, grouped):
    """270 fixed-length batches (two launches: 256 + 14), lengths 1..32, sizes
    1..4096, every third reversed, repeated 40 times on the same workspaces
    (the key counters must come back to zero after every launch)."""
    import torch
    rng = np.random.default_rng(34)
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=120_000).astype(np.uint8)
    blob = T.gpu_build(pkg, text.tobytes(), 5, 4, 3, 64, 3, 2, table)
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64))
    dev = torch.device("cuda:0")
    sizes = [2500, 1, 700, 256, 257, 3000, 40, 1999, 5, 1024, 33, 600, 77, 4096, 12, 300, 2, 900, 128, 255, 3,
             64, 1500, 3, 255, 511, 7, 2048, 90, 333, 17, 1200, 4, 640, 9, 2222, 31, 800, 65, 6]
    sizes += [int(x) for x in np.random.default_rng(6).integers(1, 600, size=230)]
    bats, jobs = [], []
    for bi, n in enumerate(sizes):
        rev, m = bi % 3 == 2, 1 + (bi * 7) % 32
        starts = rng.integers(0, text.size - m, size=n)
        pats = [text[s:s + m].tobytes() for s in starts]
        data, offsets = pkg.pack_patterns(pats)
        want = orc.locate_batch(data, offsets)
        q = [p[::-1] for p in pats] if rev else pats
        data, offsets = pkg.pack_patterns(q)
        cap = int(want[1].size) + 8
        b = dict(n=n, want=want, data=torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).to(dev),
                 off=torch.from_numpy(offsets.view(np.int64).copy()).to(dev),
                 loff=torch.full((n + 1,), -1, dtype=torch.int64, device=dev),
                 locs=torch.zeros(cap, dtype=torch.int32, device=dev), need=torch.zeros(1, dtype=torch.int64, device=dev),
                 cnt=torch.zeros(n, dtype=torch.int32, device=dev))
        ws = ix.locate_workspace_size(n)
        b["ws"] = torch.zeros(ws, dtype=torch.uint8, device=dev)
        jobs.append(ix.locate_job(b["data"].data_ptr(), b["off"].data_ptr(), n, b["loff"].data_ptr(),
                                  b["locs"].data_ptr(), cap, b["need"].data_ptr(), b["ws"].data_ptr(), ws,
                                  d_counts=b["cnt"].data_ptr(), reversed=rev, stage_kb=max(1, -(-256 * m // 1024)),
                                  fixed_len=m))
        bats.append(b)
    q = ix.job_queue(jobs)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    for rep in range(40):
        ix.locate_group_async(q, stream=stream.cuda_stream)
    ix.sync(stream.cuda_stream)
    for b in bats:
        wo, wl = b["want"]
        assert np.array_equal(b["loff"].cpu().numpy().view(np.uint64), wo)
        assert np.array_equal(b["locs"].cpu().numpy()[:wl.size].view(np.uint32), wl)
        assert int(b["need"].item()) == wl.size
        assert np.array_equal(b["cnt"].cpu().numpy().view(np.uint32), np.diff(wo).astype(np.uint32))
    ix.close()


def test_out_of_alphabet_grouped(pkg, O, grouped):
    """PassThrough bytes >= sigma in a fixed-length grouped batch are
    reported (FMX_E_SYMBOL) exactly as in launch order; a clean batch
    afterwards is answered exactly."""
    rng = np.random.default_rng(8)
    text = bytes(rng.integers(0, 4, size=5000).astype(np.uint8))
    blob = T.gpu_build(pkg, text, 4, 4, 3, 64, 3, 2, None)
    ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), pkg.text_encoders.PassThrough)
    pats = [text[s:s + 9] for s in rng.integers(0, 4990, size=300)]
    bad = pats[:100] + [b"\x01\x02\x09\x00\x01\x02\x03\x00\x01"] + pats[100:]
    with pytest.raises(pkg.FmxError):
        ix.locate_batch(bad)
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 1))
    data, offsets = pkg.pack_patterns(pats)
    goff, glocs = ix.locate_batch((data, offsets))
    ooff, olocs = orc.locate_batch(data, offsets)
    assert np.array_equal(goff, ooff) and np.array_equal(glocs, olocs)
    ix.close()


def test_grouped_equals_launch_order(pkg, O, monkeypatch):
    """A 300k-pattern fixed-length launch on a 4 Mbp text grouped (the
    default from 2^20 patterns; FMX_GROUPED_MIN moves the threshold)
    answers exactly like the same launch in launch order (FMX_GROUPED=0), and
    like the oracle; the index reports the grouping it applies."""
    rng = np.random.default_rng(5)
    chars = b"ACGT"
    text = rand_text(rng, chars, 4_000_000, 4_000_000)
    table = table_from_symbols([bytes([c]) for c in chars])
    blob = T.gpu_build(pkg, text, 4, 4, 3, 64, 3, 2, table)
    pats = [rand_pattern(rng, text, 20, 20) for _ in range(300_000)]
    data, offsets = pkg.pack_patterns(pats)
    res = {}
    monkeypatch.delenv("FMX_GROUPED", raising=False)
    monkeypatch.delenv("FMX_GROUPED_MIN", raising=False)
    ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=1)
    assert ix.info()["grouped_min"] == 3 << 20  # the default for a key of at least 5 symbols
    ix.close()
    monkeypatch.setenv("FMX_GROUPED", "0")
    for mode in ("0", None):
        if mode is None:
            monkeypatch.delenv("FMX_GROUPED")
            monkeypatch.setenv("FMX_GROUPED_MIN", "100000")
        ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=1)
        info = ix.info()
        assert info["group_key_len"] == 6 and info["group_key_base"] == 4
        if mode is None:
            assert info["grouped_min"] == 100000
        else:
            assert info["grouped_min"] == 2 ** 64 - 1
        res[mode] = ix.locate_batch((data, offsets))
        ix.close()
    assert np.array_equal(res["0"][0], res[None][0]) and np.array_equal(res["0"][1], res[None][1])
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    ooff, olocs = orc.locate_batch(data, offsets)
    assert np.array_equal(res[None][0], ooff) and np.array_equal(res[None][1], olocs)


def test_default_policy_by_alphabet(pkg, O, monkeypatch):
    """Grouping is on by default for launches of at least 3 x 2^20 patterns where
    the key spans at least 5 symbols (ACGT: 6), and from 2^26 for a
    20-residue alphabet (key of 3 symbols: no LF step beyond a k = 3 seed
    shared by the key alone — only a launch of ~100 M patterns shares
    enough deeper steps to pay for the dealing out)."""
    monkeypatch.delenv("FMX_GROUPED", raising=False)
    monkeypatch.delenv("FMX_GROUPED_MIN", raising=False)
    rng = np.random.default_rng(9)
    for chars, want_len, on in ((b"ACGT", 6, True), (b"ACDEFGHIKLMNPQRSTVWY", 3, False)):
        table = table_from_symbols([bytes([c]) for c in chars])
        text = rand_text(rng, chars, 20_000, 20_000)
        blob = T.gpu_build(pkg, text, len(chars), 4, 5, 64, 2, 2, table)
        ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block5(pkg.Vector.U64), options=1)
        info = ix.info()
        assert info["group_key_len"] == want_len and info["group_key_base"] == len(chars)
        assert info["grouped_min"] == (3 << 20 if on else 1 << 26)
        ix.close()


@pytest.mark.parametrize("pb,planes,vb", ALL_LAYOUTS)
def test_every_layout_grouped_raw(pkg, O, grouped, monkeypatch, pb, planes, vb):
    """Grouped launches with id-only sorted records (FMX_GROUPED_RAW=1 forces
    the long-pattern path on patterns that would pack): the key pass reads
    only the key's bytes, the search reads each pattern's bytes; the smallest
    and the largest alphabet of the sweep at m = 2 and 7, forward and
    reversed, blob layout and interleaved records."""
    monkeypatch.setenv("FMX_GROUPED_RAW", "1")
    rng = np.random.default_rng(pb * 31 + planes * 7 + vb + 1)
    for sigma in sorted({2, 1 << planes}):
        chars = rand_chr_list(rng, sigma)
        table = table_from_symbols([bytes([c]) for c in chars])
        text = rand_text(rng, chars, 300, 4000)
        k, sr = int(rng.integers(1, 5)), int(rng.integers(1, 5))
        if (sigma + 1) ** k > 1 << 20:
            k = 2
        blob = T.gpu_build(pkg, text, sigma, pb, planes, vb, k, sr, table)
        for m in (2, 7):
            pats = [rand_pattern(rng, text, m, m) for _ in range(300)]
            pats = [p for p in pats if len(p) == m]
            pats += [bytes(rng.choice(np.frombuffer(chars, np.uint8), size=m)) for _ in range(30)]
            for occ in (0, 1):
                T.check_parity(pkg, O, blob, pb, planes, vb, 0, pats, occ, expect_path="grouped_raw")


@pytest.mark.parametrize("m,pb,planes,vb", [(150, 8, 3, 128), (150, 4, 3, 64), (97, 4, 3, 64), (33, 8, 4, 32),
                                            (250, 8, 3, 128), (250, 4, 3, 64)])
def test_long_patterns_grouped(pkg, O, grouped, m, pb, planes, vb):
    """C5's shape: patterns too long to pack into a 96-bit record (150 bp)
    are grouped with id-only records, on a 2 Mbp ACGT text with the ACGTN
    table; 20,000 cut patterns + absent, wildcard and single-symbol ones,
    forward and reversed, every count and location against the oracle.
    m = 250 is longer than the search's LDS room for a raw pattern
    (kGroupRawStage = 216): those lanes read their pattern bytes from HBM."""
    rng = np.random.default_rng(m * 13 + pb)
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=2_000_000).astype(np.uint8).tobytes()
    blob = T.gpu_build(pkg, text, 5, pb, planes, vb, 3, 2, table)
    pats = [text[s:s + m] for s in rng.integers(0, len(text) - m, size=20_000)]
    pats += [bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), size=m)) for _ in range(200)]
    pats += [b"N" * m, b"A" * m, b"\x00" * m]
    T.check_parity(pkg, O, blob, pb, planes, vb, 0, pats, 1, expect_path="grouped_raw")
