"""CPU tests of the kernels as written: tests/simt/libfmx_simt.so is the
engine's own source (fmx_api.cpp, fmx_query.hip, fmx_layout.hip,
fmx_kernels.hpp, fmx_device.hpp — the C ABI, the launch logic and every
kernel) compiled for the CPU against a SIMT shim (tests/simt): one fiber per
work-item, workgroups in a shuffled order, work-items interleaved at random
between barriers, atomics returning in a random order, LDS and device memory
random until written, stream work queued and run late (a copy reads and
writes host memory when it runs).  The same Python API the GPU tests use runs on it, and
every answer is compared with the oracle under many schedules (seeds), so a
result that depends on scheduling, atomic order or unwritten memory fails here
deterministically — on the CPU, with the failing seed in the message.

The grouped launch path (k_group_key<count/place>, k_group_scan,
k_search_grouped, k_group_tiles, k_emit; FMX_GROUPED=1) is replayed on the
inputs of the GPU failure recorded in VERDICT r3 (test_every_layout_grouped
[4-5-32]: sigma 2, m 2, occ 1, a capacity retry and two internal passes: three
grouped launches on one workspace), on every layout, and on multi-batch
launches reusing workspaces."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from _util import ALL_LAYOUTS, rand_chr_list, rand_pattern, rand_text, table_from_symbols

HERE = os.path.dirname(os.path.abspath(__file__))
SIMT_DIR = os.path.join(HERE, "simt")
SIMT_LIB = os.path.join(SIMT_DIR, "libfmx_simt.so")


@pytest.fixture(scope="module")
def simt(pkg):
    subprocess.check_call(["make", "-s", "-j", str(min(8, os.cpu_count() or 1)), "-C", SIMT_DIR])
    n = pkg._native
    L = C.CDLL(SIMT_LIB)
    for name, (res, args) in n.SIGNATURES.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    L.simt_config.argtypes = [C.c_uint64, C.c_double]
    L.simt_config.restype = None
    L.simt_stats.argtypes = [C.POINTER(C.c_uint64)] * 3
    L.simt_stats.restype = None
    L.simt_memset_fault.argtypes = [C.c_uint64, C.POINTER(C.c_uint32), C.c_uint64]
    L.simt_memset_fault.restype = None
    L.simt_defer.argtypes = [C.c_int, C.c_double]
    L.simt_defer.restype = None
    L.simt_selftest_defer.argtypes = []
    L.simt_selftest_defer.restype = C.c_int
    L.simt_block_order.argtypes = [C.c_int]
    L.simt_block_order.restype = None
    # deferred streams for every test here: work queued on a stream runs at a
    # random later host call or when the host synchronises, copies read and
    # write host memory when they run (simt_rt.cpp)
    L.simt_defer(1, 0.25)
    # workgroups run one at a time in a shuffled order here, so the fused
    # launch (k_locate: a workgroup waits for its batch's earlier tiles) is off
    # by default and tested with index-ordered workgroups (fused fixture)
    # (and k_emit_chain, which ends grouped launches the same way)
    saved_env = {k: os.environ.get(k) for k in ("FMX_FUSED", "FMX_EMIT_CHAIN")}
    os.environ["FMX_FUSED"] = os.environ["FMX_EMIT_CHAIN"] = "0"
    saved = n._lib
    n._lib = L
    yield L
    n._lib = saved
    for k, v in saved_env.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def pos_of(pkg, pb):
    return pkg.u32 if pb == 4 else pkg.u64


def block_of(pkg, planes, vb):
    return getattr(pkg.blocks, f"Block{planes}")(pkg.Vector(vb))


def grouped_case_inputs(pb, planes, vb, sigma_pick=None, m_pick=None):
    """The inputs of test_gpu_grouped.py::test_every_layout_grouped (same
    seeds and draws), yielded per (sigma, m)."""
    rng = np.random.default_rng(pb * 31 + planes * 7 + vb)
    for sigma in sorted({2, 3, (1 << planes) // 2 + 1, 1 << planes}):
        chars = rand_chr_list(rng, sigma)
        table = table_from_symbols([bytes([c]) for c in chars])
        text = rand_text(rng, chars, 300, 4000)
        k, sr = int(rng.integers(1, 5)), int(rng.integers(1, 5))
        if (sigma + 1) ** k > 1 << 20:
            k = 2
        top = 96 // int(sigma).bit_length()
        for m in sorted({1, 2, k, 7, top}):
            pats = [rand_pattern(rng, text, m, m) for _ in range(400)]
            pats = [p for p in pats if len(p) == m]
            pats += [bytes(rng.choice(np.frombuffer(chars, np.uint8), size=m)) for _ in range(40)]
            pats += [b"\x00" * m, chars[:1] * m, chars[-1:] * m]
            if (sigma_pick is None or sigma == sigma_pick) and (m_pick is None or m == m_pick):
                yield sigma, m, text, table, k, sr, pats


def check_simt(pkg, O, blob, pb, planes, vb, pats, occ, reversed_too=True):
    L = O.layout(pb, planes, vb, 0)
    orc = O.OracleIndex(blob, L)
    ix = pkg.FmIndex.load(blob, pos_of(pkg, pb), block_of(pkg, planes, vb), options=occ)
    data, offsets = pkg.pack_patterns(pats)
    ooff, olocs = orc.locate_batch(data, offsets)
    goff, glocs = ix.locate_batch((data, offsets))
    gc, oc = np.diff(goff.astype(np.int64)), np.diff(ooff.astype(np.int64))
    bad = np.flatnonzero(gc != oc)
    assert bad.size == 0, (f"counts differ for {bad.size} patterns, first {bad[:6].tolist()}: "
                           f"simt {gc[bad[:6]].tolist()} oracle {oc[bad[:6]].tolist()}")
    assert np.array_equal(glocs, olocs), "locations differ (SA-row order)"
    if reversed_too:
        roff, rlocs = ix.locate_batch([p[::-1] for p in pats], reversed=True)
        assert np.array_equal(roff, ooff) and np.array_equal(rlocs, olocs), "reversed locate differs"
    ix.close()


@pytest.mark.parametrize("seed", range(3))
def test_grouped_verdict_r3_case(pkg, O, simt, monkeypatch, seed):
    """The failing GPU case of round 3, replayed under three schedules.  Before
    the fix in fmx_load (the blob upload waited for on the index stream) the
    late-landing upload made k_relayout build the records from stale memory
    and this test crashed in the emulator (the GPU read garbage silently)."""
    monkeypatch.setenv("FMX_GROUPED", "1")
    monkeypatch.setenv("FMX_GROUP_CHECK", "1")
    simt.simt_config(1000 + seed, 0.5)
    pb, planes, vb = 4, 5, 32
    for sigma, m, text, table, k, sr, pats in grouped_case_inputs(pb, planes, vb, sigma_pick=2, m_pick=2):
        blob = O.build(text, sigma, O.layout(pb, planes, vb), k, sr, table)
        for occ in (0, 1):
            check_simt(pkg, O, blob, pb, planes, vb, pats, occ)


@pytest.mark.parametrize("pb,planes,vb", ALL_LAYOUTS)
def test_every_layout_simt(pkg, O, simt, monkeypatch, pb, planes, vb):
    """Every layout, grouped (blob layout and interleaved records), grouped
    with id-only records and in launch order (interleaved records): the
    largest alphabet of the GPU sweep at m = k and m = 7 (the
    smallest alphabet, whose patterns have ~800 occurrences each, runs in the
    round-3 case above)."""
    simt.simt_config(pb * 131 + planes * 17 + vb, 0.5)
    monkeypatch.setenv("FMX_GROUP_CHECK", "1")
    cases = list(grouped_case_inputs(pb, planes, vb))
    sig = sorted({c[0] for c in cases})
    for sigma, m, text, table, k, sr, pats in cases:
        if not (sigma == sig[-1] and m in (k, 7)):
            continue
        blob = O.build(text, sigma, O.layout(pb, planes, vb), k, sr, table)
        for grouped, occs in (("1", (0, 1)), ("raw", (1,)), ("0", (1,))):
            # "raw": grouped with id-only sorted records (the search reads the pattern bytes)
            monkeypatch.setenv("FMX_GROUPED", "0" if grouped == "0" else "1")
            monkeypatch.setenv("FMX_GROUPED_RAW", "1" if grouped == "raw" else "0")
            for occ in occs:
                check_simt(pkg, O, blob, pb, planes, vb, pats[:110] + pats[-43:], occ, reversed_too=grouped != "0")


def test_group_launch_garbage_workspaces_simt(pkg, O, simt, monkeypatch):
    """fmx_locate_group_async on the emulator: 40 fixed-length batches in one
    grouped launch, lengths 1..32, every third reversed, workspaces and
    outputs filled with random bytes before the first launch (a
    grouped launch on a garbage workspace) and reused twice: every count,
    offset and location against the oracle each time."""
    monkeypatch.setenv("FMX_GROUPED", "1")
    monkeypatch.setenv("FMX_GROUP_CHECK", "1")
    simt.simt_config(77, 0.5)
    rng = np.random.default_rng(34)
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=30_000).astype(np.uint8)
    blob = O.build(text.tobytes(), 5, O.layout(4, 3, 64), 3, 2, table)
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=1)
    sizes = [int(x) for x in np.random.default_rng(6).integers(1, 400, size=40)]
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
        ws = ix.locate_workspace_size(n)
        b = dict(n=n, want=want, data=np.concatenate([data, np.zeros(16, np.uint8)]),
                 off=offsets.view(np.int64).copy(), loff=rng.integers(0, 2**62, size=n + 1).astype(np.int64),
                 locs=rng.integers(0, 2**31, size=cap).astype(np.int32), need=np.zeros(1, np.int64),
                 cnt=rng.integers(0, 2**31, size=n).astype(np.int32),
                 ws=rng.integers(0, 256, size=ws).astype(np.uint8))
        jobs.append(ix.locate_job(b["data"].ctypes.data, b["off"].ctypes.data, n, b["loff"].ctypes.data,
                                  b["locs"].ctypes.data, cap, b["need"].ctypes.data, b["ws"].ctypes.data, ws,
                                  d_counts=b["cnt"].ctypes.data, reversed=rev, stage_kb=max(1, -(-256 * m // 1024)),
                                  fixed_len=m))
        bats.append(b)
    q = ix.job_queue(jobs)
    for rep in range(2):
        ix.locate_group_async(q)
        ix.sync()
        for b in bats:
            wo, wl = b["want"]
            assert np.array_equal(b["loff"].view(np.uint64), wo), f"rep {rep}: offsets"
            assert np.array_equal(b["locs"][:wl.size].view(np.uint32), wl), f"rep {rep}: locations"
            assert int(b["need"][0]) == wl.size
            assert np.array_equal(b["cnt"].view(np.uint32), np.diff(wo).astype(np.uint32))
    ix.close()


@pytest.mark.parametrize("m,pb,planes,vb", [(150, 8, 3, 128), (97, 4, 3, 64), (33, 4, 3, 32), (250, 4, 3, 64)])
def test_long_patterns_grouped_simt(pkg, O, simt, monkeypatch, m, pb, planes, vb):
    """Patterns too long to pack into a 96-bit record (C5: 150 bp) are grouped
    with id-only records: the key pass reads only the key's bytes, the search
    reads each pattern's bytes itself; forward and reversed, against the
    oracle."""
    monkeypatch.setenv("FMX_GROUPED", "1")
    simt.simt_config(m * 7 + pb, 0.5)
    rng = np.random.default_rng(m)
    chars = b"ACGT"
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    text = rng.choice(np.frombuffer(chars, np.uint8), size=20_000).astype(np.uint8).tobytes()
    blob = O.build(text, 5, O.layout(pb, planes, vb), 3, 2, table)
    pats = [rand_pattern(rng, text, m, m) for _ in range(300)]
    pats += [bytes(rng.choice(np.frombuffer(chars, np.uint8), size=m)) for _ in range(20)]
    pats += [b"N" * m, b"A" * m]
    g0 = grids(simt)
    check_simt(pkg, O, blob, pb, planes, vb, pats, 1, reversed_too=False)
    assert grids(simt) - g0 == 12, ("not a grouped launch (load: relayout; locate: 4 x put (the batch table), key, "
                                    "scan, place, search, tiles, k_scan, emit)")
    check_simt(pkg, O, blob, pb, planes, vb, pats, 1)


GROUP_BINS = 8192  # fmx_internal.hpp kGroupBins
GROUP_SLOTS = 1  # kGroupSlots (build option): key k's sub-run of slot s counts at k * GROUP_SLOTS + s
COUNTERS = GROUP_BINS * GROUP_SLOTS


def test_group_check_catches_dirty_counters(pkg, O, simt, monkeypatch):
    """Fault injection: the grouped launch's key
    counters are left dirty, as a launch cut short between its count pass
    and its end would leave them without the zeroing memset.
      * -1 in key 1 and +1 in key 2 (patterns ending CAAAAA and GAAAAA,
        three of each): key 2's run starts one early, two patterns share a
        sorted position and the run's last one is never written — every
        position stays inside the launch and every bucket total is right,
        so the placing passes' guards pass it (no error without the check)
        and only FMX_GROUP_CHECK=1 sees it: FMX_E_DEVICE;
      * +5 in key 0: positions run past the launch's end; the place pass's
        guard refuses them: FMX_E_DEVICE without the check.
    The index answers correctly again on the next (clean) launch."""
    monkeypatch.setenv("FMX_GROUPED", "1")
    simt.simt_config(31337, 0.5)
    rng = np.random.default_rng(8)
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=6_000).astype(np.uint8).tobytes()
    blob = O.build(text, 5, O.layout(4, 3, 64), 3, 2, table)
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    pats = [text[s:s + 12] for s in rng.integers(0, len(text) - 12, size=700)]
    pats += [b"CCCCCCAAAAAA"] * 3 + [b"CCCCCCCAAAAA"] * 3 + [b"CCCCCCGAAAAA"] * 3
    data, offsets = pkg.pack_patterns(pats)
    want = orc.locate_batch(data, offsets)

    def inject(words):
        w = (C.c_uint32 * COUNTERS)(*words)
        simt.simt_memset_fault(4 * COUNTERS, w, COUNTERS)

    # (the one chunk is slot 0's)
    shifted = [0] * COUNTERS
    shifted[1 * GROUP_SLOTS], shifted[2 * GROUP_SLOTS] = 0xFFFFFFFF, 1
    over = [0] * COUNTERS
    over[0] = 5
    for check, words, caught in (("1", shifted, True), ("0", shifted, False), ("0", over, True),
                                 ("1", over, True)):
        monkeypatch.setenv("FMX_GROUP_CHECK", check)
        ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=1)
        got = ix.locate_batch((data, offsets))  # clean: the fault is not armed yet
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
        inject(words)
        if caught:
            with pytest.raises(pkg.FmxError) as ei:
                ix.locate_batch((data, offsets))
            assert ei.value.code == pkg._native.FMX_E_DEVICE
        else:
            ix.locate_batch((data, offsets))  # (answers from a broken order: what the check exists for)
        got = ix.locate_batch((data, offsets))
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]), "not clean after the fault"
        ix.close()


def grids(simt):
    g, i, s = C.c_uint64(), C.c_uint64(), C.c_uint64()
    simt.simt_stats(C.byref(g), C.byref(i), C.byref(s))
    return g.value


@pytest.mark.parametrize("seed", range(2))
def test_grouped_refine_simt(pkg, O, simt, monkeypatch, seed):
    """k_group_refine (each key's run re-sorted by the next key-length
    symbols): a launch of 3,000 fixed-length 16-bp patterns on a 4 kbp text
    (runs of a few records per key), forward and reversed; and one whose
    runs exceed a refine segment (8,192 records: 24,000 copies of three
    patterns, 9 variants of each in their next symbols); against the
    oracle."""
    monkeypatch.setenv("FMX_GROUPED", "1")
    monkeypatch.setenv("FMX_GROUP_REFINE_MIN", "1")
    monkeypatch.setenv("FMX_GROUP_CHECK", "1")
    simt.simt_config(4242 + seed, 0.5)
    rng = np.random.default_rng(99 + seed)
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=4_000).astype(np.uint8).tobytes()
    blob = O.build(text, 5, O.layout(4, 3, 64), 3, 2, table)
    pats = [text[s:s + 16] for s in rng.integers(0, len(text) - 16, size=3_000)]
    check_simt(pkg, O, blob, 4, 3, 64, pats, 1)
    base = [text[s:s + 16] for s in rng.integers(0, len(text) - 16, size=3)]
    var = [bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), size=10)) + b[10:] for b in base for _ in range(9)]
    check_simt(pkg, O, blob, 4, 3, 64, [var[i % len(var)] for i in range(24_000)], 1, reversed_too=False)


def test_timing_long_region_simt(pkg, O, simt):
    """Launch timing over a region of many launches: spans are folded into
    their timers as they complete (at most a few dozen pending), and every
    bracketed launch is counted — 150 host-API locates (timer `locate`) and
    40 split group launches (`locate`, `locate.search`, `locate.emit`)."""
    simt.simt_config(7, 0.0)
    rng = np.random.default_rng(3)
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=3_000).astype(np.uint8).tobytes()
    blob = O.build(text, 5, O.layout(4, 3, 64), 3, 2, table)
    ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=1)
    pats = [text[s:s + 8] for s in rng.integers(0, len(text) - 8, size=20)]
    ix.timing_enable(True, every=1)
    for _ in range(150):
        ix.locate_batch(pats)
    t = ix.timing_read()
    # (the first call may run a second pass: its output guess was too small)
    assert 150 <= t["locate"]["launches"] <= 151 and t["locate"]["units"] == t["locate"]["launches"] * len(pats)
    data, offsets = pkg.pack_patterns(pats)
    n = len(pats)
    ws = np.zeros(ix.locate_workspace_size(n), np.uint8)
    loff, locs, need = np.zeros(n + 1, np.int64), np.zeros(4096, np.int32), np.zeros(1, np.int64)
    job = ix.locate_job(data.ctypes.data, offsets.ctypes.data, n, loff.ctypes.data, locs.ctypes.data, 4096,
                        need.ctypes.data, ws.ctypes.data, ws.size)
    q = ix.job_queue([job])
    ix.timing_enable(True, every=1)
    for _ in range(40):
        ix.locate_group_async(q)
    ix.sync()
    t = ix.timing_read()
    assert all(t[k]["launches"] == 40 for k in ("locate", "locate.search", "locate.emit"))
    ix.timing_enable(False)
    ix.close()


@pytest.mark.skipif(os.environ.get("FMX_SIMT_SWEEP") != "1", reason="minutes each: FMX_SIMT_SWEEP=1")
@pytest.mark.parametrize("pb,planes,vb", [(4, 2, 64), (4, 2, 32), (8, 3, 128)])
def test_gpu_grouped_sweep_simt(pkg, O, simt, monkeypatch, pb, planes, vb):
    """test_gpu_grouped.py::test_every_layout_grouped's whole sweep for these
    layouts (every alphabet size and length, forward and reversed, blob and
    interleaved index) with the same environment: grouped, refine and the
    device check on (the layouts of the unexplained GPU failure of round 4,
    DESIGN.md §2; opt-in, ~2 minutes each)."""
    monkeypatch.setenv("FMX_GROUPED", "1")
    monkeypatch.setenv("FMX_GROUP_REFINE_MIN", "1")
    monkeypatch.setenv("FMX_GROUP_CHECK", "1")
    simt.simt_config(pb * 7 + planes * 5 + vb, 0.5)
    for sigma, m, text, table, k, sr, pats in grouped_case_inputs(pb, planes, vb):
        blob = O.build(text, sigma, O.layout(pb, planes, vb), k, sr, table)
        for occ in (0, 1):
            check_simt(pkg, O, blob, pb, planes, vb, pats, occ)


def test_deferred_stream_model_simt(simt):
    """The emulator's stream model (what the staging tests below rely on): a
    queued host-to-device copy reads its source when it runs, a queued
    device-to-host copy has not written its destination before the host
    waits, an event orders both."""
    assert simt.simt_selftest_defer() == 0


@pytest.mark.parametrize("seed", range(2))
def test_pinned_stage_simt(pkg, O, simt, monkeypatch, seed):
    """Every host <-> HBM copy goes through the index's double-buffered pinned
    stage (fmx_internal.hpp Stage).  With 4 KiB chunks the blob
    upload and a 48 KB batch (2,400 x 20 bp) take many chunks in turn through
    the two buffers, and the deferred streams run each copy late: a buffer
    refilled before its previous copy ran, or a result read before its copy
    ran, gives wrong answers here.  Counts, locations (forward and reversed)
    and the caller's buffer unchanged, against the oracle."""
    monkeypatch.setenv("FMX_STAGE_CHUNK", "4096")
    simt.simt_config(900 + seed, 0.5)
    simt.simt_defer(1, 0.5)
    rng = np.random.default_rng(55 + seed)
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=40_000).astype(np.uint8).tobytes()
    blob = O.build(text, 5, O.layout(4, 3, 64), 3, 2, table)
    pats = [text[s:s + 20] for s in rng.integers(0, len(text) - 20, size=2_400)]
    pats += [b"ACGTN" * 4, b"A" * 20]
    data, offsets = pkg.pack_patterns(pats)
    ref = data.copy()
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    ooff, olocs = orc.locate_batch(data, offsets)
    for occ in (0, 1):
        ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=occ)
        goff, glocs = ix.locate_batch((data, offsets))
        assert np.array_equal(goff, ooff) and np.array_equal(glocs, olocs)
        assert np.array_equal(ix.count_batch((data, offsets)).astype(np.uint64), np.diff(ooff))
        roff, rlocs = ix.locate_batch([p[::-1] for p in pats], reversed=True)
        assert np.array_equal(roff, ooff) and np.array_equal(rlocs, olocs)
        ix.close()
    assert np.array_equal(data, ref), "the caller's pattern buffer changed"
    simt.simt_defer(1, 0.25)


@pytest.mark.parametrize("refine", ["1", "0"])
def test_protein_grouped_refine_simt(pkg, O, simt, monkeypatch, refine):
    """C4's shape (20 residues + X wildcard, sigma 21, u32/Block5<u64>): a
    grouped launch keys on the last 3 residues (8,000 of the 8,192 bins), the
    refine pass orders each key's run by the next 3, and the in-workgroup sort
    then orders a workgroup by the residue after those 6 (or after the key's 3
    without the refine pass); 3,000 x 12 aa + absent and X patterns, forward
    and reversed, the sorted order checked on the device, against the
    oracle."""
    monkeypatch.setenv("FMX_GROUPED", "1")
    monkeypatch.setenv("FMX_GROUP_CHECK", "1")
    monkeypatch.setenv("FMX_GROUP_REFINE_MIN", "1" if refine == "1" else "18446744073709551615")
    simt.simt_config(2121 + int(refine), 0.5)
    rng = np.random.default_rng(21)
    amino = b"ACDEFGHIKLMNPQRSTVWY"
    table = table_from_symbols([bytes([c]) for c in amino] + [b"X"])
    text = rng.choice(np.frombuffer(amino, np.uint8), size=30_000).astype(np.uint8).tobytes()
    blob = O.build(text, 21, O.layout(4, 5, 64), 3, 2, table)
    pats = [text[s:s + 12] for s in rng.integers(0, len(text) - 12, size=3_000)]
    pats += [bytes(rng.choice(np.frombuffer(amino, np.uint8), size=12)) for _ in range(50)]
    pats += [b"X" * 12, b"W" * 12, text[:12], text[-12:]]
    ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block5(pkg.Vector.U64), options=1)
    info = ix.info()
    assert info["group_key_len"] == 3 and info["group_key_base"] == 20
    ix.close()
    check_simt(pkg, O, blob, 4, 5, 64, pats, 1)


def test_workspace_alignment_simt(pkg, O, simt):
    """the grouped passes read and write a workspace as 16-B
    vectors, so fmx_locate_batch_async and fmx_locate_group_async refuse a
    workspace that is not 16-byte aligned (FMX_E_ARG) instead of issuing
    misaligned vector accesses; the same workspace 16 bytes further on works."""
    rng = np.random.default_rng(4)
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=5_000).astype(np.uint8).tobytes()
    blob = O.build(text, 5, O.layout(4, 3, 64), 3, 2, table)
    ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=1)
    pats = [text[s:s + 10] for s in rng.integers(0, len(text) - 10, size=50)]
    data, offsets = pkg.pack_patterns(pats)
    n = len(pats)
    ws_need = ix.locate_workspace_size(n)
    raw = np.zeros(ws_need + 64, np.uint8)
    base = raw.ctypes.data + (-raw.ctypes.data) % 16
    loff, locs, need = np.zeros(n + 1, np.int64), np.zeros(4096, np.int32), np.zeros(1, np.int64)
    args = (data.ctypes.data, offsets.ctypes.data, n, loff.ctypes.data, locs.ctypes.data, 4096, need.ctypes.data)
    with pytest.raises(pkg.FmxError) as ei:
        ix.locate_batch_async(*args, base + 8, ws_need)
    assert ei.value.code == pkg._native.FMX_E_ARG
    with pytest.raises(pkg.FmxError) as ei:
        ix.locate_group_async(ix.job_queue([ix.locate_job(*args, base + 8, ws_need)]))
    assert ei.value.code == pkg._native.FMX_E_ARG
    ix.locate_batch_async(*args, base + 16, ws_need)
    ix.sync()
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    ooff, olocs = orc.locate_batch(data, offsets)
    assert np.array_equal(loff.view(np.uint64), ooff) and np.array_equal(locs[:olocs.size].view(np.uint32), olocs)
    ix.close()


def test_grouping_policy_simt(pkg, O, simt, monkeypatch):
    """The default grouping policy (fmx_api.cpp finish_load): a DNA index
    (key of 6 symbols) groups launches of at least 2^20 patterns — below
    that the dealing out's fixed cost eats the sharing (C1's 256 x 1,000
    patterns: 8.0 vs 4.2 x 10^9 in launch order, profiles/r5/r5q_*);
    FMX_GROUPED_MIN moves the threshold, FMX_GROUPED=1 groups every launch
    that can be, FMX_GROUPED=0 none."""
    for k in ("FMX_GROUPED", "FMX_GROUPED_MIN"):
        monkeypatch.delenv(k, raising=False)
    rng = np.random.default_rng(12)
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=5_000).astype(np.uint8).tobytes()
    blob = O.build(text, 5, O.layout(4, 3, 64), 3, 2, table)

    def policy():
        ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=1)
        i = ix.info()
        ix.close()
        return i["group_key_len"], i["grouped_min"]
    assert policy() == (6, 3 << 20)
    monkeypatch.setenv("FMX_GROUPED_MIN", "5000")
    assert policy() == (6, 5000)
    monkeypatch.delenv("FMX_GROUPED_MIN")
    monkeypatch.setenv("FMX_GROUPED", "1")
    assert policy() == (6, 1)
    monkeypatch.setenv("FMX_GROUPED", "0")
    assert policy() == (6, 2 ** 64 - 1)


@pytest.fixture
def fused(simt, monkeypatch):
    """The fused launch (k_locate) and the chained grouped emit
    (k_emit_chain) on, workgroups run in a SHUFFLED order: a workgroup answers
    the tile of its ticket (take_ticket, the number of its batch's workgroups
    started before it), so it only ever waits on tiles already running and
    the launch needs no dispatch order at all."""
    monkeypatch.setenv("FMX_FUSED", "1")
    monkeypatch.setenv("FMX_EMIT_CHAIN", "1")
    simt.simt_block_order(0)
    yield simt


def fused_case(O, rng, pb, planes, vb, sigma, n_text):
    chars = rand_chr_list(rng, sigma)
    table = table_from_symbols([bytes([c]) for c in chars])
    text = rand_text(rng, chars, n_text, n_text)
    blob = O.build(text, len(chars) + 1, O.layout(pb, planes, vb), 2, 2, table)
    return chars, text, blob


@pytest.mark.parametrize("pb,planes,vb,occ", [(4, 3, 64, 1), (4, 2, 32, 0), (8, 3, 128, 1), (4, 5, 64, 1)])
def test_fused_locate_simt(pkg, O, fused, pb, planes, vb, occ):
    """k_locate (search, tile counts handed from workgroup to workgroup,
    offsets and locations in one kernel) against the oracle: fixed-length
    batches of five tiles, short patterns (counts of 0, 1 and hundreds: the
    settled and the dealt emission), long ones (one row each: the row walked
    during the search), forward and reversed; every launch took the fused
    path (fmx_index_info.launches_fused)."""
    fused.simt_config(pb * 1000 + planes * 100 + vb + occ, 0.5)
    rng = np.random.default_rng(pb * 31 + planes * 7 + vb)
    chars, text, blob = fused_case(O, rng, pb, planes, vb, min(1 << planes, 12) - 1, 4000)
    orc = O.OracleIndex(blob, O.layout(pb, planes, vb, 0))
    ix = pkg.FmIndex.load(blob, pos_of(pkg, pb), block_of(pkg, planes, vb), options=occ)
    launches = 0
    for m in (3, 17):
        pats = [rand_pattern(rng, text, m, m) for _ in range(1150)]
        pats = [p for p in pats if len(p) == m]
        pats += [bytes(rng.choice(np.frombuffer(chars, np.uint8), size=m)) for _ in range(40)]
        pats += [chars[:1] * m, chars[-1:] * m]
        data, offsets = pkg.pack_patterns(pats)
        ooff, olocs = orc.locate_batch(data, offsets)
        goff, glocs = ix.locate_batch((data, offsets))
        assert np.array_equal(goff, ooff), f"m={m}: offsets"
        assert np.array_equal(glocs, olocs), f"m={m}: locations"
        roff, rlocs = ix.locate_batch([p[::-1] for p in pats], reversed=True)
        assert np.array_equal(roff, ooff) and np.array_equal(rlocs, olocs), f"m={m}: reversed"
        launches += 2
        assert int(np.diff(ooff).max()) > (1 if m == 3 else 0)
    info = ix.info()
    assert info["launches_fused"] == info["launches_ordered"] >= launches, info
    ix.close()


def test_fused_group_garbage_workspaces_simt(pkg, O, fused, monkeypatch):
    """A fused group launch (fmx_locate_group_async in launch order): 24
    fixed-length batches of 1-5 tiles, lengths 2..23, every third reversed,
    workspaces (where the tile counts and their tags live) and outputs full of
    random bytes, run three times on the same workspaces — a tag left by an
    earlier launch must never pass for this one's."""
    monkeypatch.setenv("FMX_GROUPED", "0")
    fused.simt_config(4242, 0.5)
    rng = np.random.default_rng(35)
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=20_000).astype(np.uint8)
    blob = O.build(text.tobytes(), 5, O.layout(4, 3, 64), 3, 2, table)
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=1)
    sizes = [int(x) for x in np.random.default_rng(7).integers(1, 1200, size=24)]
    bats, jobs = [], []
    for bi, n in enumerate(sizes):
        rev, m = bi % 3 == 2, 2 + (bi * 5) % 22
        starts = rng.integers(0, text.size - m, size=n)
        pats = [text[s:s + m].tobytes() for s in starts]
        data, offsets = pkg.pack_patterns(pats)
        want = orc.locate_batch(data, offsets)
        q = [p[::-1] for p in pats] if rev else pats
        data, offsets = pkg.pack_patterns(q)
        cap = int(want[1].size) + 8
        ws = ix.locate_workspace_size(n)
        b = dict(n=n, want=want, data=np.concatenate([data, np.zeros(16, np.uint8)]),
                 off=offsets.view(np.int64).copy(), loff=rng.integers(0, 2**62, size=n + 1).astype(np.int64),
                 locs=rng.integers(0, 2**31, size=cap).astype(np.int32), need=np.zeros(1, np.int64),
                 cnt=rng.integers(0, 2**31, size=n).astype(np.int32),
                 ws=rng.integers(0, 256, size=ws).astype(np.uint8))
        jobs.append(ix.locate_job(b["data"].ctypes.data, b["off"].ctypes.data, n, b["loff"].ctypes.data,
                                  b["locs"].ctypes.data, cap, b["need"].ctypes.data, b["ws"].ctypes.data, ws,
                                  d_counts=b["cnt"].ctypes.data, reversed=rev, stage_kb=max(1, -(-256 * m // 1024)),
                                  fixed_len=m))
        bats.append(b)
    q = ix.job_queue(jobs)
    for rep in range(3):
        ix.locate_group_async(q)
        ix.sync()
        for b in bats:
            wo, wl = b["want"]
            assert np.array_equal(b["loff"].view(np.uint64), wo), f"rep {rep}: offsets"
            assert np.array_equal(b["locs"][:wl.size].view(np.uint32), wl), f"rep {rep}: locations"
            assert int(b["need"][0]) == wl.size
            assert np.array_equal(b["cnt"].view(np.uint32), np.diff(wo).astype(np.uint32))
    info = ix.info()
    assert info["launches_fused"] == info["launches_ordered"] == 3, info
    ix.close()


def test_fused_wait_is_bounded_simt(pkg, O, simt, monkeypatch):
    """k_locate's waits end.  Without tickets (FMX_FUSED_TICKETS=0: each
    workgroup answers the tile of its index) and workgroups run in a shuffled
    order (a later tile before an earlier one, one workgroup at a time: the
    residency trap of ADVICE r5 in its extreme form) the waiting workgroups
    give up after FMX_FUSED_TIMEOUT_MS and the launch reports FMX_E_DEVICE
    instead of hanging; the next launch, dispatched in order, answers
    correctly.  With tickets (the default) the same shuffled launch answers
    correctly: every tile waits only on tiles whose workgroups already ran."""
    monkeypatch.setenv("FMX_FUSED", "1")
    monkeypatch.setenv("FMX_FUSED_TIMEOUT_MS", "20")
    monkeypatch.setenv("FMX_FUSED_TICKETS", "0")
    simt.simt_config(99, 0.5)
    rng = np.random.default_rng(3)
    chars, text, blob = fused_case(O, rng, 4, 3, 64, 4, 3000)
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=1)
    pats = [text[s:s + 9] for s in rng.integers(0, len(text) - 9, size=8 * 256)]
    data, offsets = pkg.pack_patterns(pats)
    ooff, olocs = orc.locate_batch(data, offsets)
    with pytest.raises(pkg.FmxError) as ei:
        ix.locate_batch((data, offsets))
    assert ei.value.code == pkg._native.FMX_E_DEVICE
    simt.simt_block_order(1)
    try:
        goff, glocs = ix.locate_batch((data, offsets))
    finally:
        simt.simt_block_order(0)
    assert np.array_equal(goff, ooff) and np.array_equal(glocs, olocs)
    ix.close()
    monkeypatch.setenv("FMX_FUSED_TICKETS", "1")
    ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=1)
    for rep in range(3):  # (shuffled; the counters back at zero after every launch)
        goff, glocs = ix.locate_batch((data, offsets))
        assert np.array_equal(goff, ooff) and np.array_equal(glocs, olocs), f"tickets, launch {rep}"
    # (the host API may launch a batch twice: its first output guess too small)
    assert ix.info()["launches_fused"] == ix.info()["launches_ordered"] >= 3
    ix.close()


@pytest.mark.parametrize("seed", range(2))
def test_chained_grouped_emit_simt(pkg, O, fused, monkeypatch, seed):
    """Grouped launches ended by k_emit_chain (the tile counts handed from
    tile to tile inside the kernel) instead of k_group_tiles + k_emit: the
    group launch of 40 fixed-length batches (1-1,500 patterns, lengths 1..32,
    every third reversed) on random-byte workspaces, twice, against the
    oracle; every launch grouped and chained."""
    monkeypatch.setenv("FMX_GROUPED", "1")
    monkeypatch.setenv("FMX_GROUP_CHECK", "1")
    fused.simt_config(1000 + seed, 0.5)
    rng = np.random.default_rng(60 + seed)
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=30_000).astype(np.uint8)
    blob = O.build(text.tobytes(), 5, O.layout(4, 3, 64), 3, 2, table)
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=1)
    sizes = [int(x) for x in np.random.default_rng(6 + seed).integers(1, 1500, size=40)]
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
        ws = ix.locate_workspace_size(n)
        b = dict(n=n, want=want, data=np.concatenate([data, np.zeros(16, np.uint8)]),
                 off=offsets.view(np.int64).copy(), loff=rng.integers(0, 2**62, size=n + 1).astype(np.int64),
                 locs=rng.integers(0, 2**31, size=cap).astype(np.int32), need=np.zeros(1, np.int64),
                 cnt=rng.integers(0, 2**31, size=n).astype(np.int32),
                 ws=rng.integers(0, 256, size=ws).astype(np.uint8))
        jobs.append(ix.locate_job(b["data"].ctypes.data, b["off"].ctypes.data, n, b["loff"].ctypes.data,
                                  b["locs"].ctypes.data, cap, b["need"].ctypes.data, b["ws"].ctypes.data, ws,
                                  d_counts=b["cnt"].ctypes.data, reversed=rev, stage_kb=max(1, -(-256 * m // 1024)),
                                  fixed_len=m))
        bats.append(b)
    q = ix.job_queue(jobs)
    for rep in range(2):
        ix.locate_group_async(q)
        ix.sync()
        for b in bats:
            wo, wl = b["want"]
            assert np.array_equal(b["loff"].view(np.uint64), wo), f"rep {rep}: offsets"
            assert np.array_equal(b["locs"][:wl.size].view(np.uint32), wl), f"rep {rep}: locations"
            assert int(b["need"][0]) == wl.size
            assert np.array_equal(b["cnt"].view(np.uint32), np.diff(wo).astype(np.uint32))
    info = ix.info()
    assert info["launches_grouped"] == info["launches_chained"] == 2, info
    ix.close()


@pytest.mark.parametrize("grouped", ["1", "0"])
def test_launch_of_many_groups_simt(pkg, O, simt, monkeypatch, grouped):
    """More than 256 batches in one fmx_locate_group_async call (700: three
    kernel-argument groups).  Grouped: ONE grouped launch over all of them —
    the key counts and the place pass per group, the scan, the refine and
    check passes and the search once over the launch's whole order (its batch
    table, GroupTab, in the first batch's workspace), tiles and emit per
    group; in launch order: one launch per group.  Fixed-length batches of
    1-60 patterns, lengths 2..29, every third reversed, random-byte
    workspaces, twice, against the oracle."""
    monkeypatch.setenv("FMX_GROUPED", grouped)
    monkeypatch.setenv("FMX_GROUP_CHECK", "1")
    monkeypatch.setenv("FMX_GROUP_REFINE_MIN", "1")
    simt.simt_config(515 + len(grouped), 0.5)
    rng = np.random.default_rng(71)
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=20_000).astype(np.uint8)
    blob = O.build(text.tobytes(), 5, O.layout(4, 3, 64), 3, 2, table)
    orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
    ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), options=1)
    sizes = [int(x) for x in np.random.default_rng(8).integers(1, 60, size=700)]
    bats, jobs = [], []
    for bi, n in enumerate(sizes):
        rev, m = bi % 3 == 2, 2 + (bi * 11) % 28
        starts = rng.integers(0, text.size - m, size=n)
        pats = [text[s:s + m].tobytes() for s in starts]
        data, offsets = pkg.pack_patterns(pats)
        want = orc.locate_batch(data, offsets)
        q = [p[::-1] for p in pats] if rev else pats
        data, offsets = pkg.pack_patterns(q)
        cap = int(want[1].size) + 8
        ws = ix.locate_workspace_size(n)
        b = dict(n=n, want=want, data=np.concatenate([data, np.zeros(16, np.uint8)]),
                 off=offsets.view(np.int64).copy(), loff=rng.integers(0, 2**62, size=n + 1).astype(np.int64),
                 locs=rng.integers(0, 2**31, size=cap).astype(np.int32), need=np.zeros(1, np.int64),
                 cnt=rng.integers(0, 2**31, size=n).astype(np.int32),
                 ws=rng.integers(0, 256, size=ws).astype(np.uint8))
        jobs.append(ix.locate_job(b["data"].ctypes.data, b["off"].ctypes.data, n, b["loff"].ctypes.data,
                                  b["locs"].ctypes.data, cap, b["need"].ctypes.data, b["ws"].ctypes.data, ws,
                                  d_counts=b["cnt"].ctypes.data, reversed=rev, stage_kb=max(1, -(-256 * m // 1024)),
                                  fixed_len=m))
        bats.append(b)
    q = ix.job_queue(jobs)
    for rep in range(2):
        ix.locate_group_async(q)
        ix.sync()
        for bi, b in enumerate(bats):
            wo, wl = b["want"]
            assert np.array_equal(b["loff"].view(np.uint64), wo), f"rep {rep} batch {bi}: offsets"
            assert np.array_equal(b["locs"][:wl.size].view(np.uint32), wl), f"rep {rep} batch {bi}: locations"
            assert int(b["need"][0]) == wl.size
            assert np.array_equal(b["cnt"].view(np.uint32), np.diff(wo).astype(np.uint32))
    info = ix.info()
    if grouped == "1":
        assert info["launches_grouped"] == 2 and info["launches_ordered"] == 0, info
    else:
        assert info["launches_grouped"] == 0 and info["launches_ordered"] == 6, info
    ix.close()
