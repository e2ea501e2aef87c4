"""Full-size parity on BASELINE.json's configurations (C2, C4, C5): the blob
is built on the GPU from a seeded synthetic text, copied to the host, and the
oracle (oracle/fmx_oracle.c, the C restatement of the reference's query path)
answers the same patterns on the same blob bytes.  Every count and every
location (suffix-array-row order) of the GPU must equal the oracle's, under
the default index (FMX_OPT_DEFAULT: interleaved records) in launch order and
with the launch grouped (FMX_GROUPED=1), and on the blob as laid out
(FMX_OCC_BLOB).  Sizes are the configs' own: 1 Gbp / 1 G residues / 3 Gbp
texts; 100,000 patterns each (C5: a 100,000-pattern subset of its 1 M)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ACGTN = [b"Aa", b"Cc", b"Gg", b"Tt", b"Nn"]
AMINO = b"ACDEFGHIKLMNPQRSTVWY"


def progress(msg):
    print(f"[full] {msg}", flush=True)


def oracle_threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def run_config(pkg, O, n, alphabet, symbols, pos, planes, vec, m, npat, seed, extra=()):
    import torch
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    alpha = torch.tensor(list(alphabet), dtype=torch.uint8, device=dev)
    d_text = torch.empty(n, dtype=torch.uint8, device=dev)
    for c0 in range(0, n, 1 << 28):
        c1 = min(n, c0 + (1 << 28))
        d_text[c0:c1] = alpha[torch.randint(0, len(alphabet), (c1 - c0,), device=dev, generator=gen)]
    table = pkg.text_encoders.EncodingTable.from_symbols(symbols)
    position = pkg.u32 if pos == 4 else pkg.u64
    block = getattr(pkg.blocks, f"Block{planes}")(pkg.Vector(vec))
    b = (pkg.FmIndexBuilder(n, table.symbol_count(), table, position, block)
         .set_lookup_table_config(pkg.build_config.LookupTableConfig.KmerSize(3))
         .set_suffix_array_config(pkg.build_config.SuffixArrayConfig.Compressed(2)))
    size = b.blob_size()
    d_blob = torch.empty(size, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()  # (fmx_build_device also waits for the device)
    b.build_device(d_text.data_ptr(), d_blob.data_ptr(), size)
    progress(f"n={n:,}: blob {size:,} B built on the GPU")
    starts = torch.randint(0, n - m + 1, (npat,), device=dev, generator=gen)
    pats = d_text[(starts[:, None] + torch.arange(m, device=dev)[None, :]).reshape(-1)].cpu().numpy()
    blob = O.aligned_zeros(size, 16)
    blob[:] = d_blob.cpu().numpy()
    del d_text, d_blob
    torch.cuda.empty_cache()
    offsets = np.arange(npat + 1, dtype=np.uint64) * m
    # a few edge patterns (absent, wildcard-only, short — not so short that
    # they occur millions of times: the oracle walks every row), answered in
    # a call of their own: the fixed-length batch alone is what a grouped
    # launch takes (a batch of mixed lengths always runs in launch order)
    ex_d, ex_o = pkg.pack_patterns([bytes(x) for x in extra]) if extra else (None, None)
    orc = O.OracleIndex(blob, O.layout(pos, planes, vec, 0))
    ooff, olocs = orc.locate_batch(pats, offsets, threads=oracle_threads())
    eoff, elocs = orc.locate_batch(ex_d, ex_o, threads=oracle_threads()) if extra else (None, None)
    cnts = np.diff(ooff)
    top = np.argsort(cnts)[-3:]
    progress(f"oracle: {npat:,} patterns, {olocs.size:,} locations; most: "
             + ", ".join(f"{bytes(pats[int(offsets[i]):int(offsets[i + 1])])!r} x{int(cnts[i])}" for i in top)
             + f"; zero counts: {int((cnts == 0).sum())}")
    starts_h = starts.cpu().numpy()
    # (load options, environment at load, the path the batch must take): the
    # default index as loaded (100k patterns: below the grouping threshold,
    # launch order), grouping forced on (packed records for C2 and C4, id-only
    # records for C5's 150 bp), and the blob as laid out
    raw = m * int(table.symbol_count()).bit_length() > 96
    runs = ((pkg._native.FMX_OPT_DEFAULT, {}, "ordered"),
            (pkg._native.FMX_OPT_DEFAULT, {"FMX_GROUPED": "1", "FMX_GROUPED_RAW": "1" if raw else "0"},
             "grouped_raw" if raw else "grouped"),
            (pkg._native.FMX_OCC_BLOB, {}, "ordered"))
    for options, env, path in runs:
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)  # (read at load)
        try:
            ix = pkg.FmIndex.load(blob, position, block, table, options=options)
        finally:
            for k, v in saved.items():
                if v is None:
                    del os.environ[k]
                else:
                    os.environ[k] = v
        goff, glocs = ix.locate_batch((pats, offsets))
        info = ix.info()
        took = {k: info["launches_" + k] for k in ("grouped", "grouped_raw", "ordered")}
        # (one call may launch more than once: the host API reruns a batch whose locations overflow its
        # first output guess)
        assert took[path] >= 1 and sum(took.values()) == took[path], \
            f"options {options} {env}: expected {path}, ran {took}"
        assert np.array_equal(goff, ooff), f"offsets differ, options {options} {env}"
        assert np.array_equal(glocs, olocs), f"locations differ, options {options} {env}"
        cnt = ix.count_batch((pats, offsets))
        assert np.array_equal(cnt.astype(np.uint64), np.diff(ooff))
        if extra:
            xoff, xlocs = ix.locate_batch((ex_d, ex_o))
            assert np.array_equal(xoff, eoff) and np.array_equal(xlocs, elocs), f"edge patterns, {options} {env}"
        progress(f"options {options} {env}: {path}, bit-exact")
        ix.close()
    # the size-independent property: every cut pattern finds its own start
    own = np.zeros(npat, dtype=bool)
    cnt = np.diff(ooff[:npat + 1]).astype(np.int64)
    owner = np.repeat(np.arange(npat), cnt)
    own[owner[olocs[:owner.size].astype(np.int64) == starts_h[owner]]] = True
    assert own.all()
    return ooff, olocs


def test_c2_full(pkg, O):
    """C2: 1 Gbp ACGT (ACGTN table), u32/Block3<u64>, sr 2, k 3, 100,000 x 20 bp."""
    run_config(pkg, O, 1_000_000_000, b"ACGT", ACGTN, 4, 3, 64, 20, 100_000, 42,
               extra=[b"N" * 20, b"ACGTNACGTN", b"GATTACA" * 3, b"ACGTACGTACGT"])


def test_c4_full(pkg, O):
    """C4: 1 G residues over 20 amino acids (+X wildcard: sigma 21),
    u32/Block5<u64>, sr 2, k 3, 100,000 x 12 aa."""
    run_config(pkg, O, 1_000_000_000, AMINO, [bytes([c, c + 32]) for c in AMINO] + [b"Xx"], 4, 5, 64, 12,
               100_000, 43, extra=[b"X" * 12, b"WWWWWWWWWWWW", b"MKV", b"ACDEFGHIKLMNPQRSTVWY"])


def test_c5_full(pkg, O):
    """C5: 3 Gbp ACGT, u64/Block3<u128> (ALIGN 16), sr 2, k 3, 100,000 x 150 bp."""
    run_config(pkg, O, 3_000_000_000, b"ACGT", ACGTN, 8, 3, 128, 150, 100_000, 44,
               extra=[b"N" * 150, b"ACGT" * 37, b"GATTACAGATTACA"])


def _device_text(n, seed, alphabet=b"ACGT"):
    import torch
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    alpha = torch.tensor(list(alphabet), dtype=torch.uint8, device=dev)
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    for c0 in range(0, n, 1 << 28):
        c1 = min(n, c0 + (1 << 28))
        d[c0:c1] = alpha[torch.randint(0, len(alphabet), (c1 - c0,), device=dev, generator=gen)]
    return d, gen


def test_builder_sa64_matches_sa32(pkg, O, monkeypatch):
    """200 Mbp (with a long repeat and an N run): the 64-bit suffix-array
    path and the 32-bit one give byte-identical blobs at a size where both
    run with many workgroups and large buckets."""
    import torch
    n = 200_000_000
    d_text, _ = _device_text(n, 7)
    d_text[50_000_000:50_100_000] = d_text[10_000_000:10_100_000]   # a 100 kbp repeat
    d_text[120_000_000:120_050_000] = ord("N")                       # an N run (wildcard)
    table = pkg.text_encoders.EncodingTable.from_symbols(ACGTN)
    b = (pkg.FmIndexBuilder(n, 5, table, pkg.u64, pkg.blocks.Block3(pkg.Vector.U128))
         .set_lookup_table_config(pkg.build_config.LookupTableConfig.KmerSize(3))
         .set_suffix_array_config(pkg.build_config.SuffixArrayConfig.Compressed(2)))
    size = b.blob_size()
    blobs = []
    for force in ("0", "1"):
        monkeypatch.setenv("FMX_BUILD_SA64", force)
        d_blob = torch.zeros(size, dtype=torch.uint8, device="cuda:0")
        b.build_device(d_text.data_ptr(), d_blob.data_ptr(), size)
        blobs.append(d_blob)
        progress(f"SA64={force}: built {size:,} B")
    assert torch.equal(blobs[0], blobs[1])


def _big_text_case(pkg, O, n, position, block, layout, npat=2000, m=24, seed=11):
    """Build an n-symbol text on the GPU, then answer npat patterns cut from
    it (the text's last m symbols among them) + wildcard ones like the oracle
    on the same blob, each finding its own start."""
    import torch
    d_text, gen = _device_text(n, seed)
    table = pkg.text_encoders.EncodingTable.from_symbols(ACGTN)
    b = (pkg.FmIndexBuilder(n, 5, table, position, block)
         .set_lookup_table_config(pkg.build_config.LookupTableConfig.KmerSize(3))
         .set_suffix_array_config(pkg.build_config.SuffixArrayConfig.Compressed(2)))
    size = b.blob_size()
    d_blob = torch.empty(size, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    b.build_device(d_text.data_ptr(), d_blob.data_ptr(), size)
    progress(f"n={n:,}: blob {size:,} B built on the GPU")
    starts = torch.randint(0, n - m + 1, (npat,), device="cuda:0", generator=gen)
    starts[-1] = n - m  # the text's last m symbols
    starts[-2] = 0      # and its first
    pats = d_text[(starts[:, None] + torch.arange(m, device="cuda:0")[None, :]).reshape(-1)].cpu().numpy()
    del d_text
    blob = O.aligned_zeros(size, 16)
    blob[:] = d_blob.cpu().numpy()
    del d_blob
    torch.cuda.empty_cache()
    offsets = np.arange(npat + 1, dtype=np.uint64) * m
    extra = [b"N" * m, b"ACGTN" * 4]
    ex_d, ex_o = pkg.pack_patterns(extra)
    pats = np.concatenate([pats, ex_d])
    offsets = np.concatenate([offsets, ex_o[1:] + offsets[-1]])
    orc = O.OracleIndex(blob, O.layout(*layout, 0))
    ooff, olocs = orc.locate_batch(pats, offsets, threads=oracle_threads())
    ix = pkg.FmIndex.load(blob, position, block, table)
    assert ix.info()["text_len"] == n
    goff, glocs = ix.locate_batch((pats, offsets))
    assert np.array_equal(goff, ooff) and np.array_equal(glocs, olocs)
    ix.close()
    st = starts.cpu().numpy()
    for i in range(npat):
        assert int(st[i]) in set(int(x) for x in olocs[ooff[i]:ooff[i + 1]])
    progress(f"{npat} patterns bit-exact, every start found")


def test_builder_text_beyond_u32(pkg, O):
    """n + 1 >= 2^32 (4.4 Gbp, u64 / Block3<u128>): the builder takes its
    64-bit suffix-array path; the blob validates, and 2,000 patterns cut from
    the text (+ wildcard ones) are answered bit-exactly like the oracle on the
    same blob, each finding its own start."""
    _big_text_case(pkg, O, 4_400_000_000, pkg.u64, pkg.blocks.Block3(pkg.Vector.U128), (8, 3, 128))


@pytest.mark.parametrize("n", [(1 << 32) - 3, (1 << 32) - 2])
def test_builder_u32_limit(pkg, O, n):
    """Both sides of the builder's switch to 64-bit suffix indices (n + 1 =
    2^32 - 2: the 32-bit path at its last size; n + 1 = 2^32 - 1: the 64-bit
    path), with u32 positions as close to 2^32 as they go (C[sigma] = n):
    2,000 patterns answered like the oracle, each finding its own start."""
    _big_text_case(pkg, O, n, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64), (4, 3, 64), seed=13)


@pytest.mark.parametrize("n_run", [1 << 20, 200_000_000, 2_000_000_000])
def test_builder_single_symbol_run(pkg, n_run):
    """The builder's worst case: a run of one symbol leaves every suffix of the
    run unresolved for ~log2(n) prefix-doubling rounds.  Text = A^n_run C G:
    the answers are known in closed form — count(A^k) = n_run - k + 1,
    locate(A^k C) = [n_run - k], count(C G) = 1 — so the check needs no oracle
    (which would need minutes for 200 M equal suffixes)."""
    import time
    import torch
    dev = torch.device("cuda:0")
    n = n_run + 2
    d_text = torch.full((n,), ord("A"), dtype=torch.uint8, device=dev)
    d_text[n_run] = ord("C")
    d_text[n_run + 1] = ord("G")
    table = pkg.text_encoders.EncodingTable.from_symbols(ACGTN)
    block = pkg.blocks.Block3(pkg.Vector.U64)
    b = (pkg.FmIndexBuilder(n, table.symbol_count(), table, pkg.u32, block)
         .set_lookup_table_config(pkg.build_config.LookupTableConfig.KmerSize(3))
         .set_suffix_array_config(pkg.build_config.SuffixArrayConfig.Compressed(2)))
    size = b.blob_size()
    d_blob = torch.empty(size, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    b.build_device(d_text.data_ptr(), d_blob.data_ptr(), size)
    torch.cuda.synchronize()
    progress(f"A^{n_run:,}CG: blob built in {time.perf_counter() - t0:.2f} s")
    blob = d_blob.cpu().numpy()
    del d_text, d_blob
    torch.cuda.empty_cache()
    for options in (pkg._native.FMX_OPT_DEFAULT, pkg._native.FMX_OCC_BLOB):
        ix = pkg.FmIndex.load(blob, pkg.u32, block, table, options=options)
        ks = [1, 2, 3, 4, 7, 20, 64, 1000]
        cnt = ix.count_batch([b"A" * k for k in ks])
        assert [int(x) for x in cnt] == [n_run - k + 1 for k in ks]
        pats = [b"A" * k + b"C" for k in (1, 5, 33, 500)] + [b"CG", b"G", b"AACG", b"T", b"GA"]
        off, locs = ix.locate_batch(pats)
        want = [[n_run - k] for k in (1, 5, 33, 500)] + [[n_run], [n_run + 1], [n_run - 2], [], []]
        got = [sorted(int(x) for x in locs[int(off[i]):int(off[i + 1])]) for i in range(len(pats))]
        assert got == want, (options, got, want)
        ix.close()
