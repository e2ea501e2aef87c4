"""Bench CLI (sview-fmindex_amd/bench_cli.py, the reference's bench/src/main.rs
subcommands) and the streamed blob-file ingest (fmx_load_file).

CPU tests: file formats (text.txt, pattern.txt, *-results.txt) and the host
side of fmx_load_file (open / header validation happen before any HIP call).
GPU tests: the whole generate -> build -> locate flow against the oracle, and
fmx_load_file == fmx_load on the same blob."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sview-fmindex_amd"))
import bench_cli as cli  # noqa: E402


def test_generate_text_and_patterns(tmp_path):
    d = str(tmp_path)
    cli.generate_text(d, 5000, 3, True)
    text = open(os.path.join(d, "text.txt"), "rb").read()
    assert len(text) == 5000 and set(text) <= set(b"ACGT")
    # cold 30 % of 10 -> 3 cold, 7 warm repeats of them (generate.rs:94-118)
    cli.generate_pattern(d, 20, 10, 0.3, 3, True)
    raw = open(os.path.join(d, "pattern.txt"), "rb").read()
    assert not raw.endswith(b"\n")
    pats = raw.split(b"\n")
    assert len(pats) == 10 and all(len(p) == 20 and p in text for p in pats)
    assert pats[3:] == [pats[i % 3] for i in range(7)]
    # no overwrite unless asked
    cli.generate_pattern(d, 5, 4, 1.0, 9, False)
    assert open(os.path.join(d, "pattern.txt"), "rb").read() == raw


def test_read_patterns_line_rules(tmp_path):
    p = tmp_path / "pattern.txt"
    p.write_bytes(b"ACG\r\nTT\n\nGA\n")
    assert cli.read_patterns(str(p)) == [b"ACG", b"TT", b"", b"GA"]
    p.write_bytes(b"ACG")
    assert cli.read_patterns(str(p)) == [b"ACG"]


def test_format_results():
    off = np.array([0, 2, 2, 3], np.uint64)
    locs = np.array([7, 1, 4000000000], np.uint32)
    assert cli.format_results(off, locs) == b"7,1\n\n4000000000\n"
    assert cli.format_results(np.array([0], np.uint64), np.array([], np.uint32)) == b""


def test_load_file_host_errors(pkg, O, tmp_path):
    """fmx_load_file opens and validates the header before touching the device."""
    block = pkg.blocks.Block2(pkg.Vector.U64)
    with pytest.raises(pkg.FmxError):
        pkg.FmIndex.load_file(str(tmp_path / "missing.blob"), pkg.u32, block)
    L = O.layout(4, 2, 64, 0)
    blob = O.build(b"ACGT" * 50, 4, L, 2, 2, bytes([3] * 256))
    bad = blob.copy()
    bad[0] ^= 0xFF
    (tmp_path / "bad.blob").write_bytes(bad.tobytes())
    with pytest.raises(pkg.LoadError.InvalidFormat):
        pkg.FmIndex.load_file(str(tmp_path / "bad.blob"), pkg.u32, block)
    (tmp_path / "long.blob").write_bytes(blob.tobytes() + b"\0" * 8)
    with pytest.raises(pkg.LoadError.MismatchedBlobSize) as e:
        pkg.FmIndex.load_file(str(tmp_path / "long.blob"), pkg.u32, block)
    assert e.value.expected == blob.size and e.value.actual == blob.size + 8


def _oracle_results(O, blob, block_planes, patterns):
    L = O.layout(4, block_planes, 64, 0)
    orc = O.OracleIndex(blob, L)
    offs = np.zeros(len(patterns) + 1, np.uint64)
    offs[1:] = np.cumsum([len(p) for p in patterns])
    data = np.frombuffer(b"".join(patterns), np.uint8) if patterns else np.zeros(0, np.uint8)
    ooff, olocs = orc.locate_batch(data, offs)
    return cli.format_results(ooff, olocs)


@pytest.mark.gpu
@pytest.mark.parametrize("wildcard_t", [False, True])
def test_cli_end_to_end(pkg, O, tmp_path, wildcard_t):
    d = str(tmp_path)
    cli.generate_text(d, 30000, 5, True)
    cli.generate_pattern(d, 20, 300, 0.5, 5, True)
    # a few extra lines: short, absent, wildcard bytes
    with open(os.path.join(d, "pattern.txt"), "ab") as f:
        f.write(b"\nA\nNNNNNNNNNNNN\nacgtACGT\nTTTTTTTTTTTTTTTTTTTTTTTTTT")
    paths = cli.build(d, "all", 2, 3, wildcard_t)
    blobs = [np.fromfile(p, np.uint8) for p in paths]
    assert np.array_equal(blobs[0], blobs[1])
    text = open(os.path.join(d, "text.txt"), "rb").read()
    table = cli.SYMBOLS_ACGT if wildcard_t else cli.SYMBOLS_ACGTN
    planes = 2 if wildcard_t else 3
    tbl = bytearray([len(table) - 1] * 256)
    for i, s in enumerate(table):
        for x in s:
            tbl[x] = i
    ref_blob = O.build(text, len(table), O.layout(4, planes, 64, 0), 3, 2, bytes(tbl))
    assert np.array_equal(blobs[0], ref_blob), "GPU-built blob differs from the oracle's"
    results = cli.locate(d, "all", wildcard_t, batch=128)
    want = _oracle_results(O, ref_blob, planes, cli.read_patterns(os.path.join(d, "pattern.txt")))
    for r in results:
        assert open(r, "rb").read() == want


@pytest.mark.gpu
def test_load_file_matches_load(pkg, O, tmp_path):
    rng = np.random.default_rng(11)
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=50000).astype(np.uint8)
    table = pkg.text_encoders.EncodingTable.from_symbols([b"Aa", b"Cc", b"Gg", b"Tt", b"Nn"])
    block = pkg.blocks.Block3(pkg.Vector.U64)
    b = (pkg.FmIndexBuilder(text.size, 5, table, pkg.u32, block)
         .set_lookup_table_config(pkg.build_config.LookupTableConfig.KmerSize(3))
         .set_suffix_array_config(pkg.build_config.SuffixArrayConfig.Compressed(2)))
    blob = pkg.aligned_buffer(b.blob_size())
    b.build(text, blob)
    path = str(tmp_path / "x.blob")
    blob.tofile(path)
    starts = rng.integers(0, text.size - 20, size=2000)
    pats = [text[s:s + int(rng.integers(1, 21))].tobytes() for s in starts]
    a = pkg.FmIndex.load(blob, pkg.u32, block, table)
    want = a.locate_batch(pats)
    a.close()
    for chunk in (0, 4096, 12345):  # default, and chunks that split the sections
        f = pkg.FmIndex.load_file(path, pkg.u32, block, pkg.text_encoders.EncodingTable, chunk_bytes=chunk)
        assert f.blob() is None
        got = f.locate_batch(pats)
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
        assert f.info()["blob_len"] == blob.size
        f.close()


def _direct_dir(tmp_path):
    """A directory whose file system accepts O_DIRECT reads (tmpfs may not)."""
    for d in (str(tmp_path), os.environ.get("GRAFT_REPO_ROOT", ""), ROOT, "/var/tmp"):
        if not d or not os.path.isdir(d) or not os.access(d, os.W_OK):
            continue
        probe = os.path.join(d, ".fmx_odirect_probe")
        try:
            with open(probe, "wb") as f:
                f.write(b"\0" * 8192)
            fd = os.open(probe, os.O_RDONLY | os.O_DIRECT)
            os.close(fd)
            return d
        except OSError:
            continue
        finally:
            if os.path.exists(probe):
                os.remove(probe)
    return None


@pytest.mark.gpu
def test_load_file_direct(pkg, O, tmp_path):
    """fmx_load_file with FMX_LOAD_DIRECT: the body read with O_DIRECT (page
    cache bypassed, 4 KiB-rounded requests, the file's length not a multiple
    of 4 KiB); chunk sizes that split the sections.  Results equal fmx_load's."""
    d = _direct_dir(tmp_path)
    if d is None:
        pytest.skip("no writable file system here accepts O_DIRECT")
    rng = np.random.default_rng(13)
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=3_000_001).astype(np.uint8)
    table = pkg.text_encoders.EncodingTable.from_symbols([b"Aa", b"Cc", b"Gg", b"Tt", b"Nn"])
    block = pkg.blocks.Block3(pkg.Vector.U64)
    b = (pkg.FmIndexBuilder(text.size, 5, table, pkg.u32, block)
         .set_lookup_table_config(pkg.build_config.LookupTableConfig.KmerSize(3))
         .set_suffix_array_config(pkg.build_config.SuffixArrayConfig.Compressed(2)))
    blob = pkg.aligned_buffer(b.blob_size())
    b.build(text, blob)
    assert blob.size % 4096 != 0
    path = os.path.join(d, f"direct_{os.getpid()}.blob")
    try:
        blob.tofile(path)
        pats = [text[s:s + int(rng.integers(6, 25))].tobytes() for s in rng.integers(0, text.size - 24, 5000)]
        a = pkg.FmIndex.load(blob, pkg.u32, block, table)
        want = a.locate_batch(pats)
        a.close()
        for chunk in (0, 1 << 20, (3 << 20) + 4096):
            f = pkg.FmIndex.load_file(path, pkg.u32, block, pkg.text_encoders.EncodingTable, chunk_bytes=chunk,
                                      direct=True)
            got = f.locate_batch(pats)
            assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]), f"chunk {chunk}"
            f.close()
    finally:
        if os.path.exists(path):
            os.remove(path)


@pytest.mark.gpu
def test_load_file_threaded_ring(pkg, O, tmp_path):
    """A blob of ~80 MB: the default 16 MiB chunks are read by 4 threads
    each and the 4-buffer ring wraps several times; a 40 MiB chunk splits
    into 8 slices with a short last one.  Results equal fmx_load's."""
    n = 30_000_000
    rng = np.random.default_rng(12)
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=n).astype(np.uint8)
    table = pkg.text_encoders.EncodingTable.from_symbols([b"Aa", b"Cc", b"Gg", b"Tt", b"Nn"])
    block = pkg.blocks.Block3(pkg.Vector.U64)
    b = (pkg.FmIndexBuilder(n, 5, table, pkg.u32, block)
         .set_lookup_table_config(pkg.build_config.LookupTableConfig.KmerSize(3))
         .set_suffix_array_config(pkg.build_config.SuffixArrayConfig.Compressed(2)))
    blob = pkg.aligned_buffer(b.blob_size())
    b.build(text, blob)
    path = str(tmp_path / "big.blob")
    blob.tofile(path)
    starts = rng.integers(0, n - 24, size=20000)
    pats = [text[s:s + int(rng.integers(8, 25))].tobytes() for s in starts]
    a = pkg.FmIndex.load(blob, pkg.u32, block, table)
    want = a.locate_batch(pats)
    a.close()
    for chunk in (0, 40 << 20, (5 << 20) + 4096):
        f = pkg.FmIndex.load_file(path, pkg.u32, block, pkg.text_encoders.EncodingTable, chunk_bytes=chunk)
        got = f.locate_batch(pats)
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]), f"chunk {chunk}"
        f.close()


C_HOST = os.path.join(ROOT, "sview-fmindex_amd", "lib", "fmx_locate")


def test_c_host_links_and_reports_abi(pkg):
    """examples/fmx_locate.c (built by build()) links against libfmx.so and
    agrees on the ABI version — no GPU call."""
    import subprocess
    if not os.path.exists(C_HOST):
        import __graft_entry__ as g
        g.build_c_host()
    p = subprocess.run([C_HOST, "--abi"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0 and p.stdout.strip() == "fmx ABI 8"


@pytest.mark.gpu
@pytest.mark.parametrize("block2", [False, True])
def test_c_host_locate_matches_oracle(pkg, O, tmp_path, block2):
    """The C host locates a pattern file against a blob file and writes the
    reference bench's results format; the file equals the oracle's answer."""
    import subprocess
    d = str(tmp_path)
    cli.generate_text(d, 200_000, 3, True)
    cli.generate_pattern(d, 20, 3000, 1.0, 3, True)
    with open(os.path.join(d, "pattern.txt"), "ab") as f:
        f.write(b"\nA\nNNNN\nacgtACGT\r\nTTTTTTTTTTTTTTTTTTTTTTTTTTTTTT\n")
    blob_path = cli.build(d, "sview-memory", 2, 3, block2)[0]
    out = os.path.join(d, "c-results.txt")
    args = [C_HOST, blob_path, os.path.join(d, "pattern.txt"), out] + (["--block2"] if block2 else [])
    p = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    assert "Blob loading time:" in p.stdout and "Locate processing time:" in p.stdout
    planes = 2 if block2 else 3
    want = _oracle_results(O, np.fromfile(blob_path, np.uint8), planes,
                           cli.read_patterns(os.path.join(d, "pattern.txt")))
    assert open(out, "rb").read() == want
