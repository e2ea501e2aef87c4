#!/usr/bin/env python3
"""Bench CLI of the MI355X engine — the reference's `sview-fmindex-bench`
(bench/src/main.rs:8-99) with the same subcommands, arguments and files:

  generate-text     text.txt: uniform ACGT, no newline         (generate.rs:7-55)
  generate-pattern  pattern.txt: cold patterns cut at uniform starts, then
                    warm repeats of them, '\\n'-joined          (generate.rs:58-143)
  generate          both (cold ratio 1.0)                      (generate.rs:146-156)
  build             text.txt -> <algorithm>-block{2,3}.blob, built on the GPU
                    (bench/src/build/sview_memory.rs, sview_mmap.rs)
  locate            blob + pattern.txt -> <stem>-results.txt, one line per
                    pattern, its locations comma-joined in the order
                    FmIndex::locate returns them (locate/mod.rs:115-124)

Algorithms: "sview-memory" reads the whole blob file into host memory and
loads it (fmx_load); "sview-mmap" streams it file -> pinned chunks -> HBM
(fmx_load_file).  Both run the same kernels and read/write the reference's
file names, so a blob built by the reference bench is located here and vice
versa (the blob bytes are the reference's layout).  "all" runs both.

Patterns are located in batches (one fmx_locate_batch per --batch patterns)
instead of one `locate` call per line; the output is identical.

The synthetic text and patterns come from numpy's PCG64, not the reference's
StdRng (ChaCha12) stream, so the same seed gives different (equally uniform)
data; files written by the reference bench are read unchanged.

usage: python sview-fmindex_amd/bench_cli.py <subcommand> [--data-dir DIR] ...
"""
from __future__ import annotations

import argparse
import math
import os
import sys
import time

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SYMBOLS_ACGT = [b"Aa", b"Cc", b"Gg", b"Tt"]      # bench/src/build/mod.rs:29
SYMBOLS_ACGTN = [b"Aa", b"Cc", b"Gg", b"Tt", b"Nn"]  # bench/src/build/mod.rs:30
ALGORITHMS = ("sview-memory", "sview-mmap")


def _pkg():
    """The engine package with its library loaded (before any timer, like the
    reference bench's statically linked binary)."""
    if _ROOT not in sys.path:
        sys.path.insert(0, _ROOT)
    import __graft_entry__ as g
    pkg = g.load_package()
    pkg._native.lib()
    return pkg


# ------------------------------------------------------------------ generate

def generate_text(data_dir: str, text_length: int, seed: int, overwrite: bool) -> str:
    os.makedirs(data_dir, exist_ok=True)
    path = os.path.join(data_dir, "text.txt")
    if os.path.exists(path) and not overwrite:
        print(f"Text file already exists: {path}\nUse --overwrite to overwrite.")
        return path
    rng = np.random.Generator(np.random.PCG64(seed))
    nuc = np.frombuffer(b"ACGT", np.uint8)
    with open(path, "wb") as f:
        for c0 in range(0, text_length, 1 << 26):
            n = min(1 << 26, text_length - c0)
            f.write(nuc[rng.integers(0, 4, size=n, dtype=np.uint8)].tobytes())
    print(f"Text file created: {path}")
    return path


def generate_pattern(data_dir: str, pattern_length: int, pattern_count: int, cold_ratio: float, seed: int,
                     overwrite: bool) -> str:
    text_path = os.path.join(data_dir, "text.txt")
    if not os.path.exists(text_path):
        raise SystemExit(f"Text file not found: {text_path}. Run generate-text first.")
    path = os.path.join(data_dir, "pattern.txt")
    if os.path.exists(path) and not overwrite:
        print(f"Pattern file already exists: {path}\nUse --overwrite to overwrite.")
        return path
    text = np.memmap(text_path, dtype=np.uint8, mode="r")
    cold = min(int(math.ceil(cold_ratio * pattern_count)), pattern_count)
    warm = pattern_count - cold
    print(f"Cold patterns: {cold} (new)\nWarm patterns: {warm} (repeated)")
    rng = np.random.Generator(np.random.PCG64(seed))
    max_start = max(len(text) - pattern_length, 0)
    starts = rng.integers(0, max_start + 1, size=cold, dtype=np.int64)
    cold_p = [bytes(text[s:s + pattern_length]) for s in starts]
    warm_p = [cold_p[i % cold] for i in range(warm)] if cold else []
    with open(path, "wb") as f:
        f.write(b"\n".join(cold_p + warm_p))
    print(f"Pattern file created: {path}")
    return path


# --------------------------------------------------------------------- build

def _layout(pkg, treat_t_as_wildcard: bool):
    symbols = SYMBOLS_ACGT if treat_t_as_wildcard else SYMBOLS_ACGTN
    block = pkg.blocks.Block2(pkg.Vector.U64) if treat_t_as_wildcard else pkg.blocks.Block3(pkg.Vector.U64)
    return symbols, block, "block2" if treat_t_as_wildcard else "block3"


def build(data_dir: str, algorithm: str, sasr: int, klts: int, treat_t_as_wildcard: bool, device: int = 0):
    pkg = _pkg()
    text_path = os.path.join(data_dir, "text.txt")
    if not os.path.exists(text_path):
        raise SystemExit(f"Text file not found: {text_path}")
    text = np.fromfile(text_path, dtype=np.uint8)
    print(f"Loaded text: {text.size} bytes")
    symbols, block, tag = _layout(pkg, treat_t_as_wildcard)
    table = pkg.text_encoders.EncodingTable.from_symbols(symbols)
    sa_cfg = (pkg.build_config.SuffixArrayConfig.Uncompressed() if sasr == 1
              else pkg.build_config.SuffixArrayConfig.Compressed(sasr))
    lt_cfg = pkg.build_config.LookupTableConfig.None_() if klts == 1 else pkg.build_config.LookupTableConfig.KmerSize(klts)
    builder = (pkg.FmIndexBuilder(text.size, table.symbol_count(), table, pkg.u32, block)
               .set_suffix_array_config(sa_cfg).set_lookup_table_config(lt_cfg))
    algos = ALGORITHMS if algorithm == "all" else (algorithm,)
    blob = pkg.aligned_buffer(builder.blob_size())
    print(f"Blob size: {blob.size} bytes")
    t0 = time.perf_counter_ns()
    builder.build(text, blob, device=device)
    print(f"Build time: {time.perf_counter_ns() - t0} ns")
    paths = []
    for a in algos:
        path = os.path.join(data_dir, f"{a}-{tag}.blob")
        t0 = time.perf_counter_ns()
        blob.tofile(path)
        print(f"Save time: {time.perf_counter_ns() - t0} ns\nIndex saved to: {path}")
        paths.append(path)
    return paths


# -------------------------------------------------------------------- locate

def read_patterns(path: str):
    """pattern.txt lines (BufRead::lines: '\\n' separated, a trailing '\\r'
    dropped, no empty last line after a final '\\n')."""
    raw = open(path, "rb").read()
    lines = raw.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    return [ln[:-1] if ln.endswith(b"\r") else ln for ln in lines]


def read_file(pkg, path: str, threads: int = 8) -> np.ndarray:
    """The whole blob file into an aligned host buffer (the sview-memory
    loader, bench/src/locate/sview_memory.rs:17-40), read as `threads`
    slices in parallel (os.preadv releases the GIL)."""
    size = os.path.getsize(path)
    blob = pkg.aligned_buffer(size)
    mv = memoryview(blob)
    fd = os.open(path, os.O_RDONLY)
    try:
        step = max(4 << 20, -(-size // threads) + 4095 & ~4095)

        def part(o):
            end = min(size, o + step)
            while o < end:
                got = os.preadv(fd, [mv[o:end]], o)
                if got <= 0:
                    raise OSError(f"short read of {path} at {o}")
                o += got

        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(part, range(0, size, step)))
    finally:
        os.close(fd)
    return blob


def resident_fraction(path: str) -> float:
    """Share of the file's pages in the page cache (mincore over a read-only
    mapping, which itself reads nothing); -1 if it cannot be determined."""
    import ctypes
    import mmap
    size = os.path.getsize(path)
    if size == 0:
        return 0.0
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        libc.mincore.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        with open(path, "rb") as f:
            mm = mmap.mmap(f.fileno(), size, prot=mmap.PROT_READ)
        try:
            view = np.frombuffer(mm, np.uint8)
            vec = np.zeros((size + mmap.PAGESIZE - 1) // mmap.PAGESIZE, np.uint8)
            rc = libc.mincore(ctypes.c_void_p(view.ctypes.data), size, ctypes.c_void_p(vec.ctypes.data))
            del view
            return float((vec & 1).mean()) if rc == 0 else -1.0
        finally:
            mm.close()
    except (OSError, ValueError, AttributeError, BufferError):
        return -1.0


def drop_file_cache(path: str) -> None:
    """Evict the file's pages from the page cache without root: flush dirty
    pages (a freshly built blob is dirty), then POSIX_FADV_DONTNEED — for this
    file what the reference bench's `sync; echo 3 > /proc/sys/vm/drop_caches`
    does machine-wide (bench/run_benchmark.sh:53-56)."""
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
    finally:
        os.close(fd)


def format_results(loc_offsets: np.ndarray, locs: np.ndarray) -> bytes:
    """One line per pattern, locations comma-joined (write_locations_to_file,
    locate/mod.rs:115-124).  Vectorised: every location becomes its digits
    plus ',' (or '\n' after a pattern's last one), every pattern without
    locations one '\n', placed by index arithmetic and joined once."""
    off = loc_offsets.astype(np.int64)
    cnt = np.diff(off)
    n = cnt.size
    if n == 0:
        return b""
    start = np.zeros(n + 1, np.int64)
    start[1:] = np.cumsum(np.maximum(cnt, 1))  # a pattern's first piece
    pieces = np.empty(int(start[-1]), dtype=object)
    pat = np.repeat(np.arange(n), cnt)
    sep = np.full(locs.size, ",", dtype=object)
    sep[off[1:][cnt > 0] - 1] = "\n"
    pieces[start[pat] + (np.arange(locs.size) - off[pat])] = locs.astype(np.uint64).astype(str).astype(object) + sep
    pieces[start[:-1][cnt == 0]] = "\n"
    return "".join(pieces.tolist()).encode()


def locate(data_dir: str, algorithm: str, treat_t_as_wildcard: bool, drop_caches: bool = False,
           batch: int = 1 << 20, device: int = 0, options=None, direct: bool = False):
    """`drop_caches`: the blob and pattern files are evicted from the page
    cache before each load (drop_file_cache), so "Blob loading time" is a
    cold read from storage, as in the reference's README runs; `direct`: the
    sview-mmap loader reads the blob with O_DIRECT (FMX_LOAD_DIRECT)."""
    pkg = _pkg()
    pattern_path = os.path.join(data_dir, "pattern.txt")
    if not os.path.exists(pattern_path):
        raise SystemExit(f"Pattern file not found: {pattern_path}")
    _, block, tag = _layout(pkg, treat_t_as_wildcard)
    algos = ALGORITHMS if algorithm == "all" else (algorithm,)
    results = []
    for a in algos:
        stem = f"{a}-{tag}"
        blob_path = os.path.join(data_dir, f"{stem}.blob")
        if not os.path.exists(blob_path):
            if algorithm == "all":
                continue
            raise SystemExit(f"{tag} blob file not found: {blob_path}")
        print(f"Using blob file: {blob_path}")
        if drop_caches:
            td = time.perf_counter_ns()
            for f in (blob_path, pattern_path):
                drop_file_cache(f)
            print(f"Page cache dropped for the blob and pattern files in {time.perf_counter_ns() - td} ns (outside "
                  f"the timings below, as the reference's drop_caches): {resident_fraction(blob_path):.4f} of "
                  f"the blob resident")
        t0 = time.perf_counter_ns()
        if a == "sview-mmap":
            ix = pkg.FmIndex.load_file(blob_path, pkg.u32, block, pkg.text_encoders.EncodingTable, device=device,
                                       options=options, direct=direct)
        else:
            blob = read_file(pkg, blob_path)
            if os.environ.get("FMX_LOAD_TRACE"):
                print(f"[fmx load] file -> host memory     {(time.perf_counter_ns() - t0) / 1e6:9.3f} ms",
                      file=sys.stderr, flush=True)
            ix = pkg.FmIndex.load(blob, pkg.u32, block, pkg.text_encoders.EncodingTable, device=device,
                                  options=options)
        load_ns = time.perf_counter_ns() - t0
        t0 = time.perf_counter_ns()
        pats = read_patterns(pattern_path)
        result_path = os.path.join(data_dir, f"{stem}-results.txt")
        with open(result_path, "wb") as out:
            for b0 in range(0, len(pats), batch):
                off, locs = ix.locate_batch(pats[b0:b0 + batch])
                out.write(format_results(off, locs))
        locate_ns = time.perf_counter_ns() - t0
        ix.close()
        print(f"Blob loading time: {load_ns} ns\nLocate processing time: {locate_ns} ns")
        print(f"Results saved to: {result_path}")
        results.append(result_path)
    if not results:
        raise SystemExit("no blob file found")
    return results


def main(argv=None):
    # The CLI process uses no torch: libfmx binds the system HIP runtime
    # directly (importing torch only to share its runtime costs ~1.3 s).  Not
    # for a process that imports these functions and uses torch itself: two
    # HIP runtimes in one process do not share the device.
    if "torch" not in sys.modules:
        os.environ.setdefault("FMX_NO_TORCH_RUNTIME", "1")
    ap = argparse.ArgumentParser(prog="sview-fmindex-bench (MI355X)")
    sub = ap.add_subparsers(dest="command", required=True)
    g = sub.add_parser("generate")
    g.add_argument("-d", "--data-dir", default="test_data")
    g.add_argument("-t", "--text-length", type=int, default=100000)
    g.add_argument("-p", "--pattern-length", type=int, default=20)
    g.add_argument("-n", "--pattern-count", type=int, default=100)
    g.add_argument("-s", "--seed", type=int, default=0)
    gt = sub.add_parser("generate-text")
    gt.add_argument("-d", "--data-dir", default="test_data")
    gt.add_argument("-t", "--text-length", type=int, default=100000)
    gt.add_argument("-s", "--seed", type=int, default=0)
    gt.add_argument("--overwrite", action="store_true")
    gp = sub.add_parser("generate-pattern")
    gp.add_argument("-d", "--data-dir", default="test_data")
    gp.add_argument("-p", "--pattern-length", type=int, default=20)
    gp.add_argument("-n", "--pattern-count", type=int, default=100)
    gp.add_argument("-c", "--cold-ratio", type=float, default=1.0)
    gp.add_argument("-s", "--seed", type=int, default=0)
    gp.add_argument("--overwrite", action="store_true")
    b = sub.add_parser("build")
    b.add_argument("-d", "--data-dir", default="test_data")
    b.add_argument("-a", "--algorithm", default="sview-memory", choices=ALGORITHMS + ("all",))
    b.add_argument("-s", "--sasr", type=int, default=2)
    b.add_argument("-k", "--klts", type=int, default=3)
    b.add_argument("-t", "--treat-t-as-wildcard", action="store_true")
    b.add_argument("--device", type=int, default=0)
    lo = sub.add_parser("locate")
    lo.add_argument("-d", "--data-dir", default="test_data")
    lo.add_argument("-a", "--algorithm", default="all", choices=ALGORITHMS + ("all",))
    lo.add_argument("-t", "--treat-t-as-wildcard", action="store_true")
    lo.add_argument("--drop-caches", action="store_true",
                    help="evict the blob and pattern files from the page cache before each load (no root needed)")
    lo.add_argument("--direct", action="store_true", help="sview-mmap: read the blob with O_DIRECT")
    lo.add_argument("--batch", type=int, default=1 << 20, help="patterns per fmx_locate_batch call")
    lo.add_argument("--device", type=int, default=0)
    lo.add_argument("--options", type=int, default=None,
                    help="fmx_load options (default FMX_OPT_DEFAULT: the blob's own structures)")
    a = ap.parse_args(argv)
    t0 = time.perf_counter_ns()
    if a.command == "generate":
        generate_text(a.data_dir, a.text_length, a.seed, True)
        generate_pattern(a.data_dir, a.pattern_length, a.pattern_count, 1.0, a.seed, True)
    elif a.command == "generate-text":
        generate_text(a.data_dir, a.text_length, a.seed, a.overwrite)
    elif a.command == "generate-pattern":
        generate_pattern(a.data_dir, a.pattern_length, a.pattern_count, a.cold_ratio, a.seed, a.overwrite)
    elif a.command == "build":
        build(a.data_dir, a.algorithm, a.sasr, a.klts, a.treat_t_as_wildcard, a.device)
    elif a.command == "locate":
        locate(a.data_dir, a.algorithm, a.treat_t_as_wildcard, a.drop_caches, a.batch, a.device, a.options,
               a.direct)
    print(f"Total time: {time.perf_counter_ns() - t0} ns")
    # the reference's run_benchmark.sh reads max RSS from /usr/bin/time -v
    import resource
    print(f"Maximum resident set size (kbytes): {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss}")


if __name__ == "__main__":
    main()
