"""CPU tests of the kernels' arithmetic: tests/emu/libfmx_emu.so runs the
engine's __host__ __device__ code (sview-fmindex_amd/csrc/fmx_device.hpp —
rank/popcount for every Block x Vector, seed, LF loop, deep k-mer table, full
SA, single-row text verification, walk) on the CPU, and every count and
location (SA-row order) is compared with the oracle.  The GPU tests
(test_gpu.py) run the same code on the device."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from _util import ALL_LAYOUTS, rand_chr_list, rand_pattern, rand_text, table_from_symbols

HERE = os.path.dirname(os.path.abspath(__file__))
EMU = os.path.join(HERE, "emu", "libfmx_emu.so")
# fmx_load option bits; bits 8.. set the row-scan limit (FMX_SCAN_ROWS)
# (bit 7: the long-pattern kernels' vectorised tail compare instead of the short one;
#  bit 6: plain interleaved records where the loader would pick paired-chunk or symbol-mask ones;
#  bit 30: multi-line symbol masks with a walk line where they fit, fmx_device.hpp kRecWalk)
OPTIONS = (0, 1, 1 | 64, 31 | 64, 1 | 2, 1 | 4, 1 | 2 | 4 | 8, 4 | 8, 2 | 8, 31, 16, 1 | 16 | (1 << 8), 2 | 16 | (64 << 8),
           1 | 2 | 16 | (5 << 8), 2 | 8 | 32, 63, 1 | 2 | 16 | 32 | (3 << 8),
           4 | 8 | 128, 31 | 128, 63 | 128, 1 | 2 | 16 | 32 | 128 | (3 << 8),
           1 | (1 << 30))


@pytest.fixture(scope="module")
def emu():
    subprocess.check_call(["make", "-s", "-j", str(min(8, os.cpu_count() or 1)), "-C", os.path.join(HERE, "emu")])
    lib = C.CDLL(EMU)
    u32, u64, p = C.c_uint32, C.c_uint64, C.c_void_p
    lib.emu_locate.argtypes = [p, u64, u32, u32, u32, u32, u32, p, p, u64, u32, p, p, u64, C.POINTER(u64)]
    lib.emu_locate.restype = C.c_int
    return lib


def emu_locate(lib, blob, layout, options, pats, reverse=False):
    pb, planes, vb, enc = layout
    data = np.frombuffer(b"".join(pats), np.uint8) if pats else np.zeros(1, np.uint8)
    offs = np.zeros(len(pats) + 1, np.uint64)
    np.cumsum([len(x) for x in pats], out=offs[1:])
    counts = np.zeros(max(len(pats), 1), np.uint64)
    cap = 1 << 20
    locs = np.zeros(cap, np.uint64)
    need = C.c_uint64()
    st = lib.emu_locate(blob.ctypes.data, blob.size, pb, planes, vb, enc, options, data.ctypes.data,
                        offs.ctypes.data, len(pats), 1 if reverse else 0, counts.ctypes.data, locs.ctypes.data,
                        cap, C.byref(need))
    return st, counts[:len(pats)], locs[:need.value]


def check(lib, O, blob, layout, pats, options):
    L = O.layout(*layout)
    orc = O.OracleIndex(blob, L)
    data = np.frombuffer(b"".join(pats), np.uint8)
    offs = np.zeros(len(pats) + 1, np.uint64)
    np.cumsum([len(x) for x in pats], out=offs[1:])
    ooff, olocs = orc.locate_batch(data, offs)
    st, cnt, locs = emu_locate(lib, blob, layout, options, pats)
    assert st == 0
    assert np.array_equal(cnt, np.diff(ooff)), f"counts differ, options={options}"
    assert np.array_equal(locs, olocs.astype(np.uint64)), f"locations differ, options={options}"
    st, rcnt, rlocs = emu_locate(lib, blob, layout, options, [x[::-1] for x in pats], reverse=True)
    assert st == 0 and np.array_equal(rcnt, cnt) and np.array_equal(rlocs, locs)


@pytest.mark.parametrize("pb,planes,vb", ALL_LAYOUTS)
def test_device_code_every_layout(emu, O, pb, planes, vb):
    rng = np.random.default_rng(pb * 1000 + planes * 100 + vb)
    for sigma in sorted({2, 3, (1 << planes) // 2 + 1, 1 << planes}):
        chars = rand_chr_list(rng, sigma)
        table = table_from_symbols([bytes([c]) for c in chars])
        text = rand_text(rng, chars, 300, 2000)
        k, sr = int(rng.integers(1, 5)), int(rng.integers(1, 5))
        if (sigma + 1) ** k > 1 << 20:
            k = 2
        blob = O.build(text, sigma, O.layout(pb, planes, vb), k, sr, table)
        pats = [rand_pattern(rng, text, 1, 24) for _ in range(200)]
        pats += [bytes(rng.choice(np.frombuffer(chars, np.uint8), size=int(rng.integers(1, 12))))
                 for _ in range(30)]
        pats += [b"\x00", b"\x7f\x7f", chars[:1] * 2]
        for options in OPTIONS:
            check(emu, O, blob, (pb, planes, vb, 0), pats, options)


def test_device_code_repetitive(emu, O):
    table = table_from_symbols([b"A", b"C", b"G", b"T"])
    text = b"AC" * 3000 + b"GT" * 40 + b"A" * 2000
    pats = [b"A", b"AC", b"CA", b"ACA", b"G", b"GT", b"TA", b"AAAA", b"A" * 30, b"CA" * 12 + b"G"]
    for layout in [(4, 2, 64, 0), (8, 3, 128, 0), (8, 2, 64, 0)]:
        for sr in (1, 2, 3, 5):
            blob = O.build(text, 4, O.layout(*layout[:3]), 3, sr, table)
            for options in OPTIONS:
                check(emu, O, blob, layout, pats, options)


def test_device_code_text_start_and_symbols(emu, O):
    """Tails that run into the text start, and PassThrough bytes >= sigma reached
    (or not) by the search: per pattern, the same status as the oracle."""
    rng = np.random.default_rng(77)
    text = bytes([3, 2, 1, 0]) + bytes(rng.integers(0, 3, size=3000).astype(np.uint8))  # [3,2,1,0] unique start
    for layout in [(4, 2, 64, 1), (8, 3, 32, 1)]:
        blob = O.build(text, 4, O.layout(*layout[:3]), 2, 3, None)
        orc = O.OracleIndex(blob, O.layout(*layout))
        pats = [bytes([0, 3, 2, 1, 0]), bytes([1, 1, 3, 2, 1, 0, 2]), bytes([9, 3, 2, 1, 0]),
                bytes([3, 2, 1, 0]), bytes([9, 9, 2, 2, 1]), bytes([2, 9, 0, 1, 2, 0, 1])]
        pats += [bytes([9]) + text[s:s + 12] for s in rng.integers(4, 2900, size=40)]
        pats += [text[s:s + 12] + bytes([7]) for s in rng.integers(4, 2900, size=10)]
        for p in pats:
            for options in OPTIONS:
                try:
                    want = ("ok", sorted(orc.locate(p)), orc.locate(p))
                except O.OracleError as e:
                    want = ("err", e.code)
                st, cnt, locs = emu_locate(emu, blob, layout, options, [p])
                got = ("ok", sorted(int(x) for x in locs), [int(x) for x in locs]) if st == 0 else ("err", st)
                assert got == want, (p, options, got, want)


def test_device_code_absent_symbols(emu, O):
    """Symbols of the alphabet that never occur in the text (the deep table is
    indexed by the occurring ones): patterns holding them anywhere — inside the
    deep-table window, left of it, in the blob's k-mer window — and, for
    PassThrough, bytes >= sigma next to them.  Same status and locations as the
    oracle."""
    rng = np.random.default_rng(123)
    # EncodingTable ACGTN, the text has no N (the C2 situation)
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    text = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), size=4000))
    for layout in [(4, 3, 64, 0), (8, 3, 128, 0), (4, 3, 32, 0)]:
        blob = O.build(text, 5, O.layout(*layout[:3]), 3, 2, table)
        pats = [text[s:s + int(rng.integers(1, 30))] for s in rng.integers(0, 3950, size=300)]
        for p in list(pats[:120]):
            j = int(rng.integers(0, len(p)))
            pats.append(p[:j] + b"N" + p[j + 1:])
        pats += [b"N", b"NN", b"N" * 20, b"ACGTN" * 4]
        for options in OPTIONS:
            check(emu, O, blob, layout, pats, options)
    # PassThrough sigma 5 over a text of 0..3: symbol 4 is absent, 9 is >= sigma
    text = bytes(rng.integers(0, 4, size=4000).astype(np.uint8))
    for layout in [(4, 3, 64, 1), (8, 3, 64, 1)]:
        blob = O.build(text, 5, O.layout(*layout[:3]), 2, 2, None)
        orc = O.OracleIndex(blob, O.layout(*layout))
        pats = [text[s:s + 24] for s in rng.integers(0, 3950, size=60)]
        muts = []
        for p in pats:
            a, b = sorted(int(x) for x in rng.integers(0, len(p), size=2))
            muts.append(p[:a] + bytes([4]) + p[a + 1:b] + bytes([9]) + p[b + 1:] if a < b else p)
            muts.append(p[:a] + bytes([9]) + p[a + 1:b] + bytes([4]) + p[b + 1:] if a < b else p)
        for p in pats + muts:
            for options in OPTIONS:
                try:
                    want = ("ok", orc.locate(p))
                except O.OracleError as e:
                    want = ("err", e.code)
                st, cnt, locs = emu_locate(emu, blob, layout, options, [p])
                got = ("ok", [int(x) for x in locs]) if st == 0 else ("err", st)
                assert got == want, (p, options, got, want)


def test_device_code_long_tails(emu, O):
    """Long patterns (C5-like, up to 200 symbols): single-row tails compared
    against the text 64 positions per round, with one substituted symbol at
    every depth of the tail, and tails that run past the text start."""
    rng = np.random.default_rng(5150)
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    text = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), size=20000))
    alt = {ord("A"): b"C", ord("C"): b"G", ord("G"): b"T", ord("T"): b"A"}
    pats = []
    for s in rng.integers(0, 19700, size=60):
        m = int(rng.integers(40, 201))
        p = text[s:s + m]
        pats.append(p)
        j = int(rng.integers(0, len(p)))
        pats.append(p[:j] + alt[p[j]] + p[j + 1:])
    for m in (63, 64, 65, 129, 150):  # the text start falls inside the tail
        pats.append(b"G" * (m - 50) + text[:50])
        pats.append(text[:m])
    for layout in [(4, 3, 64, 0), (8, 3, 128, 0)]:
        blob = O.build(text, 5, O.layout(*layout[:3]), 3, 2, table)
        for options in OPTIONS:
            check(emu, O, blob, layout, pats, options)
