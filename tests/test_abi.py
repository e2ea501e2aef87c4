"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every
entry point include/fmx.h declares, and its host-only logic (blob sizing,
status strings, argument checks) agrees with the oracle.  No kernel runs here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from _util import ALL_LAYOUTS

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "fmx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fmx_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol(pkg):
    lib = pkg._native.lib()
    declared = header_functions()
    assert len(declared) >= 19
    for name in declared:
        assert hasattr(lib, name), f"libfmx.so does not export {name}"
    assert set(declared) == set(pkg._native.SIGNATURES), "ctypes signatures out of sync with fmx.h"
    assert lib.fmx_abi_version() == 8


def test_status_strings(pkg):
    for code in range(0, 11):
        assert pkg._native.status_str(code)


@pytest.mark.parametrize("pb,planes,vb", ALL_LAYOUTS)
def test_blob_size_matches_oracle(pkg, O, pb, planes, vb):
    rng = np.random.default_rng(pb * 100 + planes * 10 + vb)
    for _ in range(5):
        n = int(rng.integers(0, 5000))
        sigma = int(rng.integers(1, (1 << planes) + 1))
        k = int(rng.integers(1, 4))
        sr = int(rng.integers(1, 6))
        for enc in (0, 1):
            L = pkg._native.fmx_layout(pb, planes, vb, enc)
            out = C.c_uint64()
            st = pkg._native.lib().fmx_build_blob_size(n, sigma, L, k, sr, C.byref(out))
            assert st == 0
            assert out.value == O.blob_size(n, sigma, O.layout(pb, planes, vb, enc), k, sr)


def test_python_builder_sizes(pkg, O):
    """FmIndexBuilder.blob_size (builder/mod.rs:165-181) through the ABI; C2's
    blob is 2,687,501,296 B."""
    table = pkg.text_encoders.EncodingTable.from_symbols([b"Aa", b"Cc", b"Gg", b"Tt", b"Nn"])
    b = (pkg.FmIndexBuilder(10 ** 9, 5, table, pkg.u32, pkg.blocks.Block3(pkg.Vector.U64))
         .set_lookup_table_config(pkg.build_config.LookupTableConfig.KmerSize(3))
         .set_suffix_array_config(pkg.build_config.SuffixArrayConfig.Compressed(2)))
    assert b.blob_size() == 2_687_501_296
    t4 = pkg.text_encoders.EncodingTable.from_symbols([b"Aa", b"Cc", b"Gg", b"Tt"])
    b1 = (pkg.FmIndexBuilder(10 ** 6, 4, t4, pkg.u32, pkg.blocks.Block2(pkg.Vector.U64))
          .set_lookup_table_config(pkg.build_config.LookupTableConfig.KmerSize(3))
          .set_suffix_array_config(pkg.build_config.SuffixArrayConfig.Compressed(2)))
    assert b1.blob_size() == 2_500_920
    with pytest.raises(pkg.BuildError):
        pkg.FmIndexBuilder(10, 5, table, pkg.u32, pkg.blocks.Block2(pkg.Vector.U64))  # 5 > 4 symbols


def test_load_rejects_bad_blobs_before_touching_the_device(pkg, O):
    """Validation happens on the host, before any HIP call, so these run on CPU."""
    table = bytes([3] * 256)
    L = O.layout(4, 2, 64, 0)
    blob = O.build(b"ACGT" * 10, 4, L, 2, 2, table)
    bad = blob.copy()
    bad[1] = ord("X")
    with pytest.raises(pkg.LoadError):
        pkg.FmIndex.load(bad, pkg.u32, pkg.blocks.Block2(pkg.Vector.U64))
    longer = pkg.aligned_buffer(blob.size + 8)
    longer[:blob.size] = blob
    with pytest.raises(pkg.LoadError.MismatchedBlobSize) as e:
        pkg.FmIndex.load(longer, pkg.u32, pkg.blocks.Block2(pkg.Vector.U64))
    assert e.value.actual == blob.size + 8 and e.value.expected == blob.size
    # P/B/E are not in the blob: a wrong layout tag is caught by the consistency checks
    with pytest.raises((pkg.LoadError, pkg.FmxError)):
        pkg.FmIndex.load(blob, pkg.u64, pkg.blocks.Block2(pkg.Vector.U64))
    # the multi-device handle validates the same way, before any device
    with pytest.raises(pkg.LoadError.InvalidFormat):
        pkg.MultiDeviceIndex(bad, [0, 1], pkg.u32, pkg.blocks.Block2(pkg.Vector.U64))
    with pytest.raises(pkg.LoadError.MismatchedBlobSize):
        pkg.MultiDeviceIndex(longer, [0], pkg.u32, pkg.blocks.Block2(pkg.Vector.U64))
    with pytest.raises(pkg.FmxError):
        pkg.MultiDeviceIndex(blob, [], pkg.u32, pkg.blocks.Block2(pkg.Vector.U64))


def test_pack_patterns(pkg):
    data, off = pkg.pack_patterns([b"AC", b"", b"GGT"])
    assert data.tobytes() == b"ACGGT"
    assert off.tolist() == [0, 2, 2, 5]


def test_workspace_bytes_host_sizing(pkg):
    """fmx_workspace_bytes (ABI 8): the locate workspace a batch needs, from
    the library's own arithmetic with no index loaded — what distributed.py's
    per-rank HBM accounting uses.  Grows with n (a per-pattern record, a
    16-B grouped record and two counters per tile), is wider for 8-B
    positions, and rejects other position widths."""
    ws = pkg.distributed.workspace_bytes
    base4, base8 = ws(0, 4), ws(0, 8)
    assert base4 > 0 and base8 >= base4
    prev = base4
    for n in (1, 255, 256, 257, 100_000, 102_400_000):
        cur = ws(n, 4)
        assert cur > prev and cur - base4 >= 16 * n
        assert ws(n, 8) > cur
        prev = cur
    # linear in the tile count: 256 more patterns add one tile's worth exactly
    assert ws(512, 4) - ws(256, 4) == ws(768, 4) - ws(512, 4)
    for bad in (0, 2, 16):
        with pytest.raises(ValueError):
            ws(10, bad)
    out = C.c_uint64()
    assert pkg._native.lib().fmx_workspace_bytes(10, 4, None) != 0
    assert pkg._native.lib().fmx_workspace_bytes(10, 4, C.byref(out)) == 0 and out.value == ws(10, 4)
