"""fmx_multi_*: one handle over several replicas (here all on cuda:0, which
this one-GPU box allows: replicas on one GPU run concurrently; the shard and
concatenation logic is the same for distinct GPUs).  Every answer equals the
single-device index's (which the other GPU tests pin to the oracle)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _case(pkg, n=400_000, seed=5):
    rng = np.random.default_rng(seed)
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=n).astype(np.uint8)
    table = pkg.text_encoders.EncodingTable.from_symbols([b"Aa", b"Cc", b"Gg", b"Tt", b"Nn"])
    block = pkg.blocks.Block3(pkg.Vector.U64)
    b = (pkg.FmIndexBuilder(text.size, 5, table, pkg.u32, block)
         .set_lookup_table_config(pkg.build_config.LookupTableConfig.KmerSize(3))
         .set_suffix_array_config(pkg.build_config.SuffixArrayConfig.Compressed(2)))
    blob = pkg.aligned_buffer(b.blob_size())
    b.build(text, blob)
    return rng, text, table, block, blob


@pytest.mark.parametrize("replicas", [1, 3])
def test_multi_matches_single_device(pkg, replicas):
    rng, text, table, block, blob = _case(pkg)
    one = pkg.FmIndex.load(blob, pkg.u32, block, table)
    multi = pkg.MultiDeviceIndex(blob, [0] * replicas, pkg.u32, block, table)
    assert multi.replicas == replicas
    # ragged, with 1-3 bp patterns (tens of thousands of occurrences each: the
    # shards' first guess of room overflows), absent and wildcard patterns
    pats = [text[s:s + int(rng.integers(1, 30))].tobytes() for s in rng.integers(0, text.size - 30, 20001)]
    pats += [b"NNNN", b"ACGTN", b"acgt"]
    for rev in (False, True):
        q = [p[::-1] for p in pats] if rev else pats
        w_off, w_locs = one.locate_batch(q, reversed=rev)
        g_off, g_locs = multi.locate_batch(q, reversed=rev)
        assert np.array_equal(g_off, w_off) and np.array_equal(g_locs, w_locs)
        assert np.array_equal(multi.count_batch(q, reversed=rev), one.count_batch(q, reversed=rev))
    # fewer patterns than replicas
    few = pats[:2]
    assert np.array_equal(multi.locate_batch(few)[1], one.locate_batch(few)[1])
    assert multi.locate_batch([])[0].tolist() == [0]
    one.close()
    multi.close()


def test_multi_capacity_and_errors(pkg):
    rng, text, table, block, blob = _case(pkg, n=100_000, seed=6)
    one = pkg.FmIndex.load(blob, pkg.u32, block, table)
    multi = pkg.MultiDeviceIndex(blob, [0, 0], pkg.u32, block, table)
    pats = [text[s:s + 4].tobytes() for s in rng.integers(0, text.size - 4, 300)]
    w_off, w_locs = one.locate_batch(pats)
    data, offsets = pkg.pack_patterns(pats)
    loc_off = np.zeros(len(pats) + 1, np.uint64)
    locs = np.zeros(10, np.uint32)
    needed = C.c_uint64()
    st = pkg._native.lib().fmx_multi_locate_batch(multi._h, data.ctypes.data, offsets.ctypes.data, len(pats), 0,
                                                  loc_off.ctypes.data, locs.ctypes.data, 10, C.byref(needed))
    assert st == pkg._native.FMX_E_CAPACITY and needed.value == w_locs.size
    assert np.array_equal(loc_off, w_off)  # offsets are written whatever the capacity
    with pytest.raises(pkg.FmxError) as e:
        multi.locate_batch(pats[:5] + [b""] + pats[5:])
    assert e.value.code == pkg._native.FMX_E_EMPTY_PATTERN
    bad = blob.copy()
    bad[0] ^= 0xFF
    with pytest.raises(pkg.LoadError.InvalidFormat):
        pkg.MultiDeviceIndex(bad, [0, 0], pkg.u32, block, table)
    one.close()
    multi.close()
