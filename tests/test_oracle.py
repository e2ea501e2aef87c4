"""CPU tests of the oracle (oracle/fmx_oracle.c) — the checker every GPU parity
test compares against.  They mirror the reference's own test suite
(sview-fmindex/src/tests/): the README known answers, the accuracy contract
(sorted locate == every occurrence), configuration invariance, encoder /
reverse-iterator consistency, plus the edge cases of SURVEY.md §8.0."""
import json
import os

import numpy as np
import pytest

from _util import (ALL_LAYOUTS, encode, occurrences, rand_chr_list, rand_pattern, rand_text,
                   table_from_symbols)

HERE = os.path.dirname(os.path.abspath(__file__))


def test_readme_known_answers(O):
    """src/tests/readme/mod.rs:29-44."""
    g = json.load(open(os.path.join(HERE, "golden", "readme.json")))
    table = table_from_symbols([s.encode() for s in g["symbols"]])
    L = O.layout(g["layout"]["pos_bytes"], g["layout"]["planes"], g["layout"]["vec_bits"], 0)
    blob = O.build(g["text"].encode(), g["symbol_count"], L, g["kmer_size"], g["sampling_ratio"], table)
    ix = O.OracleIndex(blob, L)
    for case in g["cases"]:
        p = case["pattern"].encode()
        if "count" in case:
            assert ix.count(p) == case["count"]
        assert sorted(ix.locate(p)) == case["sorted_locations"]


def test_golden_regression(O):
    """Byte-level regression of the restatement (tests/golden/make_golden.py)."""
    g = json.load(open(os.path.join(HERE, "golden", "oracle_cases.json")))
    for c in g["cases"]:
        pb, planes, vb = c["layout"]
        L = O.layout(pb, planes, vb, 0)
        blob = O.build(bytes.fromhex(c["text"]), c["sigma"], L, c["kmer_size"], c["sampling_ratio"],
                       bytes.fromhex(c["table"]))
        assert bytes(blob).hex() == c["blob"]
        ix = O.OracleIndex(blob, L)
        for q in c["queries"]:
            p = bytes.fromhex(q["pattern"])
            assert ix.count(p) == q["count"]
            assert ix.locate(p) == q["locations"]


@pytest.mark.parametrize("sigma", [3, 4, 5, 7, 8, 9, 15, 16, 17])
def test_accurate_results(O, sigma):
    """get_accurate_result/mod.rs:143-225: every layout, k=3, sr=2, texts of
    100-300, patterns of 1-10 taken from the text, against brute force."""
    rng = np.random.default_rng(1000 + sigma)
    for _ in range(2):
        chars = rand_chr_list(rng, sigma)
        text = rand_text(rng, chars, 100, 300)
        pats = [rand_pattern(rng, text, 1, 10) for _ in range(100)]
        table = table_from_symbols([bytes([c]) for c in chars])
        t_idx = encode(table, text)
        answers = [occurrences(t_idx, encode(table, p)) for p in pats]
        for pb, planes, vb in ALL_LAYOUTS:
            if (1 << planes) < sigma:
                continue
            L = O.layout(pb, planes, vb, 0)
            ix = O.OracleIndex(O.build(text, sigma, L, 3, 2, table), L)
            data = np.frombuffer(b"".join(pats), np.uint8)
            offs = np.zeros(len(pats) + 1, np.uint64)
            np.cumsum([len(p) for p in pats], out=offs[1:])
            loff, locs = ix.locate_batch(data, offs)
            for i, ans in enumerate(answers):
                assert sorted(int(x) for x in locs[loff[i]:loff[i + 1]]) == ans


@pytest.mark.parametrize("sigma", [4, 6, 8, 10])
def test_config_invariance(O, sigma):
    """config_invariance/mod.rs:50-143: k in {1,2,3,4} x sr in {1,2,3,4} give the
    default u32/Block4<u32> answer."""
    rng = np.random.default_rng(2000 + sigma)
    for _ in range(3):
        chars = rand_chr_list(rng, sigma)
        text = rand_text(rng, chars, 1000, 1000)
        pat = rand_pattern(rng, text, 10, 10)
        table = table_from_symbols([bytes([c]) for c in chars])
        base_L = O.layout(4, 4, 32, 0)
        answer = sorted(O.OracleIndex(O.build(text, sigma, base_L, 1, 1, table), base_L).locate(pat))
        for pb, planes, vb in ALL_LAYOUTS[::3]:
            if (1 << planes) < sigma:
                continue
            for k in (1, 2, 3, 4):
                for sr in (1, 2, 3, 4):
                    L = O.layout(pb, planes, vb, 0)
                    ix = O.OracleIndex(O.build(text, sigma, L, k, sr, table), L)
                    assert sorted(ix.locate(pat)) == answer


@pytest.mark.parametrize("sigma", [2, 3])
def test_text_encoders_consistency(O, sigma):
    """text_encoders_consistency/mod.rs:163-251: EncodingTable vs PassThrough,
    forward vs reverse iterator, count and locate."""
    rng = np.random.default_rng(3000 + sigma)
    chars = rand_chr_list(rng, sigma)
    text = rand_text(rng, chars, 100, 300)
    table = table_from_symbols([bytes([c]) for c in chars])
    pats = [rand_pattern(rng, text, 1, 10) for _ in range(100)]
    for pb, planes, vb in ALL_LAYOUTS:
        L = O.layout(pb, planes, vb, 0)
        et = O.OracleIndex(O.build(text, sigma, L, 3, 2, table), L)
        Lp = O.layout(pb, planes, vb, 1)
        pt = O.OracleIndex(O.build(encode(table, text), sigma, Lp, 3, 2, None), Lp)
        for p in pats:
            pi = encode(table, p)
            c = et.count(p)
            assert c == et.count_rev(p[::-1]) == pt.count(pi) == pt.count_rev(pi[::-1])
            assert sorted(et.locate(p)) == sorted(pt.locate(pi))


def test_edge_cases(O):
    """SURVEY §8.0 edge cases: n % BL == 0 (extra zero block), m < k, absent
    patterns, wildcard bytes, high-count short patterns, one-symbol text."""
    rng = np.random.default_rng(4)
    table = table_from_symbols([b"A", b"C", b"G", b"T"])  # T is the wildcard
    for n in (0, 1, 2, 31, 32, 33, 63, 64, 65, 127, 128, 129, 256):
        text = bytes(rng.choice(np.frombuffer(b"ACGTXN", np.uint8), size=n)) if n else b""
        t_idx = encode(table, text)
        for (pb, planes, vb) in [(4, 2, 32), (8, 2, 64), (4, 3, 128)]:
            for k, sr in [(1, 1), (3, 2), (4, 3), (5, 7)]:
                L = O.layout(pb, planes, vb, 0)
                ix = O.OracleIndex(O.build(text, 4, L, k, sr, table), L)
                assert ix.text_len == n
                for p in [b"A", b"AC", b"ACGTACGT", b"T", b"Z", b"ZZ", b"CCCCCCCCCCCCCCCCCCCCC"]:
                    assert sorted(ix.locate(p)) == occurrences(t_idx, encode(table, p))
    text = b"A" * 300
    L = O.layout(4, 2, 64, 0)
    ix = O.OracleIndex(O.build(text, 4, L, 3, 4, table), L)
    assert ix.count(b"A") == 300 and ix.count(b"AA") == 299 and ix.count(b"C") == 0
    assert sorted(ix.locate(b"AAA")) == list(range(298))


def test_errors(O):
    table = table_from_symbols([b"A", b"C"])
    L = O.layout(4, 2, 64, 0)
    blob = O.build(b"ACCA", 2, L, 1, 1, table)
    ix = O.OracleIndex(blob, L)
    with pytest.raises(O.OracleError) as e:
        ix.count(b"")
    assert e.value.code == 5  # empty pattern: count_array.rs:211 panics
    bad = blob.copy()
    bad[0] = ord("X")
    with pytest.raises(O.OracleError) as e:
        O.OracleIndex(bad, L)
    assert e.value.code == 1  # LoadError::InvalidFormat
    trunc = O.aligned_zeros(blob.size - 8)
    trunc[:] = blob[:blob.size - 8]
    with pytest.raises(O.OracleError) as e:
        O.OracleIndex(trunc, L)
    assert e.value.code == 2  # MismatchedBlobSize
    short = O.aligned_zeros(blob.size + 8)
    short[:blob.size] = blob
    with pytest.raises(O.OracleError) as e:
        O.OracleIndex(short, L)
    assert e.value.code == 2  # MismatchedBlobSize
    # PassThrough: byte >= symbol_count
    Lp = O.layout(4, 2, 64, 1)
    pt = O.OracleIndex(O.build(bytes([0, 1, 1, 0]), 2, Lp, 1, 1, None), Lp)
    with pytest.raises(O.OracleError) as e:
        pt.count(bytes([0, 2]))
    assert e.value.code == 6
    with pytest.raises(O.OracleError):
        O.build(b"AC", 5, O.layout(4, 2, 64), 1, 1, table)  # SymbolCountOver (5 > 4)


def test_suffix_array_small(O):
    rng = np.random.default_rng(5)
    for _ in range(50):
        n = int(rng.integers(1, 200))
        t = rng.integers(1, int(rng.integers(2, 6)), size=n).astype(np.uint8)
        t = np.concatenate([t, np.zeros(1, np.uint8)])
        sa = O.suffix_array(t, 8)
        ref = sorted(range(len(t)), key=lambda i: bytes(t[i:]))
        assert [int(x) for x in sa] == ref


def test_kmer_size_config(pkg):
    """lookup_table_config.rs:55-76 (pure host logic of the Python mirror)."""
    LT = pkg.build_config.LookupTableConfig
    assert LT.None_().kmer_size(pkg.u32, 1) == 1
    assert LT.None_().kmer_size(pkg.u32, 2) == 1
    with pytest.raises(pkg.BuildError):
        LT.KmerSize(1).kmer_size(pkg.u32, 1)
    assert LT.KmerSize(2).kmer_size(pkg.u32, 2) == 2
    assert LT.MaxMemory(0).kmer_size(pkg.u32, 1) == 1
    assert LT.MaxMemory(0).kmer_size(pkg.u32, 2) == 1
    assert LT.MaxMemory(6 ** 3 * 4).kmer_size(pkg.u32, 5) == 3
    SA = pkg.build_config.SuffixArrayConfig
    assert SA.Uncompressed().sampling_ratio() == 1
    with pytest.raises(pkg.BuildError):
        SA.Compressed(1).sampling_ratio()
