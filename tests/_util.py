"""Shared test helpers: random data in the shape of the reference's own
generators (sview-fmindex/src/tests/random_data/mod.rs:7-37, seeded here), and
a brute-force occurrence finder (the reference's accuracy contract,
src/tests/get_accurate_result/mod.rs:136-140)."""
import numpy as np

# every (P bytes, planes, vector bits) the reference's tests sweep
# (get_accurate_result/mod.rs:179-222)
ALL_LAYOUTS = [(p, n, v) for p in (4, 8) for n in (2, 3, 4, 5, 6) for v in (32, 64, 128)]


def table_from_symbols(symbols, with_wildcard=False):
    """EncodingTable::from_symbols[_with_wildcard] (encoding_table.rs:15-35)."""
    count = len(symbols) + (1 if with_wildcard else 0)
    t = bytearray([count - 1] * 256)
    for i, s in enumerate(symbols):
        for x in bytes(s):
            t[x] = i
    return bytes(t)


def rand_chr_list(rng, count):
    """gen_rand_chr_list: `count` distinct printable bytes (random_data/mod.rs:7-18)."""
    return bytes(rng.choice(np.arange(33, 127), size=count, replace=False).astype(np.uint8))


def rand_text(rng, chr_list, min_len, max_len):
    """gen_rand_text: every chr at least once, shuffled (random_data/mod.rs:20-30)."""
    n = int(rng.integers(min_len, max_len + 1))
    t = list(chr_list) + list(rng.choice(np.frombuffer(chr_list, np.uint8), size=max(0, n - len(chr_list))))
    rng.shuffle(t)
    return bytes(bytearray(int(x) for x in t))


def rand_pattern(rng, text, min_len, max_len):
    """gen_rand_pattern: a substring (random_data/mod.rs:31-37)."""
    m = int(rng.integers(min_len, max_len + 1))
    s = int(rng.integers(0, len(text) - m))
    return text[s:s + m]


def occurrences(text_idx: bytes, pat_idx: bytes):
    """All start positions of pat in text, over symbol indices."""
    m = len(pat_idx)
    out, i = [], text_idx.find(pat_idx)
    while i != -1:
        out.append(i)
        i = text_idx.find(pat_idx, i + 1)
    return out if m else []


def encode(table: bytes, data: bytes) -> bytes:
    return bytes(table[b] for b in data)
