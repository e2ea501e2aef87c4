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


# Full-size blob provenance (the C2-C5 blobs' SHA-256 recorded).
# The text recipe is shared by tests/golden/make_blob_digests.py (the oracle's
# CPU builder, in this container) and tests/test_gpu_provenance.py (the GPU
# builder, on the box): numpy's PCG64 stream is the same on both.
ACGTN_SYMBOLS = [b"Aa", b"Cc", b"Gg", b"Tt", b"Nn"]
AMINO20 = b"ACDEFGHIKLMNPQRSTVWY"
PROVENANCE = {
    # name: (n, alphabet, symbols, (P bytes, planes, vector bits), seed)
    "c2": (1_000_000_000, b"ACGT", ACGTN_SYMBOLS, (4, 3, 64), 20261),
    "c4": (1_000_000_000, AMINO20, [bytes([c, c + 32]) for c in AMINO20] + [b"Xx"], (4, 5, 64), 20262),
}
PROVENANCE_K, PROVENANCE_SR = 3, 2


def provenance_text(name):
    """The seeded text of a provenance config: uniform over its alphabet."""
    n, alphabet, _, _, seed = PROVENANCE[name]
    rng = np.random.Generator(np.random.PCG64(seed))
    out = np.empty(n, dtype=np.uint8)
    lut = np.frombuffer(alphabet, dtype=np.uint8)
    step = 1 << 26
    for c0 in range(0, n, step):
        c1 = min(n, c0 + step)
        out[c0:c1] = lut[rng.integers(0, len(alphabet), c1 - c0, dtype=np.uint8)]
    return out
