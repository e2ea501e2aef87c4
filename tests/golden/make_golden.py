"""Generate tests/golden/oracle_cases.json — regression fixtures of the CPU
oracle (oracle/fmx_oracle.c): blob bytes (hex) and counts / locations in
suffix-array-row order for small seeded inputs across layouts and configs.

Provenance: these vectors are produced by this repo's restatement, not by the
reference (its Rust toolchain is absent here).  The restatement itself is
pinned by the reference's README known answers (golden/readme.json) and by the
brute-force accuracy contract (tests/test_oracle.py); these fixtures freeze
its byte-level output (blob layout, unsorted SA-row order) so any later change
is caught.  Re-run: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))
from oracle import oracle as O  # noqa: E402
from _util import rand_chr_list, rand_text, rand_pattern, table_from_symbols  # noqa: E402

CASES = [
    # (seed, sigma, pos_bytes, planes, vec_bits, k, sr, n_min, n_max)
    (1, 4, 4, 2, 64, 3, 2, 200, 300),
    (2, 5, 4, 3, 64, 3, 2, 256, 256),     # n % BL == 0
    (3, 3, 8, 2, 32, 2, 3, 100, 150),
    (4, 7, 4, 3, 128, 4, 4, 300, 400),
    (5, 21, 4, 5, 64, 2, 2, 300, 400),
    (6, 16, 8, 4, 128, 1, 1, 128, 128),   # n % 128 == 0
    (7, 40, 4, 6, 32, 1, 2, 200, 300),
    (8, 2, 8, 2, 64, 4, 5, 64, 64),
]


def main():
    out = []
    for seed, sigma, pb, planes, vb, k, sr, lo, hi in CASES:
        rng = np.random.default_rng(seed)
        chars = rand_chr_list(rng, sigma)
        table = table_from_symbols([bytes([c]) for c in chars])
        text = rand_text(rng, chars, lo, hi)
        L = O.layout(pb, planes, vb, 0)
        blob = O.build(text, sigma, L, k, sr, table)
        ix = O.OracleIndex(blob, L)
        pats = [rand_pattern(rng, text, 1, 8) for _ in range(12)] + [b"\x01\x02", chars[:1] * 3]
        res = []
        for p in pats:
            res.append({"pattern": p.hex(), "count": ix.count(p), "locations": ix.locate(p)})
        out.append({"seed": seed, "sigma": sigma, "layout": [pb, planes, vb], "kmer_size": k,
                    "sampling_ratio": sr, "table": table.hex(), "text": text.hex(),
                    "blob": bytes(blob).hex(), "queries": res})
    with open(os.path.join(HERE, "oracle_cases.json"), "w") as f:
        json.dump({"_source": __doc__.strip().splitlines()[0], "cases": out}, f, indent=0)


if __name__ == "__main__":
    main()
