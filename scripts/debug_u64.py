# Debug: the test_builder_and_queries_every_layout[8-2-64] case on the GPU,
# every load option, first mismatches vs the oracle.
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'tests'))
os.environ.setdefault("FMX_DEEP_LUT_MB", "1")
import __graft_entry__ as g
from oracle import oracle as O
from _util import *
pkg = g.load_package()
pb, planes, vb = 8, 2, 64
rng = np.random.default_rng(pb * 1000 + planes * 100 + vb)
for sigma in sorted({2, 3, (1 << planes) // 2 + 1, 1 << planes}):
    chars = rand_chr_list(rng, sigma)
    table = table_from_symbols([bytes([c]) for c in chars])
    text = rand_text(rng, chars, 300, 2000)
    k, sr = int(rng.integers(1, 5)), int(rng.integers(1, 5))
    if (sigma + 1) ** k > 1 << 20: k = 2
    pats = [rand_pattern(rng, text, 1, 24) for _ in range(300)]
    pats += [bytes(rng.choice(np.frombuffer(chars, np.uint8), size=int(rng.integers(1, 12)))) for _ in range(50)]
    pats += [b"\x00", b"\x7f\x7f", chars[:1] * 2]
    blob = O.build(text, sigma, O.layout(pb, planes, vb), k, sr, table)
    orc = O.OracleIndex(blob, O.layout(pb, planes, vb, 0))
    data, offs = pkg.pack_patterns(pats)
    ooff, olocs = orc.locate_batch(data, offs)
    for opt in (0, 1, 3, 5, 15, 12):
        ix = pkg.FmIndex.load(blob, pkg.u64, pkg.blocks.Block2(pkg.Vector(64)), options=opt)
        goff, glocs = ix.locate_batch((data, offs))
        cnt = ix.count_batch((data, offs))
        bad = np.nonzero(glocs != olocs)[0] if glocs.size == olocs.size else None
        print(f"sigma={sigma} k={k} sr={sr} n={len(text)} opt={opt} offsets_eq={np.array_equal(goff, ooff)} "
              f"count_eq={np.array_equal(cnt.astype(np.uint64), np.diff(ooff))} locs_eq={np.array_equal(glocs, olocs)} "
              f"nbad={None if bad is None else bad.size} first={None if bad is None or not bad.size else (int(bad[0]), int(glocs[bad[0]]), int(olocs[bad[0]]))}")
        # single-pattern re-query of the first bad one
        if bad is not None and bad.size:
            pi = int(np.searchsorted(ooff, bad[0], side='right') - 1)
            print("   pattern", pi, pats[pi], "gpu", ix.locate(pats[pi])[:5], "orc", orc.locate(pats[pi])[:5])
        ix.close()
