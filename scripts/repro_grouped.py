"""Repro: test_every_layout_grouped[4-4-64] mismatch — per-pattern details, grouped vs launch order, repeated."""
import os, sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import __graft_entry__ as ge
pkg = ge.load_package()
from oracle import oracle as O
import test_gpu as T
from _util import rand_chr_list, rand_pattern, rand_text, table_from_symbols
pb, planes, vb = 4, 4, 64
rng = np.random.default_rng(pb * 31 + planes * 7 + vb)
for sigma in sorted({2, 3, (1 << planes) // 2 + 1, 1 << planes}):
    chars = rand_chr_list(rng, sigma)
    table = table_from_symbols([bytes([c]) for c in chars])
    text = rand_text(rng, chars, 300, 4000)
    k, sr = int(rng.integers(1, 5)), int(rng.integers(1, 5))
    if (sigma + 1) ** k > 1 << 20:
        k = 2
    blob = T.gpu_build(pkg, text, sigma, pb, planes, vb, k, sr, table)
    top = 96 // int(sigma).bit_length()
    for m in sorted({1, 2, k, 7, top}):
        pats = [rand_pattern(rng, text, m, m) for _ in range(400)]
        pats = [p for p in pats if len(p) == m]
        pats += [bytes(rng.choice(np.frombuffer(chars, np.uint8), size=m)) for _ in range(40)]
        pats += [b"\x00" * m, chars[:1] * m, chars[-1:] * m]
        data, offsets = pkg.pack_patterns(pats)
        orc = O.OracleIndex(blob, O.layout(pb, planes, vb, 0))
        ooff, olocs = orc.locate_batch(data, offsets)
        for occ in (0, 1):
            for mode in ("1", "0", "1", "1"):
                os.environ["FMX_GROUPED"] = mode
                ix = pkg.FmIndex.load(blob, pkg.u32, pkg.blocks.Block4(pkg.Vector.U64), options=occ)
                goff, glocs = ix.locate_batch((data, offsets))
                ix.close()
                bad = np.flatnonzero(np.diff(goff.astype(np.int64)) != np.diff(ooff.astype(np.int64)))
                print(f"sigma={sigma} n={len(text)} k={k} sr={sr} m={m} occ={occ} grouped={mode} n_pat={len(pats)} bad={bad.tolist()[:10]}", flush=True)
                for b in bad[:4]:
                    print("   pat", b, pats[b], "gpu", int(goff[b+1]-goff[b]), "oracle", int(ooff[b+1]-ooff[b]), flush=True)
