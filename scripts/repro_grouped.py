import os, sys
os.environ["FMX_GROUPED"] = "1"; os.environ["FMX_DEBUG"] = "1"
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import __graft_entry__ as ge
pkg = ge.load_package()
from oracle import oracle as O
import test_gpu as T
from _util import rand_chr_list, rand_pattern, rand_text, table_from_symbols
pb, planes, vb = 4, 2, 32
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
        for occ in (0, 1):
            try:
                T.check_parity(pkg, O, blob, pb, planes, vb, 0, pats, occ)
                print("ok", sigma, len(text), k, sr, m, occ, flush=True)
            except Exception as e:
                print("FAIL", sigma, len(text), k, sr, m, occ, repr(e), flush=True)
