"""Stress / repro driver for grouped launches (GPU): replays the inputs of
tests/test_gpu_grouped.py::test_every_layout_grouped (same seeds) over and over
for a time budget, and prints every per-pattern mismatch against the oracle
(layout, sigma, m, load options, direction, which patterns, GPU vs oracle
count) instead of stopping at the first assert.

    python scripts/stress_grouped.py --seconds 240 [--layouts 4-5-32,4-4-64] [--env FMX_GROUP_CHECK=1] [--rebuild]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=240)
    ap.add_argument("--layouts", default="")
    ap.add_argument("--env", action="append", default=[])
    ap.add_argument("--grouped", default="1")
    ap.add_argument("--rebuild", action="store_true",
                    help="build every blob on the GPU again each round (as the suite does), not once")
    a = ap.parse_args()
    os.environ["FMX_GROUPED"] = a.grouped
    for kv in a.env:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    import __graft_entry__ as ge
    pkg = ge.load_package()
    from oracle import oracle as O
    import test_gpu as T
    from _util import ALL_LAYOUTS, rand_chr_list, rand_pattern, rand_text, table_from_symbols
    layouts = ALL_LAYOUTS
    if a.layouts:
        layouts = [tuple(int(x) for x in s.split("-")) for s in a.layouts.split(",")]
    t0 = time.time()
    rep = calls = bad_calls = 0
    cache = {}
    while time.time() - t0 < a.seconds:
        for (pb, planes, vb) in layouts:
            if time.time() - t0 >= a.seconds:
                break
            key = (pb, planes, vb)
            if a.rebuild:
                cache.pop(key, None)
            if key not in cache:
                rng = np.random.default_rng(pb * 31 + planes * 7 + vb)
                cases = []
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
                        cases.append((sigma, m, blob, pats, data, offsets, ooff, olocs))
                cache[key] = cases
            blk = getattr(pkg.blocks, f"Block{planes}")(pkg.Vector(vb))
            pos = pkg.u32 if pb == 4 else pkg.u64
            for (sigma, m, blob, pats, data, offsets, ooff, olocs) in cache[key]:
                for occ in (0, 1):
                    ix = pkg.FmIndex.load(blob, pos, blk, options=occ)
                    for rev in (False, True):
                        q = (data, offsets) if not rev else [p[::-1] for p in pats]
                        try:
                            goff, glocs = ix.locate_batch(q, reversed=rev)
                            err = None
                        except Exception as e:  # a latched device check (FMX_GROUP_CHECK) or another error
                            goff, glocs, err = None, None, repr(e)
                        calls += 1
                        ok = err is None and np.array_equal(goff, ooff) and np.array_equal(glocs, olocs)
                        if not ok:
                            bad_calls += 1
                            msg = f"MISMATCH rep={rep} layout={pb}-{planes}-{vb} sigma={sigma} m={m} occ={occ} rev={rev}"
                            if err:
                                print(msg, "error", err, flush=True)
                                continue
                            gc, oc = np.diff(goff.astype(np.int64)), np.diff(ooff.astype(np.int64))
                            bad = np.flatnonzero(gc != oc)
                            print(msg, f"patterns={len(pats)} bad={len(bad)} total gpu={int(goff[-1])} "
                                  f"oracle={int(ooff[-1])}", flush=True)
                            for b in bad[:12]:
                                same = sorted({pats[j] for j in np.flatnonzero(oc == gc[b])})[:4]
                                print(f"   pat {b} {pats[b]!r} gpu {gc[b]} oracle {oc[b]} "
                                      f"(oracle count of {same!r})", flush=True)
                                gl = glocs[goff[b]:goff[b + 1]] if not rev else None
                                if gl is not None and gl.size:
                                    hits = [(j, pats[j]) for j in range(len(pats)) if pats[j] != pats[b] and
                                            oc[j] == gc[b] and np.array_equal(np.sort(olocs[ooff[j]:ooff[j + 1]]),
                                                                              np.sort(gl))]
                                    print(f"      its locations are pattern {hits[:1]!r}'s" if hits else
                                          "      its locations match no other pattern's", flush=True)
                            if len(bad) == 0:
                                d = np.flatnonzero(glocs != olocs)
                                print(f"   locations differ at {d[:8].tolist()} of {olocs.size}", flush=True)
                    ix.close()
            print(f"[{time.time() - t0:7.1f}s] rep {rep} layout {pb}-{planes}-{vb} calls {calls} bad {bad_calls}",
                  flush=True)
        rep += 1
    print(f"DONE reps={rep} calls={calls} bad_calls={bad_calls}", flush=True)


if __name__ == "__main__":
    main()
