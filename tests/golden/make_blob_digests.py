"""Record the SHA-256 of full-size blobs built by the oracle's CPU builder
(oracle/fmx_oracle.c orc_build: FmIndexBuilder::build restated,
builder/mod.rs:187-264) from the seeded texts of tests/_util.py PROVENANCE.
tests/test_gpu_provenance.py builds the same texts with the GPU builder and
asserts the same digests.  Test infrastructure; run here (no GPU):

    python tests/golden/make_blob_digests.py c2 [c4]

C2 (1 Gbp) needs ~36 GB of host RAM (prefix doubling keeps three 8-B arrays
of n + 1 words plus a counter array of the same size); C5 (3 Gbp) would need
~110 GB and does not fit this container's 62 GB, so it has no digest."""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from _util import PROVENANCE, PROVENANCE_K, PROVENANCE_SR, provenance_text, table_from_symbols  # noqa: E402
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(HERE, "blob_digests.json")


def main(names):
    db = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for name in names:
        n, alphabet, symbols, (pb, planes, vec), seed = PROVENANCE[name]
        t0 = time.time()
        text = provenance_text(name)
        text_sha = hashlib.sha256(text).hexdigest()
        table = table_from_symbols(symbols)
        sigma = max(table) + 1
        print(f"[{name}] text {n:,} generated in {time.time() - t0:.1f} s, sha256 {text_sha}", flush=True)
        t1 = time.time()
        blob = O.build(text, sigma, O.layout(pb, planes, vec, 0), k=PROVENANCE_K, sr=PROVENANCE_SR, table=table)
        build_s = time.time() - t1
        del text
        digest = hashlib.sha256(blob).hexdigest()
        print(f"[{name}] blob {blob.size:,} B built by the oracle in {build_s:.0f} s, sha256 {digest}", flush=True)
        db[name] = {
            "n": n, "alphabet": alphabet.decode(), "seed": seed, "rng": "numpy PCG64, integers(0, |alphabet|, uint8)",
            "layout": {"pos_bytes": pb, "planes": planes, "vec_bits": vec}, "sigma": sigma,
            "k": PROVENANCE_K, "sr": PROVENANCE_SR, "text_sha256": text_sha,
            "blob_bytes": int(blob.size), "blob_sha256": digest,
            "builder": "oracle/fmx_oracle.c orc_build (prefix doubling)", "build_s": round(build_s),
        }
        del blob
        with open(OUT, "w") as f:
            json.dump(db, f, indent=1, sort_keys=True)
            f.write("\n")


if __name__ == "__main__":
    main(sys.argv[1:] or ["c2", "c4"])
