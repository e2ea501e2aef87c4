"""Per-kernel sums of the PMC passes of `scripts/gpu.sh TAG pmc` (the
rocprofv3 counter_collection.csv of each pass) and the bench line each pass
printed, copied under profiles/ for the record:

    python scripts/pmc_by_kernel.py TAG PREFIX
      -> PREFIX_pmc_{fetch,ea,write,tcc}_by_kernel.csv  (kernel, counter, sum, dispatches, per_dispatch)
         PREFIX_bench_pmc_{fetch,ea,write,tcc}.json     (the bench line of that pass)
"""
import csv
import gzip
import json
import os
import sys
from collections import defaultdict

def open_csv(path):
    """A pass's counter CSV, gzipped on the box when the raw files would not fit gpurun's 64 MiB return."""
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path)


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag, prefix = sys.argv[1], sys.argv[2]
    g = os.path.join(ROOT, "gpurun_out", tag)
    for p in ("fetch", "ea", "write", "tcc"):
        if not os.path.isdir(os.path.join(g, f"pmc_{p}")):
            continue  # (the TCC pass is optional)
        path = None
        for root, _, files in os.walk(os.path.join(g, f"pmc_{p}")):
            for f in files:
                if f.endswith("counter_collection.csv") or f.endswith("counter_collection.csv.gz"):
                    path = os.path.join(root, f)
        if path is None:
            raise SystemExit(f"no counter_collection.csv for pass {p} under {g}")
        tot, disp = defaultdict(float), defaultdict(set)
        for r in csv.DictReader(open_csv(path)):
            k = (r["Kernel_Name"][:120], r["Counter_Name"])
            tot[k] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
        with open(f"{prefix}_pmc_{p}_by_kernel.csv", "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "counter", "sum", "dispatches", "per_dispatch"])
            for k in sorted(tot, key=lambda k: -tot[k]):
                w.writerow([k[0], k[1], tot[k], len(disp[k]), tot[k] / len(disp[k])])
        lines = [ln for ln in open(os.path.join(g, f"pmc_{p}.log")) if ln.startswith("{")]
        if lines:
            json.dump(json.loads(lines[-1]), open(f"{prefix}_bench_pmc_{p}.json", "w"), indent=1)


if __name__ == "__main__":
    main()
