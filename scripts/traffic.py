"""Per-launch HBM traffic of the locate launch from the PMC passes of
scripts/r2_profile.sh, written into profiles/pmc_traffic.json under the
bench's profile key (bench.py reads it for roofline.traffic).

    python scripts/traffic.py <TAG> [--out profiles/pmc_traffic.json]

FETCH_SIZE (KB) is the L2's memory-side read bytes (TCC_EA0_RDREQ x 64 B per
request on gfx950, MI355X_MICROARCH.md HBM section); the request split into
64-B and 128-B requests comes from TCC_EA0_RDREQ_64B/_128B, so the bytes
actually requested are 64 n64 + 128 n128 (+ 32 n32) — reported as
fabric_bytes_per_launch (memory-side requests: on gfx950 they include
Infinity Cache hits, so they bound the HBM bytes from above), with
FETCH_SIZE kept alongside."""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LAUNCH = ("k_search", "k_emit", "k_scan", "k_group_")  # k_group_*: a grouped launch's other kernels


def sums(path, variant):
    """counter -> total over the launch kernels of the headline variant, and the launch count."""
    tot = defaultdict(float)
    launches = set()
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if not any(k in name for k in LAUNCH):
            continue
        if "k_search_grouped" in name:  # (faithful only)
            launches.add(r["Dispatch_Id"])
        elif "k_search" in name:
            if variant not in name:
                continue
            launches.add(r["Dispatch_Id"])
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
    return tot, len(launches)


def bench_json(log):
    lines = [ln for ln in open(log) if ln.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def main():
    tag = sys.argv[1]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else os.path.join(ROOT, "profiles", "pmc_traffic.json")
    g = os.path.join(ROOT, "gpurun_out")
    b = bench_json(os.path.join(g, f"{tag}_fetch.log"))
    key = b["profile_key"]
    variant = ", 0>" if b["config"]["load_options"] in (0, 1) else ""
    rf = b["roofline"]
    ppl = rf["kernel"]["patterns_per_launch"] if "kernel" in rf else rf["patterns_per_launch"]
    fetch, nl = sums(os.path.join(g, f"{tag}_fetch", "run_counter_collection.csv"), variant)
    ea, nl2 = sums(os.path.join(g, f"{tag}_ea", "run_counter_collection.csv"), variant)
    wr, nl3 = sums(os.path.join(g, f"{tag}_write", "run_counter_collection.csv"), variant)
    tcc, nl4 = sums(os.path.join(g, f"{tag}_tcc", "run_counter_collection.csv"), variant)
    n64, n128, nreq = ea["TCC_EA0_RDREQ_64B_sum"] / nl2, ea["TCC_EA0_RDREQ_128B_sum"] / nl2, ea["TCC_EA0_RDREQ_sum"] / nl2
    n32 = max(nreq - n64 - n128, 0.0)
    run = {
        "tag": tag, "source": "rocprofv3 --pmc, scripts/r2_profile.sh + scripts/traffic.py",
        "launches_profiled": nl, "patterns_per_launch": ppl,
        "fetch_size_bytes_per_launch": fetch["FETCH_SIZE"] * 1024 / nl,
        "fabric_requests_per_launch": nreq, "requests_32b": n32, "requests_64b": n64, "requests_128b": n128,
        "fabric_bytes_per_launch": 32 * n32 + 64 * n64 + 128 * n128,
        "write_bytes_per_launch": wr["WRITE_SIZE"] * 1024 / nl3,
        "l2_hit_rate": tcc["TCC_HIT_sum"] / max(tcc["TCC_HIT_sum"] + tcc["TCC_MISS_sum"], 1),
        "l2_requests_per_pattern": (tcc["TCC_HIT_sum"] + tcc["TCC_MISS_sum"]) / nl4 / ppl,
    }
    run["fabric_bytes_per_pattern"] = run["fabric_bytes_per_launch"] / ppl
    run["fabric_requests_per_pattern"] = nreq / ppl
    db = json.load(open(out)) if os.path.exists(out) else {"runs": {}}
    db.setdefault("runs", {})[key] = run
    json.dump(db, open(out, "w"), indent=1, sort_keys=True)
    print(key, json.dumps(run, indent=1))


if __name__ == "__main__":
    main()
