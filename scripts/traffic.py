"""Per-launch memory traffic of the locate launch from the PMC passes of
`scripts/gpu.sh TAG pmc` (gpurun_out/TAG/pmc_{fetch,ea,write,tcc}/ and the
bench lines in gpurun_out/TAG/pmc_*.log), written into
profiles/pmc_traffic.json under the bench's profile key (bench.py reads it
for roofline.traffic).

    python scripts/traffic.py TAG [--out profiles/pmc_traffic.json]

Counters (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KB) is the L2's
memory-side read bytes tallied at 64 B per request on gfx950 — so 128-B
requests are under-counted by half; the exact read bytes come from the
request split TCC_EA0_RDREQ_{32B,64B,128B}: 32 n32 + 64 n64 + 128 n128
(fabric_read_bytes; 2 x FETCH_SIZE is kept beside it as the guide's
correction, equal when every request is 128 B).  WRITE_SIZE (KB) is the
memory-side write bytes.  Memory-side requests include Infinity Cache hits,
so these bound the HBM bytes from above.  Sums are per launch over the
launch's kernels (k_group_key x2, k_group_scan, k_search_grouped,
k_group_tiles, k_emit — or k_search, k_emit), and for the search kernel
alone."""
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
LAUNCH = ("k_search", "k_emit", "k_scan", "k_group_")


def sums(path):
    """counter -> total over the launch kernels, the same over the search
    kernel alone, and the launch count (search-kernel dispatches)."""
    tot, srch = defaultdict(float), defaultdict(float)
    launches = set()
    for r in csv.DictReader(open_csv(path)):
        name = r["Kernel_Name"]
        if not any(k in name for k in LAUNCH):
            continue
        v = float(r["Counter_Value"])
        tot[r["Counter_Name"]] += v
        if "k_search" in name:
            launches.add(r["Dispatch_Id"])
            srch[r["Counter_Name"]] += v
    return tot, srch, max(len(launches), 1)


def bench_json(log):
    lines = [ln for ln in open(log) if ln.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def csv_of(d):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv") or f.endswith("counter_collection.csv.gz"):
                return os.path.join(root, f)
    raise SystemExit(f"no counter_collection.csv under {d}")


def main():
    tag = sys.argv[1]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else os.path.join(ROOT, "profiles",
                                                                                         "pmc_traffic.json")
    g = os.path.join(ROOT, "gpurun_out", tag)
    b = bench_json(os.path.join(g, "pmc_fetch.log"))
    key = b["profile_key"]
    ppl = b["roofline"]["kernel"]["patterns_per_launch"]
    alg = b["roofline"]["alg_bytes_per_pattern"]
    fetch, fetch_s, nl = sums(csv_of(os.path.join(g, "pmc_fetch")))
    ea, ea_s, nl2 = sums(csv_of(os.path.join(g, "pmc_ea")))
    wr, wr_s, nl3 = sums(csv_of(os.path.join(g, "pmc_write")))
    # (the TCC hit / miss pass is optional: PMC_SKIP_TCC=1 in scripts/gpu.sh)
    has_tcc = os.path.isdir(os.path.join(g, "pmc_tcc"))
    tcc, tcc_s, nl4 = sums(csv_of(os.path.join(g, "pmc_tcc"))) if has_tcc else ({}, {}, 1)

    def reads(e, n):
        n64, n128, nreq = e["TCC_EA0_RDREQ_64B_sum"] / n, e["TCC_EA0_RDREQ_128B_sum"] / n, e["TCC_EA0_RDREQ_sum"] / n
        n32 = max(nreq - n64 - n128, 0.0)
        return nreq, n32, n64, n128, 32 * n32 + 64 * n64 + 128 * n128

    nreq, n32, n64, n128, rd = reads(ea, nl2)
    sreq, _, _, _, srd = reads(ea_s, nl2)
    wb = wr["WRITE_SIZE"] * 1024 / nl3
    swb = wr_s["WRITE_SIZE"] * 1024 / nl3
    run = {
        "tag": tag, "source": f"rocprofv3 --pmc, scripts/gpu.sh {tag} pmc + scripts/traffic.py",
        "bench_config": b["config"], "launches_profiled": nl, "patterns_per_launch": ppl,
        "alg_bytes_per_pattern": alg,
        # the whole launch
        "fetch_size_bytes_per_launch": fetch["FETCH_SIZE"] * 1024 / nl,
        "fetch_size_x2_bytes_per_launch": 2 * fetch["FETCH_SIZE"] * 1024 / nl,
        "fabric_requests_per_launch": nreq, "requests_32b": n32, "requests_64b": n64, "requests_128b": n128,
        "fabric_bytes_per_launch": rd,
        "write_bytes_per_launch": wb,
        "traffic_bytes_per_launch": rd + wb,
        "l2_hit_rate": tcc["TCC_HIT_sum"] / max(tcc["TCC_HIT_sum"] + tcc["TCC_MISS_sum"], 1) if has_tcc else None,
        "l2_requests_per_pattern": (tcc["TCC_HIT_sum"] + tcc["TCC_MISS_sum"]) / nl4 / ppl if has_tcc else None,
        # the search kernel alone
        "search_kernel": {
            "fabric_requests_per_launch": sreq, "fabric_bytes_per_launch": srd, "write_bytes_per_launch": swb,
            "fetch_size_x2_bytes_per_launch": 2 * fetch_s["FETCH_SIZE"] * 1024 / nl,
            "fabric_requests_per_pattern": sreq / ppl, "traffic_bytes_per_pattern": (srd + swb) / ppl,
            "l2_hit_rate": (tcc_s["TCC_HIT_sum"] / max(tcc_s["TCC_HIT_sum"] + tcc_s["TCC_MISS_sum"], 1)
                            if has_tcc else None),
        },
    }
    run["fabric_bytes_per_pattern"] = rd / ppl
    run["fabric_requests_per_pattern"] = nreq / ppl
    run["traffic_bytes_per_pattern"] = (rd + wb) / ppl
    run["traffic_over_alg"] = run["traffic_bytes_per_pattern"] / alg
    db = json.load(open(out)) if os.path.exists(out) else {"runs": {}}
    db.setdefault("runs", {})[key] = run
    json.dump(db, open(out, "w"), indent=1, sort_keys=True)
    print(key, json.dumps(run, indent=1))


if __name__ == "__main__":
    main()
