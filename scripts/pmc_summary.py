"""Fold one scripts/profile.sh run (gpurun_out/<TAG>_trace, _pmc1.._pmc4) into
profiles/pmc_fetch_size.json under the bench's profile key, and copy the
kernel-stats summary to profiles/<TAG>_kernel_stats.csv.

usage: python scripts/pmc_summary.py TAG [--kernel k_locate]
The key is read from the bench JSON line in gpurun_out/<TAG>_trace.log
("profile_key": "<config>:<n>:<batch>:<m>:<options>:<deep_lut_k>")."""
import argparse
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def bench_line(path):
    for line in open(path, errors="replace"):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise SystemExit(f"no bench JSON line in {path}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="k_search,k_scan,k_emit,k_locate",
                    help="comma-separated kernel names making up one locate step; per-dispatch means are summed")
    ap.add_argument("--json", default=os.path.join(ROOT, "profiles", "pmc_fetch_size.json"))
    args = ap.parse_args()
    b = bench_line(os.path.join(OUT, f"{args.tag}_trace.log"))
    key = b["profile_key"]
    run = {"counters": {}}
    name = None
    durations = []
    kernels = [k for k in args.kernel.split(",") if k]

    def which(kname):
        for k in kernels:
            if f"fmx::{k}<" in kname or f"fmx::{k}(" in kname:
                return k
        return None

    names = set()
    for d in sorted(glob.glob(os.path.join(OUT, f"{args.tag}_pmc*"))):
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # counter -> kernel -> dispatch
        for r in csv.DictReader(open(f)):
            k = which(r["Kernel_Name"])
            if k is None:
                continue
            names.add(r["Kernel_Name"])
            per[r["Counter_Name"]][k][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for cn, byk in per.items():
            # one locate step = one dispatch of each of its kernels: sum the per-kernel means
            launches = max(len(by) for by in byk.values())
            run["counters"][cn] = {"launches": launches,
                                   "mean_per_launch": sum(sum(by.values()) / len(by) for by in byk.values())}
    stats = os.path.join(OUT, f"{args.tag}_trace", "run_kernel_stats.csv")
    avg, calls = 0.0, 0
    for r in csv.DictReader(open(stats)):
        if which(r["Name"]):
            avg += float(r["AverageNs"])
            calls = max(calls, int(r["Calls"]))
    run["avg_duration_ns"] = avg  # summed over the step's kernels
    run["launches"] = calls
    name = " + ".join(sorted(names))
    run["kernel"] = name
    c = run["counters"]
    if "FETCH_SIZE" in c:
        run["hbm_bytes_per_launch"] = c["FETCH_SIZE"]["mean_per_launch"] * 1024
    if "TCC_EA0_RDREQ_sum" in c:
        run["rdreq_x64B_per_launch"] = c["TCC_EA0_RDREQ_sum"]["mean_per_launch"] * 64
    run["bench_value"] = b["value"]
    run["tag"] = args.tag
    doc = json.load(open(args.json)) if os.path.exists(args.json) else {"runs": {}}
    doc["runs"][key] = run
    json.dump(doc, open(args.json, "w"), indent=1)
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"{args.tag}_kernel_stats.csv"))
    print(key, json.dumps({k: v for k, v in run.items() if k != "counters"}))
    for cn, v in sorted(c.items()):
        print(f"  {cn:28s} {v['mean_per_launch']:.1f}")


if __name__ == "__main__":
    sys.exit(main())
