"""Per-leg kernel averages from a rocprofv3 kernel trace of the default bench
command: the faithful leg (k_search<..., 0>) and the derived-index leg
(k_search<..., 1|2>) share k_emit's name, so rocprofv3's own stats mix them;
this splits the dispatches at the derived leg's first k_search.

    python scripts/trace_legs.py gpurun_out/<tag>_trace/run_kernel_trace.csv"""
import csv
import json
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
split = next((int(r["Start_Timestamp"]) for r in rows
              if "k_search" in r["Kernel_Name"] and not r["Kernel_Name"].rstrip(")").endswith("0>(fmx::QueryArgs, fmx::LocateGroup, unsigned int")
              and ", 0>(" not in r["Kernel_Name"]), None)
legs = {"faithful": defaultdict(list), "derived": defaultdict(list)}
for r in rows:
    name = r["Kernel_Name"]
    key = next((k for k in ("k_search", "k_emit", "k_scan") if f"fmx::{k}" in name), None)
    if key is None:
        continue
    leg = "derived" if split is not None and int(r["Start_Timestamp"]) >= split else "faithful"
    legs[leg][key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = {leg: {k: {"dispatches": len(v), "avg_us": sum(v) / len(v) / 1e3, "min_us": min(v) / 1e3}
             for k, v in d.items()} for leg, d in legs.items()}
print(json.dumps(out, indent=1))
