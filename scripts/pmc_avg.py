"""Average rocprofv3 PMC counters per dispatch for kernels matching a name
fragment: python scripts/pmc_avg.py <run_counter_collection.csv> [fragment ...]"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
frags = sys.argv[2:] or ["k_"]
acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(dict)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    key = next((f for f in frags if f in name), None)
    if key is None:
        continue
    acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur[key][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for key, cs in acc.items():
    d = list(dur[key].values())
    print(f"{key}: dispatches={len(d)} avg_ns={sum(d) / len(d):.0f} vgpr/sgpr from csv")
    for c, v in cs.items():
        print(f"   {c} avg={sum(v) / len(v):.4g}")
