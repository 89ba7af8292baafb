#!/usr/bin/env python3
"""Aggregate rocprofv3 counter_collection.csv files per kernel (mean per dispatch)."""
import collections
import csv
import glob
import json
import sys

# usage: pmc_summary.py [root] [last]   (last: only each kernel's last N dispatches, steady state)
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
last = int(sys.argv[2]) if len(sys.argv) > 2 else 0
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r.get("Dispatch_Id", 0)))
    for r in rows:
        name = r.get("Kernel_Name", "?")
        key = name.replace("kfx::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
if last:
    for d in agg.values():
        for c in d:
            d[c] = d[c][-last:]
out = {}
for k, d in sorted(agg.items()):
    out[k] = {c: sum(v) / len(v) for c, v in d.items()}
    out[k]["dispatches"] = max(len(v) for v in d.values())
import os
if os.path.isdir(root):
    json.dump(out, open(f"{root}/summary.json", "w"), indent=1)
for k, d in out.items():
    if not k.startswith("k_"):
        continue
    print(k)
    for c in sorted(d):
        print(f"   {c:28s} {d[c]:16.1f}")
