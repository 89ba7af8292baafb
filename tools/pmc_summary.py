#!/usr/bin/env python3
"""Aggregate rocprofv3 counter_collection.csv files per kernel (mean per dispatch)."""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "?")
        key = name.replace("kfx::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
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
