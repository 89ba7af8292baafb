#!/usr/bin/env python3
"""Per-kernel launch durations from a rocprofv3 --kernel-trace run of bench.py:
mean over every dispatch and over the timed region's dispatches (the frames
after `warmup`, `steps` of them), to set beside the bench line's HIP-event
figure (roofline.avg_launch_ms, timed_region_kernel_ms).
usage: prof_summary.py <kernel_trace.csv> <warmup> <steps> [out.json]"""
import csv
import json
import re
import sys

import numpy as np


def main():
    path, warmup, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    rows = list(csv.DictReader(open(path)))
    per = {}
    for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
        m = re.search(r"(k_\w+(<[^>]*>)?|__amd\w+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        per.setdefault(name, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {}
    for name, d in sorted(per.items()):
        d = np.array(d)
        e = {"dispatches": len(d), "mean_us_all": round(float(d.mean()), 2),
             "median_us_all": round(float(np.median(d)), 2)}
        if (name in ("k_icp_track", "k_raycast<true, false, false>") or name.startswith("k_integrate<false, true")) and len(d) >= warmup + steps:
            t = d[warmup:warmup + steps]
            e["mean_us_timed_region"] = round(float(t.mean()), 2)
        out[name] = e
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 4:
        json.dump(out, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
