#!/usr/bin/env python3
"""Kernel timeline of a rocprofv3 --kernel-trace CSV: prints N consecutive frames
(starting at the k-th ICP launch) with each kernel's start/end relative to that
frame's ICP start, its queue/stream, and the gaps between frames.
usage: tools/timeline.py <kernel_trace.csv> [first_icp_index] [frames]"""
import csv
import re
import sys


def main():
    path = sys.argv[1]
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    nfr = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    rows = list(csv.DictReader(open(path)))
    if not rows:
        print("empty trace")
        return
    keys = rows[0].keys()
    kn = next(k for k in keys if k.lower() in ("kernel_name", "kernel-name"))
    ks = next(k for k in keys if "start" in k.lower() and "timestamp" in k.lower())
    ke = next(k for k in keys if "end" in k.lower() and "timestamp" in k.lower())
    kq = next((k for k in keys if k.lower() in ("queue_id", "stream_id")), None)
    ev = sorted(((int(r[ks]), int(r[ke]), (re.search(r"(k_\w+|__amd\w+)", r[kn]) or [r[kn][:40]])[0], r[kq] if kq else "?")
                 for r in rows))
    icp = [i for i, e in enumerate(ev) if "icp_track" in e[2]]
    if len(icp) < first + nfr + 1:
        first = max(0, len(icp) - nfr - 1)
    for f in range(first, first + nfr):
        i0, i1 = icp[f], icp[f + 1]
        t0 = ev[i0][0]
        print(f"--- frame {f}: icp start {t0}")
        for s, e, n, q in ev[i0 - 6:i1]:
            print(f"  {(s - t0) / 1e3:9.2f} {(e - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f}  q={q:>3} {n}")
    per = [(ev[icp[f + 1]][0] - ev[icp[f]][0]) / 1e3 for f in range(first, first + nfr)]
    print("icp-to-icp us:", ["%.1f" % p for p in per])


if __name__ == "__main__":
    main()
