#!/usr/bin/env python3
"""Summarise global load / s_waitcnt vmcnt ordering per kernel in a saved .s
(L = global_load, Wn = s_waitcnt vmcnt(n), | = conditional branch)."""
import re
import sys

s = open(sys.argv[1]).read()
pats = sys.argv[2:] or ["k_"]
for m in re.finditer(r"^(_ZN3kfx\S+):\s", s, re.M):
    name = m.group(1)
    if not any(p in name for p in pats):
        continue
    body = s[m.end():s.find(".Lfunc_end", m.end())]
    lines = [l.strip() for l in body.splitlines() if l.startswith("\t") and not l.strip().startswith((".", ";"))]
    seq = []
    for l in lines:
        if "global_load" in l:
            seq.append("L")
        elif "s_waitcnt" in l and "vmcnt" in l:
            seq.append(" W" + re.search(r"vmcnt\((\d+)\)", l).group(1) + " ")
        elif l.startswith("s_cbranch"):
            seq.append("|")
    print(f"{name[:70]}: {len(lines)} instrs, {sum('global_load' in l for l in lines)} loads")
    print("   " + "".join(seq)[:1200])
