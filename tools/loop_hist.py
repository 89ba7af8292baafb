#!/usr/bin/env python3
"""Instruction histogram of the largest loop body of one kernel in a gfx950 .s.
usage: loop_hist.py file.s kernel_substring"""
import collections
import re
import sys

src = open(sys.argv[1]).read()
m = [x for x in re.finditer(r"^(_ZN3kfx\S+):\s", src, re.M) if sys.argv[2] in x.group(1)][0]
body = src[m.end():src.find(".Lfunc_end", m.end())].splitlines()
hdr = [i for i, l in enumerate(body) if "Loop Header" in l]
best = None
for h in hdr:
    lab = body[h].split(":")[0]
    ends = [i for i, l in enumerate(body) if re.search(r"s_c?branch\w*\s+" + re.escape(lab) + r"\b", l)]
    if ends:
        e = max(ends)
        if best is None or e - h > best[1] - best[0]:
            best = (h, e)
h, e = best
ops = [l.strip().split()[0] for l in body[h:e + 1]
       if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
c = collections.Counter(ops)
valu = sum(v for k, v in c.items() if k.startswith("v_"))
salu = sum(v for k, v in c.items() if k.startswith("s_") and not k.startswith(("s_waitcnt", "s_nop")))
print(f"loop {body[h].split(':')[0]}: {len(ops)} instrs, VALU {valu}, SALU {salu}")
print(c.most_common(40))
