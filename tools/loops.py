#!/usr/bin/env python3
"""Loops of one kernel in a gfx950 .s: instruction mix per loop (nested loops
are counted in every enclosing loop).  usage: loops.py file.s kernel_substring"""
import collections
import re
import sys

src = open(sys.argv[1]).read()
m = [x for x in re.finditer(r"^(_ZN3kfx\S+):\s", src, re.M) if sys.argv[2] in x.group(1)][0]
body = src[m.end():src.find(".Lfunc_end", m.end())].splitlines()
ins = [l for l in body if l.startswith("\t") and not l.strip().startswith((".", ";"))]
print("function instrs", len(ins))
for i, l in enumerate(body):
    mm = re.match(r"^(\.LBB\w+):", l)
    if not mm:
        continue
    lab = mm.group(1)
    ends = [j for j, x in enumerate(body) if j > i and re.search(r"s_c?branch\w*\s+" + re.escape(lab) + r"\b", x)]
    if not ends:
        continue
    seg = [x.strip().split()[0] for x in body[i:max(ends) + 1] if x.startswith("\t") and not x.strip().startswith((".", ";"))]
    c = collections.Counter(seg)
    print(f"{lab:12s} lines {i}-{max(ends)} len {len(seg):5d} VALU {sum(n for k, n in c.items() if k.startswith('v_')):5d} "
          f"SALU {sum(n for k, n in c.items() if k.startswith('s_')):4d} VMEM {sum(n for k, n in c.items() if k.startswith(('buffer', 'global'))):3d} "
          f"SMEM {sum(n for k, n in c.items() if k.startswith('s_load') or k.startswith('s_buffer_load')):3d}")
