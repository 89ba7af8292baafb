#!/usr/bin/env python3
"""Opcode histogram of kernels in a saved gfx950 .s (whole function body)."""
import collections
import re
import sys

s = open(sys.argv[1]).read()
for m in re.finditer(r"^(_ZN3kfx\S+):\s", s, re.M):
    name = m.group(1)
    if not any(p in name for p in sys.argv[2:] or ["k_"]):
        continue
    body = s[m.end():s.find(".Lfunc_end", m.end())]
    ops = [l.strip().split()[0] for l in body.splitlines()
           if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
    c = collections.Counter(ops)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    salu = sum(v for k, v in c.items() if k.startswith("s_") and not k.startswith(("s_waitcnt", "s_nop")))
    print(f"{name[:60]}: {len(ops)} instrs, VALU {valu}, SALU {salu}, div_f32 {c['v_div_fixup_f32']}, "
          f"sqrt {c['v_sqrt_f32_e32']}, nop {c['s_nop']}")
    print("   ", c.most_common(24))
