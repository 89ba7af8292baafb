#!/usr/bin/env python3
"""Per-basic-block instruction budget of the shipped k_integrate<false, true>
main loop (VALU / SALU / memory per block, in code order), from the gfx950
assembly of csrc/kfx_kernels.hip.  usage: tools/isa_budget.py [out.txt]"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(ROOT, "slam-kinectfusion_amd", "csrc", "kfx_kernels.hip")
asm = "/tmp/kfx_isa_budget.s"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                "-fno-fast-math", "--cuda-device-only", "-S", src, "-o", asm], check=True, capture_output=True)
text = open(asm).read()
m = [x for x in re.finditer(r"^(_ZN3kfx\S+):\s", text, re.M) if "k_integrateILb0ELb1EE" in x.group(1)][0]
body = text[m.end():text.find(".Lfunc_end", m.end())].splitlines()
# the main loop: the loop whose blocks hold the depth gathers (buffer_load_dwordx2)
blocks, cur = [], None
for line in body:
    mm = re.match(r"^(\.LBB\w+|; %bb\.\d+):(.*)", line)
    if mm:
        hdr = re.search(r"Header=(BB\w+)", mm.group(2))
        loop = hdr.group(1) if hdr else (mm.group(1)[2:] if "Loop Header" in mm.group(2) else None)
        cur = [mm.group(1), loop, collections.Counter()]
        blocks.append(cur)
        continue
    t = line.strip()
    if cur and line.startswith("\t") and t and not t.startswith((".", ";")):
        cur[2][t.split()[0]] += 1
loops = collections.defaultdict(int)
for b in blocks:
    if b[1]:
        loops[b[1]] += b[2]["buffer_load_dwordx2"]
# the z loops: one per path since round 4 (packed exact / IEEE), each with the
# batch's depth gathers; the fast one's sqrt is v_rsq_f32 + Newton
mains = [l for l, n in loops.items() if n > 0]
out = []
for main in mains:
    rsq = sum(n for _, loop, c in blocks if loop == main for k, n in c.items() if k.startswith("v_rsq"))
    kind = "fast path (packed exact projection, rsq-Newton sqrt)" if rsq else "IEEE path (tiny / huge operands)"
    out += [f"k_integrate<false, true> z loop {main}, {kind}: per basic block (code order)",
            f"{'block':14s} {'VALU':>5s} {'SALU':>5s} {'VMEM':>5s} {'LDS':>4s}  notable"]
    tot = collections.Counter()
    for name, loop, c in blocks:
        if loop != main:
            continue
        v = sum(n for k, n in c.items() if k.startswith("v_"))
        sa = sum(n for k, n in c.items() if k.startswith("s_"))
        vm = sum(n for k, n in c.items() if k.startswith(("buffer_", "global_")))
        ds = sum(n for k, n in c.items() if k.startswith("ds_"))
        tot.update({"VALU": v, "SALU": sa, "VMEM": vm, "LDS": ds})
        note = ", ".join(f"{k} {n}" for k, n in c.most_common() if k.startswith(("v_rcp", "v_rsq", "v_pk_", "buffer_load",
                                                                                    "buffer_store", "v_readlane", "ds_")))[:90]
        out.append(f"{name:14s} {v:5d} {sa:5d} {vm:5d} {ds:4d}  {note}")
    out.append(f"{'loop total':14s} {tot['VALU']:5d} {tot['SALU']:5d} {tot['VMEM']:5d} {tot['LDS']:4d}  (static)")
    out.append("")
text_out = "\n".join(out)
print(text_out)
if len(sys.argv) > 1:
    open(sys.argv[1], "w").write(text_out + "\n")
