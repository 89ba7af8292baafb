#!/usr/bin/env python3
"""Summary of a tools/valu_calib.sh directory -> profiles/<name>.json: per
calibration kernel the in-kernel cycles per wave-instruction (plain run) and
the SQ counters per dispatch, with the counts per instruction they imply.
usage: python3 tools/valu_calib_summary.py gpurun_out/r06_valu_calib profiles/r06_valu_calib.json"""
import collections
import csv
import glob
import json
import re
import sys

root, out = sys.argv[1], sys.argv[2]
rec = {"source": "tools/valu_calib.hip (8 waves per SIMD on every SIMD, 16 independent instructions "
                 "x 4096 iterations per wave) via tools/valu_calib.sh", "kernels": {}}
for line in open(f"{root}/plain.txt"):
    m = re.match(r"(\S+)\s+waves.*cycles/instr per SIMD: min ([\d.]+) med ([\d.]+) max ([\d.]+)", line)
    if m:
        rec["kernels"].setdefault(m.group(1), {})["cycles_per_wave_instruction"] = {
            "min": float(m.group(2)), "med": float(m.group(3)), "max": float(m.group(4))}
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in ("pmc_a", "pmc_b"):
    for f in glob.glob(f"{root}/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].strip()
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    if k not in rec["kernels"]:
        continue
    c = {n: sum(v) / len(v) for n, v in cs.items()}
    e = rec["kernels"][k]
    e["counters_per_dispatch"] = c
    I = c.get("SQ_INSTS_VALU")
    if I:
        e["active_inst_valu_per_instruction"] = round(c.get("SQ_ACTIVE_INST_VALU", 0.0) / I, 3)
        cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        med = e["cycles_per_wave_instruction"]["med"]
        e["issue_busy_frac"] = round(med * I / (1024 * cyc), 4) if cyc else None
        e["four_x_active_over_simd_cycles"] = round(4.0 * c.get("SQ_ACTIVE_INST_VALU", 0.0) / (1024 * cyc), 4)
rec["reading"] = ("SQ_INSTS_VALU counts one per wave-instruction.  SQ_ACTIVE_INST_VALU counts 1 per "
                  "v_add_f32 (2 cycles), v_pk_fma_f32 (4) and v_mad_u32_u24 (4), 2 per v_rcp_f32 (8): "
                  "4 x ACTIVE is the issue time only for 4-cycle instructions and doubles it for 2-cycle ones, "
                  "so 4 x ACTIVE / SIMD-cycles (round 5's valu_active_frac) exceeds 1 on 2-cycle-heavy "
                  "kernels.  Issue cycles lie in [6 ACTIVE - 4 INSTS, 4 ACTIVE] (tools/traffic.py sq_issue).")
json.dump(rec, open(out, "w"), indent=1)
print(json.dumps({k: (v.get("cycles_per_wave_instruction", {}).get("med"), v.get("active_inst_valu_per_instruction"),
                      v.get("issue_busy_frac"), v.get("four_x_active_over_simd_cycles"))
                  for k, v in rec["kernels"].items()}, indent=1))
