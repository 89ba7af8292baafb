#!/usr/bin/env python3
"""Tabulate hipcc -Rpass-analysis=kernel-resource-usage for a HIP source."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "slam-kinectfusion_amd/csrc/kfx_kernels.hip"
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
       "-c", src, "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = {}, None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?):\s+(.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = re.sub(r"^_ZN3kfx12_GLOBAL__N_1\d+", "", v)[:44]
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for f, d in rows.items():
    print(f"{f:46s} VGPR {d.get('VGPRs', '?'):>4} SGPR {d.get('TotalSGPRs', '?'):>4} "
          f"scratch {d.get('ScratchSize [bytes/lane]', '?'):>4} occ {d.get('Occupancy [waves/SIMD]', '?')} "
          f"LDS {d.get('LDS Size [bytes/block]', '?')}")
