#!/bin/bash
# Per-kernel durations of the raycast launches (k_raycast, k_ray_tail, the
# deferred k_resize) in a short bench run, per library variant (GPU box, from
# the repo root through gpurun):
#   tools/ray_kernels.sh base|<var> ...   (var = slam-kinectfusion_amd/lib/var_<var>)
# -> gpurun_out/rk_<var>/ and one summary line per variant
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then L=$ROOT/slam-kinectfusion_amd/lib/libkfx.so; else L=$ROOT/slam-kinectfusion_amd/lib/var_$v/libkfx.so; fi
  OUT=$ROOT/gpurun_out/rk_$v
  mkdir -p "$OUT"
  KFX_LIB_PATH=$L timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --c5-frames 0 \
    --host-frames 0 --extract 0 > "$OUT/run.log" 2>&1 || { tail -5 "$OUT/run.log"; exit 1; }
  python3 - "$OUT/run_kernel_trace.csv" "$v" <<'EOF'
import csv, sys
from collections import defaultdict
d = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    for k in ("k_raycast<", "k_ray_tail", "k_resize", "k_integrate<", "k_icp_track"):
        if k in n:
            d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(sys.argv[2], " ".join(f"{k.rstrip('<')} {sum(x[-20:]) / len(x[-20:]):.1f}us(n{len(x)})" for k, x in d.items() if x))
EOF
done
