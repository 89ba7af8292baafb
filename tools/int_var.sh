#!/bin/bash
# k_integrate kernel time on a fixed volume state per library (tools/int_bench.py
# under rocprofv3 kernel trace): tools/int_var.sh frames base|<var> ...
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
F=$1; shift
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then L="$ROOT/slam-kinectfusion_amd/lib/libkfx.so"; else L="$ROOT/slam-kinectfusion_amd/lib/var_$v/libkfx.so"; fi
  mkdir -p "$ROOT/gpurun_out/intv"
  KFX_LIB_PATH=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/intv/$v.$F" -o run -- \
      python3 "$ROOT/tools/int_bench.py" $F 8 > "$ROOT/gpurun_out/intv/$v.$F.log" 2>&1 || { echo "rc=$? $v"; tail -5 "$ROOT/gpurun_out/intv/$v.$F.log"; exit 1; }
  python3 - "$ROOT/gpurun_out/intv/$v.$F" "$v" <<'PY'
import csv, glob, sys
rows = [r for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True) for r in csv.DictReader(open(f))]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_integrate<false, true>" in r["Kernel_Name"]]
d = d[-8:]
print(f"{sys.argv[2]:8s} integrate us: " + " ".join(f"{x:.1f}" for x in d) + f"  median {sorted(d)[len(d)//2]:.1f}")
PY
done
