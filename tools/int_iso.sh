# isolated k_integrate timing (tools/int_bench.py under rocprofv3 --kernel-trace
# --stats: the same C2 volume state integrated `reps` times, nothing running
# beside it) for each named library:  tools/int_iso.sh base|<var> ...
set -o pipefail
ROOT=$PWD
mkdir -p gpurun_out
for v in "$@"; do
  if [ $v = base ]; then L=$ROOT/slam-kinectfusion_amd/lib/libkfx.so; else L=$ROOT/slam-kinectfusion_amd/lib/var_$v/libkfx.so; fi
  (cd /tmp && export TMPDIR=/tmp && KFX_LIB_PATH=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $ROOT/gpurun_out/iso_$v -- python3 $ROOT/tools/int_bench.py 10 12 > $ROOT/gpurun_out/iso_$v.log 2>&1) || { tail -5 gpurun_out/iso_$v.log; exit 1; }
  python3 - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
for f in glob.glob(f"gpurun_out/iso_{v}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_integrate" in r["Name"] and "true, " not in r["Name"][:40]:
            print(v, r["Name"][:40], "calls", r["Calls"], "avg us %.1f" % (float(r["AverageNs"]) / 1e3),
                  "min %.1f max %.1f" % (float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
PY
done
