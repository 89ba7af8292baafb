#!/bin/bash
# VALU issue-counter calibration passes (tools/valu_calib.hip): the plain run
# (in-kernel cycles per instruction) and one rocprofv3 --pmc pass per counter
# group, under gpurun_out/<tag>/.  usage: tools/valu_calib.sh <tag>
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/gpurun_out/${1:-valu_calib}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 "$ROOT/tools/build/valu_calib" > "$OUT/plain.txt"
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES \
  --output-format csv -d "$OUT/pmc_a" -- "$ROOT/tools/build/valu_calib" > "$OUT/pmc_a.txt" 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc_b" -- "$ROOT/tools/build/valu_calib" > "$OUT/pmc_b.txt" 2>&1
timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -- "$ROOT/tools/build/valu_calib" \
  > "$OUT/trace.txt" 2>&1
echo "valu calibration done: $OUT"
