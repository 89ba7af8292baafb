#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration for the access widths kfx uses (tools/pmc_calib.hip).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p "$ROOT/gpurun_out/calib"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d "$ROOT/gpurun_out/calib/$c" -- \
      "$ROOT/tools/build/pmc_calib" > "$ROOT/gpurun_out/calib/$c.log" 2>&1 || exit $?
done
python3 "$ROOT/tools/pmc_summary.py" "$ROOT/gpurun_out/calib"
