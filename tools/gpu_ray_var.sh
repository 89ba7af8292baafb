#!/bin/bash
# raycast timing + SQ instruction counters per variant: tools/gpu_ray_var.sh base|<var> ...
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
for v in "$@"; do
  if [ "$v" = base ]; then L="$ROOT/slam-kinectfusion_amd/lib/libkfx.so"; else L="$ROOT/slam-kinectfusion_amd/lib/var_$v/libkfx.so"; fi
  KFX_LIB_PATH=$L timeout -k 10 120 python3 "$ROOT/bench.py" --steps 100 --warmup 5 --cpu-frames 0 --profile-frames 2 > "$ROOT/gpurun_out/rv_$v.json" 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('$ROOT/gpurun_out/rv_$v.json').read().strip().splitlines()[-1]);print('$v',d['value'],d['timed_region_kernel_ms'])"
  (cd /tmp && TMPDIR=/tmp KFX_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d "$ROOT/gpurun_out/rvp/$v" -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --profile-frames 2 --cpu-frames 0 > "$ROOT/gpurun_out/rvp_$v.log" 2>&1) || exit 1
  python3 "$ROOT/tools/pmc_summary.py" "$ROOT/gpurun_out/rvp/$v" | grep -A9 "k_raycast<true, false, false>"
done
