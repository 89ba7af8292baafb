#!/bin/bash
# Memory-pipeline PMC passes in integrate's steady state (frames past the
# saturation transient), per variant library:
#   tools/pmc_steady.sh base|<var> ...   -> gpurun_out/pmcs/<var>/p<k>
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
PASSES=(
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
  "TD_TD_BUSY_sum TD_TC_STALL_sum"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum"
  "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY"
  "TCC_HIT_sum TCC_MISS_sum"
  "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM"
)
for v in "$@"; do
  if [ "$v" = base ]; then L="$ROOT/slam-kinectfusion_amd/lib/libkfx.so"; else L="$ROOT/slam-kinectfusion_amd/lib/var_$v/libkfx.so"; fi
  i=0
  mkdir -p "$ROOT/gpurun_out/pmcs/$v"
  for p in "${PASSES[@]}"; do
    i=$((i+1))
    echo "=== $v pass $i: $p"
    KFX_LIB_PATH=$L timeout -k 10 120 rocprofv3 --pmc $p --output-format csv -d "$ROOT/gpurun_out/pmcs/$v/p$i" -- \
        python3 "$ROOT/bench.py" --steps 40 --warmup 100 --profile-frames 2 --cpu-frames 0 \
        > "$ROOT/gpurun_out/pmcs/$v/p$i.log" 2>&1 || { echo "rc=$?"; tail -5 "$ROOT/gpurun_out/pmcs/$v/p$i.log"; exit 1; }
  done
done
