#!/bin/bash
# Memory-pipeline / issue PMC passes of k_integrate in the driver's regime
# (bench --steps 20 --warmup 5: the unsaturated transient), per library:
#   tools/pmc_int.sh base|<var> ...   -> gpurun_out/pmci/<var>/p<k>
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
PASSES=(
  "TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum GRBM_GUI_ACTIVE"
  "TD_TD_BUSY_sum TD_TC_STALL_sum"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD"
  "SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
)
for v in "$@"; do
  if [ "$v" = base ]; then L="$ROOT/slam-kinectfusion_amd/lib/libkfx.so"; else L="$ROOT/slam-kinectfusion_amd/lib/var_$v/libkfx.so"; fi
  i=0
  for p in "${PASSES[@]}"; do
    i=$((i+1))
    echo "=== $v pass $i: $p"
    mkdir -p "$ROOT/gpurun_out/pmci/$v"
    KFX_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d "$ROOT/gpurun_out/pmci/$v/p$i" -- \
        python3 "$ROOT/bench.py" --steps 20 --warmup 5 --profile-frames 2 --cpu-frames 0 \
        > "$ROOT/gpurun_out/pmci/$v/p$i.log" 2>&1 || { echo "rc=$?"; tail -5 "$ROOT/gpurun_out/pmci/$v/p$i.log"; exit 1; }
  done
done
