#!/bin/bash
# Memory-pipeline and issue PMC passes of the driver regime (or BENCH_ARGS), per
# variant library:  tools/pmc_mem.sh base|<var> ...   -> gpurun_out/pmcm/<var>/p<k>
# Summarise with tools/pmc_summary.py gpurun_out/pmcm/<var>.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 20 --warmup 5"}
PASSES=(
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
  "TD_TD_BUSY_sum TD_TC_STALL_sum"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum"
  "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY"
  "SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_INSTS_SMEM"
)
for v in "$@"; do
  if [ "$v" = base ]; then L="$ROOT/slam-kinectfusion_amd/lib/libkfx.so"; else L="$ROOT/slam-kinectfusion_amd/lib/var_$v/libkfx.so"; fi
  mkdir -p "$ROOT/gpurun_out/pmcm/$v"
  i=0
  for p in "${PASSES[@]}"; do
    i=$((i+1))
    echo "=== $v pass $i: $p"
    KFX_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d "$ROOT/gpurun_out/pmcm/$v/p$i" -- \
        python3 "$ROOT/bench.py" $ARGS --profile-frames 2 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --c5-frames 0 --host-frames 0 --extract 0 \
        > "$ROOT/gpurun_out/pmcm/$v/p$i.log" 2>&1 || { echo "rc=$?"; tail -5 "$ROOT/gpurun_out/pmcm/$v/p$i.log"; exit 1; }
  done
done
