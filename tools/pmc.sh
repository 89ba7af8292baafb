#!/bin/bash
# PMC passes on a short bench run, one rocprofv3 run per counter group (counters
# never combined with trace domains).  Output: gpurun_out/pmc/<pass>/...
# usage: tools/pmc.sh [bench args...]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
ARGS=${@:-"--steps 20 --warmup 5 --profile-frames 2 --cpu-frames 0"}
PASSES=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
  "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT TCC_MISS"
  "GRBM_GUI_ACTIVE GRBM_COUNT"
)
mkdir -p "$ROOT/gpurun_out/pmc"
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  echo "=== pmc pass $i: $p"
  timeout -k 10 240 rocprofv3 --pmc $p --output-format csv -d "$ROOT/gpurun_out/pmc/p$i" -- \
      python3 "$ROOT/bench.py" $ARGS > "$ROOT/gpurun_out/pmc/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$ROOT/gpurun_out/pmc/p$i.log"; exit $rc; fi
done
