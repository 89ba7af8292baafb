#!/bin/bash
# slab records of the named libraries: tools/slab_ab.sh c4|c5 base|<var> ...
# (SLAB_GROUPS: the cut sets slab_record.py times, default "equal,calibrated")
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
C=$1; shift
G=${SLAB_GROUPS:-equal,calibrated}
for v in "$@"; do
  L=$PWD/slam-kinectfusion_amd/lib/libkfx.so; [ $v = base ] || L=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so
  echo "== $v"
  KFX_LIB_PATH=$L timeout -k 10 600 python3 tools/slab_record.py $C --groups $G --out gpurun_out/slab_${C}_$v.json > gpurun_out/slab_${C}_$v.log 2>&1 || { tail -5 gpurun_out/slab_${C}_$v.log; exit 1; }
  tail -n 4 gpurun_out/slab_${C}_$v.log
done
