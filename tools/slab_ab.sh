#!/bin/bash
# slab records of the named libraries: tools/slab_ab.sh c4|c5 base|<var> ...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
C=$1; shift
for v in "$@"; do
  L=$PWD/slam-kinectfusion_amd/lib/libkfx.so; [ $v = base ] || L=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so
  KFX_LIB_PATH=$L timeout -k 10 600 python3 tools/slab_record.py $C --out gpurun_out/slab_${C}_$v.json > gpurun_out/slab_${C}_$v.log 2>&1 || { tail -5 gpurun_out/slab_${C}_$v.log; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/slab_${C}_$v.json'))

for n in ('balanced_cuts_unbounded', 'calibrated_cuts_unbounded'):
  k=d[n];print('$v', n[:5], 'int', [round(s['integrate_ms'],3) for s in k['slabs']], 'ray', [round(s['raycast_local_ms'],3) for s in k['slabs']], 'crit+comb', round(k['max_rank_icp_integrate_raycast_combine_ms'],3), 'single', round(d['single']['raycast_ms'],3))"
done
