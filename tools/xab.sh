#!/bin/bash
# extraction A/B (points + mesh records of bench.py) of the named libraries, alternating:
#   tools/xab.sh rounds [bench args] -- base|<var> ...
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
R=$1; shift
A=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do A+=("$1"); shift; done; shift
for r in $(seq $R); do
  for v in "$@"; do
    L=$PWD/slam-kinectfusion_amd/lib/libkfx.so; [ $v = base ] || L=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so
    KFX_LIB_PATH=$L timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-frames 0 --c1-frames 0 --c3-frames 0 \
      --c5-frames 0 --host-frames 0 "${A[@]}" > gpurun_out/xab_$v.json 2>&1 || { tail -5 gpurun_out/xab_$v.json; exit 1; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/xab_$v.json').read().strip().splitlines()[-1]);x=d['extract']
print('$v', {k: (x[k]['total_ms'], x[k]['items']) for k in ('points','mesh')})"
  done
done
