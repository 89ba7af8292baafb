#!/bin/bash
# wave priority A/B (integrate long chunks, raycast tail waves); fetch grid 4 vs 16
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
bash tools/ab_quick.sh 3 base iprio2 rprio3 rprio6 2>&1 | tee gpurun_out/ab_r3x.log || exit 1
for v in base fetch4; do
  if [ $v = base ]; then L=$PWD/slam-kinectfusion_amd/lib/libkfx.so; else L=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so; fi
  echo "== $v"
  KFX_LIB_PATH=$L timeout -k 10 180 python3 -u tools/host_input_probe.py --frames 150 > gpurun_out/host_probe_$v.log 2>&1 || { tail -5 gpurun_out/host_probe_$v.log; exit 1; }
  grep -E "direct|staged " gpurun_out/host_probe_$v.log
done
