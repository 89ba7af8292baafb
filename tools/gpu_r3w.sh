#!/bin/bash
# host fetch: low-priority copy stream; grid size A/B in the host-input probe
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for v in base fetch16 fetch256 base; do
  if [ $v = base ]; then L=$PWD/slam-kinectfusion_amd/lib/libkfx.so; else L=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so; fi
  echo "== $v"
  KFX_LIB_PATH=$L timeout -k 10 180 python3 -u tools/host_input_probe.py --frames 150 > gpurun_out/host_probe_$v.log 2>&1 || { tail -5 gpurun_out/host_probe_$v.log; exit 1; }
  grep -E "direct|staged " gpurun_out/host_probe_$v.log
done
