#!/bin/bash
# per-wave integrate timelines (driver regime) + multi-GPU readiness records (C4, C5 in-process slabs)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for v in tr0 tr1; do
  echo "== $v"
  KFX_LIB_PATH=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so timeout -k 10 120 python3 tools/int_trace.py - 25 || exit 1
done
timeout -k 10 300 python3 tools/slab_record.py c4 --out gpurun_out/r03_c4_slabs.json || exit 1
timeout -k 10 400 python3 tools/slab_record.py c5 --frames 10 --warmup 3 --out gpurun_out/r03_c5_slabs.json || exit 1
