#!/bin/bash
# per-wave integrate timelines in the driver regime (25 frames): unplanned 3 chunks vs planned 4 chunks
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
for v in tr0 tr1; do
  echo "== $v"
  KFX_LIB_PATH=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so timeout -k 10 120 python3 tools/int_trace.py - 25 || exit 1
done
