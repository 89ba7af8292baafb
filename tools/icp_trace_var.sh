#!/bin/bash
# ICP phase trace per variant library: tools/icp_trace_var.sh var...
for v in "$@"; do
  echo "== $v"
  KFX_LIB_PATH="$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so" timeout -k 10 100 python3 tools/icp_trace.py | grep -E "per-iteration|lane|block reduce|solve|sums read" || exit $?
done
