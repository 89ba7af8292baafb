#!/bin/bash
# Build tuning variants of libkfx.so (in-tree, so they travel with gpurun):
#   tools/variants.sh name "-DKNOB=v ..." [name "-D..."]...
# -> slam-kinectfusion_amd/lib/var_<name>/libkfx.so ; run with KFX_LIB_PATH=<that>
set -e
cd "$(dirname "$0")/../slam-kinectfusion_amd"
while [ $# -ge 2 ]; do
  make -s ARCH=gfx950 OUT="lib/var_$1" EXTRA="$2" >/dev/null
  echo "built lib/var_$1 ($2)"
  shift 2
done
