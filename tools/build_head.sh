#!/bin/bash
# build the committed (HEAD) library as lib/var_head for A/B runs against the working tree
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p "$T/include" "$T/slam-kinectfusion_amd/csrc" "$T/slam-kinectfusion_amd/examples"
git -C "$R" show HEAD:include/kfx.h > "$T/include/kfx.h"
for f in Makefile csrc/kfx_kernels.hip csrc/kfx_api.hip csrc/kfx_dataset.cpp csrc/kfx_internal.h csrc/kfx_ffadd.h examples/kfx_run.cpp; do
  git -C "$R" show "HEAD:slam-kinectfusion_amd/$f" > "$T/slam-kinectfusion_amd/$f"
done
make -C "$T/slam-kinectfusion_amd" -j8 OUT="$R/slam-kinectfusion_amd/lib/var_head" "$R/slam-kinectfusion_amd/lib/var_head/libkfx.so" EXTRA="$*" > /dev/null
rm -rf "$T"
echo "built lib/var_head"
