#!/bin/bash
# ICP coarse levels on one / two XCD groups: ICP tests on the variants, A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for v in xc1 xc2; do
  KFX_LIB_PATH=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "icp or pipeline" --timeout 120 --timeout-method thread > gpurun_out/tests_r3z_$v.log 2>&1; rc=$?
  tail -2 gpurun_out/tests_r3z_$v.log; [ $rc -eq 0 ] || exit $rc
done
bash tools/ab_quick.sh 4 base xc1 xc2 2>&1 | tee gpurun_out/ab_r3z.log || exit 1
