#!/bin/bash
# integrate weight-divisor variants: parity tests on both, A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for v in rt0 rt2; do
  KFX_LIB_PATH=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "integrate or pipeline" --timeout 300 --timeout-method thread > gpurun_out/tests_r3ab_$v.log 2>&1; rc=$?
  tail -2 gpurun_out/tests_r3ab_$v.log; [ $rc -eq 0 ] || exit $rc
done
bash tools/ab_quick.sh 4 base rt0 rt2 2>&1 | tee gpurun_out/ab_r3ab.log || exit 1
