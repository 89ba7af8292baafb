#!/bin/bash
# integrate lean-update variants: parity tests on lean3, A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
KFX_LIB_PATH=$PWD/slam-kinectfusion_amd/lib/var_lean3/libkfx.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_regimes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r3aa.log 2>&1; rc=$?
tail -2 gpurun_out/tests_r3aa.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_quick.sh 3 base lean1 lean2 lean3 2>&1 | tee gpurun_out/ab_r3aa.log || exit 1
