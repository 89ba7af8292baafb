#!/bin/bash
# integrate plan (k_int_plan): GPU tests on the default build, then A/B of chunk counts
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r3d.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3d.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_quick.sh 2 nofree base p3 p6 p8 p4g 2>&1 | tee gpurun_out/ab_r3d.log
