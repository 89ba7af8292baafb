#!/bin/bash
# round 3, first GPU session: A/B of the integrate variants, GPU tests on the
# candidate library, then the HEAD profile (counters) of the baseline library.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
echo "== A/B"; bash tools/ab_quick.sh 3 base free nofree 2>&1 | tee gpurun_out/ab_r3a.log || exit 1
echo "== tests (var_free)"
KFX_LIB_PATH=$PWD/slam-kinectfusion_amd/lib/var_free/libkfx.so timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/tests_r3a.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3a.log; [ $rc -eq 0 ] || exit $rc
echo "== profile (var_free)"
KFX_LIB_PATH=$PWD/slam-kinectfusion_amd/lib/var_free/libkfx.so KFX_COMMIT=4dc4658+ PMC_RECORD=r03_free_pmc.json bash tools/prof.sh --steps 20 --warmup 5
