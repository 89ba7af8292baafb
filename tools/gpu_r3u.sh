#!/bin/bash
# integrate ZCLASS variant: parity + pipeline tests on it, A/B against base, its counters
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
KFX_LIB_PATH=$PWD/slam-kinectfusion_amd/lib/var_zc/libkfx.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_regimes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r3u.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3u.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_quick.sh 3 base zc pix3 2>&1 | tee gpurun_out/ab_r3u.log || exit 1
bash tools/pmc_mem.sh zc > gpurun_out/pmcm_zc.log 2>&1 || { tail -20 gpurun_out/pmcm_zc.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmcm/zc > gpurun_out/pmcm_zc.txt
