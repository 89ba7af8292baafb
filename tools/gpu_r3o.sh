#!/bin/bash
# integrate gather-dedupe A/B (alternating driver-command runs) + memory PMC passes of the variant
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
KFX_LIB_PATH=$PWD/slam-kinectfusion_amd/lib/var_dedup/libkfx.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r3o.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3o.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_quick.sh 3 base dedup dedup2 2>&1 | tee gpurun_out/ab_r3o.log || exit 1
bash tools/pmc_mem.sh dedup > gpurun_out/pmcm_dedup.log 2>&1 || { tail -20 gpurun_out/pmcm_dedup.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmcm/dedup > gpurun_out/pmcm_dedup.txt
timeout -k 10 180 python3 tools/host_input_probe.py > gpurun_out/host_probe.log 2>&1 || { tail -5 gpurun_out/host_probe.log; exit 1; }
cat gpurun_out/host_probe.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/hostprof -o run -- python3 $GRAFT_REPO_ROOT/tools/host_input_probe.py --frames 60 > $GRAFT_REPO_ROOT/gpurun_out/host_probe_prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/host_probe_prof.log; exit 1; }
