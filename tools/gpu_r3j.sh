#!/bin/bash
# GPU tests on the default build, raycast scalar-replay A/B, slab records with balanced cuts
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r3j.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3j.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_quick.sh 2 base rsr 2>&1 | tee gpurun_out/ab_r3j.log || exit 1
timeout -k 10 300 python3 tools/slab_record.py c4 --out gpurun_out/r03_c4_slabs.json || exit 1
timeout -k 10 500 python3 tools/slab_record.py c5 --frames 10 --warmup 3 --out gpurun_out/r03_c5_slabs.json || exit 1
