#!/bin/bash
# GPU tests with the exact fast-forward replay (default build), integrate chunking A/B, slab records
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r3k.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3k.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_quick.sh 3 base noff c100 w16 lpt 2>&1 | tee gpurun_out/ab_r3k.log || exit 1
timeout -k 10 300 python3 tools/slab_record.py c4 --out gpurun_out/r03_c4_slabs.json || exit 1
timeout -k 10 500 python3 tools/slab_record.py c5 --frames 10 --warmup 3 --out gpurun_out/r03_c5_slabs.json || exit 1
