#!/bin/bash
# ICP 3+3 block solve + slab raycast pre-skip: all GPU tests, A/B vs HEAD, C4/C5 slab records
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r3t.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3t.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_quick.sh 4 base head 2>&1 | tee gpurun_out/ab_r3t.log || exit 1
timeout -k 10 300 python3 tools/slab_record.py c4 --out gpurun_out/r03_c4_slabs_skip.json || exit 1
timeout -k 10 500 python3 tools/slab_record.py c5 --frames 10 --warmup 3 --out gpurun_out/r03_c5_slabs_skip.json || exit 1
