#!/bin/bash
# slab raycast pre-skip: slab tests, C4 / C5 slab records
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_slab.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r3s.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3s.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/slab_record.py c4 --out gpurun_out/r03_c4_slabs_skip.json || exit 1
timeout -k 10 500 python3 tools/slab_record.py c5 --frames 10 --warmup 3 --out gpurun_out/r03_c5_slabs_skip.json || exit 1
