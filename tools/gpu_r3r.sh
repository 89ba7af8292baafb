#!/bin/bash
# ICP 3+3 block solve: all GPU tests, A/B against HEAD (LDLt solve)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r3r.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3r.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_quick.sh 4 base head 2>&1 | tee gpurun_out/ab_r3r.log || exit 1
