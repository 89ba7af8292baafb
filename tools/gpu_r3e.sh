#!/bin/bash
# kernel-trace of the planned integrate (default build): plan vs integrate split
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r3e
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/r3e/stats -o run -- \
  python3 bench.py --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --host-frames 0 --extract 0 \
  > gpurun_out/r3e/bench.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/r3e/stats/run_kernel_trace.csv 5 20 gpurun_out/r3e/summary.json | head -80
