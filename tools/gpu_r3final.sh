#!/bin/bash
# round-3 final tree: all GPU tests, the driver's bench line, the profiling
# session (stats + PMC traffic + SQ issue, tools/prof.sh), memory-pipeline counters
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
bash tools/gpu_full.sh || exit $?
bash tools/prof.sh --steps 20 --warmup 5 > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
tail -5 gpurun_out/prof.log
bash tools/pmc_mem.sh base > gpurun_out/pmcm.log 2>&1 || { tail -20 gpurun_out/pmcm.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmcm/base > gpurun_out/pmcm_base.txt
