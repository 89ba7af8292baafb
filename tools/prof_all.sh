#!/bin/bash
# The round's profiling session on one GPU box (tools/prof.sh per config):
#   C2 driver command -> gpurun_out/prof     + profiles/r05_integrate_pmc.json copy
#   C3 record regime  -> gpurun_out/prof_c3  + r05_c3_pmc.json
#   C5 record regime  -> gpurun_out/prof_c5  + r05_c5_pmc.json
# (bench.py attaches each PMC record only to a run of the same workload, step
# counts and libkfx.so sha256).  usage: KFX_COMMIT=<sha> bash tools/prof_all.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
PROF_OUT=gpurun_out/prof PMC_RECORD=r05_integrate_pmc.json bash tools/prof.sh --steps 20 --warmup 5 || exit $?
PROF_OUT=gpurun_out/prof_c3 PMC_RECORD=r05_c3_pmc.json bash tools/prof.sh --config c3 --steps 20 --warmup 5 \
  --profile-frames 0 --extract 0 --cpu-frames 0 --c1-frames 0 --host-frames 0 || exit $?
PROF_OUT=gpurun_out/prof_c5 PMC_RECORD=r05_c5_pmc.json bash tools/prof.sh --config c5 --steps 10 --warmup 5 \
  --profile-frames 0 --extract 0 --cpu-frames 0 --c1-frames 0 --host-frames 0 || exit $?
echo "prof_all done"
