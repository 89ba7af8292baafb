#!/bin/bash
# The round's profiling session on one GPU box (tools/prof.sh per config):
#   C2 driver command -> gpurun_out/prof     + profiles/${R}_integrate_pmc.json
#   C3 record regime  -> gpurun_out/prof_c3  + ${R}_c3_pmc.json
#   C5 record regime  -> gpurun_out/prof_c5  + ${R}_c5_pmc.json
# (R = the round prefix, default r06)
# (bench.py attaches each PMC record only to a run of the same workload, step
# counts and libkfx.so sha256).  usage: KFX_COMMIT=<sha> bash tools/prof_all.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
R=${R:-r06}
cd "$ROOT" || exit 1
PROF_OUT=gpurun_out/prof PMC_RECORD=${R}_integrate_pmc.json bash tools/prof.sh --steps 20 --warmup 5 || exit $?
PROF_OUT=gpurun_out/prof_c3 PMC_RECORD=${R}_c3_pmc.json bash tools/prof.sh --config c3 --steps 20 --warmup 5 \
  --profile-frames 0 --extract 0 --cpu-frames 0 --c1-frames 0 --host-frames 0 || exit $?
PROF_OUT=gpurun_out/prof_c5 PMC_RECORD=${R}_c5_pmc.json bash tools/prof.sh --config c5 --steps 10 --warmup 5 \
  --profile-frames 0 --extract 0 --cpu-frames 0 --c1-frames 0 --host-frames 0 || exit $?
echo "prof_all done"
