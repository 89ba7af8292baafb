#!/bin/bash
# add-chain latency microbenchmark, then A/B of the scalar-add replays
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 60 tools/build/chain_bench || exit 1
bash tools/ab_quick.sh 2 sr0 sr1u psru 2>&1 | tee gpurun_out/ab_r3i.log
