#!/bin/bash
# integrate chunking / replay timing variants (timing-only builds marked n: wrong values)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
bash tools/ab_quick.sh 2 nofree w3n w6 w8 w8e w8n w16n 2>&1 | tee gpurun_out/ab_r3b.log
