#!/bin/bash
# integrate: equal / geometric chunks without replay (timing only) and the
# store-last update restructure (rs: with the free-space shortcut, rs0: without)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
bash tools/ab_quick.sh 2 nofree rs rs0 e4n e6n e8n e12n g6n 2>&1 | tee gpurun_out/ab_r3c.log
