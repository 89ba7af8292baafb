#!/bin/bash
# certified free-space integrate: all GPU tests (cert on by default), A/B against cert off
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r3q.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3q.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_quick.sh 3 base nocert 2>&1 | tee gpurun_out/ab_r3q.log || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/ab_base.json').read().strip().splitlines()[-1]);print(d['integrate_voxels'])"
timeout -k 10 180 python3 -u tools/host_input_probe.py > gpurun_out/host_probe.log 2>&1 || { tail -5 gpurun_out/host_probe.log; exit 1; }
cat gpurun_out/host_probe.log
