#!/bin/bash
# host input by the fetch kernel: async tests, the probe, the driver's bench line
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "async or pipeline" --timeout 120 --timeout-method thread > gpurun_out/tests_r3p.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3p.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python3 -u tools/host_input_probe.py > gpurun_out/host_probe.log 2>&1 || { tail -5 gpurun_out/host_probe.log; exit 1; }
cat gpurun_out/host_probe.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 --c3-frames 0 > gpurun_out/b_r3p.json 2> gpurun_out/b_r3p.err || { tail -5 gpurun_out/b_r3p.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/b_r3p.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['host_input'])"
