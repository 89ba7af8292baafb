#!/bin/bash
# full GPU tests; the driver bench line; the N>1 code path (replicas + zslab record) at N=1
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r3y.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3y.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/b_r3y.json 2> gpurun_out/b_r3y.err || { tail -5 gpurun_out/b_r3y.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/b_r3y.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['timed_region_kernel_ms']);print(d['host_input']['ms_per_step']);print(d['extract']['points'],d['extract']['mesh'])"
timeout -k 10 400 python3 bench.py --mode replicas --zslab c4 --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --host-frames 0 > gpurun_out/b_r3y_rep.json 2> gpurun_out/b_r3y_rep.err || { tail -5 gpurun_out/b_r3y_rep.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/b_r3y_rep.json').read().strip().splitlines()[-1]);print(d['value'],d['scaling'],d['config']['parallelism']);print(d.get('zslab'))"
