#!/bin/bash
# extraction brick skip: extract/mesh/slab tests, the driver bench line (extract record)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_extract.py tests/test_gpu_slab.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r3v.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3v.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 > gpurun_out/b_r3v.json 2> gpurun_out/b_r3v.err || { tail -5 gpurun_out/b_r3v.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/b_r3v.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['timed_region_kernel_ms']);print(d['extract']);print(d['host_input']);print(d['c3_record']['value'], d['c3_record']['timed_region_kernel_ms'])"
