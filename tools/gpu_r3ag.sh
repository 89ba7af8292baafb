#!/bin/bash
# strided persistent ICP (1280x720): parity tests, C2 driver bench (unchanged path), C5 single-volume bench
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_regimes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r3ag.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3ag.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --host-frames 0 --extract 0 > gpurun_out/ab_c2.json 2>&1 || { tail -5 gpurun_out/ab_c2.json; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_c2.json').read().strip().splitlines()[-1]);print('c2',d['value'],d['ms_per_step'],d['timed_region_kernel_ms'])"
done
timeout -k 10 300 python3 bench.py --config c5 --steps 10 --warmup 3 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --host-frames 0 --extract 0 > gpurun_out/ab_c5.json 2>&1 || { tail -5 gpurun_out/ab_c5.json; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/ab_c5.json').read().strip().splitlines()[-1]);print('c5',d['value'],d['ms_per_step'],d['timed_region_kernel_ms'])"
echo done
