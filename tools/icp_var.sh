#!/bin/bash
# ICP A/B on the GPU box: parity tests of the working-tree library, then the
# per-iteration ICP trace and alternating driver-command bench runs of the
# libraries named (base = working tree, else lib/var_<name>).
#   tools/icp_var.sh "test -k expr" rounds name...
set -o pipefail
mkdir -p gpurun_out
K=$1; R=$2; shift 2
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_regimes.py -k "$K" > gpurun_out/icpvar_t.log 2>&1 || { tail -30 gpurun_out/icpvar_t.log; exit 1; }
tail -2 gpurun_out/icpvar_t.log
for v in "$@"; do
  if [ $v = base ]; then L=$PWD/slam-kinectfusion_amd/lib/libkfx.so; else L=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so; fi
  KFX_LIB_PATH=$L timeout -k 10 100 python3 tools/icp_trace.py > gpurun_out/icpt_$v.log 2>&1 || { tail gpurun_out/icpt_$v.log; exit 1; }
  echo "== $v"; grep -E "^(per-iteration|lane|block reduce|atomics|arrive|sums read|solve|post-solve)" gpurun_out/icpt_$v.log
done
for r in $(seq $R); do
  for v in "$@"; do
    if [ $v = base ]; then L=$PWD/slam-kinectfusion_amd/lib/libkfx.so; else L=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so; fi
    KFX_LIB_PATH=$L timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --c5-frames 0 --host-frames 0 > gpurun_out/ab_$v.json 2>&1 || { tail -5 gpurun_out/ab_$v.json; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d['timed_region_kernel_ms'])"
  done
done
