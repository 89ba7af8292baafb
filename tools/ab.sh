#!/bin/bash
# A/B timing of variant libraries on the GPU box (bench.py, kernel timing samples):
#   tools/ab.sh [-t] rounds base|<var> ...   (-t: run the GPU tests on the default library first)
set -e
L=slam-kinectfusion_amd/lib
if [ "$1" = -t ]; then
  shift
  timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -1 gpurun_out/gpu_tests.log
fi
R=$1; shift
for r in $(seq $R); do
  for v in "$@"; do
    if [ $v = base ]; then P=$L/libkfx.so; else P=$L/var_$v/libkfx.so; fi
    KFX_LIB_PATH=$PWD/$P timeout -k 10 120 python3 bench.py --steps 400 --warmup 30 --cpu-frames 0 > gpurun_out/ab_$v.json
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]);print('$v',d['value'],d.get('timed_region_kernel_ms'))"
  done
done
