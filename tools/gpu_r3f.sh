#!/bin/bash
# plan kernel cost split: kernel traces of the default build and timing-only variants
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
for v in base pe1 pe2; do
  if [ $v = base ]; then L=$PWD/slam-kinectfusion_amd/lib/libkfx.so; else L=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so; fi
  mkdir -p gpurun_out/r3f/$v
  KFX_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/r3f/$v -o run -- \
    python3 bench.py --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --host-frames 0 --extract 0 \
    > gpurun_out/r3f/$v.log 2>&1 || exit 1
  python3 tools/prof_summary.py gpurun_out/r3f/$v/run_kernel_trace.csv 5 20 gpurun_out/r3f/$v.json > /dev/null
  python3 -c "import json;d=json.load(open('gpurun_out/r3f/$v.json'));print('$v',{k:v['median_us_all'] for k,v in d.items() if 'int' in k or 'icp' in k or 'raycast<true, false, false>' in k})"
done
