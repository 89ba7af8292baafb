#!/bin/bash
# integrate per-column far clip: parity on it, then A/B (no clip / 16-cell / 64-cell boxes) with visited voxels
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_regimes.py tests/test_gpu_slab.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r3af.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3af.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in base nofc fc64; do
    if [ $v = base ]; then L=$PWD/slam-kinectfusion_amd/lib/libkfx.so; else L=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so; fi
    KFX_LIB_PATH=$L timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --host-frames 0 --extract 0 > gpurun_out/ab_$v.json 2>&1 || { tail -5 gpurun_out/ab_$v.json; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]);w=d['integrate_voxels'];print('$v',d['value'],d['ms_per_step'],d['timed_region_kernel_ms']['integrate'],d['timed_region_kernel_ms']['icp'],w['visited'],w['updated'],w['wave_batches'])"
  done
done
echo done
