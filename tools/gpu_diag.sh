# ICP per-block and per-iteration traces in the benchmark's staged regime, then
# A/B bench rounds of the named libraries (tools/icp_var.sh's bench loop).
set -o pipefail
mkdir -p gpurun_out
KFX_LIB_PATH=$PWD/slam-kinectfusion_amd/lib/var_btrace/libkfx.so timeout -k 10 100 python3 tools/icp_blocks.py > gpurun_out/blk.log 2>&1 || { tail gpurun_out/blk.log; exit 1; }
timeout -k 10 100 python3 tools/icp_trace.py > gpurun_out/icpt_staged.log 2>&1 || { tail gpurun_out/icpt_staged.log; exit 1; }
cat gpurun_out/blk.log; head -22 gpurun_out/icpt_staged.log
R=$1; shift
for r in $(seq $R); do
  for v in "$@"; do
    if [ $v = base ]; then L=$PWD/slam-kinectfusion_amd/lib/libkfx.so; else L=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so; fi
    KFX_LIB_PATH=$L timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --c5-frames 0 --host-frames 0 > gpurun_out/ab_$v.json 2>&1 || { tail -5 gpurun_out/ab_$v.json; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d['timed_region_kernel_ms'])"
  done
done
