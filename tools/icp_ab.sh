set -e
for v in base icp512 icp1024; do
  if [ $v = base ]; then L=$PWD/slam-kinectfusion_amd/lib/libkfx.so; else L=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so; fi
  echo "== $v"
  KFX_LIB_PATH=$L timeout -k 10 100 python3 tools/icp_trace.py > gpurun_out/icpt_$v.log 2>&1
  grep -E "per-iteration" -A2 gpurun_out/icpt_$v.log
  tail -1 gpurun_out/icpt_$v.log | head -1 > /dev/null
  python3 -c "
import re
t=open('gpurun_out/icpt_$v.log').read().splitlines()
rows=[l.split() for l in t if re.match(r'^\s*\d+\s', l)]
print('total ICP us (solved of last iter):', rows[-1][5])"
  KFX_LIB_PATH=$L timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --cpu-frames 0 > gpurun_out/icpb_$v.json 2>&1
  python3 -c "import json;d=json.loads(open('gpurun_out/icpb_$v.json').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d['timed_region_kernel_ms'])"
done
