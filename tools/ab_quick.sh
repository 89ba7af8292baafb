# alternating driver-command bench runs (no side records) of the named libraries:
#   tools/ab_quick.sh rounds base|<var> ...   (var = lib/var_<var>)
set -o pipefail
mkdir -p gpurun_out
R=$1; shift
for r in $(seq $R); do
  for v in "$@"; do
    if [ $v = base ]; then L=$PWD/slam-kinectfusion_amd/lib/libkfx.so; else L=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so; fi
    KFX_LIB_PATH=$L timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --c5-frames 0 --host-frames 0 --extract 0 > gpurun_out/ab_$v.json 2>&1 || { tail -5 gpurun_out/ab_$v.json; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d['timed_region_kernel_ms'])"
  done
done
