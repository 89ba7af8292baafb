# alternating driver-command bench runs with the host-input (PCIe-inclusive)
# record of the named libraries:  tools/ab_host.sh rounds base|<var> ...
set -o pipefail
mkdir -p gpurun_out
R=$1; shift
for r in $(seq $R); do
  for v in "$@"; do
    if [ $v = base ]; then L=$PWD/slam-kinectfusion_amd/lib/libkfx.so; else L=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so; fi
    KFX_LIB_PATH=$L timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --c5-frames 0 --extract 0 > gpurun_out/abh_$v.json 2>&1 || { tail -5 gpurun_out/abh_$v.json; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/abh_$v.json').read().strip().splitlines()[-1]);h=d['host_input'] or {};print('$v',d['value'],d['ms_per_step'],'host_input',h.get('ms_per_step'))"
  done
done
