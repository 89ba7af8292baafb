set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
for v in base xw262 xw16; do
  L=$PWD/slam-kinectfusion_amd/lib/libkfx.so; [ $v = base ] || L=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so
  for c in c2 c5; do
    A="--steps 5 --warmup 2"; [ $c = c5 ] && A="--config c5 --steps 3 --warmup 2"
    KFX_LIB_PATH=$L timeout -k 10 300 python3 bench.py $A --cpu-frames 0 --c1-frames 0 --c3-frames 0 --c5-frames 0 --host-frames 0 > gpurun_out/x_${v}_$c.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/x_${v}_$c.json').read().strip().splitlines()[-1]);e=d['extract'];print('$v $c', {k:(e[k]['passes'],e[k]['count_ms'],e[k]['scan_ms'],e[k]['copy_or_emit_ms']) for k in ('points','mesh')})"
  done
done
