# A/B of libraries on the big-volume workloads: C4 (1024^3 @ 2 mm) as 8
# calibrated Z-slabs in one process (tools/slab_record.py; every member timed
# alone) next to the single volume, optionally C5 single volume (bench).
#   tools/ab_big.sh rounds base|<var> ...   (var = lib/var_<var>); C5=1 adds C5
set -o pipefail
mkdir -p gpurun_out
R=$1; shift
for r in $(seq $R); do
  for v in "$@"; do
    if [ $v = base ]; then L=$PWD/slam-kinectfusion_amd/lib/libkfx.so; else L=$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so; fi
    KFX_LIB_PATH=$L timeout -k 10 240 python3 tools/slab_record.py c4 --groups calibrated --frames 10 --warmup 3 \
      --out gpurun_out/abbig_${v}_c4.json > gpurun_out/abbig_${v}_c4.log 2>&1 || { tail -5 gpurun_out/abbig_${v}_c4.log; exit 1; }
    python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.load(open(f"gpurun_out/abbig_{v}_c4.json"))
s = d["single"]
g = [k for k in d if isinstance(d[k], dict) and "slabs" in d[k]]
for k in g:
    it = [x["integrate_ms"] for x in d[k]["slabs"]]
    rl = [x["raycast_local_ms"] for x in d[k]["slabs"]]
    print(v, "c4", k, "single int %.3f ray %.3f" % (s["integrate_ms"], s["raycast_ms"]),
          "slab int sum %.3f max %.3f" % (sum(it), max(it)), "ray max %.3f" % max(rl))
PY
    if [ "${C5:-0}" = 1 ]; then
      KFX_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config c5 --steps 8 --warmup 3 --cpu-frames 0 --c1-frames 0 --c3-frames 0 \
        --c5-frames 0 --host-frames 0 --extract 0 > gpurun_out/abbig_${v}_c5.json 2>&1 || { tail -5 gpurun_out/abbig_${v}_c5.json; exit 1; }
      python3 -c "import json;d=json.loads(open('gpurun_out/abbig_${v}_c5.json').read().strip().splitlines()[-1]);print('$v c5',d['ms_per_step'],d['timed_region_kernel_ms'])"
    fi
  done
done
