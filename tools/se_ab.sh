#!/bin/bash
# bench value with and without the in-run timing samples, alternating
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for r in 1 2 3 4; do
  for se in 8 0; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --sample-every $se --cpu-frames 0 --c1-frames 0 --c3-frames 0 --c5-frames 0 --host-frames 0 --extract 0 > gpurun_out/se_$se.json 2>&1 || { tail -5 gpurun_out/se_$se.json; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/se_$se.json').read().strip().splitlines()[-1]);print('se$se',d['value'],d['ms_per_step'])"
  done
done
