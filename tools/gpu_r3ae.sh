#!/bin/bash
# graph modes A/B on the final library: default (preprocess graph), eager, full overlapped graphs
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in g1 g0 g2; do
    X=""; [ $v = g0 ] && X="--no-graph"; [ $v = g2 ] && X="--graph-full"
    timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --extract 0 $X > gpurun_out/ab_$v.json 2>&1 || { tail -5 gpurun_out/ab_$v.json; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d.get('host_input',{}).get('ms_per_step'),d['config']['graph'])"
  done
done
echo done
