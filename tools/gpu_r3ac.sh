#!/bin/bash
# overlapped frames replayed as graphs: all GPU tests, then graph vs eager A/B (staged + host input)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r3ac.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r3ac.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in graph eager; do
    X=""; [ $v = eager ] && X="--no-graph"
    timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --extract 0 $X > gpurun_out/ab_$v.json 2>&1 || { tail -5 gpurun_out/ab_$v.json; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d['config']['graph'],d.get('host_input',{}).get('ms_per_step'))"
  done
done
echo done
