set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for r in 1 2 3; do
  for g in 1 2; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --graph $g --cpu-frames 0 --c1-frames 0 --c3-frames 0 --c5-frames 0 --host-frames 0 --extract 0 > gpurun_out/gab_$g.json 2>&1 || { tail -3 gpurun_out/gab_$g.json; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/gab_$g.json').read().strip().splitlines()[-1]);print('g$g',d['value'],d['ms_per_step'],d['timed_region_kernel_ms'],d['config']['graph'])"
  done
done
