#!/bin/bash
# rocprofv3 --kernel-trace --stats of the C3 bench line (1024^3 @ 2 mm, single GPU)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/prof_c3"
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
  python3 "$ROOT/bench.py" --config c3 --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 --host-frames 0 \
  > "$OUT/stats.log" 2>&1 || { tail -20 "$OUT/stats.log"; exit 1; }
grep "^{\"metric\"" "$OUT/stats.log" | tail -1 > "$OUT/stats_bench.json"
python3 "$ROOT/tools/prof_summary.py" "$OUT/stats/run_kernel_trace.csv" 5 20 "$OUT/kernel_summary.json" > /dev/null
echo "c3 profile done"
