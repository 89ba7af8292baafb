#!/bin/bash
# C5 single volume (2048^3 @ 2 mm, 1280x720) on one GPU with the extraction record, under
# rocprofv3 kernel trace + stats: surface export timed at 2048^3
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/c5x
mkdir -p $OUT
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
  python3 $ROOT/bench.py --config c5 --steps 10 --warmup 3 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --host-frames 0 \
  > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{"metric"' $OUT/bench.log | tail -1 > $OUT/bench.json
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['timed_region_kernel_ms']);print(json.dumps(d.get('extract')))"
