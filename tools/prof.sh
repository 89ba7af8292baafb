#!/bin/bash
# One profiling session on the GPU box (run from the repo root through gpurun):
#   1. rocprofv3 --kernel-trace --stats of a short bench run  -> gpurun_out/prof/stats
#   2. FETCH_SIZE / WRITE_SIZE calibration streams             -> gpurun_out/prof/calib
#   3. FETCH_SIZE, WRITE_SIZE and SQ issue passes over the same bench -> gpurun_out/prof/pmc
# Every rocprofv3 run is its own process under its own time limit; counters are
# never combined with trace domains (MI355X_MICROARCH.md, rocprofv3 section).
# usage: tools/prof.sh [bench args...]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
ARGS="$*"   # the stats pass runs bench.py with these (default: its defaults)
# same frames and step counts as the stats pass; no side runs (the PMC record
# averages every dispatch of a kernel, so only the main stream may launch it)
PMC_ARGS="$ARGS --cpu-frames 0 --c1-frames 0 --c3-frames 0 --c5-frames 0 --host-frames 0"
OUT="$ROOT/${PROF_OUT:-gpurun_out/prof}"
mkdir -p "$OUT"
run() {  # name, timeout, rocprof args...
  local name=$1 secs=$2
  shift 2
  echo "=== $name"
  timeout -k 10 "$secs" rocprofv3 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"
  [ $rc -eq 0 ] || { tail -20 "$OUT/$name.log"; exit $rc; }
}
run stats 300 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 "$ROOT/bench.py" $ARGS
grep "^{\"metric\"" "$OUT/stats.log" | tail -1 > "$OUT/stats_bench.json"
W=$(python3 -c "import sys;a=sys.argv[1:];print(a[a.index('--warmup')+1] if '--warmup' in a else 20)" $ARGS)
S=$(python3 -c "import sys;a=sys.argv[1:];print(a[a.index('--steps')+1] if '--steps' in a else 300)" $ARGS)
python3 "$ROOT/tools/prof_summary.py" "$OUT/stats/run_kernel_trace.csv" $W $S "$OUT/kernel_summary.json" > /dev/null
if [ -x "$ROOT/tools/build/pmc_calib" ]; then
  run calib_fetch 90 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib/FETCH_SIZE" -- "$ROOT/tools/build/pmc_calib"
  run calib_write 90 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib/WRITE_SIZE" -- "$ROOT/tools/build/pmc_calib"
fi
run pmc_fetch 240 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc/FETCH_SIZE" -- python3 "$ROOT/bench.py" $PMC_ARGS
run pmc_write 240 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc/WRITE_SIZE" -- python3 "$ROOT/bench.py" $PMC_ARGS
# issue counters (8 SQ slots + GRBM): VALU issue fraction next to the HBM fraction
run pmc_sq 240 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc/SQ" -- python3 "$ROOT/bench.py" $PMC_ARGS
PROF_ARGS="$ARGS" python3 "$ROOT/tools/traffic.py" "$OUT" --commit
