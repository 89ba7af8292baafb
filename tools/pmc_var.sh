#!/bin/bash
# One SQ counter pass per variant library: tools/pmc_var.sh "counters" var1 var2 ...
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
CTR=$1
shift
for v in "$@"; do
  echo "=== $v"
  L="$ROOT/slam-kinectfusion_amd/lib/var_$v/libkfx.so"
  [ "$v" = base ] && L="$ROOT/slam-kinectfusion_amd/lib/libkfx.so"
  KFX_LIB_PATH="$L" timeout -k 10 120 rocprofv3 --pmc $CTR --output-format csv \
      -d "$ROOT/gpurun_out/pmcv/$v" -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --profile-frames 2 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --c5-frames 0 \
      --host-frames 0 --extract 0 \
      > "$ROOT/gpurun_out/pmcv/$v.log" 2>&1 || { echo "rc=$?"; tail -5 "$ROOT/gpurun_out/pmcv/$v.log"; exit 1; }
done
for v in "$@"; do
  echo "--- $v"
  python3 "$ROOT/tools/pmc_summary.py" "$ROOT/gpurun_out/pmcv/$v" | grep -A12 "^k_integrate<false, true>" | head -12 || true
done
