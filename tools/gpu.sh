#!/bin/bash
# Parameterised GPU job (run from the repo root through gpurun), replacing the
# one-shot job files.  Jobs run in order; each GPU step has its own time limit
# and the first failure ends the call (no retries):
#   tests[=EXPR]      pytest -m gpu (-k EXPR)            -> gpurun_out/tests.log
#   vtests=VAR:EXPR   pytest -m gpu -k EXPR on the variant lib/var_VAR
#   smoke             __graft_entry__.smoke()
#   bench[=ARGS]      bench.py (ARGS comma-separated; default: the driver's
#                     --steps 20 --warmup 5)              -> gpurun_out/bench.json
#   quick[=ARGS]      bench.py without side records (A/B timing)
#   prof[=ARGS]       tools/prof.sh (rocprofv3 stats + PMC passes)
#   slab=c4|c5        tools/slab_record.py (8 slabs on one GPU)
#   ab=ROUNDS:V1:V2   tools/ab_quick.sh ROUNDS V1 V2 ... (alternating variants)
#   py=SCRIPT:ARG     python3 tools/SCRIPT ARG (e.g. py=icp_trace.py:hd720)
#   pmcv=V1:V2        SQ instruction counters of k_integrate per variant (tools/pmc_var.sh)
# e.g.  gpurun -- bash tools/gpu.sh tests bench quick=--config,c5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local name=$1 secs=$2
  shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@"
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name failed: rc=$rc"; exit $rc; }
}
args() { echo "$1" | tr ',' ' '; }
for job in "$@"; do
  key=${job%%=*}
  val=""
  [ "$key" != "$job" ] && val=${job#*=}
  case $key in
    tests)
      K=()
      [ -n "$val" ] && K=(-k "$val")
      echo "=== tests"
      timeout -k 10 1500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests "${K[@]}" \
        > gpurun_out/tests.log 2>&1
      rc=$?
      tail -n 3 gpurun_out/tests.log
      [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/tests.log | head -20; exit $rc; } ;;
    vtests)
      V=${val%%:*}; E=${val#*:}
      echo "=== vtests $V"
      KFX_LIB_PATH=$PWD/slam-kinectfusion_amd/lib/var_$V/libkfx.so timeout -k 10 900 python3 -u -m pytest -x -q \
        --timeout 300 --timeout-method thread -m gpu tests -k "$E" > gpurun_out/vtests_$V.log 2>&1
      rc=$?
      tail -n 2 gpurun_out/vtests_$V.log
      [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/vtests_$V.log | head -20; exit $rc; } ;;
    smoke)
      step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      A=${val:---steps,20,--warmup,5}
      step bench 600 python3 bench.py $(args "$A") > gpurun_out/bench.json 2> gpurun_out/bench.err
      python3 -c "import json;d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1]);print('bench',d['value'],d['ms_per_step'],d['timed_region_kernel_ms'])" ;;
    quick)
      A=${val:---steps,20,--warmup,5}
      step quick 300 python3 bench.py $(args "$A") --cpu-frames 0 --c1-frames 0 --c3-frames 0 --c5-frames 0 \
        --host-frames 0 --extract 0 > gpurun_out/quick.json 2> gpurun_out/quick.err
      python3 -c "import json;d=json.loads(open('gpurun_out/quick.json').read().strip().splitlines()[-1]);print('quick',d['value'],d['ms_per_step'],d['timed_region_kernel_ms'])" ;;
    prof)
      A=${val:---steps,20,--warmup,5}
      step prof 1500 bash tools/prof.sh $(args "$A") > gpurun_out/prof.log 2>&1
      tail -n 5 gpurun_out/prof.log ;;
    slab)
      step slab 900 python3 tools/slab_record.py "$val" --out gpurun_out/slab_$val.json > gpurun_out/slab_$val.log 2>&1
      tail -n 5 gpurun_out/slab_$val.log ;;
    py)  # py=SCRIPT:ARG  a tools/ python script on the GPU
      S=${val%%:*}; A=${val#*:}; [ "$A" = "$val" ] && A=""
      step py 600 python3 tools/$S $A > gpurun_out/py_${S%.py}.log 2>&1
      tail -n 40 gpurun_out/py_${S%.py}.log ;;
    ab)
      step ab 1200 bash tools/ab_quick.sh $(echo "$val" | tr ':' ' ') ;;
    pmcv)
      mkdir -p gpurun_out/pmcv
      step pmcv 900 bash tools/pmc_var.sh "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS" $(echo "$val" | tr ':' ' ') ;;
    *)
      echo "unknown job $job"; exit 2 ;;
  esac
done
echo done
