#!/bin/bash
# Run the bench once per variant library (tools/variants.sh); one summary line each.
# usage: tools/tune.sh "bench args" var1 var2 ...
ARGS=$1
shift
mkdir -p gpurun_out/tune
for v in "$@"; do
  KFX_LIB_PATH="$PWD/slam-kinectfusion_amd/lib/var_$v/libkfx.so" timeout -k 10 120 python3 bench.py $ARGS \
      > "gpurun_out/tune/$v.json" 2> "gpurun_out/tune/$v.err"
  rc=$?
  if [ $rc -ne 0 ]; then echo "$v rc=$rc"; tail -3 "gpurun_out/tune/$v.err"; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['stage_ms'])" "gpurun_out/tune/$v.json" "$v"
done
