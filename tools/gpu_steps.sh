#!/bin/bash
# Run GPU steps in order, each under its own time limit; continue past an
# ordinary failure (exit 1/2) but stop at a crash, abort, fault or timeout.
# usage: tools/gpu_steps.sh "<secs>:<name>:<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  secs="${spec%%:*}"; rest="${spec#*:}"; name="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  tail -25 "gpurun_out/$name.log"
  echo "=== [$name] rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ] && [ $rc -ne 5 ]; then
    echo "=== stopping: step $name ended with rc=$rc"; exit $rc
  fi
done
