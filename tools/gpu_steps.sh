#!/bin/bash
# Run GPU steps in order; continue past ordinary test failures (exit 1) but stop
# after anything that looks like a fault, abort, segfault or time limit.
# usage: tools/gpu_steps.sh "<name>:<seconds>:<command>" ...
mkdir -p gpurun_out
for step in "$@"; do
  name="${step%%:*}"; rest="${step#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (limit ${secs}s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc after $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
