#!/bin/bash
# Run each argument as a GPU step under a time limit; stop on fault-like exits (>1).
mkdir -p gpurun_out
i=0
for cmd in "$@"; do
  i=$((i+1))
  echo "=== step $i: $cmd" >> gpurun_out/steps.log
  timeout -k 10 ${STEP_TIMEOUT:-300} bash -c "$cmd" >> gpurun_out/steps.log 2>&1
  rc=$?
  echo "=== rc $rc" >> gpurun_out/steps.log
  if [ $rc -gt 1 ]; then exit $rc; fi
done
