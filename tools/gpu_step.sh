#!/bin/bash
# One GPU call of this round's measurement plan: each argument is a step
# "name:seconds:command"; output of step `name` goes to gpurun_out/$RUN/name.log.
# Stops at the first failing step (no further GPU work after a fault).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${RUN:-run}
mkdir -p "$OUT"
cd "$R" || exit 2
for step in "$@"; do
  name=${step%%:*}; rest=${step#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "=== $name ($secs s): $cmd" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
