#!/bin/bash
# Farm worker streams (one HIP stream per worker thread for every sector it
# solves) against a private stream per sector: GPU tests of the farm and the
# configs[3] farm wall, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${RUN:-r5ws}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_golden.py \
  tests/test_gpu_diag_gf.py > "$OUT/tests.log" 2>&1 || { echo tests failed; tail -20 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for k in 1 2; do
  echo "== worker streams ($k)"
  timeout -k 10 200 python -u tools/farm_prof.py --reps 3 > "$OUT/ws$k.log" 2>&1 || { tail -5 "$OUT/ws$k.log"; exit 1; }
  grep "wall\|solves" "$OUT/ws$k.log"
  echo "== private streams ($k)"
  timeout -k 10 200 python -u tools/farm_prof.py --reps 3 --private-streams > "$OUT/ps$k.log" 2>&1 || { tail -5 "$OUT/ps$k.log"; exit 1; }
  grep "wall\|solves" "$OUT/ps$k.log"
done
