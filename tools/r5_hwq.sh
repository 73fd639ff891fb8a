#!/bin/bash
# configs[3] farm with the worker streams: HIP's default 4 hardware queues
# against 8 (one per worker stream), alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${RUN:-r5hq}
mkdir -p "$OUT"
for k in 1 2; do
  echo "== 4 queues ($k)"
  timeout -k 10 200 python -u tools/farm_prof.py --reps 3 > "$OUT/q4_$k.log" 2>&1 || { tail -5 "$OUT/q4_$k.log"; exit 1; }
  grep "wall" "$OUT/q4_$k.log"
  echo "== 8 queues ($k)"
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/farm_prof.py --reps 3 > "$OUT/q8_$k.log" 2>&1 || { tail -5 "$OUT/q8_$k.log"; exit 1; }
  grep "wall" "$OUT/q8_$k.log"
done
