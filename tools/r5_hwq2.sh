#!/bin/bash
# configs[3] farm with the worker streams: 4 hardware queues (default) with 8
# workers, against 2 queues with 8 workers and 4 queues with 4 workers.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${RUN:-r5hq2}
mkdir -p "$OUT"
for k in 1 2; do
  echo "== 4 queues 8 workers ($k)"
  timeout -k 10 200 python -u tools/farm_prof.py --reps 3 > "$OUT/a$k.log" 2>&1 || { tail -5 "$OUT/a$k.log"; exit 1; }
  grep "wall" "$OUT/a$k.log"
  echo "== 2 queues 8 workers ($k)"
  GPU_MAX_HW_QUEUES=2 timeout -k 10 200 python -u tools/farm_prof.py --reps 3 > "$OUT/b$k.log" 2>&1 || { tail -5 "$OUT/b$k.log"; exit 1; }
  grep "wall" "$OUT/b$k.log"
  echo "== 4 queues 4 workers ($k)"
  timeout -k 10 200 python -u tools/farm_prof.py --reps 3 --workers 4 > "$OUT/c$k.log" 2>&1 || { tail -5 "$OUT/c$k.log"; exit 1; }
  grep "wall" "$OUT/c$k.log"
  echo "== 4 queues 12 workers ($k)"
  timeout -k 10 200 python -u tools/farm_prof.py --reps 3 --workers 12 > "$OUT/d$k.log" 2>&1 || { tail -5 "$OUT/d$k.log"; exit 1; }
  grep "wall" "$OUT/d$k.log"
done
