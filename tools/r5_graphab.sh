#!/bin/bash
# configs[3] farm: Krylov sweeps replayed from hipGraphs (default) against
# direct launches (ED_OPT_NO_GRAPH), alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${RUN:-r5gr}
mkdir -p "$OUT"
for k in 1 2; do
  echo "== graphs ($k)"
  timeout -k 10 200 python -u tools/farm_prof.py --reps 3 > "$OUT/g$k.log" 2>&1 || { tail -5 "$OUT/g$k.log"; exit 1; }
  grep "wall" "$OUT/g$k.log"
  echo "== no graphs ($k)"
  timeout -k 10 200 python -u tools/farm_prof.py --reps 3 --options no_graph > "$OUT/n$k.log" 2>&1 || { tail -5 "$OUT/n$k.log"; exit 1; }
  grep "wall" "$OUT/n$k.log"
done
