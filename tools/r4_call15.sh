#!/bin/bash
# Round 4, call 15: farm A/B of the Krylov sweep block cap (1024 default vs
# 512 / 256), and per-sector A/B on the largest sectors.
set -o pipefail
export RUN=${RUN:-r4q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
F="python3 $R/tools/farm_prof.py"
bash tools/gpu_step.sh \
 "farm:400:$F --reps 3 && ED_TRLAN_GRID=512 $F --reps 3 && ED_TRLAN_GRID=256 $F --reps 3 && ED_TRLAN_GRID=384 $F --reps 3" \
 "grid:300:python3 $R/tools/trlan_ab.py --reps 2 --sectors '5,6;2,3' --grid 256,384,512,768"
