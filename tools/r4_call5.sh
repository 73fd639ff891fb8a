#!/bin/bash
# Round 4, call 5: configs[3] farm A/B — local-only CGS update (default) vs
# full update every step, and without the degeneracy probe; serial per-sector
# statistics of each (nhv, time).
set -o pipefail
export RUN=${RUN:-r4e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
F="python3 $R/tools/farm_prof.py"
bash tools/gpu_step.sh \
 "farm_def:180:$F --reps 3" \
 "farm_fullupd:180:$F --reps 3 --options trlan_fullupd" \
 "farm_noverify:180:$F --reps 3 --options eigh_no_verify" \
 "serial_def:240:$F --reps 1 --serial-stats $O/serial_def.json" \
 "serial_fullupd:240:$F --reps 1 --options trlan_fullupd --serial-stats $O/serial_fullupd.json" \
 "serial_noverify:240:$F --reps 1 --options eigh_no_verify --serial-stats $O/serial_noverify.json"
