#!/bin/bash
# Round 4, call 11: serial per-sector stats (cost-model refit), the
# projected N-GPU farm (per-part solo timing), farm worker-count A/B.
set -o pipefail
export RUN=${RUN:-r4k}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
F="python3 $R/tools/farm_prof.py"
bash tools/gpu_step.sh \
 "serial:300:$F --reps 1 --serial-stats $O/farm_c4_serial_stats.json" \
 "scale:400:python3 $R/tools/farm_scale_probe.py --out $O/farm_scale_projection.json" \
 "workers:300:for w in 4 12 16; do echo workers \$w; $F --reps 2 --workers \$w || exit 1; done"
du -sh $O
