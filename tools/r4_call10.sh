#!/bin/bash
# Round 4, call 10: the k_cgs last-block fold on 8-B agent atomics (no
# fences) against separate k_vdot_fin launches; cache-budget scheduler A/B;
# eigensolver parity.
set -o pipefail
export RUN=${RUN:-r4j}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
F="python3 $R/tools/farm_prof.py"
bash tools/gpu_step.sh \
 "tests:400:python -u -m pytest tests/test_gpu_eigh.py tests/test_gpu_golden.py tests/test_gpu_diag_gf.py -x -q --timeout 200 --timeout-method thread" \
 "vdotfin:300:python3 $R/tools/trlan_ab.py --reps 3 --opts trlan_vdotfin" \
 "farm:200:$F --reps 3 && $F --reps 2 --options trlan_vdotfin" \
 "budget:400:for b in 250 400 700; do echo budget \$b; $F --reps 2 --budget \$b || exit 1; done"
du -sh $O
