#!/bin/bash
# Round 4, call 21 (temporary switch ED_TMP_DWGRID): pass D grid sweep for
# the two-column form on n28 / n28b / c4.
set -o pipefail
export RUN=${RUN:-r4dwgrid}
R=${GRAFT_REPO_ROOT:-$(pwd)}
P="python3 $R/tools/spmv_probe.py --path 2 --iters 60"
bash tools/gpu_step.sh \
 "sweep:500:for s in n28 n28b c4; do for g in 2048 1024 1280 1536 768 2048; do echo GRID \$g; ED_TMP_DWGRID=\$g $P --sector \$s || exit 1; done; done"
