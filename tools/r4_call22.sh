#!/bin/bash
# Round 4, call 22 (temporary switches ED_TMP_DWGRID / ED_TMP_DWR2): pass D
# grid x rows-per-wave sweep for the two-column form on n28 / n28b / c4.
set -o pipefail
export RUN=${RUN:-r4dwgrid2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
P="python3 $R/tools/spmv_probe.py --path 2 --iters 60"
bash tools/gpu_step.sh \
 "sweep:600:for s in n28 n28b c4; do for g in 1024 1280 768; do echo GRID \$g R1; ED_TMP_DWGRID=\$g $P --sector \$s || exit 1; echo GRID \$g R2; ED_TMP_DWR2=1 ED_TMP_DWGRID=\$g $P --sector \$s || exit 1; done; done"
