#!/bin/bash
# Round 4, call 23 (temporary switch ED_TMP_DWGRID): pass D grids whose
# per-XCD block count divides the row tiles of a column chunk (every block
# the same number of tiles per chunk: the XCD's blocks stay on one chunk)
# against 1280 / 1024, with rocprofv3 counter traffic of two of them.
set -o pipefail
export RUN=${RUN:-r4dwgrid3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
P="python3 $R/tools/spmv_probe.py --path 2 --iters 60"
bash tools/gpu_step.sh \
 "sweep:500:for s in n28 n28b; do for g in 1280 1144 1024 1144 1280; do echo GRID \$g; ED_TMP_DWGRID=\$g $P --sector \$s || exit 1; done; done; for g in 1280 928 2048 928; do echo GRID \$g; ED_TMP_DWGRID=\$g $P --sector c4r || exit 1; done" \
 "pmc1:120:cd /tmp && export TMPDIR=/tmp && ED_TMP_DWGRID=1144 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d $O/f1144 -o p --output-format csv -- python3 $R/tools/spmv_probe.py --path 2 --iters 20 --sector n28" \
 "pmc2:120:cd /tmp && export TMPDIR=/tmp && ED_TMP_DWGRID=1280 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d $O/f1280 -o p --output-format csv -- python3 $R/tools/spmv_probe.py --path 2 --iters 20 --sector n28"
