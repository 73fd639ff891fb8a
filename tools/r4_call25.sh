#!/bin/bash
# Round 4, call 25 (temporary switch ED_TMP_NTM): pass D two-column form with
# non-temporal Hv stores (1), non-temporal y loads (2) or both (3), against
# the default, and the FETCH counter of the store variant.
set -o pipefail
export RUN=${RUN:-r4ntm}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
P="python3 $R/tools/spmv_probe.py --path 2 --iters 60"
bash tools/gpu_step.sh \
 "sweep:500:for s in n28 n28b c4r; do for g in 0 1 2 3 0 1; do echo NTM \$g; ED_TMP_NTM=\$g $P --sector \$s || exit 1; done; done" \
 "pmc1:120:cd /tmp && export TMPDIR=/tmp && ED_TMP_NTM=1 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d $O/f1 -o p --output-format csv -- python3 $R/tools/spmv_probe.py --path 2 --iters 20 --sector n28" \
 "pmc2:120:cd /tmp && export TMPDIR=/tmp && ED_TMP_NTM=1 timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d $O/w1 -o p --output-format csv -- python3 $R/tools/spmv_probe.py --path 2 --iters 20 --sector n28"
