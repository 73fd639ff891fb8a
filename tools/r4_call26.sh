#!/bin/bash
# Round 4, call 26: A/B of non-temporal Hv stores in every plain-store H·v
# (a variant library built from the same tree with EpiStore::row storing
# non-temporally, variant/libedgpu_nt.so) on the stored / matrix-free kernels.
set -o pipefail
export RUN=${RUN:-r4ntall}
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=/tmp/ntv_$$
mkdir -p $V && cp -r $R/dmft-ed_amd $R/tools $R/tests $V/ && cp $R/variant/libedgpu_nt.so $V/dmft-ed_amd/libedgpu.so || exit 1
A="python3 $R/tools/spmv_probe.py --iters 60"
B="python3 $V/tools/spmv_probe.py --iters 60"
bash tools/gpu_step.sh \
 "ab:600:for c in '--sector n28 --path 0' '--sector n28 --path 0 --complex' '--sector n28 --path 1' '--sector n26s --path 1' '--sector n26s --path 0' '--sector n28j --path 0'; do for k in 1 2; do echo BASE \$c; $A \$c || exit 1; echo NT \$c; $B \$c || exit 1; done; done"
rc=$?; rm -rf $V; exit $rc
