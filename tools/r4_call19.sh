#!/bin/bash
# Round 4, call 19: pass D with two columns per lane (ED_OPT_KRON_DW2) — parity
# (test_gpu_kron2) and an A/B of the two-pass H·v on n28 / n28b / c4, then
# rocprofv3 kernel traces of n28 both ways (pass U / pass D split).
set -o pipefail
export RUN=${RUN:-r4dw2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
P="python3 $R/tools/spmv_probe.py --path 2 --iters 60"
bash tools/gpu_step.sh \
 "tests:300:python -u -m pytest tests/test_gpu_kron2.py -x -q --timeout 120 --timeout-method thread" \
 "ab:300:for s in n28 n28b c4; do $P --sector \$s && $P --sector \$s --options kron_dw2 && $P --sector \$s && $P --sector \$s --options kron_dw2; done" \
 "prof1:200:cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4dw2/p1 -o p --output-format csv -- python3 $R/tools/spmv_probe.py --path 2 --iters 60 --sector n28" \
 "prof2:200:cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4dw2/p2 -o p --output-format csv -- python3 $R/tools/spmv_probe.py --path 2 --iters 60 --sector n28 --options kron_dw2"
