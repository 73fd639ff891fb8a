#!/bin/bash
# Round 4, call 9: k_direct with separate 64-row (real) / 128-row (complex)
# chunk lists: parity and per-launch times.
set -o pipefail
export RUN=${RUN:-r4i}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
P="python3 $R/tools/spmv_probe.py"
bash tools/gpu_step.sh \
 "tests:400:python -u -m pytest tests/test_gpu_hxv.py tests/test_gpu_eigh.py tests/test_gpu_lanczos.py tests/test_gpu_golden.py tests/test_gpu_dist.py tests/test_gpu_jz.py -x -q --timeout 200 --timeout-method thread" \
 "probe:180:$P --sector n26s --path 1 --iters 30 && $P --sector n28 --path 1 --iters 30 && $P --sector n28j --path 1 --iters 30 && $P --sector n26s --path 1 --iters 30 --cvec" \
 "cvec:120:python3 $R/tools/cvec_probe.py" \
 "ncv:400:python3 $R/tools/trlan_ab.py --reps 2 --ncv 16,23,32,44 --keep 1,3,6,12" \
 "vdotfin:300:python3 $R/tools/trlan_ab.py --reps 3 --opts trlan_vdotfin" \
 "farm:200:python3 $R/tools/farm_prof.py --reps 3 && python3 $R/tools/farm_prof.py --reps 2 --options trlan_vdotfin" \
 "budget:300:for b in 250 400 700; do python3 $R/tools/farm_prof.py --reps 2 --budget $b || exit 1; done"
du -sh $O
