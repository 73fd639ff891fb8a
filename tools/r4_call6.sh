#!/bin/bash
# Round 4, call 6: k_direct two rows per lane (parity + time), then the
# configs[3] farm A/B (local-only CGS update vs full update vs no probe).
set -o pipefail
export RUN=${RUN:-r4f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
P="python3 $R/tools/spmv_probe.py"
F="python3 $R/tools/farm_prof.py"
bash tools/gpu_step.sh \
 "hxv:400:python -u -m pytest tests/test_gpu_hxv.py tests/test_gpu_jz.py tests/test_gpu_dist.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread" \
 "probe:180:$P --sector n26s --path 1 --iters 30 && $P --sector n28 --path 1 --iters 30 && $P --sector n28j --path 1 --iters 30 && $P --sector n26s --path 1 --iters 30 --cvec" \
 "farm_def:180:$F --reps 3" \
 "farm_fullupd:180:$F --reps 3 --options trlan_fullupd" \
 "farm_noverify:180:$F --reps 3 --options eigh_no_verify" \
 "serial_def:240:$F --reps 1 --serial-stats $O/serial_def.json" \
 "serial_fullupd:240:$F --reps 1 --options trlan_fullupd --serial-stats $O/serial_fullupd.json"
