#!/bin/bash
# Round 4, call 3: k_direct with out-of-range gathers for idle lanes — parity
# (H·v tests) and time / L1 counters on the nonSU2 N26 and N28 sectors.
set -o pipefail
export RUN=${RUN:-r4c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
P="python3 $R/tools/spmv_probe.py"
bash tools/gpu_step.sh \
 "hxv:300:python -u -m pytest tests/test_gpu_hxv.py tests/test_gpu_jz.py -x -q --timeout 200 --timeout-method thread" \
 "probe:120:$P --sector n26s --path 1 --iters 30 && $P --sector n28 --path 1 --iters 30 && $P --sector n28j --path 1 --iters 30 && $P --sector n26s --path 1 --iters 30 --cvec" \
 "pmc_ta_n26s:120:bash tools/pmc_pass.sh $O pmc_ta_n26s 'TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE' $P --sector n26s --path 1 --iters 5" \
 "pmc_ta_n28d:120:bash tools/pmc_pass.sh $O pmc_ta_n28d 'TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE' $P --sector n28 --path 1 --iters 5"
