#!/bin/bash
# Round 4, call 4: k_direct with compile-time group kinds — parity and time.
set -o pipefail
export RUN=${RUN:-r4d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
P="python3 $R/tools/spmv_probe.py"
bash tools/gpu_step.sh \
 "hxv:500:python -u -m pytest tests/test_gpu_hxv.py tests/test_gpu_jz.py tests/test_gpu_dist.py tests/test_gpu_lanczos.py tests/test_gpu_eigh.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread" \
 "probe:180:$P --sector n26s --path 1 --iters 30 && $P --sector n28 --path 1 --iters 30 && $P --sector n28j --path 1 --iters 30 && $P --sector n26s --path 1 --iters 30 --cvec && $P --sector n26s --path 1 --iters 30 --complex && $P --sector n26s --path 0 --iters 30" \
 "pmc_sq_n26s:120:bash tools/pmc_pass.sh $O pmc_sq_n26s 'SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM' $P --sector n26s --path 1 --iters 5" \
 "pmc_ta_n26s:120:bash tools/pmc_pass.sh $O pmc_ta_n26s 'TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE' $P --sector n26s --path 1 --iters 5"
