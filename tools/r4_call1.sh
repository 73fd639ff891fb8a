#!/bin/bash
# Round 4, first GPU call: the GPU suite at the new build, then counter passes
# on the generic matrix-free kernel (nonSU2 N26 and N28) and the stored N28
# kernel's launch-time methods side by side.
set -o pipefail
export RUN=${RUN:-r4a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
P="python3 $R/tools/spmv_probe.py"
bash tools/gpu_step.sh \
 "tests:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "probe_n28:120:$P --sector n28 --path 0 --iters 30 && $P --sector n28 --path 0 --iters 30 --complex && $P --sector n26s --path 1 --iters 30 && $P --sector n28 --path 1 --iters 30" \
 "pmc_sq_n26s:120:bash tools/pmc_pass.sh $O pmc_sq_n26s 'SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM' $P --sector n26s --path 1 --iters 5" \
 "pmc_ta_n26s:120:bash tools/pmc_pass.sh $O pmc_ta_n26s 'TA_BUSY_avr TA_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE' $P --sector n26s --path 1 --iters 5" \
 "pmc_tcc_n26s:120:bash tools/pmc_pass.sh $O pmc_tcc_n26s 'TCC_HIT_sum TCC_MISS_sum' $P --sector n26s --path 1 --iters 5" \
 "pmc_sq_n28d:120:bash tools/pmc_pass.sh $O pmc_sq_n28d 'SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM' $P --sector n28 --path 1 --iters 5" \
 "pmc_ta_n28d:120:bash tools/pmc_pass.sh $O pmc_ta_n28d 'TA_BUSY_avr TA_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE' $P --sector n28 --path 1 --iters 5" \
 "pmc_tcc_n28d:120:bash tools/pmc_pass.sh $O pmc_tcc_n28d 'TCC_HIT_sum TCC_MISS_sum' $P --sector n28 --path 1 --iters 5" \
 "st_n28:150:cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $O/st_n28 -o st --output-format csv -- $P --sector n28 --path 0 --iters 30"
