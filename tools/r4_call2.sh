#!/bin/bash
# Round 4, call 2: the LDS-staged stored H·v experiment (tools/stage_variants)
# and L1/TA counters of the stored kernel forms.
set -o pipefail
export RUN=${RUN:-r4b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
bash tools/gpu_step.sh \
 "stage:120:$R/tools/stage_variants" \
 "pmc_ta_stage:120:bash tools/pmc_pass.sh $O pmc_ta_stage 'TA_BUSY_avr TA_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE' $R/tools/stage_variants" \
 "pmc_sq_stage:120:bash tools/pmc_pass.sh $O pmc_sq_stage 'SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SMEM' $R/tools/stage_variants" \
 "pmc_fetch_stage:120:bash tools/pmc_pass.sh $O pmc_fetch_stage 'FETCH_SIZE' $R/tools/stage_variants"
