#!/bin/bash
# Counter breakdown of the complex(8) MODE 4 Lanczos step (configs[1], one
# 512-thread workgroup, 512-step dispatches of tools/cvec_probe.py): three
# rocprofv3 --pmc passes, each its own run under a hard limit, then
# tools/mode4_floor.py turns the per-dispatch medians into per-step cycles.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6m4
mkdir -p $O
bash $R/tools/pmc_pass.sh $O p1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY" python3 $R/tools/cvec_probe.py
bash $R/tools/pmc_pass.sh $O p2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY" python3 $R/tools/cvec_probe.py
bash $R/tools/pmc_pass.sh $O p3 "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SENDMSG" python3 $R/tools/cvec_probe.py
timeout -k 10 60 python3 $R/tools/cvec_probe.py > $O/cvec_probe.txt 2>&1
