#!/bin/bash
# Round 4, call 8 (call 7's outputs exceeded the copy-back limit): k_direct
# times, complex MODE 4 LDS counters, the k_direct setup profile, and the
# 8-worker profiled farm with its shared-object map; large traces deleted.
set -o pipefail
export RUN=${RUN:-r4h}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
P="python3 $R/tools/spmv_probe.py"
bash tools/gpu_step.sh \
 "probe:180:$P --sector n26s --path 1 --iters 30 && $P --sector n28 --path 1 --iters 30 && $P --sector n28j --path 1 --iters 30 && $P --sector n26s --path 1 --iters 30 --cvec" \
 "pmc_cvec:120:bash tools/pmc_pass.sh $O pmc_cvec 'SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_SALU' python3 $R/tools/cvec_probe.py" \
 "st_direct:150:cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $O/st_direct_n28 -o st --output-format csv -- python3 $R/tools/spmv_probe.py --sector n28 --path 1 --iters 30 && find $O/st_direct_n28 -name '*kernel_trace.csv' -size +2M -delete" \
 "trlan_ab:300:python3 $R/tools/trlan_ab.py --reps 3 --opts trlan_fullupd,eigh_no_verify,trlan_g128" \
 "farm_g128:180:python3 $R/tools/farm_prof.py --reps 3 --options trlan_g128" \
 "farm_def:180:python3 $R/tools/farm_prof.py --reps 3" \
 "crash:200:ulimit -c 0; cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $O/fp_w8ng -o fp --output-format csv -- python3 $R/tools/farm_prof.py --workers 8 --reps 1 --options no_graph --maps $O/maps_w8ng.json; rc=\$?; find $O/fp_w8ng -name '*kernel_trace.csv' -delete; exit \$rc"
du -sh $O

