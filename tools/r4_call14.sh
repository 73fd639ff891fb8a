#!/bin/bash
# Round 4, call 14: kernel statistics and HBM traffic of the thick-restart
# eigensolver alone on the configs[3] (6,6) sector (k_cgs bandwidth).
set -o pipefail
export RUN=${RUN:-r4p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
mkdir -p $O
bash tools/gpu_step.sh \
 "stats:150:cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $O/st -o st --output-format csv -- python3 $R/tools/eigh_prof.py && find $O/st -name '*kernel_trace.csv' -delete" \
 "fetch:120:cd /tmp && export TMPDIR=/tmp && timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pf -o pf --output-format csv -- python3 $R/tools/eigh_prof.py" \
 "grid:300:python3 $R/tools/trlan_ab.py --reps 2 --sectors '6,6;4,5;3,4' --grid 256,512,2048" \
 "sum:60:python3 $R/tools/pmc_summary.py $O/pf > $O/fetch_summary.txt; find $O/pf -name '*kernel_trace.csv' -delete; find $O/pf -name '*counter_collection.csv' -size +20M -delete"
du -sh $O
