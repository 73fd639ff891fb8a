#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6p${1:+_$1_$2}
mkdir -p $O
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/ep" -o ep --output-format csv -- python3 "$R/tools/eigh_prof.py" $1 $2 ) > $O/ep.log 2>&1 || { echo fail; tail -5 $O/ep.log; exit 1; }
grep eigh $O/ep.log
t=$(find $O/ep -name "*kernel_trace.csv" | head -1)
python3 $R/tools/timeline.py $t $O/ep_timeline.json
s=$(find $O/ep -name "*kernel_stats.csv" | head -1); cp $s $O/ep_kernel_stats.csv
python3 $R/tools/kstats.py $s
