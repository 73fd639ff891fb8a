#!/bin/bash
# A/B of environment switches on one H·v probe: kernel stats + optional PMC.
# usage: ENVS="name1:VAR=val name2:..." PROBE="--sector n28 --path 2" PMC="FETCH_SIZE" bash tools/gpu_kab.sh out
set -eo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-kab}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for e in ${ENVS:-base:ED_NONE=1}; do
  n=${e%%:*}; kv=${e#*:}
  export ${kv//,/ }
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/st_$n -o st --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/spmv_probe.py ${PROBE:---sector n28 --path 2} --iters 20 > $O/probe_$n.log 2>&1
  echo "$n $(grep ms/launch $O/probe_$n.log)"
  for c in $PMC; do
    timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace -d $O/pmc_${n}_$c -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/spmv_probe.py ${PROBE:---sector n28 --path 2} --iters 5 > /dev/null 2>&1
  done
  for v in ${kv//,/ }; do unset ${v%%=*}; done
done
find $O -name "*kernel_trace.csv" -delete
echo DONE
