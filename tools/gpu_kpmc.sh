#!/bin/bash
# PMC passes (one counter group per run) on the probe kernel(s)
set -eo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-kpmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace -d $O/p$i -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/spmv_probe.py ${PROBE:---sector n28 --path 2} --iters 5 > $O/p$i.log 2>&1
  echo "pass $i ok: $ctrs"
done < ${PASSES:-$GRAFT_REPO_ROOT/tools/pmc_passes.txt}
find $O -name "*kernel_trace.csv" -delete
echo DONE
