#!/bin/bash
# per-kernel stats (and, with PMC="CTR ...", one counter pass per counter) of
# an H·v probe for library variants (ED_GPU_LIB_VARIANT); PROBE selects the
# sector/path (default: matrix-free Kronecker H·v on the Nlevels=28 sector)
set -eo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-kprof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then unset ED_GPU_LIB_VARIANT; else export ED_GPU_LIB_VARIANT=$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/st_$v -o st --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/spmv_probe.py ${PROBE:---sector n28 --path 2} --iters 20 > $O/probe_$v.log 2>&1
  grep ms/launch $O/probe_$v.log
  for c in $PMC; do
    timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace -d $O/pmc_${v}_$c -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/spmv_probe.py ${PROBE:---sector n28 --path 2} --iters 5 > /dev/null 2>&1
  done
done
find $O -name "*kernel_trace.csv" -delete
echo DONE
