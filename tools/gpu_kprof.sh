#!/bin/bash
# per-kernel stats of the matrix-free N28 H·v for library variants (ED_GPU_LIB_VARIANT)
set -eo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-kprof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then unset ED_GPU_LIB_VARIANT; else export ED_GPU_LIB_VARIANT=$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/st_$v -o st --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/spmv_probe.py ${PROBE:---sector n28 --path 2} --iters 20 > $O/probe_$v.log 2>&1
  grep ms/launch $O/probe_$v.log
done
find $O -name "*kernel_trace.csv" -delete
echo DONE
