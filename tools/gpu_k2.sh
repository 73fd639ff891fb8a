#!/bin/bash
# two-pass Kronecker H·v: parity tests, timing, kernel stats and HBM counters (N28)
set -eo pipefail
O=gpurun_out/${1:-k2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_kron2.py} -x -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for a in "--sector n28 --path 2" "--sector n28 --path 2 --cvec" "--sector n28b --path 2" "--sector c4 --path 2"; do
  timeout -k 10 120 python tools/spmv_probe.py $a --iters 50 >> $O/probe.log 2>&1
done
grep ms/launch $O/probe.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/st -o st --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/spmv_probe.py --sector n28 --path 2 --iters 20 > /dev/null 2>&1
for c in FETCH_SIZE WRITE_SIZE; do timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $GRAFT_REPO_ROOT/$O/pmc_$c -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/spmv_probe.py --sector n28 --path 2 --iters 5 > /dev/null 2>&1; done
find $GRAFT_REPO_ROOT/$O -name "*kernel_trace.csv" -delete
echo DONE
