#!/bin/bash
# stored SpMV on the Nlevels=28 sector: parity tests, timing, kernel stats and
# HBM counters (FETCH_SIZE / WRITE_SIZE in separate passes) — real packed and
# complex packed H
set -eo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-spmv}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
cd /tmp && export TMPDIR=/tmp
for v in "real:--path 0" "cplx:--path 0 --complex" ${EXTRA}; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/st_$n -o st --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/spmv_probe.py --sector n28 $a --iters 20 > $O/probe_$n.log 2>&1
  grep ms/launch $O/probe_$n.log
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $O/pmc_${n}_$c -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/spmv_probe.py --sector n28 $a --iters 5 > /dev/null 2>&1
  done
done
find $O -name "*kernel_trace.csv" -delete
echo DONE
