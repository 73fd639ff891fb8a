#!/bin/bash
# Round-5 final measurements, part B: the bench line, the GPU suite, the
# serial per-sector statistics of the configs[3] farm.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
O=gpurun_out/r5final2
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench_line.json
echo bench ok
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_suite.txt 2>&1 \
  || { echo "gpu suite failed"; tail -15 $O/gpu_suite.txt; exit 1; }
tail -2 $O/gpu_suite.txt
timeout -k 10 300 python -u tools/farm_prof.py --reps 1 --serial-stats $O/farm_c4_serial_stats.json > $O/farm_serial.log 2>&1 \
  || { echo "serial stats failed"; exit 1; }
echo serial ok
