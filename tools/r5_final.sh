#!/bin/bash
# Round-5 closing measurements (profiles/r5/INDEX.md cites the part):
#   A: the remaining roofline profiles and bench.py under rocprofv3;
#   B: the bench line, the GPU suite, the serial farm statistics;
#   C: after the pass-D tile deal and the farm worker streams: the Kronecker
#      roofline entries, bench.py under rocprofv3, the bench line, the GPU
#      suite and the serial farm statistics (the committed profiles/r5 set).
#   bash tools/r5_final.sh A|B|C
# Each step under its own limit, stopping at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
case "$1" in
  A)
    mkdir -p gpurun_out/r5final
    timeout -k 10 900 bash tools/gpu_profiles.sh r5 spmv_c4 kron_c4 kron_n28b spmv_n28j spmv_n28j_cplx direct_n28j \
      spmv_n26s spmv_n26s_cplx direct_n26s > gpurun_out/r5final/profiles.log 2>&1 || { echo "profiles failed"; exit 1; }
    echo profiles ok
    timeout -k 10 500 bash tools/bench_profile.sh r5 --no-farm --no-cpu > gpurun_out/r5final/bench_profile.log 2>&1 \
      || { echo "bench profile failed"; exit 1; }
    echo bench profile ok
    ;;
  B)
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
    ;;
  C)
    O=gpurun_out/r5final3
    mkdir -p $O
    timeout -k 10 400 bash tools/gpu_profiles.sh r5 kron_n28 kron_n28b kron_c4 > $O/profiles.log 2>&1 \
      || { echo "profiles failed"; tail -5 $O/profiles.log; exit 1; }
    echo profiles ok
    timeout -k 10 500 bash tools/bench_profile.sh r5 --no-farm --no-cpu > $O/bench_profile.log 2>&1 \
      || { echo "bench profile failed"; tail -5 $O/bench_profile.log; exit 1; }
    echo bench profile ok
    timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
    grep '^{' $O/bench.log > $O/bench_line.json
    echo bench ok
    timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_suite.txt 2>&1 \
      || { echo "gpu suite failed"; tail -15 $O/gpu_suite.txt; exit 1; }
    tail -2 $O/gpu_suite.txt
    timeout -k 10 300 python -u tools/farm_prof.py --reps 3 --serial-stats $O/farm_c4_serial_stats.json > $O/farm_serial.log 2>&1 \
      || { echo "serial stats failed"; exit 1; }
    grep "serial totals\|wall" $O/farm_serial.log
    ;;
  *) echo "usage: bash tools/r5_final.sh A|B|C"; exit 2 ;;
esac
