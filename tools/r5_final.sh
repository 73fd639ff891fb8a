#!/bin/bash
# Round-5 final measurements, part A: the remaining roofline profiles and
# bench.py under rocprofv3.  Each step under its own limit, stopping at the
# first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
mkdir -p gpurun_out/r5final
timeout -k 10 900 bash tools/gpu_profiles.sh r5 spmv_c4 kron_c4 kron_n28b spmv_n28j spmv_n28j_cplx direct_n28j \
  spmv_n26s spmv_n26s_cplx direct_n26s > gpurun_out/r5final/profiles.log 2>&1 || { echo "profiles failed"; exit 1; }
echo profiles ok
timeout -k 10 500 bash tools/bench_profile.sh r5 --no-farm --no-cpu > gpurun_out/r5final/bench_profile.log 2>&1 \
  || { echo "bench profile failed"; exit 1; }
echo bench profile ok
