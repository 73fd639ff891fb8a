#!/bin/bash
# rocprofv3 passes for profiles/ (run on the GPU box from the repo root).
# 1) kernel trace + stats of the bench command; 2-3) HBM counters of the
# roofline kernel in separate --pmc passes (FETCH_SIZE, WRITE_SIZE).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-prof}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/bench" -o bench --output-format csv -- \
  python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu --no-farm > "$OUT/bench_under_rocprof.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/spmv" -o spmv --output-format csv -- \
  python3 "$R/tools/spmv_probe.py" --sector n28 --path 0 --iters 20 > "$OUT/spmv_probe.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/fetch" -o fetch --output-format csv -- \
  python3 "$R/tools/spmv_probe.py" --sector n28 --path 0 --iters 5 > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/write" -o write --output-format csv -- \
  python3 "$R/tools/spmv_probe.py" --sector n28 --path 0 --iters 5 > "$OUT/write.log" 2>&1
# keep the summaries, drop the per-dispatch traces (size cap on gpurun_out/)
find "$OUT" -name "*kernel_trace.csv" -size +2M -delete
echo PROFILE_DONE
