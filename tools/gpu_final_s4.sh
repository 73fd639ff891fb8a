#!/bin/bash
# Final measurement pass (session 4 of round 2): -m gpu suite, smoke, the full
# bench line, and rocprofv3 kernel stats of the bench without the farm
# sections (rocprofv3 kernel tracing segfaults inside the farm's threaded
# hipGraph launches) plus the complex-vector two-pass H·v.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-final_s4}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 500 python3 bench.py > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
echo "bench ok"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/st_bench" -o st --output-format csv -- \
  python3 "$R/bench.py" --no-farm --no-cpu > "$OUT/bench_nofarm.log" 2>&1
tail -1 "$OUT/bench_nofarm.log" > "$OUT/bench_nofarm.json"
echo "bench prof ok"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/st_kron_cvec" -o st --output-format csv -- \
  python3 "$R/tools/spmv_probe.py" --sector n28 --path 2 --cvec --iters 30 > "$OUT/probe_kron_cvec.log" 2>&1
grep -o 'ms/launch=.*' "$OUT/probe_kron_cvec.log"
find "$OUT" -name "*kernel_trace.csv" -delete
echo FINAL_DONE
