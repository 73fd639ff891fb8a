#!/bin/bash
# Round-2 baseline on the GPU box (run from the repo root):
#   1) the -m gpu suite, 2) the full bench line,
#   3) rocprofv3 kernel stats of the matrix-free (k_kron, k_direct) and the
#      complex stored SpMV on the Nlevels=28 sector,
#   4) FETCH_SIZE / WRITE_SIZE passes for those kernels and for the
#      4/8/16-B streaming calibration probe (tools/fetch_calib).
# Every GPU step has its own time limit; the script stops at the first failure.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r2base}
mkdir -p "$OUT"
STEPS=${STEPS:-tests,bench,prof,pmc}
has() { [[ ",$STEPS," == *",$1,"* ]]; }

if has tests; then
  (cd "$R" && timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread) \
    > "$OUT/gpu_tests.log" 2>&1
  echo "tests ok"
fi
if has bench; then
  (cd "$R" && timeout -k 10 400 python -u bench.py) > "$OUT/bench.log" 2>&1
  tail -1 "$OUT/bench.log" > "$OUT/bench.json"
  echo "bench ok"
fi
cd /tmp && export TMPDIR=/tmp
if has prof; then
  for v in "kron:--path 2" "direct:--path 1" "cplx:--path 0 --complex" "pk:--path 0"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/st_$n" -o st --output-format csv -- \
      python3 "$R/tools/spmv_probe.py" --sector n28 $a --iters 20 > "$OUT/probe_$n.log" 2>&1
    echo "prof $n ok"
  done
fi
if has pmc; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace -d "$OUT/calib_$c" -o calib --output-format csv -- \
      "$R/tools/fetch_calib" > "$OUT/calib_$c.log" 2>&1
    for v in "kron:--path 2" "direct:--path 1" "cplx:--path 0 --complex"; do
      n=${v%%:*}; a=${v#*:}
      timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc_${n}_$c" -o pmc --output-format csv -- \
        python3 "$R/tools/spmv_probe.py" --sector n28 $a --iters 5 > "$OUT/pmc_${n}_$c.log" 2>&1
    done
    echo "pmc $c ok"
  done
fi
find "$OUT" -name "*kernel_trace.csv" -size +2M -delete
echo R2BASE_DONE
