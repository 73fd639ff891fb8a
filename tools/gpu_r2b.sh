#!/bin/bash
# Round-2 call B: parity of the diag/GF/farm paths (device-resident state
# vectors), farm_c4 phase breakdown, FETCH/WRITE calibration, PMC passes of
# the matrix-free and complex stored kernels on the Nlevels=28 sector.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r2b}
mkdir -p "$OUT"
STEPS=${STEPS:-tests,phase,calib,pmc}
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has tests; then
  (cd "$R" && timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_diag_gf.py tests/test_gpu_golden.py tests/test_gpu_jz.py tests/test_gpu_dist.py} -x -q --timeout 200 --timeout-method thread) \
    > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
  tail -2 "$OUT/tests.log"
fi
if has phase; then
  (cd "$R" && timeout -k 10 300 python -u tools/farm_phase.py) > "$OUT/farm_phase.log" 2>&1
  cp "$R/gpurun_out/farm_c4_phases.json" "$OUT/" ; tail -1 "$OUT/farm_phase.log"
fi
cd /tmp && export TMPDIR=/tmp
if has calib; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace -d "$OUT/calib_$c" -o calib --output-format csv -- \
      "$R/tools/fetch_calib" > "$OUT/calib_$c.log" 2>&1
  done
  echo "calib ok"
fi
if has pmc; then
  i=0
  while read -r ctrs; do
    [ -z "$ctrs" ] && continue
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace -d "$OUT/kron_p$i" -o p --output-format csv -- \
      python3 "$R/tools/spmv_probe.py" --sector n28 --path 2 --iters 5 > "$OUT/kron_p$i.log" 2>&1
    echo "kron pass $i ok"
  done < "$R/tools/pmc_kron.txt"
  for v in "direct:--path 1" "cplx:--path 0 --complex" "pk:--path 0"; do
    n=${v%%:*}; a=${v#*:}
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc_${n}_$c" -o pmc --output-format csv -- \
        python3 "$R/tools/spmv_probe.py" --sector n28 $a --iters 5 > "$OUT/pmc_${n}_$c.log" 2>&1
    done
    echo "pmc $n ok"
  done
fi
find "$OUT" -name "*kernel_trace.csv" -size +2M -delete
echo R2B_DONE
