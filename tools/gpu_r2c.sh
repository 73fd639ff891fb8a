#!/bin/bash
# Round-2 measurement pass: -m gpu suite, HBM counter passes of the kernels on
# the bench line (FETCH_SIZE / WRITE_SIZE, one counter per run) -> traffic
# summaries, then bench.py under rocprofv3 --kernel-trace --stats.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r2c}
mkdir -p "$OUT"
STEPS=${STEPS:-tests,phase,pmc,bench}
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has tests; then
  (cd "$R" && timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread) \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
  tail -2 "$OUT/gpu_tests.log"
fi
if has phase; then
  (cd "$R" && timeout -k 10 300 python -u tools/farm_phase.py) > "$OUT/farm_phase.log" 2>&1
  cp "$R/gpurun_out/farm_c4_phases.json" "$OUT/"
  echo "phase ok"
fi
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/profiles/r2"
if has pmc; then
  for v in "kron:--path 2:k_kron_" "pk:--path 0:k_spmv_pk<false" "cplx:--path 0 --complex:k_spmv_pk<true" "direct:--path 1:k_direct"; do
    IFS=: read -r n a pat <<< "$v"
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc_${n}_$c" -o pmc --output-format csv -- \
        python3 "$R/tools/spmv_probe.py" --sector n28 $a --iters 5 > "$OUT/pmc_${n}_$c.log" 2>&1
    done
    case $n in
      kron) f=kron_n28_traffic.json;; pk) f=spmv_n28_traffic.json;; cplx) f=spmv_cplx_n28_traffic.json;; direct) f=direct_n28_traffic.json;;
    esac
    python3 "$R/tools/traffic_json.py" "$OUT/$f" "$pat" "$OUT/pmc_${n}_FETCH_SIZE" "$OUT/pmc_${n}_WRITE_SIZE" "N28 (7,7) --path ${a}" > /dev/null
    cp "$OUT/$f" "$R/profiles/r2/$f"
    echo "pmc $n ok"
  done
fi
if has bench; then
  # the full line (farm / GF sections included) without the profiler, then the
  # kernel stats of the same command minus the farm sections: rocprofv3's
  # kernel tracing segfaults inside hipGraph launches made from the farm's
  # concurrent host threads (ed_sector_eigh sweeps), observed on this image
  (cd "$R" && timeout -k 10 500 python3 bench.py) > "$OUT/bench.log" 2>&1
  tail -1 "$OUT/bench.log" > "$OUT/bench.json"
  echo "bench ok"
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/bench_prof" -o bench --output-format csv -- \
    python3 "$R/bench.py" --no-farm > "$OUT/bench_prof.log" 2>&1
  tail -1 "$OUT/bench_prof.log" > "$OUT/bench_nofarm.json"
  echo "bench prof ok"
fi
find "$OUT" -name "*kernel_trace.csv" -size +2M -delete
echo R2C_DONE
