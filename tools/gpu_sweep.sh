#!/bin/bash
# SURVEY 8(d) roofline sweep beyond N28 Norb=1: kernel stats and HBM counter
# passes (FETCH_SIZE / WRITE_SIZE, one counter per run) of the packed stored
# and the matrix-free H·v on the Norb=2 Nbath=6 (7,7) sector (n28b) and the
# configs[3] (6,6) sector (c4r) -> profiles/r2/{spmv,kron}_{n28b,c4}_traffic.json
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-sweep}
mkdir -p "$OUT" "$R/profiles/r2"
cd /tmp && export TMPDIR=/tmp
for s in n28b c4r; do
  t=${s%r}
  for v in "pk:--path 0:k_spmv_pk<false:spmv" "kron:--path 2:k_kron:kron"; do
    IFS=: read -r n a pat pre <<< "$v"
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/st_${s}_$n" -o st --output-format csv -- \
      python3 "$R/tools/spmv_probe.py" --sector $s $a --iters 50 > "$OUT/probe_${s}_$n.log" 2>&1
    grep ms/launch "$OUT/probe_${s}_$n.log"
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc_${s}_${n}_$c" -o pmc --output-format csv -- \
        python3 "$R/tools/spmv_probe.py" --sector $s $a --iters 5 > "$OUT/pmc_${s}_${n}_$c.log" 2>&1
    done
    f=${pre}_${t}_traffic.json
    python3 "$R/tools/traffic_json.py" "$OUT/$f" "$pat" "$OUT/pmc_${s}_${n}_FETCH_SIZE" "$OUT/pmc_${s}_${n}_WRITE_SIZE" "$s --path ${a}" > /dev/null
    cp "$OUT/$f" "$R/profiles/r2/$f"
    echo "sweep $s $n ok"
  done
done
find "$OUT" -name "*kernel_trace.csv" -size +2M -delete
cd "$R"
timeout -k 10 500 python3 bench.py > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
echo SWEEP_DONE
