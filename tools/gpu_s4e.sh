#!/bin/bash
# -m gpu suite at HEAD, then pass-U staged rows A/B (ED_KRON_UP_RU=1) for
# complex vectors / complex H on the N28 sector
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s4e}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
cd /tmp && export TMPDIR=/tmp
for v in "n28:--cvec" "n28:--complex" "n28b:--cvec"; do
  IFS=: read -r s a <<< "$v"
  for ru in 0 1; do
    if [ $ru = 1 ]; then export ED_KRON_UP_RU=1; else unset ED_KRON_UP_RU; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/st_${s}${a}_$ru" -o st --output-format csv -- \
      python3 "$R/tools/spmv_probe.py" --sector $s --path 2 $a --iters 30 > "$OUT/probe.log" 2>&1
    echo "$s $a RU1=$ru $(grep -o 'ms/launch=.*' $OUT/probe.log)"
    python3 - "$OUT/st_${s}${a}_$ru" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "kron" in r["Name"]:
        print("   ", r["Name"][:40], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
  done
done
find "$OUT" -name "*kernel_trace.csv" -delete
