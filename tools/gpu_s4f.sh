#!/bin/bash
# complex-vector pass D rows per wave: kron parity tests, then kernel stats
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s4f}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kron2.py tests/test_gpu_kron_split.py tests/test_gpu_dist.py tests/test_gpu_hxv.py -x -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
cd /tmp && export TMPDIR=/tmp
for v in "n28:--cvec" "n28:--complex" "n28b:--cvec" "n28:"; do
  IFS=: read -r s a <<< "$v"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/st_${s}${a}" -o st --output-format csv -- \
    python3 "$R/tools/spmv_probe.py" --sector $s --path 2 $a --iters 30 > "$OUT/probe.log" 2>&1
  echo "$s $a $(grep -o 'ms/launch=.*' $OUT/probe.log)"
  python3 - "$OUT/st_${s}${a}" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "kron" in r["Name"]:
        print("   ", r["Name"][:40], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
find "$OUT" -name "*kernel_trace.csv" -delete
