#!/bin/bash
# pass-D grid A/B (ED_KRON_DW_GRID) for real / complex vectors on N28
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s4g}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kron2.py tests/test_gpu_kron_split.py -x -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
cd /tmp && export TMPDIR=/tmp
for a in "--cvec" "--complex" ""; do
  for g in 512 1024 2048; do
    export ED_KRON_DW_GRID=$g
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/st" -o st --output-format csv -- \
      python3 "$R/tools/spmv_probe.py" --sector n28 --path 2 $a --iters 30 > "$OUT/probe.log" 2>&1
    python3 - "$OUT/st" "$a" "$g" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "kron_dw" in r["Name"]:
        print(sys.argv[2] or "real", "grid", sys.argv[3], r["Name"][:34], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
    rm -rf "$OUT/st"
  done
done
