#!/bin/bash
# two-pass Kronecker with 12-slot instantiations and hop-count skipping:
# parity tests, then per-kernel stats on n28b / n28 (RU=2 default vs RU=1)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-kdeg}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kron2.py tests/test_gpu_kron_split.py tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
cd /tmp && export TMPDIR=/tmp
for v in "n28b:0" "n28b:1" "n28:0"; do
  IFS=: read -r s ru <<< "$v"
  if [ $ru = 1 ]; then export ED_KRON_UP_RU=1; else unset ED_KRON_UP_RU; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/st_${s}_$ru" -o st --output-format csv -- \
    python3 "$R/tools/spmv_probe.py" --sector $s --path 2 --iters 50 > "$OUT/probe_${s}_$ru.log" 2>&1
  grep ms/launch "$OUT/probe_${s}_$ru.log"
  python3 - "$OUT/st_${s}_$ru" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "kron" in r["Name"]:
        print("   ", r["Name"][:48], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
find "$OUT" -name "*kernel_trace.csv" -size +2M -delete
echo KDEG_DONE
