set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gsweep; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for g in 1536 1720 2048 2560 3440; do
  export ED_KRON_DW_GRID=$g
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/st" -o st --output-format csv -- python3 "$R/tools/spmv_probe.py" --sector n28 --path 2 --iters 30 > /dev/null 2>&1
  python3 - "$OUT/st" $g <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "kron_dw" in r["Name"]: print("grid", sys.argv[2], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
  rm -rf "$OUT/st"
done
