#!/bin/bash
# One rocprofv3 counter pass (no trace domains besides the kernel trace the
# counters are attributed by), under a hard time limit:
#   tools/pmc_pass.sh OUTDIR NAME "COUNTER ..." python3 tools/spmv_probe.py ...
# -> OUTDIR/NAME (rocprofv3 csv) and OUTDIR/NAME.json (per-kernel medians).
set -o pipefail
OUT=$1; NAME=$2; CTR=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$OUT"
( cd /tmp && export TMPDIR=/tmp && \
  timeout -s KILL 90 rocprofv3 --pmc $CTR -d "$OUT/$NAME" -o pmc --output-format csv -- "$@" ) \
  > "$OUT/$NAME.log" 2>&1 || { echo "pmc pass $NAME failed"; tail -5 "$OUT/$NAME.log"; exit 1; }
python3 "$R/tools/pmc_summary.py" "$OUT/$NAME" > "$OUT/$NAME.json"
find "$OUT/$NAME" -name "*.csv" -size +4M -delete
echo "pmc pass $NAME ok"
