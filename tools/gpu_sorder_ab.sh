#!/bin/bash
# A/B of the stored packed SpMV slice schedules on the N28 sector:
# default (XCD row ranges), ED_GPU_SORDER=1 (column windows, window-major),
# ED_GPU_SORDER=2 (XCD column ranges, row-major inside); time + FETCH_SIZE.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-sorder}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in 0 1 2; do
  if [ $v = 0 ]; then unset ED_GPU_SORDER; else export ED_GPU_SORDER=$v; fi
  for cx in "" "--complex"; do
    timeout -k 10 120 python3 "$R/tools/spmv_probe.py" --sector n28 --path 0 $cx --iters 50 | tee -a "$OUT/ab.log"
  done
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_s$v" -o pmc --output-format csv -- \
    python3 "$R/tools/spmv_probe.py" --sector n28 --path 0 --iters 5 > "$OUT/pmc_s$v.log" 2>&1
  python3 "$R/tools/pmc_summary.py" "$OUT/pmc_s$v" > "$OUT/pmc_s$v.json"
done
find "$OUT" -name "*kernel_trace.csv" -size +2M -delete
echo AB_DONE
