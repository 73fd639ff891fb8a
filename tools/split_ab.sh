#!/bin/bash
# A/B of two-segment stored H·v builds (tools/variants/*.so vs the tree's
# libedgpu.so): rocprofv3 kernel statistics of spmv_probe.py on the N28 sector.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${RUN:-splitab}
mkdir -p "$OUT"
for v in "$@"; do
  name=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; args=${rest#*:}
  libarg=""; [ "$lib" != "-" ] && libarg="--lib $R/$lib"
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o st \
      --output-format csv -- python3 "$R/tools/spmv_probe.py" $libarg $args --iters 30 ) > "$OUT/$name.log" 2>&1 \
    || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep "ms/launch\|per-launch" "$OUT/$name.log"
  f=$(find "$OUT/$name" -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$name" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_spmv" in r["Name"] or "k_kron" in r["Name"] or "k_direct" in r["Name"]:
        print(sys.argv[2], r["Name"][:70], r["Calls"], "avg_us=%.1f" % (float(r["AverageNs"]) / 1e3))
PY
  find "$OUT/$name" -name "*kernel_trace.csv" -delete
done
