#!/bin/bash
# bench.py itself under rocprofv3 (--kernel-trace --stats): the roofline
# kernels' per-launch durations from the same command whose line reports
# them.  Per (kernel, grid) group the bench's 5 warm-up launches are dropped
# (tools/trace_summary.py), so each sector's steady-state average sits beside
# the line's HIP-event `ms_per_launch`.
#   bash tools/bench_profile.sh TAG [bench.py arguments]
# -> gpurun_out/bprof_TAG/profiles/ (merged back by gpurun; copy to
#    profiles/TAG): bench_kernel_stats.csv, bench_trace_{spmv,spmv_cplx,kron,direct}.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r5}; shift
OUT=$R/gpurun_out/bprof_$TAG
P=$OUT/profiles
mkdir -p "$OUT" "$P"
( cd /tmp && export TMPDIR=/tmp && \
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/st" -o st --output-format csv -- \
    python3 "$R/bench.py" "$@" ) > "$OUT/bench.log" 2>&1 || { echo "profiled bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" > "$OUT/bench_line.json" || true
t=$(find "$OUT/st" -name "*kernel_trace.csv" | head -1)
s=$(find "$OUT/st" -name "*kernel_stats.csv" | head -1)
[ -n "$s" ] && cp "$s" "$P/bench_kernel_stats.csv"
# (persist: the headline configs[1] launches — one 512-thread workgroup,
# grid 512 — apart from the batched ones of the same instantiation, whose
# grids are K x 512: the runs split them)
for e in "split|k_spmv_s[ab]<false, false" "spmv|k_spmv_pk<false, false" "spmv_cplx|k_spmv_pk<true, true" \
         "fused_cplx|k_spmv_fu<true, true" "fused_cvec|k_spmv_fu<false, true" \
         "kron|k_kron_(up|dw)" "direct|k_direct<" "persist|k_lanc_persist<"; do
  IFS='|' read -r name pat <<< "$e"
  python3 "$R/tools/trace_summary.py" "$t" "$pat" 5 "$P/bench_trace_$name.json" \
    --note "rocprofv3 of bench.py $*: per (kernel, grid) group, 5 warm-up launches dropped" \
    || { echo "trace summary $name failed"; exit 1; }
done
find "$OUT" -name "*kernel_trace.csv" -delete
echo BENCH_PROFILE_DONE
