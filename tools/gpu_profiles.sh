#!/bin/bash
# Kernel statistics and HBM counter passes for every roofline entry of the
# bench line (headline N28 + SURVEY 8(d) sweep):
#   rocprofv3 --kernel-trace --stats   -> <name>_kernel_stats.csv
#   --pmc FETCH_SIZE, --pmc WRITE_SIZE -> <name>_traffic.json
# (one counter per run, each pass under its own hard time limit), written to
# gpurun_out/prof_$TAG/profiles/ (merged back by gpurun; copy to profiles/$TAG).
#   bash tools/gpu_profiles.sh TAG [name ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r3}; shift
OUT=$R/gpurun_out/prof_$TAG
PROF=$OUT/profiles
mkdir -p "$OUT" "$PROF"
# name | spmv_probe arguments | kernel-name regex
ENTRIES=(
  "spmv_n28|--sector n28 --path 0 --split off --fused off|k_spmv_pk<false"
  "split_n28|--sector n28 --path 0 --split on|k_spmv_s[ab]<false"
  "split_n28j|--sector n28j --path 0 --split on|k_spmv_s[ab]<false"
  "split_n26s|--sector n26s --path 0 --split on|k_spmv_s[ab]<false"
  "split_n28b|--sector n28b --path 0 --split on|k_spmv_s[ab]<false"
  "spmv_cplx_n28|--sector n28 --path 0 --complex --split off --fused off|k_spmv_pk<true"
  "fused_cplx_n28|--sector n28 --path 0 --complex|k_spmv_fu"
  "spmv_cvec_n28|--sector n28 --path 0 --cvec --split off --fused off|k_spmv_pk<false"
  "fused_cvec_n28|--sector n28 --path 0 --cvec|k_spmv_fu"
  "kron_n28|--sector n28 --path 2|k_kron"
  "direct_n28|--sector n28 --path 1|k_direct"
  "spmv_n28b|--sector n28b --path 0 --split off --fused off|k_spmv_pk<false"
  "kron_n28b|--sector n28b --path 2|k_kron"
  "spmv_c4|--sector c4r --path 0 --split off|k_spmv_pk<false"
  "kron_c4|--sector c4r --path 2|k_kron"
  "spmv_n28j|--sector n28j --path 0 --split off --fused off|k_spmv_pk<false"
  "spmv_n28j_cplx|--sector n28j --path 0 --complex --split off --fused off|k_spmv"
  "fused_n28j|--sector n28j --path 0|k_spmv_fu"
  "fused_n28j_cplx|--sector n28j --path 0 --complex|k_spmv_fu"
  "direct_n28j|--sector n28j --path 1|k_direct"
  "spmv_n26s|--sector n26s --path 0 --split off --fused off|k_spmv_pk<false"
  "spmv_n26s_cplx|--sector n26s --path 0 --complex --split off --fused off|k_spmv"
  "direct_n26s|--sector n26s --path 1|k_direct"
)
want=" $* "
for e in "${ENTRIES[@]}"; do
  IFS='|' read -r name args pat <<< "$e"
  if [ $# -gt 0 ] && [[ "$want" != *" $name "* ]]; then continue; fi
  ( cd /tmp && export TMPDIR=/tmp && \
    timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$OUT/st_$name" -o st --output-format csv -- \
      python3 "$R/tools/spmv_probe.py" $args --iters 30 ) > "$OUT/st_$name.log" 2>&1 \
    || { echo "stats $name failed"; tail -5 "$OUT/st_$name.log"; exit 1; }
  grep ms/launch "$OUT/st_$name.log"
  f=$(find "$OUT/st_$name" -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" "$PROF/${name}_kernel_stats.csv"
  # steady-state per-launch durations (the probe's 3 warm-ups dropped): the
  # figure bench.py's HIP-event average is compared with
  t=$(find "$OUT/st_$name" -name "*kernel_trace.csv" | head -1)
  [ -n "$t" ] && python3 "$R/tools/trace_summary.py" "$t" "$pat" 3 "$PROF/${name}_trace.json" \
    --note "spmv_probe.py $args --iters 30: 3 warm-up + 60 launches" > /dev/null
  for c in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && export TMPDIR=/tmp && \
      timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc_${name}_$c" -o pmc --output-format csv -- \
        python3 "$R/tools/spmv_probe.py" $args --iters 5 ) > "$OUT/pmc_${name}_$c.log" 2>&1 \
      || { echo "pmc $name $c failed"; tail -5 "$OUT/pmc_${name}_$c.log"; exit 1; }
  done
  python3 "$R/tools/traffic_json.py" "$PROF/${name}_traffic.json" "$pat" "$OUT/pmc_${name}_FETCH_SIZE" \
    "$OUT/pmc_${name}_WRITE_SIZE" "spmv_probe.py $args" > /dev/null || { echo "traffic $name failed"; exit 1; }
  mkdir -p "$R/profiles/$TAG" && cp "$PROF/${name}_traffic.json" "$R/profiles/$TAG/"  # for a bench.py later in the same call
  [ -f "$PROF/${name}_trace.json" ] && cp "$PROF/${name}_trace.json" "$R/profiles/$TAG/"
  echo "profile $name ok"
done
find "$OUT" -name "*kernel_trace.csv" -size +2M -delete
echo PROFILES_DONE
