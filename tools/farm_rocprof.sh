#!/bin/bash
# The configs[3] farm under rocprofv3 --kernel-trace --stats, in the variants
# that separate the suspects of the round-2 profiler crash (hipGraph launches
# from concurrent host threads): graphs on / off (ED_OPT_NO_GRAPH), 8 workers
# / 1 worker.  Each run under its own time limit; exit status and the tail of
# the profiler's stderr per variant in gpurun_out/$RUN/farm_rocprof.txt.
#   RUN=name bash tools/farm_rocprof.sh [variant ...]   (default: w1 w8nograph w8; also c5w1:
#   configs[4] ground state + Green's function, tools/c5_run.py)
# Runs the variants in the order given and stops at the first failing one.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${RUN:-farmprof}
mkdir -p "$OUT"
SUM=$OUT/farm_rocprof.txt
vars=${*:-w1 w8nograph w8}
for v in $vars; do
  case $v in
    w8) args="--workers 8 --reps 1" ;;
    w8nograph) args="--workers 8 --reps 1 --options no_graph" ;;
    w1) args="--workers 1 --reps 1" ;;
    w2) args="--workers 2 --reps 1" ;;
    w4) args="--workers 4 --reps 1" ;;
    c5w1) args="" ;;
    *) echo "unknown variant $v"; exit 2 ;;
  esac
  ( cd /tmp && export TMPDIR=/tmp && \
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/fp_$v" -o fp --output-format csv -- \
      python3 "$R/tools/$([ $v = c5w1 ] && echo c5_run.py || echo farm_prof.py)" $args ) > "$OUT/fp_$v.log" 2>&1
  rc=$?
  echo "=== $v rc=$rc" | tee -a "$SUM"
  grep -E "farm workers|c5 diag|Segmentation|signal|Error|error|Abort" "$OUT/fp_$v.log" | head -20 | tee -a "$SUM"
  tail -5 "$OUT/fp_$v.log" >> "$SUM"
  t=$(find "$OUT/fp_$v" -name "*kernel_trace.csv" | head -1)
  [ -n "$t" ] && python3 "$R/tools/timeline.py" "$t" "$OUT/fp_${v}_timeline.json" | tee -a "$SUM"
  find "$OUT/fp_$v" -name "*kernel_trace.csv" -size +2M -delete 2>/dev/null
  # after a crash, abort, time limit or kill: no further GPU work in this call
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo FARM_ROCPROF_DONE
