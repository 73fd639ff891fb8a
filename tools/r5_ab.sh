#!/bin/bash
# Round-5 A/B experiments (DESIGN.md cites their gpurun_out run names):
#   bash tools/r5_ab.sh NAME     NAME in: passd wstream graph hwq hwq2 chc
# passd and chc compare against libraries built beforehand into tools/variants/
# (lib_base.so: the tree before the change; lib_chcN.so: -DED_PK_CHC=N builds).
# Each step under its own time limit; the first failure ends the run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
case "$1" in
  passd)  # Pass D XCD-balanced tiles: kron2 parity tests, then A/B of the two-pass Kronecker H·v (tree build vs tools/variants/lib_base.so) on N28, N28b, c4r.
    OUT=$R/gpurun_out/${RUN:-r5pd}; mkdir -p "$OUT"
    timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_kron2.py \
      tests/test_gpu_kron_split.py > "$OUT/tests.log" 2>&1 || { echo tests failed; tail -20 "$OUT/tests.log"; exit 1; }
    tail -2 "$OUT/tests.log"
    RUN=${RUN:-r5pd} bash tools/split_ab.sh \
      "new28:-:--sector n28 --path 2" "base28:tools/variants/lib_base.so:--sector n28 --path 2" \
      "new28b:-:--sector n28b --path 2" "base28b:tools/variants/lib_base.so:--sector n28b --path 2" \
      "newc4:-:--sector c4r --path 2" "basec4:tools/variants/lib_base.so:--sector c4r --path 2" \
      "new28r:-:--sector n28 --path 2" "base28r:tools/variants/lib_base.so:--sector n28 --path 2"
    ;;
  wstream)  # Farm worker streams (one HIP stream per worker thread for every sector it solves) against a private stream per sector: GPU tests of the farm and the configs[3] farm wall, alternating.
    OUT=$R/gpurun_out/${RUN:-r5ws}; mkdir -p "$OUT"
    timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_golden.py \
      tests/test_gpu_diag_gf.py > "$OUT/tests.log" 2>&1 || { echo tests failed; tail -20 "$OUT/tests.log"; exit 1; }
    tail -2 "$OUT/tests.log"
    for k in 1 2; do
      echo "== worker streams ($k)"
      timeout -k 10 200 python -u tools/farm_prof.py --reps 3 > "$OUT/ws$k.log" 2>&1 || { tail -5 "$OUT/ws$k.log"; exit 1; }
      grep "wall\|solves" "$OUT/ws$k.log"
      echo "== private streams ($k)"
      timeout -k 10 200 python -u tools/farm_prof.py --reps 3 --private-streams > "$OUT/ps$k.log" 2>&1 || { tail -5 "$OUT/ps$k.log"; exit 1; }
      grep "wall\|solves" "$OUT/ps$k.log"
    done
    ;;
  graph)  # configs[3] farm: Krylov sweeps replayed from hipGraphs (default) against direct launches (ED_OPT_NO_GRAPH), alternating.
    OUT=$R/gpurun_out/${RUN:-r5gr}; mkdir -p "$OUT"
    for k in 1 2; do
      echo "== graphs ($k)"
      timeout -k 10 200 python -u tools/farm_prof.py --reps 3 > "$OUT/g$k.log" 2>&1 || { tail -5 "$OUT/g$k.log"; exit 1; }
      grep "wall" "$OUT/g$k.log"
      echo "== no graphs ($k)"
      timeout -k 10 200 python -u tools/farm_prof.py --reps 3 --options no_graph > "$OUT/n$k.log" 2>&1 || { tail -5 "$OUT/n$k.log"; exit 1; }
      grep "wall" "$OUT/n$k.log"
    done
    ;;
  hwq)  # configs[3] farm with the worker streams: HIP's default 4 hardware queues against 8 (one per worker stream), alternating.
    OUT=$R/gpurun_out/${RUN:-r5hq}; mkdir -p "$OUT"
    for k in 1 2; do
      echo "== 4 queues ($k)"
      timeout -k 10 200 python -u tools/farm_prof.py --reps 3 > "$OUT/q4_$k.log" 2>&1 || { tail -5 "$OUT/q4_$k.log"; exit 1; }
      grep "wall" "$OUT/q4_$k.log"
      echo "== 8 queues ($k)"
      GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/farm_prof.py --reps 3 > "$OUT/q8_$k.log" 2>&1 || { tail -5 "$OUT/q8_$k.log"; exit 1; }
      grep "wall" "$OUT/q8_$k.log"
    done
    ;;
  hwq2)  # configs[3] farm with the worker streams: 4 hardware queues (default) with 8 workers, against 2 queues with 8 workers and 4 queues with 4 workers.
    OUT=$R/gpurun_out/${RUN:-r5hq2}; mkdir -p "$OUT"
    for k in 1 2; do
      echo "== 4 queues 8 workers ($k)"
      timeout -k 10 200 python -u tools/farm_prof.py --reps 3 > "$OUT/a$k.log" 2>&1 || { tail -5 "$OUT/a$k.log"; exit 1; }
      grep "wall" "$OUT/a$k.log"
      echo "== 2 queues 8 workers ($k)"
      GPU_MAX_HW_QUEUES=2 timeout -k 10 200 python -u tools/farm_prof.py --reps 3 > "$OUT/b$k.log" 2>&1 || { tail -5 "$OUT/b$k.log"; exit 1; }
      grep "wall" "$OUT/b$k.log"
      echo "== 4 queues 4 workers ($k)"
      timeout -k 10 200 python -u tools/farm_prof.py --reps 3 --workers 4 > "$OUT/c$k.log" 2>&1 || { tail -5 "$OUT/c$k.log"; exit 1; }
      grep "wall" "$OUT/c$k.log"
      echo "== 4 queues 12 workers ($k)"
      timeout -k 10 200 python -u tools/farm_prof.py --reps 3 --workers 12 > "$OUT/d$k.log" 2>&1 || { tail -5 "$OUT/d$k.log"; exit 1; }
      grep "wall" "$OUT/d$k.log"
    done
    ;;
  chc)  # Complex-vector one-pass stored H·v: gathers in flight per chunk (CH) 16 (tree) against 4 / 8 / 12 (tools/variants/lib_chcN.so), N28 and nonSU2 N26.
    OUT=$R/gpurun_out/${RUN:-r5chc}; mkdir -p "$OUT"
    RUN=${RUN:-r5chc} bash tools/split_ab.sh \
      "c16:tools/variants/lib_chc16.so:--sector n28 --path 0 --complex --split off" \
      "c8:tools/variants/lib_chc8.so:--sector n28 --path 0 --complex --split off" \
      "c12:tools/variants/lib_chc12.so:--sector n28 --path 0 --complex --split off" \
      "c4:tools/variants/lib_chc4.so:--sector n28 --path 0 --complex --split off" \
      "c16r:tools/variants/lib_chc16.so:--sector n28 --path 0 --complex --split off" \
      "c8r:tools/variants/lib_chc8.so:--sector n28 --path 0 --complex --split off" \
      "s16:tools/variants/lib_chc16.so:--sector n26s --path 0 --complex --split off" \
      "s8:tools/variants/lib_chc8.so:--sector n26s --path 0 --complex --split off" \
      "s12:tools/variants/lib_chc12.so:--sector n26s --path 0 --complex --split off"
    ;;
  *) echo "usage: bash tools/r5_ab.sh {passd|wstream|graph|hwq|hwq2|chc}"; exit 2 ;;
esac
