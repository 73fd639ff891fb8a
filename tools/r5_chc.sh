#!/bin/bash
# Complex-vector one-pass stored H·v: gathers in flight per chunk (CH) 16
# (tree) against 4 / 8 / 12 (tools/variants/lib_chcN.so), N28 and nonSU2 N26.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
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
