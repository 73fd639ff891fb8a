#!/bin/bash
# Round-5 measurement call (RUN names the output directory).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
RUN=${RUN:-r5} bash tools/gpu_step.sh \
  "tests:600:$T tests/test_gpu_direct2.py tests/test_gpu_split.py tests/test_gpu_hxv.py" || exit 1
RUN=${RUN:-r5} bash tools/split_ab.sh \
  "r2:-:--sector n28 --split on" \
  "r1:tools/variants/lib_r1.so:--sector n28 --split on" \
  "r3:tools/variants/lib_r3.so:--sector n28 --split on" \
  "d26s_two:-:--sector n26s --path 1" \
  "d26s_one:-:--sector n26s --path 1 --options direct_exact" \
  "d28_two:-:--sector n28 --path 1" \
  "d28_one:-:--sector n28 --path 1 --options direct_exact" \
  "d28j_two:-:--sector n28j --path 1" \
  "d28j_one:-:--sector n28j --path 1 --options direct_exact"
