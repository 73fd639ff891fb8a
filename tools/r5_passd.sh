#!/bin/bash
# Pass D XCD-balanced tiles: kron2 parity tests, then A/B of the two-pass
# Kronecker H·v (tree build vs tools/variants/lib_base.so) on N28, N28b, c4r.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${RUN:-r5pd}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_kron2.py \
  tests/test_gpu_kron_split.py > "$OUT/tests.log" 2>&1 || { echo tests failed; tail -20 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
RUN=${RUN:-r5pd} bash tools/split_ab.sh \
  "new28:-:--sector n28 --path 2" "base28:tools/variants/lib_base.so:--sector n28 --path 2" \
  "new28b:-:--sector n28b --path 2" "base28b:tools/variants/lib_base.so:--sector n28b --path 2" \
  "newc4:-:--sector c4r --path 2" "basec4:tools/variants/lib_base.so:--sector c4r --path 2" \
  "new28r:-:--sector n28 --path 2" "base28r:tools/variants/lib_base.so:--sector n28 --path 2"
