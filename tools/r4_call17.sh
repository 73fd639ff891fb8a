#!/bin/bash
# Round 4, call 17: sanity of the final library build (eigensolver, golden,
# Lanczos, H·v) and smoke.
set -o pipefail
export RUN=${RUN:-r4t}
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_step.sh \
 "tests:500:python -u -m pytest tests/test_gpu_eigh.py tests/test_gpu_golden.py tests/test_gpu_lanczos.py tests/test_gpu_hxv.py -x -q --timeout 300 --timeout-method thread" \
 "smoke:120:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
