#!/bin/bash
# Round 4, call 18: complex MODE 4, 512-thread form, natural vs slot-major
# LDS vector in one process (A/B), plus the batched complex rate.
set -o pipefail
export RUN=${RUN:-r4u}
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_step.sh \
 "cvec:200:python3 $R/tools/cvec_probe.py && python3 $R/tools/cvec_probe.py" \
 "tests:300:python -u -m pytest tests/test_gpu_lanczos.py -x -q --timeout 300 --timeout-method thread"
