#!/bin/bash
# Round 4, call 12: dynamic multi-rank farm schedule on the GPU box (2 ranks
# on one GPU over gloo through the whole bench; RCCL world-1 paths).
set -o pipefail
export RUN=${RUN:-r4l}
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_step.sh \
 "tests:600:python -u -m pytest tests/test_bench_launch.py tests/test_gpu_nccl.py tests/test_gpu_golden.py -x -q -m gpu --timeout 500 --timeout-method thread"
