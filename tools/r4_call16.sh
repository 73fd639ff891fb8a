#!/bin/bash
# Round 4, call 16: k_cgs transposing multi-value reduction + Krylov grid
# cap 512: eigensolver parity, per-sector A/B, farm.
set -o pipefail
export RUN=${RUN:-r4s}
R=${GRAFT_REPO_ROOT:-$(pwd)}
F="python3 $R/tools/farm_prof.py"
bash tools/gpu_step.sh \
 "tests:500:python -u -m pytest tests/test_gpu_eigh.py tests/test_gpu_golden.py tests/test_gpu_diag_gf.py tests/test_gpu_lanczos.py -x -q --timeout 300 --timeout-method thread" \
 "ab:300:python3 $R/tools/trlan_ab.py --reps 3 --grid 384" \
 "farm:300:$F --reps 4"
