#!/bin/bash
# Round-5 measurement call (RUN names the output directory).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
RUN=${RUN:-r5} bash tools/gpu_step.sh \
  "tests:600:$T tests/test_gpu_eigh.py tests/test_gpu_golden.py tests/test_gpu_split.py tests/test_gpu_diag_gf.py" \
  "trlan:300:python -u tools/trlan_ab.py --reps 3 --opts trlan_nofoldnrm" \
  "farm:300:python -u tools/farm_prof.py --reps 3" \
  "farm_closing:300:python -u tools/farm_prof.py --reps 3 --options trlan_nofoldnrm" \
  "farm_w6:300:python -u tools/farm_prof.py --reps 3 --workers 6"
