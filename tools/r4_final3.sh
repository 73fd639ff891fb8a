#!/bin/bash
# Round 4: bench.py under rocprofv3 again, trace summaries with per-run
# (per-sector) steady-state durations.
set -o pipefail
export RUN=${RUN:-r4final3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_step.sh "bprof:700:bash tools/bench_profile.sh r4 --no-farm --no-cpu"
