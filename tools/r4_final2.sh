#!/bin/bash
# Round 4 final measurement, part 2: bench.py under rocprofv3 (roofline
# kernels' per-(kernel, grid) steady-state durations from the same command)
# and the default bench line (roofline now measured before the farm).
set -o pipefail
export RUN=${RUN:-r4final2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
bash tools/gpu_step.sh \
 "bprof:700:bash tools/bench_profile.sh r4 --no-farm --no-cpu" \
 "bench:500:python bench.py > $O/bench_line.json"
du -sh $O
