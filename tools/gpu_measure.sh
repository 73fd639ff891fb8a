#!/bin/bash
# One GPU call of the round's measurement pass (tools/gpu_step.sh steps, each
# under its own time limit, stop at the first failure):
#   the bench line (-> gpurun_out/$RUN/bench.json; copy to profiles/<round>/bench_line.json),
#   the bench without the farm sections under rocprofv3 --kernel-trace --stats,
#   the configs[3] farm kernel statistics (1 worker), the GPU suite and smoke.
# Kernel statistics and HBM counter passes of the roofline entries come from
# tools/gpu_profiles.sh (run it first when a kernel changed).
#   RUN=name bash tools/gpu_measure.sh
set -e -o pipefail
export RUN=${RUN:-measure}
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_step.sh \
 "bench:600:python3 bench.py > gpurun_out/$RUN/bench.json" \
 "bprof:300:cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$RUN/bprof -o bp --output-format csv -- python3 $R/bench.py --no-farm --no-cpu" \
 "farmprof:300:bash tools/farm_rocprof.sh w1" \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:120:python3 -c 'import __graft_entry__ as g; g.smoke()'"
