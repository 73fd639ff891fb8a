#!/bin/bash
# Round 4 final measurement: the whole GPU suite, smoke, the default bench
# line, and bench.py under rocprofv3 (kernel statistics + per-sector
# steady-state traces into profiles/r4).
set -o pipefail
export RUN=${RUN:-r4final4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
bash tools/gpu_step.sh \
 "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "smoke:120:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "bench:500:python bench.py > $O/bench_line.json" \
 "bprof:700:bash tools/bench_profile.sh r4 --no-farm --no-cpu"
du -sh $O
