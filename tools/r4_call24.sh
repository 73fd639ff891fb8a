#!/bin/bash
# Round 4, call 24: the default bench line once more, now that profiles/r4
# holds the two-column pass D traces it cross-checks against; smoke first.
set -o pipefail
export RUN=${RUN:-r4final8}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
bash tools/gpu_step.sh \
 "smoke:120:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "bench:500:python bench.py > $O/bench_line.json"
