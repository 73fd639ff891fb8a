#!/bin/bash
# Round 4, call 27: non-temporal Hv stores in every plain-store H·v — the
# whole GPU suite, smoke, the default bench line, bench.py under rocprofv3,
# and every roofline entry's kernel statistics and traffic (copied into
# profiles/r4 on the box before the bench line, which cross-checks them).
set -o pipefail
export RUN=${RUN:-r4final10}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
bash tools/gpu_step.sh \
 "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "smoke:120:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "kprof:900:bash tools/gpu_profiles.sh r4" \
 "cp:30:cp $R/gpurun_out/prof_r4/profiles/* $R/profiles/r4/" \
 "bench:500:python bench.py > $O/bench_line.json" \
 "bprof:700:bash tools/bench_profile.sh r4 --no-farm --no-cpu"
du -sh $O
