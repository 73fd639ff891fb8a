#!/bin/bash
# Round 4, call 20: two-column pass D as the default — the whole GPU suite,
# smoke, the default bench line, bench.py under rocprofv3, and the kron
# entries' kernel statistics and traffic.
set -o pipefail
export RUN=${RUN:-r4final9}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
bash tools/gpu_step.sh \
 "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "smoke:120:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "bench:500:python bench.py > $O/bench_line.json" \
 "bprof:700:bash tools/bench_profile.sh r4 --no-farm --no-cpu" \
 "kprof:400:bash tools/gpu_profiles.sh r4 kron_n28 kron_n28b kron_c4"
du -sh $O
