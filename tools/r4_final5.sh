#!/bin/bash
# Round 4 final measurement (after the eigensolver changes): the whole GPU
# suite, smoke, the default bench line, bench.py under rocprofv3, the serial
# sector stats and the per-part farm projection.
set -o pipefail
export RUN=${RUN:-r4final5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
bash tools/gpu_step.sh \
 "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "smoke:120:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "bench:500:python bench.py > $O/bench_line.json" \
 "serial:300:python3 $R/tools/farm_prof.py --reps 1 --serial-stats $O/farm_c4_serial_stats.json" \
 "scale:400:python3 $R/tools/farm_scale_probe.py --out $O/farm_scale_projection.json" \
 "bprof:700:bash tools/bench_profile.sh r4 --no-farm --no-cpu"
du -sh $O
